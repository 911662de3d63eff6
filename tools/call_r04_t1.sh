#!/bin/bash
set -u
OUT=gpurun_out/r04_t1; mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -x -v --timeout 900 --timeout-method thread -m gpu > $OUT/gpu_tests.log 2>&1; rc=$?; tail -3 $OUT/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $OUT/gpu_tests.log | head; exit $rc; }
bash tools/ab_env.sh r04_t1 3 c3 main "X=0"
