#!/bin/bash
set -u
OUT=gpurun_out/r04_hc8; mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -x -q --timeout 900 --timeout-method thread -m gpu > $OUT/gpu_tests.log 2>&1; rc=$?; tail -2 $OUT/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $OUT/gpu_tests.log | head; exit $rc; }
for r in 1 2 3; do bash tools/exp_run_wl.sh r04_hc8 c3 base hc8 || exit 1; done
for r in 1 2; do bash tools/exp_run_wl.sh r04_hc8 c4 base hc8 || exit 1; done
