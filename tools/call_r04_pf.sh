#!/bin/bash
set -u
OUT=gpurun_out/r04_pf; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_large.py tests/test_gpu_scale.py tests/test_gpu_parity.py -k "large or c4 or tile or runs or zipf or stream or unaligned" > $OUT/tests.log 2>&1 || { echo TESTFAIL; grep -E "FAILED|Error|assert" $OUT/tests.log | head -20; tail -5 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for r in 1 2 3; do bash tools/exp_run_wl.sh r04_pf c4 base pf4 || exit 1; done
