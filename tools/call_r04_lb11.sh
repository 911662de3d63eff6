#!/bin/bash
set -u
OUT=gpurun_out/r04_lb11; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_parity.py -k "encode_host_gather" tests/test_gpu_scale.py::test_host_pipeline_slotted_pinned > $OUT/tests.log 2>&1 || { echo TESTFAIL; tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
bash tools/lb_diag4.sh r04_lb11
