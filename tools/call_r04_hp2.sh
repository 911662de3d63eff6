#!/bin/bash
# Host pipeline (four slots, slotted encode for long messages): host-path GPU tests, rates, loopback.
set -u
OUT=gpurun_out/r04_hp2; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_scale.py -k "host_pipeline" tests/test_gpu_parity.py::test_encode_host_gather tests/test_gpu_parity.py::test_one_message_host_path > $OUT/tests.log 2>&1 || { echo TESTFAIL; tail -30 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
timeout -k 10 120 ./tools/host_rate 8 16 32 50 64 > $OUT/host_rate.txt 2>&1 || { echo FAIL; cat $OUT/host_rate.txt; exit 1; }
cat $OUT/host_rate.txt
bash tools/lb_diag3.sh r04_hp2/lb
