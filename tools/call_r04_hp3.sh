#!/bin/bash
# Host pipeline timeline (four slots): tests not run by hp2, then a kernel + copy trace of 50-message calls.
set -u
OUT=gpurun_out/r04_hp3; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_parity.py -k "encode_host_gather or one_message_host_path" > $OUT/tests.log 2>&1 || { echo TESTFAIL; tail -30 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/trace -o run -- ./tools/host_rate 50 > $OUT/trace.log 2>&1 || { echo PFAIL; tail -20 $OUT/trace.log; exit 1; }
grep sub_msgs $OUT/trace.log
