#!/bin/bash
# Kernel + copy timeline of the loopback harness's receive half (pre-encoded frames, GPU decode).
set -u
OUT=gpurun_out/r04_lbtrace; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/rx -o run -- ./tests/native/tcp_loopback --count 1000 --port 18950 --codec gpu --batch 50 --half rx --rx views > $OUT/rx.log 2>&1 || { echo PFAIL; tail -20 $OUT/rx.log; exit 1; }
grep -E "harness|pipe" $OUT/rx.log
timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/both -o run -- ./tests/native/tcp_loopback --count 1000 --port 18951 --codec gpu --batch 50 --half both --rx views > $OUT/both.log 2>&1 || { echo PFAIL; tail -20 $OUT/both.log; exit 1; }
grep -E "harness|pipe" $OUT/both.log
