#!/bin/bash
# Diagnostic: host pipeline call rates (tools/host_rate) and a kernel + memory-copy timeline of
# 50-message calls under rocprofv3.
set -u
OUT=gpurun_out/${1:-r04_hp}; mkdir -p $OUT
timeout -k 10 120 ./tools/host_rate 8 16 32 50 64 > $OUT/host_rate.txt 2>&1 || { echo FAIL; cat $OUT/host_rate.txt; exit 1; }
cat $OUT/host_rate.txt
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/trace -o run -- ./tools/host_rate 50 > $OUT/trace.log 2>&1 || { echo PFAIL; tail -20 $OUT/trace.log; exit 1; }
find $OUT/trace -name "*.csv" | head
