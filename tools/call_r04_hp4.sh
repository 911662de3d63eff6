#!/bin/bash
# Merged plan claims + four-slot host pipeline: full GPU tests, benches, host rates, memcpy, loopback.
set -u
bash tools/gpu_r04b.sh r04_hp4 tests || exit 1
OUT=gpurun_out/r04_hp4
timeout -k 10 120 ./tools/host_rate 8 16 32 50 64 > $OUT/host_rate.txt 2>&1 || { echo FAIL; cat $OUT/host_rate.txt; exit 1; }
cat $OUT/host_rate.txt
timeout -k 10 60 ./tools/membw > $OUT/membw.txt 2>&1; cat $OUT/membw.txt
bash tools/lb_diag3.sh r04_hp4/lb
