#!/bin/bash
set -u
OUT=gpurun_out/r04_c4t; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c4 -o run -- python3 bench.py --workload c4 --steps 3 --warmup 2 --cpu-seconds 0 --compacted-steps 0 > $OUT/prof_c4.log 2>&1 || exit 1
python3 tools/c4_timeline.py $OUT/prof_c4
