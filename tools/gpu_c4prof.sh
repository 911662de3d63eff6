#!/bin/bash
# rocprofv3 kernel stats of the C4 and C2 benches (per message-class kernel).
set -u
TAG=${1:-c4prof}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for wl in c4 c2; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$wl" -o run -- \
    python3 bench.py --workload $wl --steps 3 --warmup 2 --cpu-seconds 0 --compacted-steps 0 > "$OUT/prof_$wl.log" 2>&1 || exit 1
  python3 tools/prof_summary.py "$OUT/prof_$wl" "$OUT/kernel_stats_$wl.md" "rocprofv3 --kernel-trace --stats: bench.py --workload $wl --steps 3 --warmup 2" > /dev/null
done
