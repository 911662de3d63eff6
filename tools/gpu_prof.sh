#!/bin/bash
# Profile pass of the current library: rocprofv3 kernel stats of a C3 bench + PMC passes (one
# rocprofv3 run per counter group) + traffic.json keyed to the library hash.
# usage (via gpurun): bash tools/gpu_prof.sh <tag> [workload]
set -u
TAG=$1; WL=${2:-c3}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
  python3 bench.py --workload $WL --steps 5 --warmup 2 --cpu-seconds 0 --compacted-steps 0 > "$OUT/prof_bench.log" 2>&1
rc=$?; tail -c 400 "$OUT/prof_bench.log"; echo; [ $rc -eq 0 ] || { echo "rocprof rc=$rc"; exit $rc; }
python3 tools/prof_summary.py "$OUT/prof" "$OUT/kernel_stats.md" "rocprofv3 --kernel-trace --stats: bench.py --workload $WL --steps 5 --warmup 2 ($TAG)"
case $WL in c2) KEY=c2_1048576x1024;; c4) KEY=c4;; *) KEY=c3_262144x65536;; esac
PMC_KEY=$KEY bash tools/profile_pmc.sh "$OUT/pmc" --workload $WL --steps 1 --warmup 1 --cpu-seconds 0 --compacted-steps 0
rc=$?; cat "$OUT/pmc/summary.txt" 2>/dev/null | head -40; exit $rc
