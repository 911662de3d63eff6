#!/bin/bash
# One GPU-box pass: gpu tests -> bench (with CPU baseline) -> rocprofv3 kernel stats of the bench.
# usage (via gpurun): bash tools/gpu_round.sh <tag> [skip-tests]
set -u
TAG=${1:-run}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ "${2:-}" != "skip-tests" ]; then
  timeout -k 10 420 python -u -m pytest tests -x -v --timeout 120 --timeout-method thread -m gpu > "$OUT/gpu_tests.log" 2>&1
  rc=$?; tail -3 "$OUT/gpu_tests.log"; [ $rc -eq 0 ] || { echo "gpu tests rc=$rc"; exit $rc; }
fi
timeout -k 10 300 python -u bench.py > "$OUT/bench.log" 2>&1
rc=$?; tail -1 "$OUT/bench.log"; [ $rc -eq 0 ] || { echo "bench rc=$rc"; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
  python3 bench.py --steps 5 --warmup 2 --cpu-seconds 0 > "$OUT/prof_bench.log" 2>&1
rc=$?; tail -1 "$OUT/prof_bench.log"; [ $rc -eq 0 ] || { echo "rocprof rc=$rc"; exit $rc; }
python3 tools/prof_summary.py "$OUT/prof" "$OUT/kernel_stats.md" "rocprofv3 --kernel-trace --stats: bench.py --steps 5 --warmup 2 ($TAG)"
