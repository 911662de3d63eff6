#!/bin/bash
# Round-4 final pass, part A (one library build): smoke(), the C3 bench with the all-core CPU
# baseline, rocprofv3 kernel stats of the same bench, C2 / C4 / C5 benches, host-inclusive and
# per-message latency legs.  Every step time-limited; stop at the first failure.
# usage (via gpurun): bash tools/gpu_r04_final_a.sh <tag> [tests]
set -u
TAG=${1:-r04_final}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "== $1"; }
if [ "${2:-}" = "tests" ]; then
  step tests
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
  rc=$?; tail -2 "$OUT/gpu_tests.log"; [ $rc -eq 0 ] || exit $rc
fi
step smoke
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; tail -1 "$OUT/smoke.log"; [ $rc -eq 0 ] || exit $rc
step bench_c3
timeout -k 10 400 python -u bench.py > "$OUT/bench.log" 2>&1
rc=$?; tail -1 "$OUT/bench.log" | cut -c1-300; [ $rc -eq 0 ] || exit $rc
step rocprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
  python3 bench.py --steps 5 --warmup 2 --cpu-seconds 0 --compacted-steps 3 > "$OUT/prof_bench.log" 2>&1
rc=$?; [ $rc -eq 0 ] || exit $rc
python3 tools/prof_summary.py "$OUT/prof" "$OUT/kernel_stats.md" "rocprofv3 --kernel-trace --stats: bench.py --steps 5 --warmup 2 --compacted-steps 3 ($TAG)" --steady 5 > /dev/null
for wl in c2 c4 c5; do
  step bench_$wl
  timeout -k 10 400 python -u bench.py --workload $wl --steps 5 --warmup 2 --cpu-seconds 0 > "$OUT/bench_$wl.log" 2>&1
  rc=$?; tail -1 "$OUT/bench_$wl.log" | cut -c1-200; [ $rc -eq 0 ] || exit $rc
done
step host_latency
timeout -k 10 400 python -u bench.py --host-inclusive --latency --cpu-seconds 0 --steps 3 --warmup 1 > "$OUT/bench_host.log" 2>&1
rc=$?; tail -1 "$OUT/bench_host.log" | cut -c1-200; exit $rc
