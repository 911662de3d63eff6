#!/bin/bash
# Full measurement of one library build on a GPU box (everything a bench line cites):
#   -m gpu suite, smoke(), C3 bench with the four CPU-baseline rows, rocprofv3 kernel stats of
#   the same bench, FETCH/WRITE + SQ PMC passes (traffic JSON keyed to the library hash),
#   C2 / C4 benches, the host-inclusive leg with the PCIe ceiling, loopback TCP rows.
# usage (via gpurun): bash tools/gpu_final.sh <tag>
set -u
TAG=${1:-final}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "== $1"; }
step tests
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
rc=$?; tail -2 "$OUT/gpu_tests.log"; [ $rc -eq 0 ] || exit $rc
step smoke
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; tail -1 "$OUT/smoke.log"; [ $rc -eq 0 ] || exit $rc
step bench_c3
timeout -k 10 400 python -u bench.py > "$OUT/bench.log" 2>&1
rc=$?; tail -1 "$OUT/bench.log" | cut -c1-400; [ $rc -eq 0 ] || exit $rc
step rocprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
  python3 bench.py --steps 5 --warmup 2 --cpu-seconds 0 --compacted-steps 0 > "$OUT/prof_bench.log" 2>&1
rc=$?; [ $rc -eq 0 ] || exit $rc
python3 tools/prof_summary.py "$OUT/prof" "$OUT/kernel_stats.md" "rocprofv3 --kernel-trace --stats: bench.py --steps 5 --warmup 2 ($TAG)" --steady 5 > /dev/null
step pmc
bash tools/profile_pmc.sh "$OUT/pmc" || exit 1
step pmc_c2_c4
PMC_KEY=c2_1048576x1024 bash tools/profile_pmc.sh "$OUT/pmc_c2" --workload c2 --steps 1 --warmup 1 --cpu-seconds 0 --compacted-steps 0 || exit 1
PMC_KEY=c4_4194304x65536 bash tools/profile_pmc.sh "$OUT/pmc_c4" --workload c4 --steps 1 --warmup 1 --cpu-seconds 0 --compacted-steps 0 || exit 1
step c2_c4
for wl in c2 c4; do
  timeout -k 10 400 python -u bench.py --workload $wl --steps 5 --warmup 2 --cpu-seconds 0 > "$OUT/bench_$wl.log" 2>&1
  rc=$?; tail -1 "$OUT/bench_$wl.log" | cut -c1-200; [ $rc -eq 0 ] || exit $rc
done
step extras
bash tools/gpu_extras.sh "$TAG/extras" > "$OUT/extras.log" 2>&1
rc=$?; tail -3 "$OUT/extras.log"; exit $rc
