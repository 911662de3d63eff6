#!/bin/bash
# Full measurement of one library build on a GPU box (everything a bench line cites):
#   -m gpu suite, smoke(), C3 bench with the four CPU-baseline rows, rocprofv3 kernel stats of
#   the same bench, FETCH/WRITE + SQ PMC passes (traffic JSON keyed to the library hash),
#   C2 / C4 benches, the host-inclusive leg with the PCIe ceiling, loopback TCP rows.
# usage (via gpurun): bash tools/gpu_final.sh <tag> [phase ...]
#   phases (default: all, in this order): tests smoke bench rocprof pmc pmc_c2_c4 c2_c4 extras
set -u
TAG=${1:-final}; shift
PHASES=" ${*:-tests smoke bench rocprof pmc pmc_c2_c4 c2_c4 extras} "
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
on() { [[ $PHASES == *" $1 "* ]] && echo "== $1"; }
if on tests; then
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
rc=$?; tail -2 "$OUT/gpu_tests.log"; [ $rc -eq 0 ] || exit $rc
fi
if on smoke; then
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; tail -1 "$OUT/smoke.log"; [ $rc -eq 0 ] || exit $rc
fi
if on bench; then
timeout -k 10 400 python -u bench.py > "$OUT/bench.log" 2>&1
rc=$?; tail -1 "$OUT/bench.log" | cut -c1-400; [ $rc -eq 0 ] || exit $rc
fi
if on rocprof; then
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
  python3 bench.py --steps 5 --warmup 2 --cpu-seconds 0 --compacted-steps 0 > "$OUT/prof_bench.log" 2>&1
rc=$?; [ $rc -eq 0 ] || exit $rc
python3 tools/prof_summary.py "$OUT/prof" "$OUT/kernel_stats.md" "rocprofv3 --kernel-trace --stats: bench.py --steps 5 --warmup 2 ($TAG)" --steady 5 > /dev/null
fi
if on pmc; then
bash tools/profile_pmc.sh "$OUT/pmc" || exit 1
fi
if on pmc_c2_c4; then
PMC_KEY=c2_1048576x1024 bash tools/profile_pmc.sh "$OUT/pmc_c2" --workload c2 --steps 1 --warmup 1 --cpu-seconds 0 --compacted-steps 0 || exit 1
PMC_KEY=c4_4194304x65536 bash tools/profile_pmc.sh "$OUT/pmc_c4" --workload c4 --steps 1 --warmup 1 --cpu-seconds 0 --compacted-steps 0 || exit 1
fi
if on c2_c4; then
for wl in c2 c4; do
  timeout -k 10 400 python -u bench.py --workload $wl --steps 5 --warmup 2 --cpu-seconds 0 > "$OUT/bench_$wl.log" 2>&1
  rc=$?; tail -1 "$OUT/bench_$wl.log" | cut -c1-200; [ $rc -eq 0 ] || exit $rc
done
fi
if on extras; then
bash tools/gpu_extras.sh "$TAG/extras" > "$OUT/extras.log" 2>&1
rc=$?; tail -3 "$OUT/extras.log"; [ $rc -eq 0 ] || exit $rc
fi
