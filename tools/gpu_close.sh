#!/bin/bash
# Round closure run on one library build: full -m gpu suite, smoke, C3 bench with the per-message
# latency rows, the host-inclusive leg, loopback TCP rows (each step time-limited; stop at the
# first failure).  usage (via gpurun): bash tools/gpu_close.sh <tag>
set -u
TAG=${1:-close}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
rc=$?; tail -2 "$OUT/gpu_tests.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; tail -1 "$OUT/smoke.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --latency --cpu-seconds 0 --compacted-steps 0 > "$OUT/bench_latency.log" 2>&1
rc=$?; tail -c 300 "$OUT/bench_latency.log"; echo; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_extras.sh "$TAG/extras" > "$OUT/extras.log" 2>&1
rc=$?; tail -4 "$OUT/extras.log"; exit $rc
