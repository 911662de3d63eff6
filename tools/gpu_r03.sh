#!/bin/bash
# Round-3 GPU pass: gpu tests -> C3 bench -> C2 / C4 benches (every step time-limited; stop at the
# first failure).  usage (via gpurun): bash tools/gpu_r03.sh <tag> [tests|notests]
set -u
TAG=${1:-r03}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ "${2:-tests}" = "tests" ]; then
  timeout -k 10 600 python -u -m pytest tests -x -v --timeout 180 --timeout-method thread -m gpu > "$OUT/gpu_tests.log" 2>&1
  rc=$?; tail -3 "$OUT/gpu_tests.log"; [ $rc -eq 0 ] || { echo "gpu tests rc=$rc"; exit $rc; }
fi
timeout -k 10 300 python -u bench.py --cpu-seconds 0 > "$OUT/bench.log" 2>&1
rc=$?; tail -c 600 "$OUT/bench.log"; echo; [ $rc -eq 0 ] || { echo "bench rc=$rc"; exit $rc; }
for w in c2 c4; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 5 --warmup 2 --cpu-seconds 0 > "$OUT/bench_$w.log" 2>&1
  rc=$?; tail -c 300 "$OUT/bench_$w.log"; echo; [ $rc -eq 0 ] || { echo "bench $w rc=$rc"; exit $rc; }
done
