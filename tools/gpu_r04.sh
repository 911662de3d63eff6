#!/bin/bash
# Round-4 GPU pass: gpu tests -> C3 bench (with the all-cores CPU baseline) -> reference C1 row
# + loopback rows.  Every step time-limited; stop at the first failure.
# usage (via gpurun): bash tools/gpu_r04.sh <tag> [tests|notests] [extras|noextras]
set -u
TAG=${1:-r04}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ "${2:-tests}" = "tests" ]; then
  timeout -k 10 1000 python -u -m pytest tests -x -v --timeout 900 --timeout-method thread -m gpu > "$OUT/gpu_tests.log" 2>&1
  rc=$?; tail -3 "$OUT/gpu_tests.log"; [ $rc -eq 0 ] || { echo "gpu tests rc=$rc"; exit $rc; }
fi
timeout -k 10 400 python -u bench.py > "$OUT/bench.log" 2>&1
rc=$?; tail -c 800 "$OUT/bench.log"; echo; [ $rc -eq 0 ] || { echo "bench rc=$rc"; exit $rc; }
if [ "${3:-extras}" = "extras" ]; then
  bash tools/ref_tcp_bench.sh "$OUT" || { echo "ref tcp rc=$?"; exit 1; }
  for c in none gpu cpu; do
    timeout -k 10 300 ./tests/native/tcp_loopback --codec $c --count 1000 --batch 50 --port $((18300 + ${#c})) \
      > "$OUT/loopback_$c.json" 2> "$OUT/loopback_$c.err"
    rc=$?; cat "$OUT/loopback_$c.json"; [ $rc -eq 0 ] || { echo "loopback $c rc=$rc"; exit $rc; }
  done
fi
