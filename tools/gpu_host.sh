#!/bin/bash
# Host-path pass: one-message / gather / substrate GPU tests, per-message latency rows, loopback
# rows (none / gpu / cpu) at C1's 1000 x 1 MiB.  usage (via gpurun): bash tools/gpu_host.sh <tag>
set -u
TAG=${1:-host}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "one_message or gather or protocol or cpp" tests/test_tcp_substrate.py > "$OUT/host_tests.log" 2>&1
rc=$?; tail -3 "$OUT/host_tests.log"; [ $rc -eq 0 ] || { echo "tests rc=$rc"; exit $rc; }
for c in none gpu cpu; do
  timeout -k 10 300 ./tests/native/tcp_loopback --codec $c --count 1000 --batch 50 --port $((18400 + ${#c})) \
    > "$OUT/loopback_$c.json" 2> "$OUT/loopback_$c.err"
  rc=$?; cat "$OUT/loopback_$c.json"; [ $rc -eq 0 ] || { echo "loopback $c rc=$rc"; tail "$OUT/loopback_$c.err"; exit $rc; }
done
timeout -k 10 400 python -u bench.py --latency --steps 3 --warmup 1 --cpu-seconds 0 --compacted-steps 0 --msgs 32768 > "$OUT/bench_latency.log" 2>&1
rc=$?; python3 -c "
import json,sys
l=[x for x in open('$OUT/bench_latency.log') if x.startswith('{')][-1]
for r in json.loads(l)['message_latency']['rows']: print(r)"; exit $rc
