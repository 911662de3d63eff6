#!/bin/bash
# Round-4 kernel pass: full GPU tests -> C3 / C4 / C2 benches (no CPU baseline), each step
# time-limited; stop at the first failure.  usage (via gpurun): bash tools/gpu_r04b.sh <tag> [tests|notests]
set -u
TAG=${1:-r04b}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ "${2:-tests}" = "tests" ]; then
  timeout -k 10 1000 python -u -m pytest tests -x -v --timeout 900 --timeout-method thread -m gpu > "$OUT/gpu_tests.log" 2>&1
  rc=$?; tail -3 "$OUT/gpu_tests.log"; [ $rc -eq 0 ] || { echo "gpu tests rc=$rc"; grep -E "FAILED|Error" "$OUT/gpu_tests.log" | head; exit $rc; }
fi
for w in c3 c4 c2; do
  timeout -k 10 300 python -u bench.py --workload $w --cpu-seconds 0 > "$OUT/bench_$w.log" 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "bench $w rc=$rc"; tail -5 "$OUT/bench_$w.log"; exit $rc; }
  python3 -c "
import json
l=[x for x in open('$OUT/bench_$w.log') if x.startswith('{')][-1]; d=json.loads(l)
print('$w', d['value'], d['kernels_ms'], d['roofline']['frac'], d.get('compacted',{}).get('GiBps_kernels'))"
done
