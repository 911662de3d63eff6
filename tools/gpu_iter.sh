#!/bin/bash
# One GPU iteration: the -m gpu suite, then C3 / C2 / C4 benches and the size sweep.
# usage (via gpurun): bash tools/gpu_iter.sh <tag> [skip-tests]
set -u
OUT=gpurun_out/$1
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ "${2:-}" != "skip-tests" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
  rc=$?; tail -4 "$OUT/gpu_tests.log"; [ $rc -eq 0 ] || exit $rc
fi
for wl in c3 c2 c4; do
  timeout -k 10 400 python -u bench.py --workload $wl --steps 5 --warmup 2 --cpu-seconds 0 > "$OUT/bench_$wl.log" 2>&1
  rc=$?; python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['kernels_ms'], d['roundtrip_ok'])" "$OUT/bench_$wl.log" $wl || tail -5 "$OUT/bench_$wl.log"
  [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python -u tools/size_sweep.py > "$OUT/sweep.log" 2>&1
rc=$?; grep msg_bytes "$OUT/sweep.log"; exit $rc
