#!/bin/bash
# C2 / C4 workload measurements (parity configs, not the headline line).
set -u
OUT=gpurun_out/${1:-wl}
mkdir -p "$OUT"
export TMPDIR=/tmp
for w in c2 c4; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 3 --warmup 1 --cpu-seconds 0 > "$OUT/bench_$w.log" 2>&1
  rc=$?; tail -1 "$OUT/bench_$w.log"; [ $rc -eq 0 ] || exit $rc
done
