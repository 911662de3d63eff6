#!/bin/bash
# Repeat the default C3 bench (no CPU leg) on one box: the spread of the headline for one build.
set -u
OUT=gpurun_out/r04_rep; mkdir -p $OUT
export TMPDIR=/tmp
for r in 1 2 3 4; do
  timeout -k 10 200 python -u bench.py --cpu-seconds 0 --compacted-steps 0 > $OUT/c3_$r.log 2>&1 || { echo "run $r failed"; tail -5 $OUT/c3_$r.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/c3_$r.log').read().strip().splitlines()[-1]); print($r, d['value'], d['kernels_ms'], d['roofline']['frac'], d['lib_sha256'])"
done
