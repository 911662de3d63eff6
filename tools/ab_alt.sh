#!/bin/bash
# Diagnostic A/B: alternate bench.py runs over library variants (psyne_amd/libpsyne_tdt_x_<v>.so),
# R rounds, so box drift hits every variant alike.  usage: bash tools/ab_alt.sh <tag> <R> <workload> v1 v2 ...
set -u
TAG=$1; R=$2; WL=$3; shift 3
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for r in $(seq 1 $R); do
  for v in "$@"; do
    PSYNE_TDT_LIB=psyne_amd/libpsyne_tdt_x_$v.so timeout -k 10 150 python -u bench.py --workload $WL --steps 10 --warmup 2 \
      --cpu-seconds 0 --compacted-steps 0 > "$OUT/${v}_$r.log" 2>&1
    rc=$?
    python3 -c "import json; d=json.loads(open('$OUT/${v}_$r.log').read().strip().splitlines()[-1]); print('$r $v', d['value'], d['kernels_ms'], d['roundtrip_ok'])" || { echo "$v failed rc=$rc"; tail -5 "$OUT/${v}_$r.log"; exit 1; }
  done
done
