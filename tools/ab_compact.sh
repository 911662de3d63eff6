#!/bin/bash
# Diagnostic A/B of the compacted API leg (tdt_encode_batch / tdt_decode_batch) over library
# variants.  usage: bash tools/ab_compact.sh <tag> <R> <workload> v1 v2 ...
set -u
TAG=$1; R=$2; WL=$3; shift 3
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for r in $(seq 1 $R); do
  for v in "$@"; do
    PSYNE_TDT_LIB=psyne_amd/libpsyne_tdt_x_$v.so timeout -k 10 200 python -u bench.py --workload $WL --steps 2 --warmup 1 \
      --cpu-seconds 0 --compacted-steps 5 > "$OUT/c_${v}_$r.log" 2>&1
    rc=$?
    python3 -c "import json; d=json.loads(open('$OUT/c_${v}_$r.log').read().strip().splitlines()[-1]); c=d['compacted']; print('$r $v slotted', d['kernels_ms'], 'compacted', c['encode_ms'], c['decode_ms'], c['GiBps_kernels'], c['roundtrip_ok'])" || { echo "$v failed rc=$rc"; tail -5 "$OUT/c_${v}_$r.log"; exit 1; }
  done
done
