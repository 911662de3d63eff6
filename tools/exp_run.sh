#!/bin/bash
# Run bench.py (timing only) against each diagnostic library variant.
set -u
OUT=gpurun_out/${1:-exp}; shift
mkdir -p "$OUT"
for v in "$@"; do
  PSYNE_TDT_LIB=psyne_amd/libpsyne_tdt_x_$v.so timeout -k 10 120 python -u bench.py --steps 3 --warmup 1 --cpu-seconds 0 > "$OUT/$v.log" 2>&1
  rc=$?
  python3 -c "import json,sys; d=json.loads(open('$OUT/$v.log').read().strip().splitlines()[-1]); print('$v', d['kernels_ms'], d['roundtrip_ok'])" || { echo "$v failed rc=$rc"; tail -5 "$OUT/$v.log"; exit 1; }
done
