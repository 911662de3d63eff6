#!/bin/bash
# bench.py (timing only) per variant and workload: exp_run_wl.sh <tag> <workload> <variant>...
set -u
OUT=gpurun_out/${1:-exp}; W=$2; shift 2
mkdir -p "$OUT"
for v in "$@"; do
  PSYNE_TDT_LIB=psyne_amd/libpsyne_tdt_x_$v.so timeout -k 10 200 python -u bench.py --workload $W --steps 3 --warmup 1 --cpu-seconds 0 > "$OUT/${v}_$W.log" 2>&1
  rc=$?
  python3 -c "import json; d=json.loads(open('$OUT/${v}_$W.log').read().strip().splitlines()[-1]); print('$v $W', d['value'], d['kernels_ms'], d['roundtrip_ok'])" || { echo "$v failed rc=$rc"; tail -5 "$OUT/${v}_$W.log"; exit 1; }
done
