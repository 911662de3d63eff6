#!/bin/bash
# C4 bench under several PSYNE_TDT_LARGE_MIN thresholds (the tiled-path cutoff)
set -u
OUT=gpurun_out/${1:-envc4}; mkdir -p "$OUT"; shift
for lm in "$@"; do
  PSYNE_TDT_LARGE_MIN=$lm timeout -k 10 200 python -u bench.py --workload c4 --steps 3 --warmup 1 --cpu-seconds 0 > "$OUT/lm_$lm.log" 2>&1 || exit 1
  python3 -c "import json; d=json.loads(open('$OUT/lm_$lm.log').read().strip().splitlines()[-1]); print('large_min $lm', d['value'], d['kernels_ms'], d['roundtrip_ok'])"
done
