#!/bin/bash
# Diagnostic A/B: alternate bench.py runs of one library under environment settings (e.g. the
# context knobs PSYNE_TDT_LARGE_MIN / PSYNE_TDT_NO_SIDE), R rounds.
# usage: bash tools/ab_env.sh <tag> <R> <workload> <lib variant|main> "ENV=V ..." "ENV=V ..." ...
set -u
TAG=$1; R=$2; WL=$3; V=$4; shift 4
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
lib=psyne_amd/libpsyne_tdt_x_$V.so
[ "$V" = main ] && lib=psyne_amd/libpsyne_tdt.so
for r in $(seq 1 $R); do
  i=0
  for e in "$@"; do
    i=$((i+1))
    env $e PSYNE_TDT_LIB=$lib timeout -k 10 150 python -u bench.py --workload $WL --steps 10 --warmup 2 \
      --cpu-seconds 0 --compacted-steps 0 > "$OUT/e${i}_$r.log" 2>&1
    rc=$?
    python3 -c "import json; d=json.loads(open('$OUT/e${i}_$r.log').read().strip().splitlines()[-1]); print('$r [$e]', d['value'], d['kernels_ms'], d['roundtrip_ok'])" || { echo "[$e] failed rc=$rc"; tail -5 "$OUT/e${i}_$r.log"; exit 1; }
  done
done
