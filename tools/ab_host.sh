#!/bin/bash
# Diagnostic A/B of the host pipeline: bench.py --host-inclusive over library variants, alternating.
# usage: bash tools/ab_host.sh <tag> <R> v1 v2 ...
set -u
TAG=$1; R=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for r in $(seq 1 $R); do
  for v in "$@"; do
    PSYNE_TDT_LIB=psyne_amd/libpsyne_tdt_x_$v.so timeout -k 10 300 python -u bench.py --host-inclusive --cpu-seconds 0 \
      --compacted-steps 0 --steps 3 > "$OUT/host_${v}_$r.log" 2>&1 || { echo "$v failed"; tail -5 "$OUT/host_${v}_$r.log"; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/host_${v}_$r.log').read().strip().splitlines()[-1]); h=d['host_inclusive']; print('$r $v', h['pinned'], h['pageable'], h['pageable_vs_pinned'])"
  done
done
