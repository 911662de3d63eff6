#!/bin/bash
# A/B: non-temporal stores / loads in the passthrough-copy and compaction-gather helpers.
set -u
OUT=gpurun_out/r04_cpnt; mkdir -p $OUT
export TMPDIR=/tmp
for wl in c4 c2; do for r in 1 2; do for v in base2 cs csl; do
  PSYNE_TDT_LIB=psyne_amd/libpsyne_tdt_x_$v.so timeout -k 10 200 python -u bench.py --workload $wl --steps 5 --warmup 2 \
    --cpu-seconds 0 --compacted-steps 3 > $OUT/${wl}_${v}_$r.log 2>&1 || { echo "$v failed"; tail -5 $OUT/${wl}_${v}_$r.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/${wl}_${v}_$r.log').read().strip().splitlines()[-1]); c=d['compacted']; print('$wl $r $v', d['value'], d['kernels_ms'], 'compacted', c['GiBps_kernels'], c['encode_ms'], c['decode_ms'], d['roundtrip_ok'], c['roundtrip_ok'])"
done; done; done
