#!/bin/bash
# SQ counter pass per diagnostic library variant for one workload.
# usage (GPU box): tools/pmc_variants_wl.sh <outdir> <workload> v1 v2 ...   (variant "main" = psyne_amd/libpsyne_tdt.so)
set -u
OUT=$1; WL=$2; shift 2
mkdir -p "$OUT"
export TMPDIR=/tmp
for v in "$@"; do
  lib=psyne_amd/libpsyne_tdt_x_$v.so
  [ "$v" = main ] && lib=psyne_amd/libpsyne_tdt.so
  PSYNE_TDT_LIB=$lib timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS \
    SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d "$OUT/$v" -o "$v" -- \
    python3 bench.py --workload $WL --steps 1 --warmup 1 --cpu-seconds 0 --compacted-steps 0 > "$OUT/$v.log" 2>&1
  rc=$?; echo "pass $v rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 tools/pmc_summary.py "$OUT/$v" > "$OUT/$v.txt"
done
