#!/bin/bash
# One SQ counter pass over bench.py (encode+decode, timing only) per diagnostic library variant
# (tools/exp_build.sh builds psyne_amd/libpsyne_tdt_x_<name>.so; "base" = the shipped library).
# usage (GPU box): tools/pmc_variants.sh <outdir> base nohist ...
set -u
OUT=${1:-gpurun_out/pmcv}; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
for v in "$@"; do
  lib=psyne_amd/libpsyne_tdt.so
  [ "$v" = base ] || lib=psyne_amd/libpsyne_tdt_x_$v.so
  PSYNE_TDT_LIB=$lib timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS \
    SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d "$OUT/$v" -o "$v" -- \
    python3 bench.py --steps 1 --warmup 1 --cpu-seconds 0 > "$OUT/$v.log" 2>&1
  rc=$?; echo "pass $v rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 tools/pmc_summary.py "$OUT/$v" > "$OUT/$v.txt"
done
