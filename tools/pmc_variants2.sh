#!/bin/bash
# Diagnostic: instruction counts + kernel time of library variants (psyne_amd/libpsyne_tdt_x_<v>.so)
# on a quarter-C3 batch; one rocprofv3 --pmc run per variant.  usage: bash tools/pmc_variants2.sh <tag> v1 v2 ...
set -u
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
for v in "$@"; do
  PSYNE_TDT_LIB=psyne_amd/libpsyne_tdt_x_$v.so timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_WR --output-format csv -d "$OUT/$v" -o $v -- python3 bench.py --msgs 65536 --steps 1 --warmup 1 --cpu-seconds 0 > "$OUT/$v.log" 2>&1 || { echo "$v failed"; tail -5 "$OUT/$v.log"; exit 1; }
  echo "== $v"; python3 tools/pmc_summary.py "$OUT/$v" | grep -A12 "encode_kernel<4, 512, 8, 0, 0, 0>"
done
