#!/bin/bash
# PMC A/B of library variants (psyne_amd/libpsyne_tdt_x_<v>.so): two counter passes per variant
# over a short bench.py run (kernel-trace style counters only), summarised per kernel.
# usage (via gpurun): bash tools/pmc_ab2.sh <tag> "<bench args>" v1 v2 ...
set -u
TAG=$1; shift; ARGS=$1; shift
OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
[ -f "$OUT/avail.txt" ] || timeout -k 5 60 rocprofv3 -L > "$OUT/avail.txt" 2>&1 || true
for v in "$@"; do
  for pass in ${PASSES:-a b}; do
    if [ $pass = a ]; then C="SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
    else C="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_WAVES SQ_ACTIVE_INST_SCA"; fi
    PSYNE_TDT_LIB=psyne_amd/libpsyne_tdt_x_$v.so timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d "$OUT/$v$pass" -o $v -- python3 bench.py $ARGS > "$OUT/$v$pass.log" 2>&1 || { echo "$v pass $pass failed"; tail -5 "$OUT/$v$pass.log"; exit 1; }
  done
  python3 tools/pmc_summary.py "$OUT/${v}a" > "$OUT/$v.txt"; [ -d "$OUT/${v}b" ] && python3 tools/pmc_summary.py "$OUT/${v}b" >> "$OUT/$v.txt"
  echo "== $v"; grep -A22 "tdt_encode_kernel<4, 512, 8, 0, 0, 0, 0, 1>" "$OUT/$v.txt" | grep -E "SQ_|GRBM|_dur" | sort -u
done
