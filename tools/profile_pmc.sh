#!/bin/bash
# PMC passes over bench.py (one rocprofv3 invocation per counter group, kernel-trace/stats
# only — never combined with sys/runtime traces).
# usage: tools/profile_pmc.sh <outdir> [bench args]   (writes <outdir>/summary.txt + traffic.json)
set -u
OUT=${1:-gpurun_out/pmc}; shift || true
ARGS=${@:-"--steps 1 --warmup 1 --cpu-seconds 0 --compacted-steps 0"}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # name counters...
  local name=$1; shift
  timeout -s KILL 240 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$name" -o "$name" -- python3 bench.py $ARGS > "$OUT/$name.log" 2>&1
  local rc=$?; echo "pass $name rc=$rc"; return $rc
}
run sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES && \
run sq2 SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM GRBM_GUI_ACTIVE && \
run fetch FETCH_SIZE && \
run write WRITE_SIZE && \
python3 tools/pmc_summary.py "$OUT" > "$OUT/summary.txt" && \
python3 tools/traffic_json.py "$OUT" "$OUT/traffic.json" "${PMC_KEY:-c3_262144x65536}" > /dev/null
