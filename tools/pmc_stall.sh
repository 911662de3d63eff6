#!/bin/bash
# Diagnostic PMC passes (I-cache, issue stalls, LDS) of the C3 encode/decode kernels, one rocprofv3
# run per counter group; summaries via tools/pmc_summary.py.  usage: bash tools/pmc_stall.sh <tag>
set -u
OUT=gpurun_out/${1:-pmc_stall}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {
  timeout -s KILL 120 rocprofv3 --pmc $2 --output-format csv -d "$OUT/$1" -o $1 -- python3 bench.py --msgs 65536 --steps 1 --warmup 1 --cpu-seconds 0 > "$OUT/$1.log" 2>&1
}
run a "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE" && \
run b "SQ_IFETCH SQ_WAIT_INST_ANY SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_INSTS_VALU" && \
run c "SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_BUSY_CYCLES" && \
python3 tools/pmc_summary.py "$OUT" > "$OUT/summary.txt" 2>&1
