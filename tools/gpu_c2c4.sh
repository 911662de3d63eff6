#!/bin/bash
# C2 / C4 workloads (timing) + one SQ counter pass over C2.
# usage (via gpurun): bash tools/gpu_c2c4.sh <tag>
set -u
OUT=gpurun_out/$1
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --workload c2 --steps 5 --warmup 2 --cpu-seconds 0 > "$OUT/bench_c2.log" 2>&1
rc=$?; tail -c 1200 "$OUT/bench_c2.log"; echo; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --workload c4 --steps 3 --warmup 1 --cpu-seconds 0 > "$OUT/bench_c4.log" 2>&1
rc=$?; tail -c 1200 "$OUT/bench_c4.log"; echo; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_WAVES GRBM_GUI_ACTIVE \
  --output-format csv -d "$OUT/pmc_c2" -o c2 -- python3 bench.py --workload c2 --steps 1 --warmup 1 --cpu-seconds 0 > "$OUT/pmc_c2.log" 2>&1
rc=$?; echo "pmc rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 tools/pmc_summary.py "$OUT/pmc_c2" > "$OUT/pmc_c2.txt"; cat "$OUT/pmc_c2.txt"
