#!/bin/bash
# Diagnostic: loopback gpu row vs the copy-pool size (PSYNE_TDT_COPY_THREADS) and the box's CPU quota.
set -u
OUT=gpurun_out/${1:-r04_lb}; mkdir -p $OUT
cat /sys/fs/cgroup/cpu.max 2>/dev/null; nproc; python3 -c "import os; print(len(os.sched_getaffinity(0)))"
port=18700
for ct in 2 4 8 16; do
  for r in 1 2; do
    port=$((port + 1))
    PSYNE_TDT_COPY_THREADS=$ct timeout -k 10 120 ./tests/native/tcp_loopback --count 1000 --port $port --codec gpu --batch 50 > $OUT/lb_ct${ct}_$r.json 2>&1 || { echo FAIL; exit 1; }
    echo "ct=$ct $(cat $OUT/lb_ct${ct}_$r.json)"
  done
done
