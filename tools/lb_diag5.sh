#!/bin/bash
# Loopback gpu row (both halves) under hardware-queue / side-stream settings: the two codec
# contexts of the one-process harness share HIP's hardware queues (GPU_MAX_HW_QUEUES, default 4).
set -u
OUT=gpurun_out/${1:-r04_lb}; mkdir -p $OUT
port=18960
i=0
for e in "X=0" "GPU_MAX_HW_QUEUES=8" "GPU_MAX_HW_QUEUES=16" "PSYNE_TDT_NO_SIDE=1" "GPU_MAX_HW_QUEUES=16 PSYNE_TDT_NO_SIDE=1"; do
  i=$((i+1))
  for r in 1 2; do
    port=$((port + 1))
    env $e timeout -k 10 120 ./tests/native/tcp_loopback --count 1000 --port $port --codec gpu --batch 50 > $OUT/lb_e${i}_$r.json 2> $OUT/lb_e${i}_$r.err || { echo FAIL; cat $OUT/lb_e${i}_$r.err; exit 1; }
    echo "[$e] $(python3 -c "import json; print(json.load(open('$OUT/lb_e${i}_$r.json'))['effective_MBps'])") $(tail -1 $OUT/lb_e${i}_$r.err | cut -c1-200)"
  done
done
