#!/bin/bash
# Loopback gpu row: the harness's own GPU_MAX_HW_QUEUES=8 vs HIP's default 4 (set explicitly).
set -u
OUT=gpurun_out/${1:-r04_lb}; mkdir -p $OUT
port=19100
for r in 1 2 3; do
  for e in "X=0" "GPU_MAX_HW_QUEUES=4"; do
    port=$((port + 1))
    env $e timeout -k 10 120 ./tests/native/tcp_loopback --count 1000 --port $port --codec gpu --batch 50 > $OUT/lb_${r}_${e%%=*}.json 2> $OUT/lb_${r}_${e%%=*}.err || { echo FAIL; cat $OUT/lb_${r}_${e%%=*}.err; exit 1; }
    echo "[$e] $(python3 -c "import json; print(json.load(open('$OUT/lb_${r}_${e%%=*}.json'))['effective_MBps'])")"
  done
  port=$((port + 1))
  timeout -k 10 120 ./tests/native/tcp_loopback --count 1000 --port $port --codec none > $OUT/lb_${r}_none.json 2>/dev/null && echo "[none] $(python3 -c "import json; print(json.load(open('$OUT/lb_${r}_none.json'))['effective_MBps'])")"
done
