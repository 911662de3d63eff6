#!/bin/bash
# Loopback C1 rows with the tensors in pageable vs pinned host memory (gpu codec both halves,
# and no codec), with the gpu pipeline's thread time split.
set -u
OUT=gpurun_out/${1:-r04_lb}; mkdir -p $OUT
port=18900
for row in "gpu pageable" "gpu pinned" "none pageable" "none pinned"; do
  set -- $row
  for r in 1 2 3; do
    port=$((port + 1))
    timeout -k 10 120 ./tests/native/tcp_loopback --count 1000 --port $port --codec $1 --batch 50 --mem $2 > $OUT/lb_$1_$2_$r.json 2> $OUT/lb_$1_$2_$r.err || { echo FAIL; cat $OUT/lb_$1_$2_$r.err; exit 1; }
    echo "$1 $2 $(python3 -c "import json; print(json.load(open('$OUT/lb_$1_$2_$r.json'))['effective_MBps'])") $(tail -1 $OUT/lb_$1_$2_$r.err)"
  done
done
