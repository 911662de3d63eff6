#!/bin/bash
# Diagnostic: loopback gpu row, both halves and each half alone, with the pipeline threads' time split.
set -u
OUT=gpurun_out/${1:-r04_lb}; mkdir -p $OUT
port=18800
for mode in "both views" "tx views" "rx views" "both copy"; do
  set -- $mode
  for r in 1 2; do
    port=$((port + 1))
    timeout -k 10 120 ./tests/native/tcp_loopback --count 1000 --port $port --codec gpu --batch 50 --half $1 --rx $2 > $OUT/lb_$1_$2_$r.json 2> $OUT/lb_$1_$2_$r.err || { echo FAIL; cat $OUT/lb_$1_$2_$r.err; exit 1; }
    echo "$1 $2 $(python3 -c "import json; print(json.load(open('$OUT/lb_$1_$2_$r.json'))['effective_MBps'])") $(tail -1 $OUT/lb_$1_$2_$r.err)"
  done
done
