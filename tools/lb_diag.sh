#!/bin/bash
# Diagnostic: loopback gpu row by half (both / tx / rx), receive mode and batch size, 3 runs
# each (the box's loopback numbers vary run to run), beside the none row.
set -u
OUT=gpurun_out/${1:-r04_lb}; mkdir -p $OUT
port=18500
run() {  # name args...
  local name=$1; shift
  for r in 1 2 3; do
    port=$((port + 1))
    timeout -k 10 120 ./tests/native/tcp_loopback --count 1000 --port $port "$@" > $OUT/lb_${name}_$r.json 2>$OUT/lb_${name}_$r.err || { echo "FAIL $name"; cat $OUT/lb_${name}_$r.err; exit 1; }
    cat $OUT/lb_${name}_$r.json
  done
}
run none --codec none --batch 50
run gpu_views_50 --codec gpu --batch 50 --rx views
run gpu_views_200 --codec gpu --batch 200 --rx views
run gpu_copy_50 --codec gpu --batch 50 --rx copy
run gpu_tx_50 --codec gpu --batch 50 --half tx
run gpu_rx_views_50 --codec gpu --batch 50 --half rx --rx views
