#!/bin/bash
set -u
OUT=gpurun_out/r04_lb13; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_scale.py -k "host_pipeline" > $OUT/tests.log 2>&1 || { echo TESTFAIL; tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 120 ./tools/host_rate 16 50 > $OUT/host_rate.txt 2>&1 && cat $OUT/host_rate.txt
port=19010
for r in 1 2 3; do for c in gpu none; do
  port=$((port+1))
  timeout -k 10 120 ./tests/native/tcp_loopback --count 1000 --port $port --codec $c --batch 50 > $OUT/lb_${c}_$r.json 2> $OUT/lb_${c}_$r.err || { echo FAIL; cat $OUT/lb_${c}_$r.err; exit 1; }
  echo "$c $(python3 -c "import json; print(json.load(open('$OUT/lb_${c}_$r.json'))['effective_MBps'])")"
done; done
