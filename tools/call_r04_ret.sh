#!/bin/bash
set -u
OUT=gpurun_out/r04_ret; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_scale.py tests/test_gpu_parity.py tests/test_tcp_substrate.py tests/test_gpu_async.py -k "host or gather or one_message or loopback or substrate or growth or latency" > $OUT/tests.log 2>&1 || { echo TESTFAIL; grep -E "FAILED|Error|assert" $OUT/tests.log | head -20; exit 1; }
tail -2 $OUT/tests.log
port=19300
for r in 1 2 3 4; do for c in gpu none; do
  port=$((port+1))
  timeout -k 10 120 ./tests/native/tcp_loopback --codec $c --count 1000 --batch 50 --port $port > $OUT/lb_${c}_$r.json 2> $OUT/lb_${c}_$r.err || { echo FAIL; cat $OUT/lb_${c}_$r.err; exit 1; }
  echo "$c $(python3 -c "import json; print(json.load(open('$OUT/lb_${c}_$r.json'))['effective_MBps'])")"
done; done
