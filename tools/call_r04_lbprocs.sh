#!/bin/bash
# Loopback C1 with each end in its own process (--procs 2) beside the one-process rows.
set -u
OUT=gpurun_out/r04_lbprocs; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_tcp_substrate.py > $OUT/tests.log 2>&1 || { echo TESTFAIL; tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
port=19110
for r in 1 2 3; do for p in 1 2; do for c in gpu none; do
  port=$((port+1))
  timeout -k 10 150 ./tests/native/tcp_loopback --count 1000 --port $port --codec $c --batch 50 --procs $p > $OUT/lb_${c}_p${p}_$r.json 2> $OUT/lb_${c}_p${p}_$r.err || { echo FAIL; cat $OUT/lb_${c}_p${p}_$r.err; exit 1; }
  echo "$c procs=$p $(python3 -c "import json; d=json.load(open('$OUT/lb_${c}_p${p}_$r.json')); print(d['effective_MBps'], d['mismatches'])")"
done; done; done
