#!/bin/bash
set -u
OUT=gpurun_out/r04_lbres; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_compact.py tests/test_gpu_parity.py -k "compact or lookback or tiny" > $OUT/tests.log 2>&1 || { echo TESTFAIL; grep -E "FAILED|Error|assert" $OUT/tests.log | head -20; tail -5 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for r in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --cpu-seconds 0 --compacted-steps 5 > $OUT/b$r.log 2>&1 || exit 1
  python3 -c "import json; d=json.loads([l for l in open('$OUT/b$r.log') if l.startswith('{')][-1]); print(d['value'], d['kernels_ms'], d['compacted']['encode_ms'], d['compacted']['decode_ms'], d['compacted']['GiBps_kernels'], d['compacted']['roundtrip_ok'])"
done
