#!/bin/bash
# GPU suite, then a rocprofv3 kernel-trace of the C4 bench (per-kernel times of the mixed batch).
set -u
OUT=gpurun_out/${1:-c4prof}; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
rc=$?; tail -2 "$OUT/gpu_tests.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o c4 -- \
  python3 bench.py --workload c4 --steps 3 --warmup 1 --cpu-seconds 0 > "$OUT/c4.log" 2>&1
rc=$?; tail -1 "$OUT/c4.log" | cut -c1-300; [ $rc -eq 0 ] || exit $rc
python3 tools/prof_summary.py "$OUT/prof" "$OUT/c4_kernels.md" "C4 kernels"
