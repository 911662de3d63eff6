#!/bin/bash
# Host-inclusive + loopback TCP measurements (SURVEY.md §8(d) C1/C5 host path).
set -u
TAG=${1:-run}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --host-inclusive --latency --cpu-seconds 0 --steps 3 --warmup 1 > "$OUT/bench_host.log" 2>&1
rc=$?; tail -1 "$OUT/bench_host.log"; [ $rc -eq 0 ] || exit $rc
# loopback C1 rows, 12 timed passes each (median / min / max): the GPU codec and
# no codec on the same box, payloads in pageable and in pinned memory, one process and two
bash tools/loopback_rows.sh "$TAG/loop" 1 \
  "gpu||--codec gpu --batch 50 --passes 12" "none||--codec none --passes 12" \
  "gpu_pinned||--codec gpu --batch 50 --passes 12 --mem pinned" "none_pinned||--codec none --passes 12 --mem pinned" \
  "gpu_procs2||--codec gpu --batch 50 --passes 12 --procs 2" "none_procs2||--codec none --passes 12 --procs 2" \
  "gpu_pinned_procs2||--codec gpu --batch 50 --passes 12 --mem pinned --procs 2" \
  "none_pinned_procs2||--codec none --passes 12 --mem pinned --procs 2" > "$OUT/loopback_rows.txt" 2>&1
rc=$?; cat "$OUT/loopback_rows.txt"; [ $rc -eq 0 ] || exit $rc
# psyne's own CPU path (the reference protocol compiled from its header: oracle/_ref)
timeout -k 10 300 ./tests/native/tcp_loopback --codec cpu --count 1000 --port 18092 > "$OUT/loopback_cpu.json" 2> "$OUT/loopback_cpu.err"
rc=$?; cat "$OUT/loopback_cpu.json"; tail -3 "$OUT/loopback_cpu.err"; exit $rc
