#!/bin/bash
# Host-inclusive + loopback TCP measurements (SURVEY.md §8(d) C1/C5 host path).
set -u
TAG=${1:-run}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --host-inclusive --latency --cpu-seconds 0 --steps 3 --warmup 1 > "$OUT/bench_host.log" 2>&1
rc=$?; tail -1 "$OUT/bench_host.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 ./tests/native/tcp_loopback --codec none --count 1000 --port 18090 > "$OUT/loopback_none.json" 2> "$OUT/loopback_none.err"
rc=$?; cat "$OUT/loopback_none.json"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 ./tests/native/tcp_loopback --codec gpu --count 1000 --batch 50 --port 18091 > "$OUT/loopback_gpu.json" 2> "$OUT/loopback_gpu.err"
rc=$?; cat "$OUT/loopback_gpu.json"; tail -3 "$OUT/loopback_gpu.err"; [ $rc -eq 0 ] || exit $rc
# psyne's own CPU path (the reference protocol compiled from its header: oracle/_ref)
timeout -k 10 300 ./tests/native/tcp_loopback --codec cpu --count 1000 --port 18092 > "$OUT/loopback_cpu.json" 2> "$OUT/loopback_cpu.err"
rc=$?; cat "$OUT/loopback_cpu.json"; tail -3 "$OUT/loopback_cpu.err"; exit $rc
