#!/bin/bash
# C1 reference row (BASELINE.json configs[0]): the reference's own benchmarks/tcp_tdt_benchmark.cpp,
# compiled from /root/reference by oracle/Makefile (target ref_tcp, output oracle/_ref/, git-ignored),
# run as server + client over 127.0.0.1: 1,000 x 1 MiB GRADIENTS tensors through its SimpleTDT
# (tcp_tdt_benchmark.cpp:542-543).  Beside it tests/native/tcp_loopback's rows on the same host.
# usage: tools/ref_tcp_bench.sh <out-dir>
set -u
OUT=${1:-gpurun_out/ref_tcp}
mkdir -p "$OUT"
BIN=./oracle/_ref/tcp_tdt_benchmark
[ -x "$BIN" ] || { echo "missing $BIN (make -C oracle ref_tcp in the build container)"; exit 3; }
PORT=18195
timeout -k 10 300 "$BIN" server $PORT > "$OUT/ref_tcp_server.log" 2>&1 &
SPID=$!
sleep 1
timeout -k 10 300 "$BIN" client 127.0.0.1 $PORT > "$OUT/ref_tcp_client.log" 2>&1
crc=$?
wait $SPID
src=$?
grep -E "Total time|Compression ratio|Effective throughput|Network throughput|Receive throughput" "$OUT/ref_tcp_server.log" "$OUT/ref_tcp_client.log"
[ $crc -eq 0 ] && [ $src -eq 0 ]
