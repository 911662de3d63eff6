#!/bin/bash
# Loopback TCP rows (tests/native/tcp_loopback, C1's 1000 x 1 MiB by default), R repeats of each
# row, printing effective MB/s (the median pass with --passes P in a row's args; then min, max,
# passes) and the harness' last stderr line.  A row is "label|ENV=V ...|args"
# or "label|ENV=V ...|args|prefix" (prefix: a launcher such as "taskset -c 0-31"):
#   bash tools/loopback_rows.sh <tag> <R> "gpu||--codec gpu --batch 50" "none||--codec none" \
#        "gpu-nosid|PSYNE_TDT_NO_SIDE=1|--codec gpu --batch 50 --half rx --rx views"
set -u
TAG=$1; R=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
port=$((18000 + RANDOM % 2000))
for r in $(seq 1 "$R"); do
  for row in "$@"; do
    IFS='|' read -r label envs args prefix <<< "$row"
    port=$((port + 1))
    f="$OUT/lb_${label}_$r"
    env X=0 $envs timeout -k 10 180 ${prefix:-} ./tests/native/tcp_loopback --count 1000 --port $port $args > "$f.json" 2> "$f.err" \
      || { echo "FAIL $label"; cat "$f.err"; exit 1; }
    echo "$label $r $(python3 -c "import json; d=json.load(open('$f.json')); print(d['effective_MBps'], d.get('min_MBps'), d.get('max_MBps'), d.get('passes'), d.get('mismatches'))") $(tail -1 "$f.err" | cut -c1-200)"
  done
done
