#!/bin/bash
# GPU parity subset (-k expression) then alternating A/B of library variants on workloads.
# usage (via gpurun): bash tools/gpu_ab_tests.sh <tag> "<pytest -k expr>" "<workloads>" R v1 v2 ...
set -u
TAG=$1; K=$2; WLS=$3; R=$4; shift 4
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -n "$K" ]; then
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" > "$OUT/tests.log" 2>&1
  rc=$?; tail -3 "$OUT/tests.log"; [ $rc -eq 0 ] || exit $rc
fi
for wl in $WLS; do
  bash tools/ab_alt.sh "$TAG/ab_$wl" "$R" "$wl" "$@" || exit 1
done
