#!/bin/bash
# GPU tests (optional) then timing of library variants (psyne_amd/libpsyne_tdt_x_<v>.so).
# usage (via gpurun): bash tools/gpu_ab.sh <tag> <tests|notests> v1 v2 ...
set -u
TAG=$1; shift; T=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ "$T" = tests ]; then
  timeout -k 10 420 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu > "$OUT/gpu_tests.log" 2>&1
  rc=$?; tail -2 "$OUT/gpu_tests.log"; [ $rc -eq 0 ] || { echo "gpu tests rc=$rc"; tail -30 "$OUT/gpu_tests.log"; exit $rc; }
fi
bash tools/exp_run.sh "$TAG" "$@"
