#!/bin/bash
# GPU test pass (via gpurun): pytest -m gpu over the given files / -k expression, time-limited,
# stopping at the first failure; the log lands in gpurun_out/<tag>/tests.log.
# usage: bash tools/gpu_tests.sh <tag> [seconds] [pytest args ...]   (no args: the whole -m gpu suite)
set -u
TAG=$1; shift
LIMIT=900
if [ $# -gt 0 ] && [[ $1 =~ ^[0-9]+$ ]]; then LIMIT=$1; shift; fi
[ $# -gt 0 ] || set -- tests
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 "$LIMIT" python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread "$@" > "$OUT/tests.log" 2>&1
rc=$?
tail -2 "$OUT/tests.log"
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" "$OUT/tests.log" | head -20; exit $rc; }
