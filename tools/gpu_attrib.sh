#!/bin/bash
# Phase attribution of the C3 encode (PSY_X_STOP=k builds return at phase mark k; VALU/SALU/LDS
# per launch per variant) plus SQ counters of C2 / C4 on the shipped library.
# usage (via gpurun): bash tools/gpu_attrib.sh <tag> v1 v2 ...
set -u
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
bash tools/pmc_variants_wl.sh "$OUT/c3" c3 "$@" || exit 1
bash tools/pmc_variants_wl.sh "$OUT/c2" c2 main || exit 1
bash tools/pmc_variants_wl.sh "$OUT/c4" c4 main || exit 1
