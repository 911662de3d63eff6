#!/bin/bash
# Diagnostic: build a variant of the FULL library (the production translation units: tdt_api.hip
# plus one tdt_enc_ws.hip object per word size, linked like psyne_amd/build.py), so that A/B
# timings compare the production code layout.  usage: tools/full_variant.sh <name> "<flags>" [src-root]
set -e
cd "$(dirname "$0")/.."
NAME=$1; FLAGS=$2; SRC=${3:-.}
OBJ=/tmp/fv_$NAME; mkdir -p $OBJ
B="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I include $FLAGS"
$B -c $SRC/psyne_amd/csrc/tdt_api.hip -o $OBJ/api.o &
for ws in 1 2 4 8 16; do $B -DPSY_INST_WS=$ws -c $SRC/psyne_amd/csrc/tdt_enc_ws.hip -o $OBJ/ws$ws.o & done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $OBJ/api.o $OBJ/ws1.o $OBJ/ws2.o $OBJ/ws4.o $OBJ/ws8.o $OBJ/ws16.o -o psyne_amd/libpsyne_tdt_x_$NAME.so
ls -la psyne_amd/libpsyne_tdt_x_$NAME.so
