#!/bin/bash
# Diagnostic variants of the library (word_size 4 only) for time attribution; never shipped.
# usage: tools/exp_build.sh name "-DFLAG ..." [name "-DFLAGS"]...
set -e
cd "$(dirname "$0")/.."
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -DPSY_FAST_BUILD $flags -I include \
    psyne_amd/csrc/tdt_api.hip -o psyne_amd/libpsyne_tdt_x_$name.so &
done
wait
ls -la psyne_amd/libpsyne_tdt_x_*.so
