#!/bin/bash
set -u
for r in 1 2 3; do bash tools/exp_run_wl.sh r04_dre c4 base dreord || exit 1; done
for r in 1 2; do bash tools/exp_run_wl.sh r04_dre c2 base dreord || exit 1; done
bash tools/exp_run_wl.sh r04_dre c3 base dreord
