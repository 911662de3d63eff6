#!/bin/bash
set -u
bash tools/lb_diag3.sh r04_lb10 && bash tools/call_r04_lbtrace.sh
