set -u
bash tools/host_pipe_prof.sh r04_hp1 && \
bash tools/ab_env.sh r04_m256 3 c3 main "X=0" "PSYNE_TDT_M256=1" && \
PSYNE_TDT_M256=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_scale.py -k "c3_full_batch or mid_class or zipf_full" > gpurun_out/r04_m256/tests.log 2>&1; tail -3 gpurun_out/r04_m256/tests.log && \
bash tools/ab_env.sh r04_m256c4 2 c4 main "X=0" "PSYNE_TDT_M256=1"
