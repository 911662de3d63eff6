set -o pipefail
mkdir -p gpurun_out/r06_c
export TMPDIR=/tmp
PSYNE_TDT_LIB=psyne_amd/libpsyne_tdt_x_fx.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_scale.py -k "c3_full or c4_full or golden or gradient or word_sizes or every_ws4 or rle_cap or cap_exclusion or speculated or large_streaming or zipf" > gpurun_out/r06_c/tests_fx.log 2>&1 || { tail -30 gpurun_out/r06_c/tests_fx.log; exit 1; }
tail -3 gpurun_out/r06_c/tests_fx.log
bash tools/ab_alt.sh r06_c/ab 3 c3 base w8 fx > gpurun_out/r06_c/ab.txt 2>&1; cat gpurun_out/r06_c/ab.txt
timeout -k 10 120 tools/ubench_hbm 8 > gpurun_out/r06_c/ubench_hbm.txt 2>&1
