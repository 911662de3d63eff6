set -o pipefail
mkdir -p gpurun_out/r06_o
export TMPDIR=/tmp
PSYNE_TDT_LIB=psyne_amd/libpsyne_tdt_x_lastblk.so timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_large.py > gpurun_out/r06_o/tests.log 2>&1 || { tail -30 gpurun_out/r06_o/tests.log; exit 1; }
tail -1 gpurun_out/r06_o/tests.log
bash tools/ab_alt.sh r06_o/ab2 3 c2 cur lastblk > gpurun_out/r06_o/ab2.txt 2>&1; cat gpurun_out/r06_o/ab2.txt
bash tools/ab_alt.sh r06_o/ab3 2 c3 cur lastblk > gpurun_out/r06_o/ab3.txt 2>&1; cat gpurun_out/r06_o/ab3.txt
