set -o pipefail
mkdir -p gpurun_out/r06_f
export TMPDIR=/tmp
PSYNE_TDT_LIB=psyne_amd/libpsyne_tdt_x_swx2.so timeout -k 10 120 python -u tools/swx_diag.py 2>/dev/null | tee gpurun_out/r06_f/diag.txt
grep -q "mismatches [1-9]" gpurun_out/r06_f/diag.txt && exit 1
PSYNE_TDT_LIB=psyne_amd/libpsyne_tdt_x_swx2.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_scale.py -k "c3_full or c4_full or golden or gradient or word_sizes or every_ws4 or rle_cap or cap_exclusion or speculated or large_streaming or zipf or misaligned or ties" > gpurun_out/r06_f/tests.log 2>&1 || { tail -30 gpurun_out/r06_f/tests.log; exit 1; }
tail -2 gpurun_out/r06_f/tests.log
cp psyne_amd/libpsyne_tdt.so psyne_amd/libpsyne_tdt_x_cur.so
bash tools/ab_alt.sh r06_f/ab 3 c3 cur swx2 > gpurun_out/r06_f/ab.txt 2>&1; cat gpurun_out/r06_f/ab.txt
