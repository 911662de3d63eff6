set -u
OUT=gpurun_out/pmcab; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 --list-avail > $OUT/avail.txt 2>&1 || true
for v in base fl2; do
  PSYNE_TDT_LIB=psyne_amd/libpsyne_tdt_x_$v.so timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT --output-format csv -d $OUT/$v -o $v -- python3 bench.py --steps 1 --warmup 1 --cpu-seconds 0 > $OUT/$v.log 2>&1 || exit 1
  python3 tools/pmc_summary.py $OUT/$v > $OUT/$v.txt
done
