mkdir -p gpurun_out/pmc_ic2
export TMPDIR=/tmp
PSYNE_TDT_LIB=psyne_amd/libpsyne_tdt_x_w6.so timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE --output-format csv -d gpurun_out/pmc_ic2/a -o a -- python3 bench.py --msgs 65536 --steps 1 --warmup 1 --cpu-seconds 0 > gpurun_out/pmc_ic2/a.log 2>&1 && \
PSYNE_TDT_LIB=psyne_amd/libpsyne_tdt_x_w6.so timeout -s KILL 90 rocprofv3 --pmc SQ_IFETCH SQ_WAIT_INST_ANY SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_INSTS_VALU --output-format csv -d gpurun_out/pmc_ic2/b -o b -- python3 bench.py --msgs 65536 --steps 1 --warmup 1 --cpu-seconds 0 > gpurun_out/pmc_ic2/b.log 2>&1 && \
python3 tools/pmc_summary.py gpurun_out/pmc_ic2
