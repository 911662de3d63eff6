set -u
OUT=gpurun_out/r03_c4ns
mkdir -p $OUT
export TMPDIR=/tmp
PSYNE_TDT_NO_SIDE=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof -o run -- python3 bench.py --workload c4 --steps 2 --warmup 2 --cpu-seconds 0 --compacted-steps 0 > $OUT/log 2>&1
