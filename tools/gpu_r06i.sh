set -o pipefail
mkdir -p gpurun_out/r06_i
export TMPDIR=/tmp
bash tools/loopback_rows.sh r06_i/loop 2 "gpu_pin||--codec gpu --batch 50 --passes 12 --mem pinned" "none_pin||--codec none --passes 12 --mem pinned" \
  "gpu_ct4|PSYNE_TDT_COPY_THREADS=4|--codec gpu --batch 50 --passes 12" "gpu_b100||--codec gpu --batch 100 --passes 12" "none||--codec none --passes 12" > gpurun_out/r06_i/loop.txt 2>&1
cat gpurun_out/r06_i/loop.txt
