set -o pipefail
mkdir -p gpurun_out/r06_h
export TMPDIR=/tmp
bash tools/ab_compact.sh r06_h/cmp 2 c3 lb6 lb8 > gpurun_out/r06_h/cmp.txt 2>&1; cat gpurun_out/r06_h/cmp.txt
bash tools/loopback_rows.sh r06_h/loop 2 "gpu||--codec gpu --batch 50 --passes 12" "none||--codec none --passes 12" \
  "gpu_p2||--codec gpu --batch 50 --passes 12 --procs 2" "none_p2||--codec none --passes 12 --procs 2" > gpurun_out/r06_h/loop.txt 2>&1
cat gpurun_out/r06_h/loop.txt
