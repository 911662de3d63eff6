#!/bin/bash
# Round-4 final pass, part B (the same library build as part A): PMC passes (FETCH/WRITE + SQ) of
# the C3 / C2 / C4 benches — traffic JSON keyed to the library hash, cited by bench.py's
# roofline — then the C1 loopback rows (gpu x3, none x3, the reference codec) and the
# reference's own tcp_tdt_benchmark row.  usage (via gpurun): bash tools/gpu_r04_final_b.sh <tag>
set -u
TAG=${1:-r04_final}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "== $1"; }
step pmc_c3
bash tools/profile_pmc.sh "$OUT/pmc" || exit 1
step pmc_c2
PMC_KEY=c2_1048576x1024 bash tools/profile_pmc.sh "$OUT/pmc_c2" --workload c2 --steps 1 --warmup 1 --cpu-seconds 0 --compacted-steps 0 || exit 1
step pmc_c4
PMC_KEY=c4_4194304x65536 bash tools/profile_pmc.sh "$OUT/pmc_c4" --workload c4 --steps 1 --warmup 1 --cpu-seconds 0 --compacted-steps 0 || exit 1
step loopback
port=18400
for r in 1 2 3; do for c in gpu none; do
  port=$((port + 1))
  timeout -k 10 180 ./tests/native/tcp_loopback --codec $c --count 1000 --batch 50 --port $port > "$OUT/loopback_${c}_$r.json" 2> "$OUT/loopback_${c}_$r.err"
  rc=$?; cat "$OUT/loopback_${c}_$r.json"; [ $rc -eq 0 ] || exit $rc
done; done
timeout -k 10 300 ./tests/native/tcp_loopback --codec cpu --count 1000 --port 18420 > "$OUT/loopback_cpu.json" 2> "$OUT/loopback_cpu.err"
rc=$?; cat "$OUT/loopback_cpu.json"; [ $rc -eq 0 ] || exit $rc
step ref_tcp
bash tools/ref_tcp_bench.sh "$OUT"
