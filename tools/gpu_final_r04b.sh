#!/bin/bash
# Round-4 measurement set, part B (one gpurun call): the C1, C2, C4 and C5 bench lines (each with its CPU baseline),
# the per-call nmf_mu latency table and the CPU baseline against its process count.  Usage: bash tools/gpu_final_r04b.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/final_r04}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p "$OUT"
for C in C1 C2; do
  timeout -k 10 300 python -u bench.py --config $C --steps 10 --warmup 2 > "$OUT/${C,,}_bench.json" 2> "$OUT/${C,,}_bench.err" \
    && echo "$C ok" || { tail -5 "$OUT/${C,,}_bench.err"; exit 1; }
done
timeout -k 10 600 python -u bench.py --config C4 --steps 1 --warmup 1 --cpu-iters 4 > "$OUT/c4_bench.json" 2> "$OUT/c4_bench.err" \
  && echo "C4 ok" || { tail -5 "$OUT/c4_bench.err"; exit 1; }
timeout -k 10 600 python -u bench.py --config C5 --steps 1 --warmup 1 > "$OUT/c5_bench.json" 2> "$OUT/c5_bench.err" \
  && echo "C5 ok" || { tail -5 "$OUT/c5_bench.err"; exit 1; }
timeout -k 10 300 python -u tools/nmf_mu_latency.py 3 > "$OUT/nmf_mu_latency.json" 2> "$OUT/nmf_mu_latency.err" && echo "latency ok"
timeout -k 10 400 python -u tools/cpu_scaling.py --procs 1,4,8,16 > "$OUT/cpu_scaling.json" 2> "$OUT/cpu_scaling.err" && echo "cpu scaling ok" && cat "$OUT/cpu_scaling.err"
