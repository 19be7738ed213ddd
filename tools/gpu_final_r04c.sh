#!/bin/bash
# Round-4 measurement set after the register-Gram change: part A (tools/gpu_final_r04a.sh) and the C4 line.
set -o pipefail
OUT=${1:-gpurun_out/final_r04c}
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_final_r04a.sh "$OUT" || exit 1
timeout -k 10 600 python -u bench.py --config C4 --steps 1 --warmup 1 --cpu-iters 4 > "$OUT/c4_bench.json" 2> "$OUT/c4_bench.err" \
  && echo "C4 ok" || { tail -5 "$OUT/c4_bench.err"; exit 1; }
