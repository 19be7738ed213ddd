#!/bin/bash
# Round-4 measurement set after the last source change: part A (tools/gpu_final_r04a.sh) and part B
# (tools/gpu_final_r04b.sh) into one directory.
set -o pipefail
OUT=${1:-gpurun_out/final_r04e}
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_final_r04a.sh "$OUT" && bash tools/gpu_final_r04b.sh "$OUT"
