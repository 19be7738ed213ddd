#!/bin/bash
# rocprofv3 kernel-trace stats of the C5 (Brunet) bench command.  Usage: bash tools/profile_brunet.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/profile_c5}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p "$OUT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 bench.py --config C5 --steps 1 --warmup 0 --no-cpu-baseline \
  > "$OUT/trace.log" 2>&1 || { echo "C5 trace failed"; tail "$OUT/trace.log"; exit 1; }
echo "C5 trace ok"
find "$OUT/trace" -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} "$OUT/c5_kernel_stats.csv"
head -8 "$OUT/c5_kernel_stats.csv" | cut -c1-200
