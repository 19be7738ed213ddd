#!/bin/bash
# rocprofv3 kernel trace of one default bench sweep (no PMC).  Usage: bash tools/gpu_trace.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/trace}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline \
  > "$OUT/trace.log" 2>&1 || { echo "trace failed"; tail "$OUT/trace.log"; exit 1; }
echo "trace ok"
