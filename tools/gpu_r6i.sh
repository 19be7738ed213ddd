#!/bin/bash
# Round 6: kernel timeline of the 8-GPU C3 shard's workload (R = 25 per k) with one and two restart groups.
set -o pipefail
OUT=${1:-gpurun_out/r6i}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p "$OUT"
for G in 1 2; do
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$OUT/g$G" -o run -- python3 bench.py --restarts 25 \
    --groups $G --steps 1 --warmup 0 --no-cpu-baseline --dump-iters "$OUT/iters_g$G.npy" > "$OUT/g$G.log" 2>&1 || { echo "G=$G failed"; tail -5 "$OUT/g$G.log"; exit 1; }
  f=$(find "$OUT/g$G" -name '*kernel_trace.csv' | head -1)
  python3 tools/trace_timeline.py "$f" 50 "$OUT/iters_g$G.npy" 20000 500 > "$OUT/timeline_g$G.txt" && grep '^{' "$OUT/g$G.log" | tail -1 | cut -c1-200
done
