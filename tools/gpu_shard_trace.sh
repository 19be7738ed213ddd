#!/bin/bash
# Kernel-trace timeline of one strong-scaling shard (tools/shard_probe.py).  Usage:
#   RANK_=2 WORLD_=8 GROUPS_=1 bash tools/gpu_shard_trace.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/shard_trace}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p "$OUT"
R_=${RANK_:-2}; W_=${WORLD_:-8}; G_=${GROUPS_:-1}
timeout -k 10 200 python3 tools/shard_probe.py --rank $R_ --world $W_ --groups $G_ --repeat 2 > "$OUT/untraced.log" 2>&1 && cat "$OUT/untraced.log" || { tail -5 "$OUT/untraced.log"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/trace" -o run -- \
  python3 tools/shard_probe.py --rank $R_ --world $W_ --groups $G_ --dump "$OUT/iters.npy" > "$OUT/traced.log" 2>&1 \
  || { echo "trace failed"; tail -5 "$OUT/traced.log"; exit 1; }
f=$(find "$OUT/trace" -name '*kernel_trace.csv' | head -1)
python3 tools/trace_timeline.py "$f" 50 "$OUT/iters.npy" > "$OUT/timeline.txt" && cat "$OUT/timeline.txt"
