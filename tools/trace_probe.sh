#!/bin/bash
# Kernel-trace timeline of one C3 sweep per restart count R (R = 200/N is one GPU's shard of the
# N-GPU strong-scaling job).  Usage: RS="25 200" bash tools/trace_probe.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/trace_probe}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p "$OUT"
for R in ${RS:-25 200}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/R$R" -o run -- \
    python3 bench.py --restarts "$R" --steps 1 --warmup 0 --no-cpu-baseline --dump-iters "$OUT/R$R.iters.npy" ${BENCH_ARGS:-} > "$OUT/R$R.log" 2>&1 \
    || { echo "trace R=$R failed"; tail -5 "$OUT/R$R.log"; exit 1; }
  f=$(find "$OUT/R$R" -name '*kernel_trace.csv' | head -1)
  python3 tools/trace_timeline.py "$f" ${BUCKET:-100} "$OUT/R$R.iters.npy" > "$OUT/R$R.timeline.txt" && echo "R=$R" && cat "$OUT/R$R.timeline.txt"
done
