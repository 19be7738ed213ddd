#!/bin/bash
# rocprofv3 kernel-trace statistics of the per-call drop-in on the gct (k_solo_mu at k = 2..4, k_team_mu at
# k = 5).  Usage: bash tools/gpu_solo_prof.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/solo_prof}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o solo -- python3 tools/nmf_mu_latency.py 3 > "$OUT/latency.json" 2> "$OUT/prof.err" || { tail -20 "$OUT/prof.err"; exit 1; }
find "$OUT/prof" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \;
cat "$OUT/kernel_stats.csv" | cut -c1-220
