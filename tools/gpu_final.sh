#!/bin/bash
# Round-end measurement set on one GPU (one call): rocprofv3 kernel-trace stats of the default C3 bench
# command, the FETCH_SIZE / WRITE_SIZE PMC passes (HBM traffic per kernel, tools/pmc_traffic.py), the
# bench-vs-rocprof agreement, then the C3 bench line with the CPU baseline, the C2 line, the per-call
# nmf_mu latency table and the strong-scaling shards R = 100 / 50 / 25.  Usage: bash tools/gpu_final.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/final}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p "$OUT"
bash tools/profile_round.sh "$OUT/profile" > "$OUT/profile.log" 2>&1 || { echo "profile failed"; tail -5 "$OUT/profile.log"; exit 1; }
echo "profile ok"
f=$(find "$OUT/profile/trace" -name '*kernel_stats.csv' | head -1)
cp "$f" "$OUT/kernel_stats.csv" && cp "$OUT/profile/pmc_traffic.json" "$OUT/pmc_traffic.json" || exit 1
grep -h '^{' "$OUT/profile/trace.log" | tail -1 > "$OUT/bench_under_rocprof.json"
python3 tools/profile_agreement.py "$OUT/bench_under_rocprof.json" "$OUT/kernel_stats.csv" > "$OUT/agreement.txt" && cat "$OUT/agreement.txt" || exit 1
bash tools/gpu_measure.sh > "$OUT/measure.log" 2>&1 || { echo "measure failed"; tail -5 "$OUT/measure.log"; exit 1; }
cp -r gpurun_out/measure "$OUT/measure" && echo "measure ok"
RS="100 50 25" bash tools/gpu_scaling_probe.sh > "$OUT/scaling.txt" 2>&1 && cat "$OUT/scaling.txt"
