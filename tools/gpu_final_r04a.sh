#!/bin/bash
# Round-4 measurement set, part A (one gpurun call): rocprofv3 kernel stats + FETCH/WRITE PMC passes of the default
# C3 bench command, the bench-vs-rocprof agreement, the C3 bench line with the CPU baseline, the C3 FIXED-1000 line,
# and the 8-GPU strong-scaling replay.  Usage: bash tools/gpu_final_r04a.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/final_r04}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p "$OUT"
bash tools/profile_round.sh "$OUT/profile" > "$OUT/profile.log" 2>&1 || { echo "profile failed"; tail -5 "$OUT/profile.log"; exit 1; }
echo "profile ok"
f=$(find "$OUT/profile/trace" -name '*kernel_stats.csv' | head -1)
cp "$f" "$OUT/kernel_stats.csv" && cp "$OUT/profile/pmc_traffic.json" "$OUT/pmc_traffic.json" || exit 1
grep -h '^{' "$OUT/profile/trace.log" | tail -1 > "$OUT/bench_under_rocprof.json"
python3 tools/profile_agreement.py "$OUT/bench_under_rocprof.json" "$OUT/kernel_stats.csv" > "$OUT/agreement.txt" && cat "$OUT/agreement.txt" || exit 1
timeout -k 10 600 python -u bench.py > "$OUT/c3_bench.json" 2> "$OUT/c3_bench.err" && echo "c3 ok" && cat "$OUT/c3_bench.json" || { tail -5 "$OUT/c3_bench.err"; exit 1; }
timeout -k 10 300 python -u bench.py --stop-rule fixed --maxiter 1000 --steps 1 --warmup 0 --no-cpu-baseline \
  > "$OUT/c3_fixed1000.json" 2> "$OUT/c3_fixed1000.err" && echo "c3 fixed-1000 ok" || { tail -5 "$OUT/c3_fixed1000.err"; exit 1; }
timeout -k 10 300 python -u bench.py --simulate-world 8 --steps 2 --warmup 1 > "$OUT/sim8.json" 2> "$OUT/sim8.err" \
  && python3 -c "import json,sys; d=json.load(open(sys.argv[1])); c=d['config']; print('sim8 per GPU', round(c['per_gpu_restarts_per_s'],1), [round(x*1e3) for x in c['shard_seconds']], c['counts_equal_whole_sweep'])" "$OUT/sim8.json"
