#!/bin/bash
# Strong-scaling replay on one GPU: bench.py --simulate-world 8 (the 8 real shards of the 1800-job C3 grid)
# and the kernel-trace timeline of one R = 25 shard.  Usage: bash tools/gpu_sim8.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/sim8}
mkdir -p "$OUT"
timeout -k 10 400 python -u bench.py --simulate-world 8 --steps 2 --warmup 1 > "$OUT/sim8.json" 2> "$OUT/sim8.err" \
  && python3 -c "import json,sys; d=json.load(open(sys.argv[1])); c=d['config']; print('sim8', round(d['value'],1), 'per GPU', round(c['per_gpu_restarts_per_s'],1), 'shards s', [round(x,3) for x in c['shard_seconds']], 'equal', c['counts_equal_whole_sweep'])" "$OUT/sim8.json" \
  || { tail -5 "$OUT/sim8.err"; exit 1; }
RS=25 BENCH_ARGS="--groups 1" bash tools/trace_probe.sh "$OUT/trace" > "$OUT/trace.log" 2>&1 && tail -30 "$OUT/trace.log" || { tail -5 "$OUT/trace.log"; exit 1; }
