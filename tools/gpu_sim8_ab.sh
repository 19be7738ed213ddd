#!/bin/bash
# A/B of engine env knobs on the 8-GPU strong-scaling replay (bench.py --simulate-world 8).
# Usage: bash tools/gpu_sim8_ab.sh <outdir> "NAME=VAL ..." "NAME=VAL --bench-arg=x ..." [...]   (each arg = one arm: env
# assignments, and bench.py options written as --opt=value)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=$1; shift; mkdir -p "$OUT"
i=0
for arm in "$@"; do
  i=$((i + 1))
  envs=""; args=""
  for tok in $arm; do case "$tok" in --*) args="$args $tok";; *) envs="$envs $tok";; esac; done
  env $envs timeout -k 10 300 python -u bench.py --simulate-world 8 --steps ${SIM_STEPS:-2} --warmup 1 $args > "$OUT/sim8_$i.json" 2> "$OUT/sim8_$i.err" \
    && python3 -c "import json,sys; d=json.load(open(sys.argv[1])); c=d['config']; print(sys.argv[2], 'per GPU', round(c['per_gpu_restarts_per_s'],1), 'shards ms', [round(x*1e3) for x in c['shard_seconds']], 'equal', c['counts_equal_whole_sweep'])" "$OUT/sim8_$i.json" "$arm" \
    || { echo "arm $arm failed"; tail -5 "$OUT/sim8_$i.err"; exit 1; }
done
