#!/bin/bash
# C3 at N = 1: one restart group vs two (host threads, one HIP stream each), alternated on one box.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=${1:-gpurun_out/groups_n1}; mkdir -p "$OUT"
for rep in 1 2; do
  for g in 1 2 3; do
    timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --groups $g > "$OUT/g${g}_$rep.json" 2> "$OUT/g${g}_$rep.err" || { echo "groups $g failed"; tail -5 "$OUT/g${g}_$rep.err"; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('$OUT/g${g}_$rep.json').read().strip().splitlines()[-1]); print('groups $g rep $rep', round(d['value'],1), 'wta', round(d['roofline']['achieved'],1))"
  done
done
