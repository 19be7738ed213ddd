#!/bin/bash
# Forced W^T A tile shape vs the automatic choice on small per-GPU shards (R restarts per k).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/shape
for R in ${RS:-25 50}; do
  for s in auto big mid small; do
    if [ $s = auto ]; then unset NMFC_WTA_TILE; else export NMFC_WTA_TILE=$s; fi
    timeout -k 10 300 python -u bench.py --restarts $R --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/shape/$R.$s.json 2> gpurun_out/shape/$R.$s.err || { echo "R=$R $s failed"; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/shape/$R.$s.json'));print('R=$R $s', round(d['value'],1), 'restarts/s', round(d['ms_per_step'],1), 'ms/step')"
  done
done
