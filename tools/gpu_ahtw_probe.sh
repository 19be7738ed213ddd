#!/bin/bash
# Forced A h^T tile height (128 / 64 genes) vs the automatic choice on per-GPU shards of R restarts per k.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/ahtw
for R in ${RS:-25 50 200}; do
  for s in auto 128 64; do
    if [ $s = auto ]; then unset NMFC_AHTW_TILE; else export NMFC_AHTW_TILE=$s; fi
    timeout -k 10 300 python -u bench.py --restarts $R --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/ahtw/$R.$s.json 2> gpurun_out/ahtw/$R.$s.err || { echo "R=$R $s failed"; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/ahtw/$R.$s.json'));print('R=$R ahtw $s', round(d['value'],1), 'restarts/s', round(d['ms_per_step'],1), 'ms/step')"
  done
done
