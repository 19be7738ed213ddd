#!/bin/bash
# Restart groups per GPU (engines on their own streams) and host-overlapped cophenetic, R = 25 (the N = 8
# shard) and R = 200.  Usage: bash tools/gpu_groups_probe.sh [outdir]   (VARIANTS="g1 g2 g2o ..." RS="25 200")
set -o pipefail
OUT=${1:-gpurun_out/groups}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p "$OUT"
for R in ${RS:-25 200}; do
  for v in ${VARIANTS:-g1 g1o g2o g3o}; do
    g=${v:1:1}; o=""; [ "${v:2:1}" = "o" ] && o="--overlap-host"
    timeout -k 10 300 python -u bench.py --restarts $R --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline --groups $g $o \
      > "$OUT/${v}_R$R.json" 2> "$OUT/${v}_R$R.err" || { echo "$v R=$R failed"; tail -5 "$OUT/${v}_R$R.err"; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/${v}_R$R.json'));k=d['roofline']['kernels'];print('$v R=$R', round(d['value'],1), 'restarts/s', round(d['ms_per_step'],1), 'ms/step', 'wta', round(k['wta']['tflops'],1), 'ahtw', round(k['ahtw']['tflops'],1))"
  done
done
