#!/bin/bash
# Split-K chunk size probe: the C3 sweep at R restarts per k with NMFC_KCHUNK = each of CHUNKS.
# Usage: RS="25 200" CHUNKS="2048 1024" bash tools/kchunk_probe.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/kchunk}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p "$OUT"
for R in ${RS:-25}; do
  for C in ${CHUNKS:-2048 1024 512}; do
    NMFC_KCHUNK=$C timeout -k 10 300 python -u bench.py --restarts "$R" --steps ${STEPS:-2} --warmup 1 --no-cpu-baseline \
      --no-timing > "$OUT/R${R}_c$C.json" 2> "$OUT/R${R}_c$C.err" || { echo "R=$R chunk=$C failed"; tail -5 "$OUT/R${R}_c$C.err"; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/R${R}_c$C.json'));print('R=$R chunk=$C', round(d['value'],1), 'restarts/s', round(d['ms_per_step'],1), 'ms/step', d['config']['cophenetic_rho'])"
  done
done
