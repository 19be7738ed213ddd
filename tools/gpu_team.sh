#!/bin/bash
# k_team_mu check on one GPU: the GPU parity suite, teambench, per-call nmf_mu latency on the gct and on
# expression-set shapes.  Usage: bash tools/gpu_team.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/team}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > "$OUT/parity.log" 2>&1 \
  && echo "parity ok: $(tail -1 "$OUT/parity.log")" || { echo "parity failed"; tail -30 "$OUT/parity.log"; exit 1; }
timeout -k 10 120 ./tools/teambench 2000 > "$OUT/teambench.txt" 2>&1 && grep -A3 "k = 2," "$OUT/teambench.txt" || exit 1
timeout -k 10 200 python -u tools/nmf_mu_latency.py 5 > "$OUT/latency.json" && cat "$OUT/latency.json" || exit 1
timeout -k 10 500 python -u tools/nmf_mu_latency_shapes.py 2 > "$OUT/latency_shapes.json" 2> "$OUT/latency_shapes.err" \
  && grep -v Exiting "$OUT/latency_shapes.err" | tail -6 || exit 1
