#!/bin/bash
# Solo path, round-3 measurement set: GPU suite, phase bench, per-call nmf_mu latency (gct: solo default vs
# NMFC_SOLO=0 team; expression-set shapes).  Usage: bash tools/gpu_solo3.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/solo3}
mkdir -p "$OUT"
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 \
  && echo "gpu suite ok: $(tail -1 "$OUT/gpu_tests.log")" || { echo "gpu suite failed"; tail -30 "$OUT/gpu_tests.log"; exit 1; }
timeout -k 10 120 ./tools/solobench 2000 > "$OUT/solobench.txt" 2>&1 || exit 1
timeout -k 10 200 python -u tools/nmf_mu_latency.py 5 > "$OUT/latency_solo.json" && cat "$OUT/latency_solo.json" || exit 1
NMFC_SOLO=0 timeout -k 10 200 python -u tools/nmf_mu_latency.py 5 > "$OUT/latency_team.json" && cat "$OUT/latency_team.json" || exit 1
timeout -k 10 500 python -u tools/nmf_mu_latency_shapes.py 2 > "$OUT/latency_shapes.json" 2> "$OUT/latency_shapes.err" \
  && grep -v Exiting "$OUT/latency_shapes.err" | tail -8 || exit 1
timeout -k 10 300 python -u bench.py --config C1 > "$OUT/c1_bench.json" 2> "$OUT/c1_bench.err" && cat "$OUT/c1_bench.json" || { tail -5 "$OUT/c1_bench.err"; exit 1; }
