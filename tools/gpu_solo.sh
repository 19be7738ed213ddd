#!/bin/bash
# Solo-kernel check on one GPU (csrc/solo.hip): its parity tests first, then the GPU parity suite, then the
# per-call nmf_mu latency on the gct with the solo path (default) and without it (NMFC_SOLO=0: the team kernel).
# Usage: bash tools/gpu_solo.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/solo}
mkdir -p "$OUT"
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -x -v -k solo --timeout 120 --timeout-method thread > "$OUT/solo_tests.log" 2>&1 \
  && echo "solo ok: $(tail -1 "$OUT/solo_tests.log")" || { echo "solo failed"; tail -40 "$OUT/solo_tests.log"; exit 1; }
timeout -k 10 200 python -u tools/nmf_mu_latency.py 5 > "$OUT/latency_solo.json" && cat "$OUT/latency_solo.json" || exit 1
NMFC_SOLO=0 timeout -k 10 200 python -u tools/nmf_mu_latency.py 5 > "$OUT/latency_team.json" && cat "$OUT/latency_team.json" || exit 1
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 \
  && echo "gpu suite ok: $(tail -1 "$OUT/gpu_tests.log")" || { echo "gpu suite failed"; tail -30 "$OUT/gpu_tests.log"; exit 1; }
