#!/bin/bash
# k_team_mu check on one GPU: the GPU parity suite, per-call nmf_mu latency, C2 line (auto policy and each
# kernel forced).  Usage: bash tools/gpu_team.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/team}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > "$OUT/parity.log" 2>&1 \
  && echo "parity ok: $(tail -1 "$OUT/parity.log")" || { echo "parity failed"; tail -30 "$OUT/parity.log"; exit 1; }
timeout -k 10 200 python -u tools/nmf_mu_latency.py 5 > "$OUT/latency.json" && cat "$OUT/latency.json" || exit 1
for K in auto team single; do
  NMFC_SMALL_KERNEL=$K timeout -k 10 200 python -u bench.py --config C2 --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/c2_$K.json" 2> "$OUT/c2_$K.err" \
    && python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'])" "$OUT/c2_$K.json" $K || { tail -5 "$OUT/c2_$K.err"; exit 1; }
done
