#!/bin/bash
# Round-end check on one GPU (one call): the -m gpu suite, smoke(), the C5 line, then tools/gpu_final.sh
# (profile set + measurement lines).  Usage: bash tools/gpu_roundend.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/roundend}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 \
  && echo "tests ok: $(tail -1 "$OUT/gpu_tests.log")" || { echo "tests failed"; tail -20 "$OUT/gpu_tests.log"; exit 1; }
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 && tail -1 "$OUT/smoke.log" || exit 1
timeout -k 10 300 python -u bench.py --config C5 --steps 1 --warmup 1 > "$OUT/c5.json" 2> "$OUT/c5.err" \
  && echo "c5 ok" || { echo "c5 failed"; tail -5 "$OUT/c5.err"; exit 1; }
bash tools/gpu_final.sh "$OUT/final"
