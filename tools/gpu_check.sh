#!/bin/bash
# GPU check: A sha on the box, the GPU suite (optional -k filter), one C3 bench line.
# Usage: bash tools/gpu_check.sh <outdir> [pytest -k expression]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=${1:-gpurun_out/check}; mkdir -p "$OUT"
K=${2:-}
timeout -k 10 120 python tools/a_sha.py > "$OUT/a_sha.txt" 2>&1; cat "$OUT/a_sha.txt"
if [ -n "$K" ]; then KARG=(-k "$K"); else KARG=(); fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${KARG[@]}" > "$OUT/gpu_tests.log" 2>&1 \
  && echo "tests ok: $(tail -1 "$OUT/gpu_tests.log")" || { echo "tests failed"; grep -E "FAILED|Error|error" "$OUT/gpu_tests.log" | head -20; tail -30 "$OUT/gpu_tests.log"; exit 1; }
timeout -k 10 600 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err" \
  && python -c "import json,sys; d=json.load(open('$OUT/bench.json')); print('bench', d['value'], d['roofline']['frac'], d['config']['mean_iterations'])" \
  || { echo "bench failed"; tail "$OUT/bench.err"; exit 1; }
