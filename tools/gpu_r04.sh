#!/bin/bash
# Round-4 GPU pass: the -m gpu suite (optional -k filter), then bench lines for the given configs.
# Usage: bash tools/gpu_r04.sh <outdir> "<pytest -k expr or ->" "<configs, e.g. C1 C2 C3>"
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=${1:-gpurun_out/r04}; mkdir -p "$OUT"
K=${2:--}
CONFIGS=${3:-}
if [ "$K" != "none" ]; then
  if [ "$K" != "-" ]; then KARG=(-k "$K"); else KARG=(); fi
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread "${KARG[@]}" > "$OUT/gpu_tests.log" 2>&1 \
    && echo "tests ok: $(tail -1 "$OUT/gpu_tests.log")" || { echo "tests failed"; grep -E "FAILED|Error|error" "$OUT/gpu_tests.log" | head -20; tail -30 "$OUT/gpu_tests.log"; exit 1; }
fi
for C in $CONFIGS; do
  timeout -k 10 600 python -u bench.py --config "$C" ${BENCH_ARGS:-} > "$OUT/bench_$C.json" 2> "$OUT/bench_$C.err" \
    && python -c "import json; d=json.load(open('$OUT/bench_$C.json')); r=d.get('roofline') or {}; print('$C', round(d['value'],1), d['ms_per_step'], r.get('frac'), (d.get('cpu_baseline') or {}).get('value'))" \
    || { echo "bench $C failed"; tail "$OUT/bench_$C.err"; exit 1; }
done
