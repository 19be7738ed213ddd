#!/bin/bash
# A/B of engine env knobs on the C3 bench (default REF_COMPAT sweep and the FIXED-1000 full-load line).
# Usage: bash tools/gpu_ab_c3.sh <outdir> "ENV=.. ..." "ENV=.. ..." ...
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=$1; shift; mkdir -p "$OUT"
i=0
for arm in "$@"; do
  i=$((i + 1))
  env $arm timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/c3_$i.json" 2> "$OUT/c3_$i.err" \
    && env $arm timeout -k 10 300 python -u bench.py --stop-rule fixed --maxiter 1000 --steps 1 --warmup 0 --no-cpu-baseline > "$OUT/fx_$i.json" 2> "$OUT/fx_$i.err" \
    && python3 -c "
import json,sys
a=json.load(open(sys.argv[1])); b=json.load(open(sys.argv[2]))
k=lambda d: {n: round(v['tflops'],2) for n,v in d['roofline']['kernels'].items() if 'tflops' in v}
print(sys.argv[3], 'C3', round(a['value'],1), k(a), '| fixed1000', round(b['value'],1), k(b))" "$OUT/c3_$i.json" "$OUT/fx_$i.json" "$arm" \
    || { echo "arm $arm failed"; tail -5 "$OUT/c3_$i.err" "$OUT/fx_$i.err"; exit 1; }
done
