#!/bin/bash
# Solo kernel: its parity tests, then the phase / variant bench.  Usage: bash tools/gpu_solobench.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/solobench}
mkdir -p "$OUT"
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -x -q -k "solo or nmf_mu" --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1 && tail -1 "$OUT/tests.log" || { tail -30 "$OUT/tests.log"; exit 1; }
timeout -k 10 200 ./tools/solobench 2000 > "$OUT/solobench.txt" 2>&1 && cat "$OUT/solobench.txt"
