#!/bin/bash
# Quick check on one GPU: the -m gpu suite, smoke(), one default C3 bench line.  Usage: bash tools/gpu_quick.sh
set -o pipefail
OUT=${1:-gpurun_out/r03a}
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 && echo "tests ok: $(tail -1 $OUT/gpu_tests.log)" || { echo tests failed; tail -30 $OUT/gpu_tests.log; exit 1; }
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && tail -1 $OUT/smoke.log || exit 1
timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err && cat $OUT/bench.json || { tail -5 $OUT/bench.err; exit 1; }
