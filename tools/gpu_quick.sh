#!/bin/bash
# Quick GPU check: optional tool binaries, GPU parity tests, default bench.  Usage: bash tools/gpu_quick.sh [tool ...]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for t in "$@"; do
  timeout -k 10 120 ./tools/$t > gpurun_out/$t.log 2>&1 || { echo "$t failed"; exit 1; }
  echo "$t ok"
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
echo "tests ok"
timeout -k 10 600 python -u bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json; tail -1 gpurun_out/bench.err
