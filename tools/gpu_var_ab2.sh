#!/bin/bash
# Two passes of tools/gpu_var_bench.sh over tools/var/*.so (C3, R = 200), then the bit-identity tests on the in-tree library.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
STEPS=3 RS=200 bash tools/gpu_var_bench.sh && STEPS=3 RS=200 bash tools/gpu_var_bench.sh || exit 1
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/var_tests.log 2>&1; tail -2 gpurun_out/var_tests.log
