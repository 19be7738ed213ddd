#!/bin/bash
# One GPU call: co-issue probe, kernel bench, GPU parity tests, default bench, rocprof profile.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 60 ./tools/coissue_probe > gpurun_out/coissue.log 2>&1 && echo "probe ok" &&
timeout -k 10 120 ./tools/kbench > gpurun_out/kbench.log 2>&1 && echo "kbench ok" &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && echo "tests ok" &&
timeout -k 10 600 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err && echo "bench ok" && cat gpurun_out/bench.json &&
bash tools/profile_round.sh gpurun_out/profile
