#!/bin/bash
# Brunet (C5) GPU check: parity tests, per-k kernel bench, full C5 bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_brunet.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_brunet.log 2>&1 || { echo "brunet tests failed"; tail -40 gpurun_out/gpu_brunet.log; exit 1; }
echo "brunet tests ok"
timeout -k 10 300 python -u tools/brunet_kbench.py > gpurun_out/kb_default.log 2>&1 || { echo "kb failed"; tail gpurun_out/kb_default.log; exit 1; }
grep -v '^{"lib' gpurun_out/kb_default.log | grep -v amdgpu.ids
timeout -k 10 600 python -u bench.py --config C5 --steps 1 --warmup 0 ${BENCH_ARGS:-} > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err || { echo "bench failed"; tail gpurun_out/bench_c5.err; exit 1; }
cat gpurun_out/bench_c5.json; tail -2 gpurun_out/bench_c5.err
