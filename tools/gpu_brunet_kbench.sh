#!/bin/bash
# Brunet kernel bench: default build plus variant libraries given as arguments (tools/*.so).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_brunet.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/brunet_tests.log 2>&1 || { echo "brunet tests failed"; tail -30 gpurun_out/brunet_tests.log; exit 1; }
echo "brunet tests ok"
timeout -k 10 300 python -u tools/brunet_kbench.py > gpurun_out/kb_default.log 2>&1 || { echo "kb default failed"; tail gpurun_out/kb_default.log; exit 1; }
echo "== default"; grep -v '^{"lib' gpurun_out/kb_default.log | grep -v amdgpu.ids
for v in "$@"; do
  b=$(basename $v .so)
  timeout -k 10 300 python -u tools/brunet_kbench.py --lib $v > gpurun_out/kb_$b.log 2>&1 || { echo "kb $b failed"; tail gpurun_out/kb_$b.log; exit 1; }
  echo "== $b"; grep -v '^{"lib' gpurun_out/kb_$b.log | grep -v amdgpu.ids
done
