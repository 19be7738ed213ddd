#!/bin/bash
# Round 6, call p: the Brunet GPU tests on the batched-reciprocal product build, then tools/brunet_kbench.py on the
# HEAD-source library (br_base), the new default (br_new) and three RG / SPL re-tunings (br_va, br_vb, br_vc), two passes.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r6p
timeout -k 10 400 python -u -m pytest tests/test_gpu_brunet.py tests/test_gpu_r_binding.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6p/brunet_tests.log 2>&1 || { echo "brunet tests failed"; tail -40 gpurun_out/r6p/brunet_tests.log; exit 1; }
tail -3 gpurun_out/r6p/brunet_tests.log
for pass in 1 2; do
  if [ $pass = 1 ]; then L="base new va vb vc"; else L="vc vb va new base"; fi
  for v in $L; do
    timeout -k 10 240 python -u tools/brunet_kbench.py --lib tools/br_$v.so > gpurun_out/r6p/kb_${v}_$pass.txt 2>&1 || { echo "kb $v failed"; tail gpurun_out/r6p/kb_${v}_$pass.txt; exit 1; }
    echo "== $v pass $pass"; grep -v '^{"lib' gpurun_out/r6p/kb_${v}_$pass.txt | grep -v amdgpu.ids
  done
done
