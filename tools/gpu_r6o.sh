#!/bin/bash
# Round 6, call o: the Brunet batch reciprocal (NMFC_BR_RCPB).  v_rcp_f64 issue rate and the batched quotient's
# agreement with IEEE a / p (tools/quot_probe), then tools/brunet_kbench.py on the HEAD-source library (br_base) and
# the batch sizes 1 / 2 / 4 / 8 built from the new source, interleaved in two passes.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r6o
timeout -k 10 120 ./tools/quot_probe 1 rate > gpurun_out/r6o/rcp_rate.txt 2>&1 || { echo "rate probe failed"; cat gpurun_out/r6o/rcp_rate.txt; exit 1; }
cat gpurun_out/r6o/rcp_rate.txt
timeout -k 10 240 ./tools/quot_probe 268435456 > gpurun_out/r6o/quot_probe.txt 2>&1 || { echo "quot probe failed"; cat gpurun_out/r6o/quot_probe.txt; exit 1; }
cat gpurun_out/r6o/quot_probe.txt
for pass in 1 2; do
  if [ $pass = 1 ]; then L="base rcp1 rcp2 rcp4 rcp8"; else L="rcp8 rcp4 rcp2 rcp1 base"; fi
  for v in $L; do
    timeout -k 10 240 python -u tools/brunet_kbench.py --lib tools/br_$v.so > gpurun_out/r6o/kb_${v}_$pass.txt 2>&1 || { echo "kb $v failed"; tail gpurun_out/r6o/kb_${v}_$pass.txt; exit 1; }
    echo "== $v pass $pass"; grep -v '^{"lib' gpurun_out/r6o/kb_${v}_$pass.txt | grep -v amdgpu.ids
  done
done
