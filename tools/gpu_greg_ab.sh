#!/bin/bash
# A/B of the register-sourced Gram (tools/var/a_greg0.so = off, b_greg1.so = on): C3 bench twice each, then the
# 8-GPU replay.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
STEPS=3 RS=200 bash tools/gpu_var_bench.sh && STEPS=3 RS=200 bash tools/gpu_var_bench.sh || exit 1
for v in a_greg0 b_greg1; do
  NMFC_LIB=$PWD/tools/var/$v.so timeout -k 10 300 python -u bench.py --simulate-world 8 --steps 2 --warmup 1 > gpurun_out/var/sim8_$v.json 2> gpurun_out/var/sim8_$v.err \
    && python3 -c "import json,sys; d=json.load(open(sys.argv[1])); c=d['config']; print(sys.argv[2], 'sim8 per GPU', round(c['per_gpu_restarts_per_s'],1), 'equal', c['counts_equal_whole_sweep'])" gpurun_out/var/sim8_$v.json $v || { echo "sim8 $v failed"; tail -5 gpurun_out/var/sim8_$v.err; exit 1; }
done
