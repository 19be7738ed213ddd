#!/bin/bash
# Per-GPU work of an N-GPU C3 run simulated on one GPU (R = 200/N restarts per k); optional trace of
# the R = 25 (N = 8) shard.  NGROUPS (default 2) = restart groups per GPU, the bench's policy for N > 1 shards.
# Usage: bash tools/gpu_scaling_probe.sh   (RS="25 50 100" NGROUPS=1|2 TRACE=1)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for R in ${RS:-25 50 100}; do
  timeout -k 10 300 python -u bench.py --restarts $R --steps 2 --warmup 1 --no-cpu-baseline --groups ${NGROUPS:-2} > gpurun_out/scal_$R.json 2> gpurun_out/scal_$R.err || { echo "R=$R failed"; tail gpurun_out/scal_$R.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/scal_$R.json'));print('R=$R', round(d['value'],1), 'restarts/s', round(d['ms_per_step'],1), 'ms/step')"
done
if [ -n "${TRACE:-}" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/scal_trace -o run -- python3 bench.py --restarts 25 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/scal_trace.log 2>&1 || { echo trace failed; exit 1; }
  echo trace ok
fi
