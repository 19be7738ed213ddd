#!/bin/bash
# C5 sweep on small per-GPU shards with variant libraries: bash tools/gpu_brunet_small.sh lib.so ...
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/brsm
for lib in default "$@"; do
  for R in ${RS:-25 50}; do
    if [ "$lib" = default ]; then unset NMFC_LIB; else export NMFC_LIB=$(realpath "$lib"); fi
    b=$(basename "$lib" .so)
    timeout -k 10 200 python -u bench.py --config C5 --restarts $R --steps 1 --warmup 0 --no-cpu-baseline --no-timing \
      > gpurun_out/brsm/$b.$R.json 2> gpurun_out/brsm/$b.$R.err || { echo "$b R=$R failed"; tail -3 gpurun_out/brsm/$b.$R.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/brsm/$b.$R.json'));print('$b R=$R', round(d['value'],2), 'restarts/s', round(d['ms_per_step']), 'ms')"
  done
done
