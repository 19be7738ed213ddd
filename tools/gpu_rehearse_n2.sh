#!/bin/bash
# Rehearsal of the driver's N > 1 bench flow on a ONE-GPU box: two ranks under torch.distributed.run, both on
# cuda:0, gloo all-reduce of the counts (RCCL needs one GPU per rank).  Checks the sharded sweep, the restart
# groups, the barrier / max-over-ranks timing and the rank-0 JSON line; the number is not a measurement.
# Usage: bash tools/gpu_rehearse_n2.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/n2}
mkdir -p "$OUT"
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --steps 1 --warmup 1 --dist-backend gloo --device 0 > "$OUT/n2.json" 2> "$OUT/n2.err" \
  && python3 -c "import json,sys; d=json.loads([x for x in open(sys.argv[1]) if x.startswith('{')][-1]); print('N=2 rehearsal', d['n_gpus'], round(d['value'],1), d['scaling'], d['config']['parallelism'], d['config']['groups_per_gpu'])" "$OUT/n2.json" \
  || { tail -20 "$OUT/n2.err"; exit 1; }
