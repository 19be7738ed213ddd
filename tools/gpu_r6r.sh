#!/bin/bash
# Round 6, call r: the GPU suite and smoke on the batched-reciprocal source, the C5 line, and restart groups per GPU at
# the strong-scaling shard sizes (R = 25: the 8-GPU C3 shard; R = 50: 4 GPUs), G = 1..4 interleaved twice.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6r
mkdir -p $O
bash tools/gpu_round.sh $O tests smoke c5 || exit 1
for rep in 1 2; do
  for R in 25 50; do
    for G in 1 2 3 4; do
      timeout -k 10 200 python -u bench.py --restarts $R --groups $G --steps 3 --warmup 1 --no-cpu-baseline > $O/g_R${R}_G${G}_$rep.json 2> $O/g_R${R}_G${G}_$rep.err || { tail -5 $O/g_R${R}_G${G}_$rep.err; exit 1; }
      echo "R=$R G=$G rep $rep: $(python3 -c "import json,sys; print(round(json.load(open(sys.argv[1]))['value'],1))" $O/g_R${R}_G${G}_$rep.json)"
    done
  done
done
