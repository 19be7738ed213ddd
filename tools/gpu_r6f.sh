# Round 6: restart groups for the strong-scaling shards now that the big W^T A tile is stream-K (R per GPU = 100, 50:
# the N = 2, 4 shards' workloads on one GPU), and the 8-GPU replay (R = 25 shards: the big-tile grid stays below one
# round there, so no stream-K).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6f; mkdir -p $O
for R in 100 50; do for G in 1 2 1 2; do
  timeout -k 10 200 python -u bench.py --restarts $R --groups $G --steps 4 --warmup 1 --no-cpu-baseline --no-timing > $O/r${R}_g${G}.json 2> $O/r${R}_g${G}.err || exit 1
  python3 -c "import json;d=json.load(open('$O/r${R}_g${G}.json'));print('R=$R G=$G', round(d['value'],2))"
done; done
timeout -k 10 400 python -u bench.py --simulate-world 8 --steps 2 --warmup 1 > $O/sim8.json 2> $O/sim8.err && python3 -c "import json; d=json.load(open('$O/sim8.json')); c=d['config']; print('sim8 per GPU', round(c['per_gpu_restarts_per_s'],1), [round(x*1e3) for x in c['shard_seconds']], c['counts_equal_whole_sweep'])"
