# Round 6: one-GPU replay of the 8 shards of the C4 8-GPU job (BASELINE configs[3]: 60000 x 2000, k = 2..15,
# R = 1000 -> 14 000 jobs, 1 750 per shard), VERDICT r05 item 4.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6b; mkdir -p $O
timeout -k 10 1050 python -u bench.py --config C4 --simulate-world 8 --steps 1 --warmup 0 --dump-iters $O/c4_sim8_iters.npy \
  > $O/c4_sim8.json 2> $O/c4_sim8.err; rc=$?
echo "rc=$rc"; tail -12 $O/c4_sim8.err; exit $rc
