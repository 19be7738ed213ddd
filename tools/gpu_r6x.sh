#!/bin/bash
# Round 6, call x: engine knobs re-measured on the 8-GPU shard (R = 25 per GPU, two restart groups, the N = 8 policy) and
# on C3 (R = 200, one group), since the stream-K tiles: A h^T gene tile (NMFC_AHTW_TILE), repack divisor, narrow-form
# block limit, poll cadence.  Two interleaved passes.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6x
mkdir -p $O
run() {   # name, R, G, env..., -- extra bench args
  local name=$1 R=$2 G=$3; shift 3
  local envs=() args=()
  while [ $# -gt 0 ] && [ "$1" != "--" ]; do envs+=("$1"); shift; done
  [ "$1" = "--" ] && shift
  args=("$@")
  env "${envs[@]}" timeout -k 10 300 python -u bench.py --restarts $R --groups $G --steps 3 --warmup 1 --no-cpu-baseline "${args[@]}" > $O/$name.json 2> $O/$name.err || { tail -5 $O/$name.err; exit 1; }
  echo "$name: $(python3 -c "import json,sys; print(round(json.load(open(sys.argv[1]))['value'],1))" $O/$name.json)"
}
for rep in 1 2; do
  run r25_def_$rep 25 2 X=1
  run r25_ahtw128_$rep 25 2 NMFC_AHTW_TILE=128
  run r25_rd10_$rep 25 2 NMFC_REPACK_DIV=10
  run r25_rd40_$rep 25 2 NMFC_REPACK_DIV=40
  run r25_nmb5_$rep 25 2 NMFC_NARROW_MAXB=5
  run r25_ce2_$rep 25 2 X=1 -- --check-every 2
  run r25_ce8_$rep 25 2 X=1 -- --check-every 8
  run r200_def_$rep 200 1 X=1
  run r200_ahtw128_$rep 200 1 NMFC_AHTW_TILE=128
  run r200_rd40_$rep 200 1 NMFC_REPACK_DIV=40
done
