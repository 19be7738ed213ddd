#!/bin/bash
# Round 6, call v (final set, part 2): FIXED-1000, the 8-GPU replay, C1 / C2, the C4 shard, C5, per-call latency.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_round.sh gpurun_out/final2 fixed sim8 small c4 c5 latency
