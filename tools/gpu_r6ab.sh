#!/bin/bash
# Round 6, call ab: the tree as it ships (rebuilt in place after the last experiments): GPU suite, smoke, C3 and C5 lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_round.sh gpurun_out/ship tests smoke c3 c5
