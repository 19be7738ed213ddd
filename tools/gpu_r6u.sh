#!/bin/bash
# Round 6, call u (final set, part 1, source after the batched reciprocal): GPU suite, smoke, the C3 profile (kernel
# stats + FETCH/WRITE PMC + agreement), the C3 line, and a default-lane C5 kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/final2
bash tools/gpu_round.sh $O tests smoke profile c3 || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c5trace -o run -- python3 bench.py --config C5 --steps 1 --warmup 0 --no-cpu-baseline > $O/c5trace.log 2>&1 && echo "c5 trace ok" || { echo "c5 trace failed"; tail -5 $O/c5trace.log; exit 1; }
