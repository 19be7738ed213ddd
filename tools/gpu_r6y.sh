#!/bin/bash
# Round 6, call y: kernel trace of the 8-GPU shard as the N = 8 policy runs it (R = 25 per GPU, two restart groups), one
# warm-up sweep and one traced sweep, for the overlap of the two groups' kernels.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6y
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 bench.py --restarts 25 --groups 2 --steps 1 --warmup 1 --no-cpu-baseline --no-timing > $O/trace.log 2>&1 && echo "trace ok" && grep '^{' $O/trace.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace1 -o run -- python3 bench.py --restarts 25 --groups 1 --steps 1 --warmup 1 --no-cpu-baseline --no-timing > $O/trace1.log 2>&1 && echo "trace1 ok" && grep '^{' $O/trace1.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])"
