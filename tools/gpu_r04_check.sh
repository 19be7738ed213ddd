#!/bin/bash
# Round-4 check on one GPU (one call): the whole -m gpu suite, smoke(), then the shard-2 trace with two restart groups.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=${1:-gpurun_out/r04_check}; mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 \
  && echo "tests ok: $(tail -1 "$OUT/gpu_tests.log")" || { echo "tests failed"; grep -E "FAILED|Error" "$OUT/gpu_tests.log" | head; tail -20 "$OUT/gpu_tests.log"; exit 1; }
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 && tail -1 "$OUT/smoke.log" || exit 1
RANK_=2 WORLD_=8 GROUPS_=2 bash tools/gpu_shard_trace.sh "$OUT/shard2_g2" > /dev/null 2>&1; cat "$OUT/shard2_g2/untraced.log" && python3 tools/phase_split.py "$OUT/shard2_g2/trace/run_kernel_trace.csv"
