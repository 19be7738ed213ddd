#!/bin/bash
# Round profile on the GPU box: rocprofv3 kernel-trace stats of the default bench command, then
# separate PMC passes (FETCH_SIZE, WRITE_SIZE) over the same command for the HBM traffic of the engine
# kernels (W^T A, A h^T, H update, labels, counts).  Usage: bash tools/profile_round.sh <outdir>   (then copy the summaries into profiles/)
set -o pipefail
OUT=${1:-gpurun_out/profile}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p "$OUT"
CMD="bench.py --steps 1 --warmup 0 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 $CMD \
  > "$OUT/trace.log" 2>&1 || { echo "trace pass failed"; exit 1; }
echo "trace ok"
for pass in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $pass --kernel-include-regex "k_wta|k_ahtw|k_hupdate|k_labels|k_counts" --output-format csv \
    -d "$OUT/$pass" -o run -- python3 $CMD > "$OUT/$pass.log" 2>&1 || { echo "pass $pass failed"; exit 1; }
  echo "pmc $pass ok"
done
python3 tools/pmc_traffic.py "$OUT" > "$OUT/pmc_traffic.json" && cat "$OUT/pmc_traffic.json"
