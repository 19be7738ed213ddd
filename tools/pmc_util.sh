#!/bin/bash
# Matrix / vector pipe utilisation counters for the MU and Brunet kernels, one rocprofv3 --pmc pass per
# group (never combined with tracing).  MU: C3 FIXED 20 iterations (every restart live); Brunet: C5, 20
# iterations.  Usage (GPU box): bash tools/pmc_util.sh <outdir>; then python3 tools/pmc_util.py <outdir>
set -o pipefail
OUT=${1:-gpurun_out/pmcu}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p "$OUT"
timeout -s KILL 60 rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
MU="--config C3 --stop-rule fixed --maxiter 20 --steps 1 --warmup 0 --no-cpu-baseline --no-timing"
BR="--config C5 --maxiter 20 --steps 1 --warmup 0 --no-cpu-baseline --no-timing"
run() {
  local name=$1 regex=$2 args=$3; shift 3
  timeout -s KILL 150 rocprofv3 --pmc "$@" --kernel-include-regex "$regex" --output-format csv \
     -d "$OUT/$name" -o run -- python3 bench.py $args > "$OUT/$name.log" 2>&1 || { echo "pass $name failed"; return 1; }
  echo "pass $name ok"
}
run mu_busy "k_wta2|k_ahtw4|k_hupdate" "$MU" SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE GRBM_COUNT && \
run mu_insts "k_wta2|k_ahtw4|k_hupdate" "$MU" SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAVES && \
run br_busy "k_br_hnum|k_br_wupd|k_br_hupd" "$BR" SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE GRBM_COUNT && \
run br_insts "k_br_hnum|k_br_wupd|k_br_hupd" "$BR" SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAVES
[ $? -eq 0 ] || exit 1
for w in mu br; do
  args=$MU; [ $w = br ] && args=$BR
  timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${w}_trace" -o run -- python3 bench.py $args \
    > "$OUT/${w}_trace.log" 2>&1 || { echo "trace $w failed"; exit 1; }
  echo "trace $w ok"
done
