#!/bin/bash
# PMC passes over a short FIXED-iteration C3 sweep (one rocprofv3 run per counter group; never combined
# with tracing domains).  Usage (GPU box): bash tools/pmc_passes.sh <outdir> [extra bench args]
set -o pipefail
OUT=${1:-gpurun_out/pmc}
shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
ARGS="--config C3 --stop-rule fixed --maxiter 20 --steps 1 --warmup 0 --no-cpu-baseline --no-timing $*"
run() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-include-regex "k_wta|k_ahtw|k_hupdate" --output-format csv \
     -d "$OUT/$name" -o run -- python3 bench.py $ARGS > "$OUT/$name.log" 2>&1 || { echo "pass $name failed"; return 1; }
  echo "pass $name ok"
}
mkdir -p "$OUT"
run sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS && \
run fetch FETCH_SIZE && \
run write WRITE_SIZE && \
run tcc TCC_HIT_sum TCC_MISS_sum && \
run lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT
