#!/bin/bash
# PMC passes over tools/kbench (one rocprofv3 run per counter group).  Usage: bash tools/pmc_kbench.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/pmck}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p "$OUT"
timeout -s KILL 60 rocprofv3 -L > "$OUT/counters.txt" 2>&1
run() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$name" -o run -- ./tools/kbench > "$OUT/$name.log" 2>&1 || { echo "pass $name failed"; return 1; }
  echo "pass $name ok"
}
run sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU && \
run sq2 SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE GRBM_COUNT && \
run lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE TCC_HIT_sum TCC_MISS_sum
python3 tools/pmc_summary.py "$OUT" > "$OUT/summary.txt"
