#!/bin/bash
# Stall breakdown of the small-grid kernels: one rocprofv3 --pmc pass (SQ wave-state counters) over
# tools/tailbench at the given live-panel counts.  Usage: bash tools/pmc_tail.sh <outdir> [R] [lives]
set -o pipefail
OUT=${1:-gpurun_out/pmc_tail}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p "$OUT"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d "$OUT/sq" -o run -- \
  ./tools/tailbench "${2:-25}" "${3:-1}" > "$OUT/sq.log" 2>&1 || { echo "pmc pass failed"; tail -5 "$OUT/sq.log"; exit 1; }
python3 tools/pmc_tail.py "$OUT/sq"
