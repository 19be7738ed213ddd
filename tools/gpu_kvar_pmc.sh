#!/bin/bash
# SQ counters of the full-load MFMA kernel arms of tools/kvar (pmc mode: n = 500, one round per arm), one rocprofv3
# --pmc pass per counter group (never combined with tracing), then a kernel trace for durations / clock.
# Usage (GPU box): bash tools/gpu_kvar_pmc.sh <outdir>; summary: python3 tools/pmc_kvar.py <outdir>
set -o pipefail
OUT=${1:-gpurun_out/kvar_pmc}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p "$OUT"
timeout -s KILL 60 rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
pass() {
  local name=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" --kernel-include-regex "k_ahtw|k_wta2" --output-format csv \
     -d "$OUT/$name" -o run -- ./tools/kvar 200 3 pmc > "$OUT/$name.log" 2>&1 || { echo "pass $name failed"; return 1; }
  echo "pass $name ok"
}
timeout -k 10 90 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- ./tools/kvar 200 3 pmc \
  > "$OUT/trace.log" 2>&1 && echo "trace ok" && \
pass busy SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES \
  SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE && \
pass insts SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES GRBM_GUI_ACTIVE && \
pass active SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM \
  SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE
