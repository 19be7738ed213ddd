#!/bin/bash
# SQ counters of the Brunet kernels (k_br_hnum / k_br_wupd / k_br_hupd) at the C5 shape, k = 2, 5, 10, 200 restarts,
# 10 iterations (tools/brunet_kbench.py), one rocprofv3 --pmc pass per counter group (never combined with tracing),
# then a kernel trace for durations.  Usage (GPU box): bash tools/gpu_brunet_pmc.sh <outdir>; summary:
# python3 tools/pmc_kvar.py <outdir>
set -o pipefail
OUT=${1:-gpurun_out/brunet_pmc}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p "$OUT"
CMD="tools/brunet_kbench.py --ks 2,5,10 --R 200 --T 10"
pass() {
  local name=$1; shift
  timeout -s KILL 150 rocprofv3 --pmc "$@" --kernel-include-regex "k_br_" --output-format csv \
     -d "$OUT/$name" -o run -- python3 $CMD > "$OUT/$name.log" 2>&1 || { echo "pass $name failed"; return 1; }
  echo "pass $name ok"
}
timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 $CMD \
  > "$OUT/trace.log" 2>&1 && echo "trace ok" && \
pass busy SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU \
  SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE && \
pass insts SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE && \
pass lds SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 GRBM_GUI_ACTIVE
