#!/bin/bash
# Wave-state (SQ) counters of the MU kernels on C3 with every restart live (FIXED 20 iterations), one
# rocprofv3 --pmc pass per counter group, for each library build given (default: the product lib).
# Usage (GPU box): bash tools/pmc_stall.sh <outdir> [lib.so ...]; summary via tools/pmc_tail.py <outdir>/<lib>
set -o pipefail
OUT=${1:-gpurun_out/stall}; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p "$OUT"
timeout -s KILL 60 rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
ARGS="--config C3 --stop-rule fixed --maxiter 20 --steps 1 --warmup 0 --no-cpu-baseline --no-timing"
LIBS=("$@"); [ ${#LIBS[@]} -eq 0 ] && LIBS=(nmfconsensus_amd/lib/libnmf.so)
for so in "${LIBS[@]}"; do
  v=$(basename "$so" .so)
  NMFC_LIB=$PWD/$so timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
    SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --kernel-include-regex "k_wta2|k_ahtw4|k_hupdate" \
    --output-format csv -d "$OUT/$v/sq" -o run -- python3 bench.py $ARGS > "$OUT/$v.sq.log" 2>&1 || { echo "$v sq pass failed"; exit 1; }
  NMFC_LIB=$PWD/$so timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAVES \
    --kernel-include-regex "k_wta2|k_ahtw4|k_hupdate" \
    --output-format csv -d "$OUT/$v/insts" -o run -- python3 bench.py $ARGS > "$OUT/$v.insts.log" 2>&1 || { echo "$v insts pass failed"; exit 1; }
  echo "== $v"; python3 tools/pmc_tail.py "$OUT/$v"
done
