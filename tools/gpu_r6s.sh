#!/bin/bash
# Round 6, call s: why k_br_hnum runs 10-17 % longer than k_br_wupd at k = 4..8 with the same work per element: SQ
# counters of both kernels at k = 4, 5, 7 (C5 shape, R = 200, 10 iterations), one rocprofv3 --pmc pass per group.
set -o pipefail
OUT=gpurun_out/r6s
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p "$OUT"
CMD="tools/brunet_kbench.py --ks 4,5,7 --R 200 --T 10"
pass() {
  local name=$1; shift
  timeout -s KILL 150 rocprofv3 --pmc "$@" --kernel-include-regex "k_br_" --output-format csv \
     -d "$OUT/$name" -o run -- python3 $CMD > "$OUT/$name.log" 2>&1 || { echo "pass $name failed"; tail -3 "$OUT/$name.log"; return 1; }
  echo "pass $name ok"
}
timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 $CMD \
  > "$OUT/trace.log" 2>&1 && echo "trace ok" && \
pass busy SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU \
  SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE && \
pass insts SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE && \
pass lvl SQ_INST_LEVEL_SMEM SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_WAVES GRBM_GUI_ACTIVE
python3 tools/pmc_summary.py "$OUT" > "$OUT/summary.txt" 2>&1; echo summary done
for pass in 1 2; do
  if [ $pass = 1 ]; then L="new h512"; else L="h512 new"; fi
  for v in $L; do
    timeout -k 10 240 python -u tools/brunet_kbench.py --lib tools/br_$v.so > $OUT/kb_${v}_$pass.txt 2>&1 || { echo "kb $v failed"; tail $OUT/kb_${v}_$pass.txt; exit 1; }
    echo "== $v pass $pass"; grep -v '^{"lib' $OUT/kb_${v}_$pass.txt | grep -v amdgpu.ids
  done
done
