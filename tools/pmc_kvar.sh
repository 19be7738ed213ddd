#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of k_ahtw4 in the tools/var/kbench_SP_SG tile-map variants (one PMC pass each).
set -o pipefail
OUT=${1:-gpurun_out/pmckv}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p "$OUT"
for v in "${@:2}"; do
  for pass in ${PASSES:-FETCH_SIZE WRITE_SIZE}; do
    timeout -s KILL 120 rocprofv3 --pmc $pass --kernel-include-regex "k_ahtw4" --output-format csv \
      -d "$OUT/$v/$pass" -o run -- ./tools/var/kbench_$v > "$OUT/$v.$pass.log" 2>&1 || { echo "pass $v $pass failed"; exit 1; }
  done
  python3 tools/pmc_traffic.py "$OUT/$v" > "$OUT/$v.json" && echo "== $v" && cat "$OUT/$v.json"
done
