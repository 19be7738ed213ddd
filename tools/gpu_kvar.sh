#!/bin/bash
# Runs every tools/var/kbench_* variant binary (tile-map / shape experiments), one after another.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/kvar
for b in tools/var/kbench_*; do
  n=$(basename "$b")
  timeout -k 10 120 "$b" > "gpurun_out/kvar/$n.log" 2>&1 || { echo "$n failed rc=$?"; exit 1; }
  echo "== $n"; grep -E "k_ahtw4|k_wta2|ahtw main" "gpurun_out/kvar/$n.log"
done
