#!/bin/bash
# tools/teambench (k_team_mu phase breakdown), the nmf_mu parity tests and the drop-in latency table.
# Usage: bash tools/gpu_teambench.sh
set -o pipefail
OUT=gpurun_out/team2; mkdir -p $OUT
timeout -k 10 120 ./tools/teambench 2000 > $OUT/teambench.txt 2>&1; rc=$?; cat $OUT/teambench.txt; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "mu1 or mfma_layout or nmf_mu" > $OUT/parity.log 2>&1 && tail -3 $OUT/parity.log || { tail -30 $OUT/parity.log; exit 1; }
timeout -k 10 200 python -u tools/nmf_mu_latency.py 5 > $OUT/latency.json && cat $OUT/latency.json || exit 1
