#!/bin/bash
# Runs tools/kvar (full-load MFMA kernel variants) on the GPU box.  Usage: bash tools/gpu_kvar.sh <outfile> [R]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 240 ./tools/kvar ${2:-200} 10 > "$1" 2>&1; rc=$?; cat "$1"; exit $rc
