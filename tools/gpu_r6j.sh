#!/bin/bash
# Round 6: the 2-panel stream-K tile (k_wta2_sk<..., 2>): bit-identity tests, then interleaved A/B of NMFC_WTA_SK_MID on
# the 8-GPU shard's workload (R = 25, one and two groups) and on C3 (R = 200).
set -o pipefail
OUT=${1:-gpurun_out/r6j}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c3.py -x -v --timeout 300 --timeout-method thread \
  -k "stream_k or tile_shapes or c3_sweep or sharded" > "$OUT/tests.log" 2>&1 && echo "tests ok: $(tail -1 "$OUT/tests.log")" \
  || { echo "tests failed"; grep -E "FAILED|Error|assert" "$OUT/tests.log" | head -20; tail -5 "$OUT/tests.log"; exit 1; }
v() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value'],2), round(d['ms_per_step'],1))" "$1" "$2"; }
for rep in 1 2; do
  for cfg in "25 1" "25 2" "200 1"; do
    set -- $cfg
    for mid in 1 0; do
      f="$OUT/r$1_g$2_mid${mid}_$rep.json"
      NMFC_WTA_SK_MID=$mid timeout -k 10 300 python -u bench.py --restarts $1 --groups $2 --steps 3 --warmup 1 --no-cpu-baseline \
        > "$f" 2> "${f%.json}.err" && v "$f" "R=$1 G=$2 mid=$mid" || { tail -5 "${f%.json}.err"; exit 1; }
    done
  done
done
