#!/bin/bash
# Round 6: Brunet operand rows by scalar loads (NMFC_BR_SLOAD) -- per-k kernel times of the variants, interleaved,
# then the Brunet GPU parity tests on the scalar-load build and the C5 line of each.
set -o pipefail
OUT=${1:-gpurun_out/r6k}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p "$OUT"
for rep in 1 2; do
  for v in base sload sload_spl0 sload_rglo; do
    lib=""; [ $v != base ] && lib="--lib tools/_var/$v.so"
    timeout -k 10 300 python -u tools/brunet_kbench.py $lib > "$OUT/kb_${v}_$rep.txt" 2>&1 || { echo "kbench $v failed"; tail -5 "$OUT/kb_${v}_$rep.txt"; exit 1; }
    python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); pk=d['per_k']
print(sys.argv[2], ' '.join('%s:%.3f/%.3f'%(k,v['hnum_ms'],v['wupd_ms']) for k,v in pk.items()), 'sum %.3f'%sum(v['hnum_ms']+v['wupd_ms'] for v in pk.values()))" "$OUT/kb_${v}_$rep.txt" $v
  done
done
NMFC_LIB=$PWD/tools/_var/sload.so timeout -k 10 600 python -u -m pytest tests/test_gpu_brunet.py tests/test_gpu_r_binding.py -x -q --timeout 300 --timeout-method thread \
  > "$OUT/tests_sload.log" 2>&1 && echo "sload tests ok: $(tail -1 "$OUT/tests_sload.log")" || { echo "sload tests failed"; grep -E "FAILED|Error|assert" "$OUT/tests_sload.log" | head; exit 1; }
