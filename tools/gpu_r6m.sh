#!/bin/bash
# Round 6: the refined Brunet per-kernel table (product build) against the round-5 configuration (tools/_var/base_old.so)
# and one neighbour (v5: RG 4 at k = 4, 5): per-k kernel times, interleaved; parity tests; the C5 line, interleaved.
set -o pipefail
OUT=${1:-gpurun_out/r6m}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p "$OUT"
for rep in 1 2; do
  for v in base_old new v5; do
    lib=""; [ $v != new ] && lib="--lib tools/_var/$v.so"
    timeout -k 10 300 python -u tools/brunet_kbench.py $lib > "$OUT/kb_${v}_$rep.txt" 2>&1 || { echo "kbench $v failed"; tail -5 "$OUT/kb_${v}_$rep.txt"; exit 1; }
    python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); pk=d['per_k']
print(sys.argv[2], ' '.join('%s:%.3f/%.3f'%(k,v['hnum_ms'],v['wupd_ms']) for k,v in pk.items()), 'sum %.3f'%sum(v['hnum_ms']+v['wupd_ms'] for v in pk.values()))" "$OUT/kb_${v}_$rep.txt" $v
  done
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_brunet.py tests/test_gpu_r_binding.py -x -q --timeout 300 --timeout-method thread \
  > "$OUT/tests.log" 2>&1 && echo "tests ok: $(tail -1 "$OUT/tests.log")" || { echo "tests failed"; grep -E "FAILED|Error|assert" "$OUT/tests.log" | head; exit 1; }
for rep in 1 2; do
  for v in new base_old; do
    f="$OUT/c5_${v}_$rep.json"
    if [ $v = new ]; then
      timeout -k 10 300 python -u bench.py --config C5 --steps 1 --warmup 1 --no-cpu-baseline > "$f" 2> "${f%.json}.err" || { tail -5 "${f%.json}.err"; exit 1; }
    else
      NMFC_LIB=$PWD/tools/_var/$v.so timeout -k 10 300 python -u bench.py --config C5 --steps 1 --warmup 1 --no-cpu-baseline > "$f" 2> "${f%.json}.err" || { tail -5 "${f%.json}.err"; exit 1; }
    fi
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value'],2), d['roofline']['frac'])" "$f" "C5 $v"
  done
done
