#!/bin/bash
# Round 6, call t: H-side gene chunk count (NMFC_BR_NCHUNK 16 / 32 / 48): Brunet kernel times (tools/brunet_kbench.py)
# and the C5 line per library, interleaved twice; then the Brunet GPU tests against the 32-chunk library.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6t
mkdir -p $O
for pass in 1 2; do
  if [ $pass = 1 ]; then L="new nc32 nc48"; else L="nc48 nc32 new"; fi
  for v in $L; do
    timeout -k 10 240 python -u tools/brunet_kbench.py --lib tools/br_$v.so > $O/kb_${v}_$pass.txt 2>&1 || { echo "kb $v failed"; tail $O/kb_${v}_$pass.txt; exit 1; }
    echo "== $v pass $pass: $(python3 -c "
import json,sys
for l in open(sys.argv[1]):
    if l.startswith('{\"lib'): d=json.loads(l)['per_k']
print('hnum', round(sum(v['hnum_ms'] for v in d.values()),3), 'hupd', round(sum(v['hupd_ms'] for v in d.values()),3), 'wupd', round(sum(v['wupd_ms'] for v in d.values()),3), 'hnum per k', [v['hnum_ms'] for v in d.values()])" $O/kb_${v}_$pass.txt)"
    NMFC_LIB=tools/br_$v.so timeout -k 10 300 python -u bench.py --config C5 --steps 1 --warmup 1 --no-cpu-baseline > $O/c5_${v}_$pass.json 2> $O/c5_${v}_$pass.err || { tail -5 $O/c5_${v}_$pass.err; exit 1; }
    echo "   C5 $v: $(python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(round(d['value'],2), round(d['roofline']['frac'],4))" $O/c5_${v}_$pass.json)"
  done
done
NMFC_LIB=tools/br_nc32.so timeout -k 10 400 python -u -m pytest tests/test_gpu_brunet.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests_nc32.log 2>&1; tail -3 $O/tests_nc32.log
