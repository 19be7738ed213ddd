#!/bin/bash
# Round 6, call aa: the Brunet inner-loop unroll re-measured on the batched-reciprocal source: the shipped per-k tables
# (new) against one global unroll 1 / 2 / 4 / 8, tools/brunet_kbench.py, two interleaved passes.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6aa
mkdir -p $O
for pass in 1 2; do
  if [ $pass = 1 ]; then L="new u1 u2 u4 u8"; else L="u8 u4 u2 u1 new"; fi
  for v in $L; do
    timeout -k 10 240 python -u tools/brunet_kbench.py --lib tools/br_$v.so > $O/kb_${v}_$pass.txt 2>&1 || { echo "kb $v failed"; tail $O/kb_${v}_$pass.txt; exit 1; }
    echo "== $v pass $pass"
  done
done
python3 - <<'PY'
import json,glob,collections
res=collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob('gpurun_out/r6aa/kb_*.txt'):
    v=f.split('kb_')[1].rsplit('_',1)[0]
    for l in open(f):
        if l.startswith('{"lib'):
            for k,d in json.loads(l)['per_k'].items():
                res[v][(int(k),'h')].append(d['hnum_ms']); res[v][(int(k),'w')].append(d['wupd_ms'])
for side in 'hw':
    print('side',side)
    for k in range(2,11):
        print('  k',k,' '.join(f"{v}:{sum(res[v][(k,side)])/len(res[v][(k,side)]):.4f}" for v in ('new','u1','u2','u4','u8')))
PY
