#!/bin/bash
# Round 6, call q: is the k = 7 Brunet kernel time a property of the library (code placement) or of the k runs before
# it?  br_new and br_va hold identical k = 7 kernels (same template arguments, same loop alignment mod 64).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r6q
for rep in 1 2 3; do
  for v in new va; do
    for ks in 7 6,7 2,3,4,5,6,7; do
      timeout -k 10 120 python -u tools/brunet_kbench.py --lib tools/br_$v.so --ks $ks > gpurun_out/r6q/kb_${v}_${ks}_$rep.txt 2>&1 || { echo "kb $v $ks failed"; tail gpurun_out/r6q/kb_${v}_${ks}_$rep.txt; exit 1; }
      echo "$v ks=$ks rep $rep: $(grep '^7 ' gpurun_out/r6q/kb_${v}_${ks}_$rep.txt)"
    done
  done
done
