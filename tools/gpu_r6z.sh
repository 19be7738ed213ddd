#!/bin/bash
# Round 6, call z: H side RG 2 at k = 6 and 10 (two quotients per gene step: one shared v_rcp_f64) against the shipped
# RG 1, tools/brunet_kbench.py --ks 6,10, alternating three times; then the C5 line for each library, twice.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6z
mkdir -p $O
for rep in 1 2 3; do
  for v in new h610; do
    timeout -k 10 120 python -u tools/brunet_kbench.py --lib tools/br_$v.so --ks 6,10 > $O/kb_${v}_$rep.txt 2>&1 || { echo "kb $v failed"; tail $O/kb_${v}_$rep.txt; exit 1; }
    echo "$v rep $rep: $(grep -E '^(6|10) ' $O/kb_${v}_$rep.txt | tr '\n' ' ')"
  done
done
for rep in 1 2; do
  for v in new h610; do
    NMFC_LIB=tools/br_$v.so timeout -k 10 300 python -u bench.py --config C5 --steps 1 --warmup 1 --no-cpu-baseline > $O/c5_${v}_$rep.json 2> $O/c5_${v}_$rep.err || { tail -5 $O/c5_${v}_$rep.err; exit 1; }
    echo "C5 $v rep $rep: $(python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(round(d['value'],2), round(d['roofline']['frac'],4))" $O/c5_${v}_$rep.json)"
  done
done
