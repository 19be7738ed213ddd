#!/bin/bash
# A/B of library variants (tools/var/*.so) on the small-shape configs C1 and C2 (two passes), then the GPU suite on the
# last variant (NMFC_LIB) for its parity.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/small_ab; mkdir -p $OUT
last=""
for pass in 1 2; do
  for so in tools/var/*.so; do
    v=$(basename $so .so); last=$so
    for C in C1 C2; do
      NMFC_LIB=$PWD/$so timeout -k 10 200 python -u bench.py --config $C --steps 10 --warmup 2 --no-cpu-baseline > $OUT/$v.$C.$pass.json 2> $OUT/$v.$C.$pass.err \
        || { echo "$v $C failed"; tail -5 $OUT/$v.$C.$pass.err; exit 1; }
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], round(d['value'],1), 'restarts/s', round(d['ms_per_step'],2), 'ms')" $OUT/$v.$C.$pass.json $v $C
    done
  done
done
NMFC_LIB=$PWD/$last timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $OUT/tests.log 2>&1; tail -3 $OUT/tests.log
