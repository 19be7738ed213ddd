# Round 6: the GPU suite on this tree, then the N = 1 restart-group A/B (interleaved, one box) for bench.py's policy.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6c; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
tail -3 $O/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/gpu_tests.log | head; exit 1; }
for rep in 1 2; do for G in 1 2 3; do
  timeout -k 10 200 python -u bench.py --groups $G --steps 4 --warmup 1 --no-cpu-baseline --no-timing > $O/g${G}_$rep.json 2> $O/g${G}_$rep.err || exit 1
  python3 -c "import json;d=json.load(open('$O/g${G}_$rep.json'));print('G=$G rep $rep', round(d['value'],2))"
done; done
