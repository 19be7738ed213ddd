# Round 6: the stream-K W^T A tile in the engine -- its bit-identity test first, the whole GPU suite, then the C3 line
# (default policy) and the one-group line, and FIXED-1000 (full-load rates).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6e; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "stream_k or tile_shapes" --timeout 240 --timeout-method thread > $O/sk_tests.log 2>&1; rc=$?
tail -2 $O/sk_tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
tail -2 $O/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/gpu_tests.log | head; exit 1; }
line() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d.get('roofline') or {}; k=r.get('kernels',{}); print(sys.argv[2], round(d['value'],2), 'frac', r.get('frac'), 'wta', k.get('wta',{}).get('tflops'), 'ahtw', k.get('ahtw',{}).get('tflops'))" "$1" "$2"; }
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/c3.json 2> $O/c3.err && line $O/c3.json C3-default || exit 1
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --groups 1 > $O/c3g1.json 2> $O/c3g1.err && line $O/c3g1.json C3-g1 || exit 1
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --groups 1 > $O/c3g1sk0.json 2> $O/c3g1sk0.err && line $O/c3g1sk0.json C3-g1-again || exit 1
NMFC_WTA_SK=0 timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --groups 1 > $O/c3nosk.json 2> $O/c3nosk.err && line $O/c3nosk.json C3-g1-noSK || exit 1
timeout -k 10 300 python -u bench.py --stop-rule fixed --maxiter 1000 --steps 1 --warmup 0 --no-cpu-baseline > $O/fixed.json 2> $O/fixed.err && line $O/fixed.json FIXED1000 || exit 1
