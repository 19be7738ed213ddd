set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6a; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/c5trace -o c5 -- python3 -u bench.py --config C5 --steps 1 --warmup 0 --no-cpu-baseline --maps-out $O/c5_maps.txt > $O/c5trace.json 2> $O/c5trace.err; rc=$?
echo "c5 trace rc=$rc"; tail -3 $O/c5trace.err
[ $rc -eq 0 ] || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_brunet.py -x -q --timeout 300 --timeout-method thread > $O/brunet_tests.log 2>&1; rc=$?
tail -3 $O/brunet_tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/c3.json 2> $O/c3.err && python3 -c "import json;d=json.load(open('$O/c3.json'));print(d['value'],d['roofline']['frac'],d['roofline']['kernels']['ahtw']['frac'])"
