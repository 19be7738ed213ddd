#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 350 --timeout-method thread -k c4 > gpurun_out/c4_test.log 2>&1 || { echo "c4 test failed"; tail -30 gpurun_out/c4_test.log; exit 1; }
echo "c4 test ok"; grep -E "passed|failed" gpurun_out/c4_test.log | tail -1
timeout -k 10 300 python -u bench.py --config C4 --restarts 8 --maxiter 100 --stop-rule fixed --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err || { echo "c4 bench failed"; tail gpurun_out/bench_c4.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/bench_c4.json'));print(d['value'], d['ms_per_step'], json.dumps(d['roofline']['kernels']))"
