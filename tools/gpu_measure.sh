#!/bin/bash
# Round measurements on one GPU: drop-in nmf_mu per-call latency vs the reference nmf_mu, the C1 line (test_nmf.r's
# case: batched sweep, drop-in flow, the reference on one core), the C2 bench
# line (small-shape path), the default C3 bench line with the CPU baseline, and the C3 FIXED T = 1000 line
# (SURVEY 8(d) timing mode (i): the roofline with every restart live).  Usage: bash tools/gpu_measure.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/measure
timeout -k 10 300 python -u tools/nmf_mu_latency.py 3 > gpurun_out/measure/nmf_mu_latency.json 2> gpurun_out/measure/nmf_mu_latency.err \
  && echo "latency ok" && cat gpurun_out/measure/nmf_mu_latency.json &&
timeout -k 10 300 python -u bench.py --config C1 --steps 5 --warmup 1 > gpurun_out/measure/c1_bench.json 2> gpurun_out/measure/c1_bench.err \
  && echo "c1 ok" && cat gpurun_out/measure/c1_bench.json &&
timeout -k 10 300 python -u bench.py --config C2 --steps 5 --warmup 1 > gpurun_out/measure/c2_bench.json 2> gpurun_out/measure/c2_bench.err \
  && echo "c2 ok" && cat gpurun_out/measure/c2_bench.json &&
timeout -k 10 600 python -u bench.py > gpurun_out/measure/c3_bench.json 2> gpurun_out/measure/c3_bench.err \
  && echo "c3 ok" && cat gpurun_out/measure/c3_bench.json &&
timeout -k 10 300 python -u bench.py --stop-rule fixed --maxiter 1000 --steps 1 --warmup 0 --no-cpu-baseline \
  > gpurun_out/measure/c3_fixed1000.json 2> gpurun_out/measure/c3_fixed1000.err \
  && echo "c3 fixed-1000 ok (SURVEY 8(d) timing mode i: every restart live for 1000 iterations)" \
  && cat gpurun_out/measure/c3_fixed1000.json
