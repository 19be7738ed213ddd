#!/bin/bash
# The round's GPU measurement set, one gpurun call, parts chosen by name (round 5: replaces gpu_final*.sh, gpu_r04*.sh
# and gpu_roundend.sh).  Usage: bash tools/gpu_round.sh <outdir> [part ...]    (no parts: all, in this order)
#   tests    the -m gpu suite                       smoke    __graft_entry__.smoke()
#   profile  rocprofv3 kernel stats + FETCH/WRITE PMC passes of the default C3 bench (tools/profile_round.sh), the
#            bench-vs-rocprof agreement (tools/profile_agreement.py)
#   c3       the C3 line with its CPU baseline       fixed    C3 FIXED-1000 (every restart live: full-load rates)
#   sim8     bench.py --simulate-world 8 (the 8 real shards of the 8-GPU job, replayed on one GPU)
#   small    C1 and C2 lines                        c4       the C4 per-GPU shard line    c5    the Brunet C5 line
#   latency  per-call nmf_mu vs the reference's     cpuscale the reference nmf_mu at 1..16 host processes
# Every GPU step runs under its own time limit; the first failure ends the call.
set -o pipefail
OUT=${1:?usage: gpu_round.sh <outdir> [part ...]}; shift
PARTS=${*:-tests smoke profile c3 fixed sim8 small c4 c5 latency cpuscale}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p "$OUT"
line() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d.get('roofline') or {}; print(sys.argv[2], round(d['value'],2), d['unit'], 'frac', r.get('frac'), 'cpu', (d.get('cpu_baseline') or {}).get('value'))" "$1" "$2"; }
for p in $PARTS; do
  case $p in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 \
        && echo "tests ok: $(tail -1 "$OUT/gpu_tests.log")" || { echo "tests failed"; grep -E "FAILED|Error" "$OUT/gpu_tests.log" | head; tail -20 "$OUT/gpu_tests.log"; exit 1; } ;;
    smoke)
      timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 && tail -1 "$OUT/smoke.log" || exit 1 ;;
    profile)
      bash tools/profile_round.sh "$OUT/profile" > "$OUT/profile.log" 2>&1 || { echo "profile failed"; tail -5 "$OUT/profile.log"; exit 1; }
      f=$(find "$OUT/profile/trace" -name '*kernel_stats.csv' | head -1)
      cp "$f" "$OUT/kernel_stats.csv" && cp "$OUT/profile/pmc_traffic.json" "$OUT/pmc_traffic.json" || exit 1
      grep -h '^{' "$OUT/profile/trace.log" | tail -1 > "$OUT/bench_under_rocprof.json"
      python3 tools/profile_agreement.py "$OUT/bench_under_rocprof.json" "$OUT/kernel_stats.csv" > "$OUT/agreement.txt" && cat "$OUT/agreement.txt" || exit 1 ;;
    c3)
      timeout -k 10 600 python -u bench.py > "$OUT/c3_bench.json" 2> "$OUT/c3_bench.err" && line "$OUT/c3_bench.json" C3 || { tail -5 "$OUT/c3_bench.err"; exit 1; } ;;
    fixed)
      timeout -k 10 300 python -u bench.py --stop-rule fixed --maxiter 1000 --steps 1 --warmup 0 --no-cpu-baseline \
        > "$OUT/c3_fixed1000.json" 2> "$OUT/c3_fixed1000.err" && line "$OUT/c3_fixed1000.json" FIXED-1000 || { tail -5 "$OUT/c3_fixed1000.err"; exit 1; } ;;
    sim8)
      timeout -k 10 300 python -u bench.py --simulate-world 8 --steps 2 --warmup 1 > "$OUT/sim8.json" 2> "$OUT/sim8.err" \
        && python3 -c "import json,sys; d=json.load(open(sys.argv[1])); c=d['config']; print('sim8 per GPU', round(c['per_gpu_restarts_per_s'],1), [round(x*1e3) for x in c['shard_seconds']], c['counts_equal_whole_sweep'])" "$OUT/sim8.json" \
        || { tail -5 "$OUT/sim8.err"; exit 1; } ;;
    small)
      for C in C1 C2; do
        timeout -k 10 300 python -u bench.py --config $C --steps 10 --warmup 2 > "$OUT/${C,,}_bench.json" 2> "$OUT/${C,,}_bench.err" \
          && line "$OUT/${C,,}_bench.json" $C || { tail -5 "$OUT/${C,,}_bench.err"; exit 1; }
      done ;;
    c4)
      timeout -k 10 600 python -u bench.py --config C4 --steps 1 --warmup 1 --cpu-iters 4 > "$OUT/c4_bench.json" 2> "$OUT/c4_bench.err" \
        && line "$OUT/c4_bench.json" C4 || { tail -5 "$OUT/c4_bench.err"; exit 1; } ;;
    c5)
      timeout -k 10 600 python -u bench.py --config C5 --steps 1 --warmup 1 > "$OUT/c5_bench.json" 2> "$OUT/c5_bench.err" \
        && line "$OUT/c5_bench.json" C5 || { tail -5 "$OUT/c5_bench.err"; exit 1; } ;;
    latency)
      timeout -k 10 300 python -u tools/nmf_mu_latency.py 3 > "$OUT/nmf_mu_latency.json" 2> "$OUT/nmf_mu_latency.err" && echo "latency ok" || exit 1 ;;
    cpuscale)
      timeout -k 10 400 python -u tools/cpu_scaling.py --procs 1,4,8,16 > "$OUT/cpu_scaling.json" 2> "$OUT/cpu_scaling.err" \
        && echo "cpu scaling ok" && cat "$OUT/cpu_scaling.err" || exit 1 ;;
    *) echo "unknown part $p"; exit 2 ;;
  esac
done
