#!/bin/bash
# rocprofv3 kernel-trace stats of one bench sweep per named environment (A/B of kernel durations).
# Usage (GPU box): bash tools/trace_kstats.sh <outdir> "name:VAR=v VAR2=w" ...   (BENCH_ARGS: extra bench.py args)
set -o pipefail
OUT=${1:-gpurun_out/kstats}; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p "$OUT"
for spec in "$@"; do
  name=${spec%%:*}; envs=${spec#*:}
  env $envs timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$name" -o run -- \
    python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline ${BENCH_ARGS:-} > "$OUT/$name.log" 2>&1 || { echo "$name failed"; tail -5 "$OUT/$name.log"; exit 1; }
  f=$(find "$OUT/$name" -name '*kernel_stats.csv' | head -1)
  echo "== $name"
  python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"].split("(")[0].replace("void ", "").replace("nmfc::", "")
    if n.startswith("k_"):
        print(f"  {n[:60]:60s} calls {int(r['Calls']):6d}  avg {float(r['AverageNs'])/1e3:9.1f} us  total {float(r['TotalDurationNs'])/1e6:8.2f} ms")
PY
done
