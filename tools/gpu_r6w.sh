#!/bin/bash
# Round 6, call w: the C5 sweep's 4 Brunet lanes landed on only 2 hardware queues (the r6u kernel trace: Queue_Id 3 and 4,
# two lanes each), so at most two lanes' kernels ran at once.  C5 with GPU_MAX_HW_QUEUES 4 (HIP's default) vs 8, twice,
# then a kernel trace at 8 to read the queue assignment.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6w
mkdir -p $O
echo "env GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES:-unset}"
for rep in 1 2; do
  for q in 4 8; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python -u bench.py --config C5 --steps 1 --warmup 1 --no-cpu-baseline > $O/c5_q${q}_$rep.json 2> $O/c5_q${q}_$rep.err || { tail -5 $O/c5_q${q}_$rep.err; exit 1; }
    echo "q=$q rep $rep: $(python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(round(d['value'],2), round(d['ms_per_step']), round(d['roofline']['frac'],4))" $O/c5_q${q}_$rep.json)"
  done
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
GPU_MAX_HW_QUEUES=8 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace8 -o run -- python3 bench.py --config C5 --steps 1 --warmup 0 --no-cpu-baseline --no-timing > $O/trace8.log 2>&1 && echo "trace ok"
python3 - <<'PY'
import csv,glob,re,collections
f=glob.glob('gpurun_out/r6w/trace8/**/*kernel_trace.csv',recursive=True)[0]
c=collections.Counter()
for r in csv.DictReader(open(f)):
    m=re.search(r'k_br_(\w+)<(\d+)',r['Kernel_Name'])
    if m: c[(int(m.group(2)),r['Queue_Id'])]+=1
print(sorted(c.items()))
PY
