set -o pipefail
mkdir -p gpurun_out/r02i
for d in 5 10 20 40; do
  for R in 25 200; do
    NMFC_REPACK_DIV=$d timeout -k 10 300 python -u bench.py --restarts $R --no-cpu-baseline --no-timing --steps 2 > gpurun_out/r02i/d${d}_R$R.json 2>&1 || exit 1
    python3 -c "import json;d=[json.loads(l) for l in open('gpurun_out/r02i/d${d}_R$R.json') if l.startswith('{')][0];print('div $d R=$R', round(d['value'],1), round(d['ms_per_step'],1))"
  done
done
