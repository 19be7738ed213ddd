#!/bin/bash
# A/B of libnmf.so build variants (tools/build_variant.sh -> tools/var/lib_<name>.so) on the default C3
# bench and optional small shards: one bench line per variant and shard, kernel rates summarised.
# Usage: RS="200 25" bash tools/gpu_var_bench.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/var
# a variant is tools/var/<name>.so, or tools/var/<name>.env holding "LIB=<so> VAR=value ..." (env overrides)
for f in $(ls tools/var/*.so tools/var/*.env 2>/dev/null | sort); do
  v=$(basename "${f%.*}")
  if [ "${f##*.}" = env ]; then envs=$(cat "$f"); so=$(echo "$envs" | sed -E 's/.*LIB=([^ ]+).*/\1/'); else envs=""; so=$f; fi
  for R in ${RS:-200}; do
    env $envs NMFC_LIB=$PWD/$so timeout -k 10 300 python -u bench.py --restarts $R --steps ${STEPS:-2} --warmup 1 --no-cpu-baseline \
      > gpurun_out/var/$v.$R.json 2> gpurun_out/var/$v.$R.err || { echo "$v R=$R failed"; tail -5 gpurun_out/var/$v.$R.err; exit 1; }
    python3 - "$v" "$R" <<'EOF'
import json, sys
v, R = sys.argv[1], sys.argv[2]
d = json.load(open(f"gpurun_out/var/{v}.{R}.json"))
k = (d.get("roofline") or {}).get("kernels", {})
f = lambda n, key: round(k[n][key], 3) if n in k and key in k[n] else None
print(f"{v:24s} R={R:>4s} {d['value']:8.1f} restarts/s  {d['ms_per_step']:8.1f} ms  wta {f('wta','tflops')} TF "
      f"({f('wta','avg_ms')} ms)  ahtw {f('ahtw','tflops')} TF ({f('ahtw','avg_ms')} ms)  hupd {f('hupdate','avg_ms')} ms")
EOF
  done
done
