"""HBM traffic per launch of the MFMA kernels from rocprofv3 FETCH_SIZE / WRITE_SIZE passes.

Corrections per /opt/skills/guides/MI355X_MICROARCH.md (HBM section): FETCH_SIZE and WRITE_SIZE are
in KiB; on gfx950 FETCH_SIZE reports half the bytes of wide coalesced streaming reads, so it is
doubled; WRITE_SIZE is taken as is.

Two averages per kernel: over ALL launches of the profiled sweep (what bench.py's roofline `achieved`
is averaged over: every launch of one REF_COMPAT sweep) and over the full-load launches (the first
100: every restart is still running before iteration 400).  Prints JSON.

  tools/pmc_traffic.py <profile dir> [config stop_rule maxiter restarts]
The workload the passes profiled (default: the C3 bench line's, C3 ref_compat 10000 200) is recorded in the JSON;
bench.py attaches the figures only to a line of the same workload (config, stop rule, maxiter, restarts)."""
import collections
import csv
import glob
import json
import os
import sys

root = sys.argv[1]
out = {}
for counter in ("FETCH_SIZE", "WRITE_SIZE"):
    files = glob.glob(os.path.join(root, counter, "**", "*counter_collection.csv"), recursive=True)
    per = collections.defaultdict(dict)
    for f in files:
        for row in csv.DictReader(open(f)):
            kn = row["Kernel_Name"].split("(")[0].split("::")[-1].split("<")[0]
            disp = int(row["Dispatch_Id"])
            per[kn][disp] = per[kn].get(disp, 0.0) + float(row["Counter_Value"])
    scale = 2.0 if counter == "FETCH_SIZE" else 1.0
    for kn, d in per.items():
        vals = [d[k] for k in sorted(d)]
        full = vals[:100]
        o = out.setdefault(kn, {})
        o[counter + "_bytes_per_launch"] = sum(vals) / max(len(vals), 1) * 1024.0 * scale
        o[counter + "_bytes_per_full_launch"] = sum(full) / max(len(full), 1) * 1024.0 * scale
        o["launches"] = len(vals)
for kn, d in out.items():
    d["hbm_bytes_per_launch"] = d.get("FETCH_SIZE_bytes_per_launch", 0.0) + d.get("WRITE_SIZE_bytes_per_launch", 0.0)
    d["hbm_bytes_per_full_launch"] = (d.get("FETCH_SIZE_bytes_per_full_launch", 0.0) +
                                      d.get("WRITE_SIZE_bytes_per_full_launch", 0.0))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nmfconsensus_amd.build import source_sha256  # noqa: E402

out["source_sha256"] = source_sha256()   # bench.py uses this profile only for the same kernel source
wl = sys.argv[2:6] if len(sys.argv) >= 6 else ["C3", "ref_compat", "10000", "200"]
out["workload"] = {"config": wl[0], "stop_rule": wl[1], "maxiter": int(wl[2]), "restarts": int(wl[3])}
print(json.dumps(out, indent=1))
