"""HBM traffic per launch of the MFMA kernels from rocprofv3 FETCH_SIZE / WRITE_SIZE passes.

Corrections per /opt/skills/guides/MI355X_MICROARCH.md (HBM section): FETCH_SIZE and WRITE_SIZE are
in KiB; on gfx950 FETCH_SIZE reports half the bytes of wide coalesced streaming reads, so it is
doubled; WRITE_SIZE is taken as is.  Only full-load launches are averaged (the first 100 launches of
each kernel: every restart is still running before iteration 400).  Prints JSON."""
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
    for kn, d in per.items():
        vals = [d[k] for k in sorted(d)][:100]
        kib = sum(vals) / max(len(vals), 1)
        scale = 2.0 if counter == "FETCH_SIZE" else 1.0
        out.setdefault(kn, {})[counter + "_bytes_per_launch"] = kib * 1024.0 * scale
        out[kn]["launches_averaged"] = len(vals)
for kn, d in out.items():
    d["hbm_bytes_per_launch"] = d.get("FETCH_SIZE_bytes_per_launch", 0.0) + d.get("WRITE_SIZE_bytes_per_launch", 0.0)
print(json.dumps(out, indent=1))
