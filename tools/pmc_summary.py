"""Summarise rocprofv3 --pmc csv passes (tools/pmc_passes.sh) per kernel: mean counter value per dispatch."""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    names = {}
    for row in csv.DictReader(open(f)):
        disp = row.get("Dispatch_Id") or row.get("Correlation_Id")
        kn = row["Kernel_Name"].split("(")[0].split("::")[-1]
        names[disp] = kn
        per[disp][row["Counter_Name"]] += float(row["Counter_Value"])
    for disp, cs in per.items():
        for c, v in cs.items():
            agg[names[disp]][c].append(v)
for kn, cs in sorted(agg.items()):
    print(kn)
    for c, vs in sorted(cs.items()):
        print(f"   {c:28s} n={len(vs):4d} mean={sum(vs) / len(vs):.4g}")
