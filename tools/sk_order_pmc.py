#!/usr/bin/env python3
"""HBM / L2-miss bytes and cycles of the W^T A full-load arms of tools/kvar in pmc mode (tools/gpu_r6h.sh): per dispatch
FETCH_SIZE x 2 + WRITE_SIZE (KiB; the x2 gfx950 correction of tools/pmc_traffic.py) and GRBM_GUI_ACTIVE / 8 / duration.
The two stream-K whole-round orders are one kernel instantiation (a runtime switch): their dispatches are told apart by
order (kvar runs each arm `reps` times, round-robin first).  Usage: tools/sk_order_pmc.py <outdir> <reps>"""
import collections
import csv
import glob
import os
import sys

root, reps = sys.argv[1], int(sys.argv[2])


def rows(sub):
    out = collections.defaultdict(lambda: collections.defaultdict(float))
    names, dur = {}, {}
    for f in glob.glob(os.path.join(root, sub, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            d = int(r["Dispatch_Id"])
            names[d] = r["Kernel_Name"]
            out[d][r["Counter_Name"]] += float(r["Counter_Value"])
            dur[d] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    return out, names, dur


def label(name):
    if "k_wta2_sk" in name:
        return "k_wta2_sk" + ("<NOWAIT>" if "Lb1E" in name.split("k_wta2_sk")[1][:20] else "")
    if "k_wta2<" in name or "k_wta2I" in name:
        return "k_wta2 16w" if "4, 4, 1, 3" in name or "Li4ELi4ELi1ELi3" in name else "k_wta2 8w"
    return None


fetch, names, dur = rows("FETCH_SIZE")
write, _, _ = rows("WRITE_SIZE")
groups = collections.defaultdict(list)
for d in sorted(fetch):
    lb = label(names[d])
    if lb:
        groups[lb].append(d)
print(f"{'arm':34s} {'launches':>8s} {'GB/launch':>10s} {'Mcycles':>8s} {'ms(pmc)':>8s} {'GHz':>6s}   (cycles: GRBM_GUI_ACTIVE / 8)")
for lb, ds in groups.items():
    parts = [(lb, ds)]
    if lb == "k_wta2_sk" and len(ds) >= 2 * reps:   # round-robin arm first, then the XCD-contiguous arm
        parts = [("k_wta2_sk round-robin rounds", ds[-2 * reps:-reps]), ("k_wta2_sk XCD-contiguous rounds", ds[-reps:])]
    for nm, dd in parts:
        gb = sum(fetch[d].get("FETCH_SIZE", 0) * 2 * 1024 + write[d].get("WRITE_SIZE", 0) * 1024 for d in dd) / len(dd) / 1e9
        cyc = sum(fetch[d].get("GRBM_GUI_ACTIVE", 0) / 8 for d in dd) / len(dd)
        t = sum(dur[d] for d in dd) / len(dd)
        print(f"{nm:34s} {len(dd):8d} {gb:10.3f} {cyc / 1e6:8.3f} {t * 1e3:8.3f} {cyc / t / 1e9:6.3f}")
