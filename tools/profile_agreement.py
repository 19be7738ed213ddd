"""Checks that bench.py's live HIP-event kernel averages agree with a rocprofv3 --kernel-trace --stats
summary of the same command (the bench times every 4th MU iteration's launches, a uniform sample; rocprof
sees every launch).  Usage: python3 tools/profile_agreement.py <bench.json> <kernel_stats.csv>"""
import csv
import json
import sys

bench = json.load(open(sys.argv[1]))["roofline"]["kernels"]
rows = list(csv.DictReader(open(sys.argv[2])))
for name, prefixes in (("wta", ("nmfc::k_wta2", "nmfc::k_wta_narrow")), ("ahtw", ("nmfc::k_ahtw4",)),
                       ("hupdate", ("nmfc::k_hupdate",)), ("labels", ("nmfc::k_labels",)),
                       ("counts", ("nmfc::k_counts",))):
    if name not in bench:
        continue
    sel = [r for r in rows if any(p in r["Name"] for p in prefixes)]
    calls = sum(int(r["Calls"]) for r in sel)
    avg = sum(float(r["TotalDurationNs"]) for r in sel) / max(calls, 1) / 1e6
    b = bench[name]["avg_ms"]
    print(f"{name:8s} bench {b:.4f} ms  rocprof {avg:.4f} ms over {calls} launches (all shapes)  ratio {b / avg:.4f}")
