"""Checks that bench.py's live HIP-event kernel averages agree with a rocprofv3 --kernel-trace --stats
summary of the same command.  Usage: python3 tools/profile_agreement.py <bench.json> <kernel_stats.csv>"""
import csv
import json
import sys

bench = json.load(open(sys.argv[1]))["roofline"]["kernels"]
rows = list(csv.DictReader(open(sys.argv[2])))
for name, prefix in (("wta", "nmfc::k_wta2"), ("ahtw", "nmfc::k_ahtw4"), ("hupdate", "nmfc::k_hupdate")):
    sel = [r for r in rows if prefix in r["Name"]]
    calls = sum(int(r["Calls"]) for r in sel)
    avg = sum(float(r["TotalDurationNs"]) for r in sel) / max(calls, 1) / 1e6
    b = bench[name]["avg_ms"]
    print(f"{name:8s} bench {b:.4f} ms  rocprof {avg:.4f} ms over {calls} launches (all shapes)  ratio {b / avg:.4f}")
