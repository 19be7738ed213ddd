#!/usr/bin/env python3
"""Phases of a sweep's kernel trace per HIP stream (one stream per restart group): from the first MU kernel to the first
k_move_rows (the first repack: the end of the all-live phase) and from there to the last MU kernel, plus the busy time
of the MU kernels in each phase.  Usage: python tools/phase_split.py <run_kernel_trace.csv>"""
import collections
import csv
import sys

MU = ("k_wta", "k_ahtw4", "k_hupdate")
rows = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    nm = r["Kernel_Name"].split("(")[0].replace("void ", "").split("::")[-1]
    rows[r["Stream_Id"]].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), nm))
t0 = min(s for v in rows.values() for s, _, _ in v)
for sid, v in sorted(rows.items()):
    v.sort()
    mu = [x for x in v if x[2].startswith(MU)]
    if not mu:
        continue
    first = mu[0][0]
    rep = next((s for s, _, nm in v if nm.startswith("k_move_rows") and s > first), None)
    last = mu[-1][1]
    if rep is None:
        rep = last
    busy1 = sum(e - s for s, e, nm in mu if s < rep) / 1e6
    busy2 = sum(e - s for s, e, nm in mu if s >= rep) / 1e6
    print(f"stream {sid}: MU kernels {len(mu)}, start {(first - t0) / 1e6:8.2f} ms, all-live {(rep - first) / 1e6:8.2f} ms "
          f"(busy {busy1:8.2f}), tail {(last - rep) / 1e6:8.2f} ms (busy {busy2:8.2f}), end {(last - t0) / 1e6:8.2f} ms")
