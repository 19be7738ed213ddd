"""Per-iteration timeline of one sweep from a rocprofv3 --kernel-trace CSV.

Groups the MU kernels into iterations (one k_hupdate per iteration), prints per-bucket device time of
each kernel, grid sizes, and the idle gaps between consecutive dispatches (launch/host overhead).
Usage: python tools/trace_timeline.py <run_kernel_trace.csv> [bucket=50] [iters.npy [m n]]
With the sweep's per-job (k, iterations) (bench.py --dump-iters), each bucket also reports the useful
fp64 rate: sum over live restart-iterations of F = 4mnk + 4(m+n)k^2 / the bucket's span."""
import collections
import csv
import sys

rows = []
for r in csv.DictReader(open(sys.argv[1])):
    nm = r["Kernel_Name"].split("(")[0].split("::")[-1]
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), nm, int(r["Grid_Size_X"]) // max(int(r["Workgroup_Size_X"]), 1)))
rows.sort()
bucket = int(sys.argv[2]) if len(sys.argv) > 2 else 50
it = 0
agg = collections.defaultdict(lambda: collections.defaultdict(float))
grids = collections.defaultdict(lambda: collections.defaultdict(list))
gap = collections.defaultdict(float)
span = collections.defaultdict(lambda: [None, None])
prev_end = None
for s, e, nm, g in rows:
    b = it // bucket
    if nm.startswith("k_hupdate"):
        it += 1
    key = nm.split("<")[0] + ("_big" if nm.startswith("k_wta2<4") else "_small" if nm.startswith("k_wta2<1") else "")
    agg[b][key] += (e - s) / 1e6
    grids[b][key].append(g)
    if prev_end is not None and s > prev_end:
        gap[b] += (s - prev_end) / 1e6
    prev_end = max(prev_end or 0, e)
    sp = span[b]
    sp[0] = s if sp[0] is None else sp[0]
    sp[1] = e
useful = None
live = {}
if len(sys.argv) > 3:
    import numpy as np
    kk, its = np.load(sys.argv[3])
    mm = int(sys.argv[4]) if len(sys.argv) > 4 else 20000
    nn = int(sys.argv[5]) if len(sys.argv) > 5 else 500
    F = 4.0 * mm * nn * kk + 4.0 * (mm + nn) * kk * kk
    useful = {}
    live = {}
    for b in agg:
        lo, hi = b * bucket, (b + 1) * bucket
        useful[b] = float(np.sum(F * np.clip(its - lo, 0, hi - lo)))
        # mean live restarts / live columns over the bucket's iterations
        live[b] = (float(np.sum(np.clip(its - lo, 0, hi - lo))) / bucket,
                   float(np.sum(kk * np.clip(its - lo, 0, hi - lo))) / bucket)
tot = 0.0
print(f"{'iters':>11s} {'span ms':>8s} {'gap ms':>7s} {'TF':>6s}  kernels (ms, mean grid)")
for b in sorted(agg):
    sp = (span[b][1] - span[b][0]) / 1e6
    tot += sp
    parts = "  ".join(f"{k}={v:.1f}({sum(grids[b][k]) / len(grids[b][k]):.0f})" for k, v in sorted(agg[b].items()) if v > 0.05)
    tf = useful[b] / (sp * 1e-3) / 1e12 if useful else float("nan")
    lv = f" live {live[b][0]:6.1f} r {live[b][1]:7.1f} c" if useful else ""
    print(f"{b * bucket:5d}-{(b + 1) * bucket:5d} {sp:8.1f} {gap[b]:7.2f} {tf:6.1f}{lv}  {parts}")
print(f"total span {tot:.1f} ms over {it} iterations")
# idle time by the kernel that FOLLOWS the gap (boundary gaps before each MU kernel, poll copies, repack moves)
by_next = collections.defaultdict(lambda: [0.0, 0])
for i in range(len(rows) - 1):
    g = rows[i + 1][0] - rows[i][1]
    if g > 0:
        nm = rows[i + 1][2].split("<")[0]
        by_next[nm][0] += g / 1e6
        by_next[nm][1] += 1
print("idle before each kernel kind (ms total, count, us mean):")
for nm, (ms, c) in sorted(by_next.items(), key=lambda x: -x[1][0])[:10]:
    print(f"  {nm[:40]:40s} {ms:8.2f} {c:7d} {ms / c * 1e3:8.1f}")
gaps = sorted(((rows[i + 1][0] - rows[i][1], i) for i in range(len(rows) - 1)), reverse=True)
print("largest idle gaps:")
for g, i in gaps[:8]:
    print(f"  {g / 1e6:8.2f} ms after #{i} {rows[i][2][:40]} before {rows[i + 1][2][:40]}")
