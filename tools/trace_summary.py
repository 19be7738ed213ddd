"""Per-kernel summary of a rocprofv3 --kernel-trace sqlite database, plus the per-iteration timeline of
the three MU kernels (full-load vs tail).  Usage: python tools/trace_summary.py <results.db>"""
import collections
import sqlite3
import sys

import numpy as np

con = sqlite3.connect(sys.argv[1])
rows = list(con.execute("select name, start, end from kernels order by start"))
by = collections.defaultdict(list)
for nm, s, e in rows:
    by[nm.split('(')[0].split('::')[-1].split('<')[0]].append((e - s) / 1e6)
tot = sum((e - s) for _, s, e in rows) / 1e6
print(f"{'kernel':28s} {'calls':>6s} {'total ms':>10s} {'avg ms':>9s} {'%':>6s}")
for nm, ds in sorted(by.items(), key=lambda x: -sum(x[1])):
    ds = np.array(ds)
    print(f"{nm:28s} {len(ds):6d} {ds.sum():10.1f} {ds.mean():9.4f} {100 * ds.sum() / tot:6.1f}")
print(f"span {(rows[-1][2] - rows[0][1]) / 1e6:.1f} ms, kernel sum {tot:.1f} ms")
w, h, a = (np.array(by.get(k, [])) for k in ("k_wta", "k_hupdate", "k_ahtw_t" if "k_ahtw_t" in by else "k_ahtw"))
if len(w):
    it = w + h + a
    print("iteration ms: first", np.round(it[:3], 3), "| median of first 100", round(float(np.median(it[:100])), 3))
    for lo, hi in ((0, 400), (400, 600), (600, 800), (800, len(it))):
        if lo < len(it):
            seg = it[lo:hi]
            print(f"  iterations {lo:4d}-{min(hi, len(it)):4d}: {seg.sum():8.1f} ms total, {seg.mean():.3f} ms avg")
