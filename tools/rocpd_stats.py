#!/usr/bin/env python3
"""rocprofv3's rocpd database (its default output format on ROCm 7.2) -> the kernel_stats.csv layout that
`rocprofv3 --stats --output-format csv` writes (Name, Calls, TotalDurationNs, AverageNs, Percentage, MinNs, MaxNs,
StdDev).  Usage: tools/rocpd_stats.py <results.db> > kernel_stats.csv"""
import csv
import math
import sqlite3
import sys
from collections import defaultdict

db = sqlite3.connect(sys.argv[1])
d = defaultdict(list)
for name, dur in db.execute("select name, duration from kernels"):
    d[name].append(float(dur))
tot = sum(sum(v) for v in d.values())
w = csv.writer(sys.stdout, quoting=csv.QUOTE_NONNUMERIC)
w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"])
for name, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    s, c = sum(v), len(v)
    mu = s / c
    sd = math.sqrt(sum((x - mu) ** 2 for x in v) / c)
    w.writerow([name, c, int(s), round(mu, 6), round(100 * s / tot, 2), int(min(v)), int(max(v)), round(sd, 6)])
