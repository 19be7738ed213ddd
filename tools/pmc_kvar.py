"""Per-arm counter summary for tools/gpu_kvar_pmc.sh (kvar's full-load MFMA kernel arms).  Counters are summed over
a dispatch and averaged over the dispatches of one kernel instantiation (the arms are distinct instantiations).
SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles (MI355X_MICROARCH.md); GPU cycles per dispatch =
GRBM_GUI_ACTIVE / 8 (summed over the 8 XCDs).  MFMA% = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x cycles).
Usage: python3 tools/pmc_kvar.py <outdir>"""
import collections
import csv
import glob
import os
import re
import sys

root = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))


def key(s):
    m = re.search(r"(k_\w+)(<[^()]*>)?", s)
    return (m.group(1) + (m.group(2) or "")).replace(" ", "") if m else s[:60]


for f in glob.glob(os.path.join(root, "*", "**", "*counter_collection.csv"), recursive=True):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    names = {}
    for r in csv.DictReader(open(f)):
        d = r["Dispatch_Id"]
        names[d] = key(r["Kernel_Name"])
        per[d][r["Counter_Name"]] += float(r["Counter_Value"])
    for d, cs in per.items():
        for c, v in cs.items():
            agg[names[d]][c].append(v)
dur = {}
for f in glob.glob(os.path.join(root, "trace", "**", "*kernel_stats.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        dur[key(r["Name"])] = float(r["AverageNs"]) * 1e-9
cols = ["ms", "GHz", "MFMA%", "wait%", "stall%", "issue%", "ldsst%", "MFMA/w", "VALU/w", "LDS/w", "SALU/w", "VALU%", "LDS%", "bankc%"]
print(f"{'kernel':52s} " + " ".join(f"{c:>7s}" for c in cols))
for k in sorted(agg):
    m = {c: sum(v) / len(v) for c, v in agg[k].items()}
    g = lambda c: m.get(c, float("nan"))
    cyc = g("GRBM_GUI_ACTIVE") / 8
    t = dur.get(k, float("nan"))
    wc = g("SQ_WAVE_CYCLES")
    wv = g("SQ_WAVES")
    row = [t * 1e3, cyc / t / 1e9, 100 * g("SQ_VALU_MFMA_BUSY_CYCLES") / (1024 * cyc), 100 * g("SQ_WAIT_ANY") / wc,
           100 * g("SQ_WAIT_INST_ANY") / wc, 100 * g("SQ_ACTIVE_INST_ANY") / wc, 100 * g("SQ_WAIT_INST_LDS") / wc,
           g("SQ_INSTS_MFMA") / wv, g("SQ_INSTS_VALU") / wv, g("SQ_INSTS_LDS") / wv, g("SQ_INSTS_SALU") / wv,
           100 * 4 * g("SQ_ACTIVE_INST_VALU") / (1024 * cyc), 100 * 4 * g("SQ_ACTIVE_INST_LDS") / (1024 * cyc),
           100 * g("SQ_LDS_BANK_CONFLICT") / max(g("SQ_LDS_IDX_ACTIVE"), 1)]
    print(f"{k[:52]:52s} " + " ".join(f"{x:7.1f}" if x == x else f"{'-':>7s}" for x in row))
