"""Per-kernel pipe utilisation from tools/pmc_util.sh passes.  rocprofv3 reports GRBM_GUI_ACTIVE summed over
the 8 XCDs (MI355X_MICROARCH.md, DVFS note), so per-dispatch GPU cycles = GRBM_GUI_ACTIVE / 8 and the
effective clock = that / kernel time.  MFMA util = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x cycles) (rocprofv3's
MfmaUtil expression); cycles per fp64 16x16x4 MFMA = MFMA_BUSY / SQ_INSTS_MFMA.  VALU issue share =
SQ_ACTIVE_INST_VALU x 4 (quad-cycles) / (1024 x cycles).  Usage: python3 tools/pmc_util.py <outdir>"""
import collections
import csv
import glob
import os
import re
import sys

SIMDS = 1024


def kname(s):
    m = re.search(r"(k_\w+)(<[^>]*>)?", s)
    return (m.group(1) + (m.group(2) or "")) if m else s[:40]


root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmcu"
for grp in ("mu", "br"):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for p in (grp + "_busy", grp + "_insts"):
        for f in glob.glob(os.path.join(root, p, "**", "*counter_collection.csv"), recursive=True):
            per = collections.defaultdict(lambda: collections.defaultdict(float))
            names = {}
            for r in csv.DictReader(open(f)):
                d = r["Dispatch_Id"]
                names[d] = kname(r["Kernel_Name"])
                per[d][r["Counter_Name"]] += float(r["Counter_Value"])
            for d, cs in per.items():
                for c, v in cs.items():
                    agg[names[d]][c].append(v)
    dur = {}
    for r in csv.DictReader(open(os.path.join(root, grp + "_trace", "run_kernel_stats.csv"))):
        dur[kname(r["Name"])] = float(r["AverageNs"]) * 1e-9
    print(f"{'kernel':28s} {'ms':>7s} {'GHz':>5s} {'MFMA%':>6s} {'cyc/MFMA':>8s} {'exec TF':>8s} {'VALU%':>6s}")
    for k in sorted(agg):
        m = {c: sum(v) / len(v) for c, v in agg[k].items()}
        cyc = m["GRBM_GUI_ACTIVE"] / 8
        # the Brunet sweep runs its k lanes concurrently, so its trace durations overlap: no clock there
        t = dur.get(k, float("nan")) if grp == "mu" else float("nan")
        mf = 100 * m["SQ_VALU_MFMA_BUSY_CYCLES"] / (SIMDS * cyc)
        cpm = m["SQ_VALU_MFMA_BUSY_CYCLES"] / m["SQ_INSTS_MFMA"] if m.get("SQ_INSTS_MFMA") else float("nan")
        tf = m.get("SQ_INSTS_MFMA", 0) * 2048 / t / 1e12
        va = 100 * m["SQ_ACTIVE_INST_VALU"] * 4 / (SIMDS * cyc)
        print(f"{k[:28]:28s} {t * 1e3:7.3f} {cyc / t / 1e9:5.2f} {mf:6.1f} {cpm:8.1f} {tf:8.1f} {va:6.1f}")
