"""Per-kernel wave-state shares from tools/pmc_tail.sh (SQ counters summed over a dispatch, averaged over
dispatches of the same kernel name).  WAIT_ANY = parked on s_waitcnt / barrier; WAIT_INST_ANY = issue stall
(MFMA dependency, pipe busy); ACTIVE_INST_ANY = issuing (MI355X_MICROARCH.md rocprofv3 PMC notes: the three
are disjoint and sum to about WAVE_CYCLES).  MFMA% = MFMA busy cycles / (1024 SIMDs x GRBM cycles / 8)."""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    names = {}
    for r in csv.DictReader(open(f)):
        d = r["Dispatch_Id"]
        names[d] = r["Kernel_Name"].split("(")[0].replace("void nmfc::", "").replace("nmfc::", "")
        per[d][r["Counter_Name"]] += float(r["Counter_Value"])
    for d, cs in per.items():
        for c, v in cs.items():
            agg[names[d]][c].append(v)
print(f"{'kernel':40s} {'wait%':>6s} {'stall%':>6s} {'issue%':>6s} {'lds%':>5s} {'MFMA%':>6s} {'cyc/mfma':>8s} {'disp':>5s}")
for k in sorted(agg):
    m = {c: sum(v) / len(v) for c, v in agg[k].items()}
    wc = m.get("SQ_WAVE_CYCLES", 0) or 1
    cyc = m.get("GRBM_GUI_ACTIVE", 0) / 8 or 1
    print(f"{k[:40]:40s} {100 * m.get('SQ_WAIT_ANY', 0) / wc:6.1f} {100 * m.get('SQ_WAIT_INST_ANY', 0) / wc:6.1f} "
          f"{100 * m.get('SQ_ACTIVE_INST_ANY', 0) / wc:6.1f} {100 * m.get('SQ_WAIT_INST_LDS', 0) / wc:5.1f} "
          f"{100 * m.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / (1024 * cyc):6.1f} "
          f"{m.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / max(m.get('SQ_INSTS_MFMA', 1), 1):8.1f} {len(agg[k]['SQ_WAVE_CYCLES']):5d}")
