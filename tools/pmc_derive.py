"""Derived per-kernel metrics from tools/pmc_summary.py-style csv passes: MFMA busy %, wait shares, VALU/LDS
activity, LDS bank-conflict ratio, L2 hit rate.  Usage: python3 tools/pmc_derive.py <pmc dir>"""
import collections, csv, glob, os, sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmck"
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    names = {}
    for row in csv.DictReader(open(f)):
        d = row.get("Dispatch_Id") or row.get("Correlation_Id")
        names[d] = row["Kernel_Name"].split("(")[0].replace("nmfc::", "")
        per[d][row["Counter_Name"]] += float(row["Counter_Value"])
    for d, cs in per.items():
        for c, v in cs.items():
            agg[names[d]][c].append(v)
SIMDS = 1024
print(f"{'kernel':44s} {'MFMA%':>6s} {'wait%':>6s} {'winst%':>6s} {'act%':>6s} {'valu/wv':>8s} {'lds/wv':>8s} {'ldsconf':>7s} {'L2hit':>6s} {'clkGHz?':>7s}")
for k, cs in sorted(agg.items()):
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    g = lambda c: m.get(c, float("nan"))
    mf = g("SQ_VALU_MFMA_BUSY_CYCLES") / (g("GRBM_GUI_ACTIVE") * SIMDS) * 100 if "GRBM_GUI_ACTIVE" in m else float("nan")
    wc = g("SQ_WAVE_CYCLES")
    print(f"{k[:44]:44s} {mf:6.1f} {100*g('SQ_WAIT_ANY')/wc:6.1f} {100*g('SQ_WAIT_INST_ANY')/wc:6.1f} {100*g('SQ_ACTIVE_INST_ANY')/wc:6.1f} "
          f"{g('SQ_ACTIVE_INST_VALU')/g('SQ_WAVES'):8.0f} {g('SQ_ACTIVE_INST_LDS')/g('SQ_WAVES'):8.0f} "
          f"{g('SQ_LDS_BANK_CONFLICT')/max(g('SQ_LDS_IDX_ACTIVE'),1):7.3f} {g('TCC_HIT_sum')/(g('TCC_HIT_sum')+g('TCC_MISS_sum')):6.3f}")
