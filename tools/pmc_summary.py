"""Summarise rocprofv3 counter CSVs: mean counter value per kernel (+ derived MFMA util / clock)."""
import collections
import csv
import glob
import sys

root = sys.argv[1]
dur = {}
for f in glob.glob(f"{root}/trace/*kernel_stats.csv"):
    for r in csv.DictReader(open(f)):
        dur[r["Name"]] = float(r["AverageNs"])
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{root}/*/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in agg.items():
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    short = k.split("(")[0][-60:]
    print(f"== {short}  (trace avg {dur.get(k, float('nan'))/1e3:.1f} us)")
    for c in sorted(m):
        print(f"   {c:28s} {m[c]:.4g}")
    g = m.get("GRBM_GUI_ACTIVE")
    if g and k in dur:
        print(f"   ~clock GHz (GRBM/8/t)        {g / 8 / dur[k]:.3f}")
    if g and "SQ_VALU_MFMA_BUSY_CYCLES" in m:
        print(f"   MFMA busy / (GRBM/8 * 1024 SIMD) {m['SQ_VALU_MFMA_BUSY_CYCLES'] / (g / 8 * 1024):.3f}")
