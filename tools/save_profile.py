"""Copy the judged parts of a gpurun profile directory into profiles/<round>/ and write a summary.

Usage: python tools/save_profile.py gpurun_out/prof_r1b profiles/r1 [bench.json ...]

Also writes PMC.json: HBM bytes per launch of the dominant kernel (FETCH_SIZE x2 + WRITE_SIZE,
bench.read_pmc_traffic) with the commit it was taken at; bench.py reads the newest one for
roofline.traffic when it runs without --pmc-csv.
"""
import collections
import csv
import glob
import json
import os
import shutil
import subprocess
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

src, dst = sys.argv[1], sys.argv[2]
os.makedirs(dst, exist_ok=True)
lines = [f"# rocprofv3 summary ({src})", ""]
for f in glob.glob(f"{src}/trace/*kernel_stats.csv"):
    shutil.copy(f, os.path.join(dst, "kernel_stats.csv"))
    lines += ["## --kernel-trace --stats", "", "| kernel | calls | avg us | % |", "|---|---|---|---|"]
    for r in csv.DictReader(open(f)):
        lines.append(f"| {r['Name'][:70]} | {r['Calls']} | {float(r['AverageNs']) / 1e3:.1f} | {float(r['Percentage']):.1f} |")
    lines.append("")
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{src}/*/*counter_collection.csv"):
    tag = os.path.basename(os.path.dirname(f))
    shutil.copy(f, os.path.join(dst, f"counters_{tag}.csv"))
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"][:70]][r["Counter_Name"]].append(float(r["Counter_Value"]))
if agg:
    lines += ["## PMC counters (mean per dispatch; separate --pmc passes)", ""]
    for k, cs in agg.items():
        lines.append(f"- **{k}**: " + ", ".join(f"{c}={sum(v) / len(v):.4g}" for c, v in sorted(cs.items())))
    lines.append("")
for b in sys.argv[3:]:
    txt = open(b).read().strip().splitlines()[-1]
    d = json.loads(txt)
    shutil.copy(b, os.path.join(dst, os.path.basename(b)))
    lines += [f"## bench line ({os.path.basename(b)})", "", "```json", json.dumps(d, indent=1), "```", ""]
fetch = glob.glob(f"{src}/fetch/*counter_collection.csv")
write = glob.glob(f"{src}/write/*counter_collection.csv")
if fetch and write:
    from bench import read_pmc_traffic

    kern = os.environ.get("NT_PROFILE_KERNEL", "")
    if not kern:  # the bench line's dominant kernel (e.g. update_fk_kernel -> update_fk)
        for b in sys.argv[3:]:
            k = json.loads(open(b).read().strip().splitlines()[-1])["roofline"]["kernel"].split()[0].rstrip(":")
            kern = k[: -len("_kernel")] if k.endswith("_kernel") else k
    kern = kern or "update"
    traffic = read_pmc_traffic(f"{fetch[0]},{write[0]}", kern)
    if traffic is not None:
        commit = subprocess.run(["git", "rev-parse", "--short", "HEAD"], capture_output=True,
                                text=True).stdout.strip()
        pmc = {"kernel": kern, "traffic_per_launch": traffic, "commit": commit, "time": time.time(),
               "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes; "
                         "FETCH_SIZE x2 (gfx950 wide-load correction) + WRITE_SIZE, KB -> B, "
                         "mean per dispatch"}
        json.dump(pmc, open(os.path.join(dst, "PMC.json"), "w"), indent=1)
        lines += [f"## HBM traffic per launch of `{kern}`: {traffic / 1e6:.1f} MB (PMC.json)", ""]
open(os.path.join(dst, "SUMMARY.md"), "w").write("\n".join(lines))
print("wrote", dst)
