"""Per-kernel mean duration and mean idle gap before each kernel (by kernel name) from a rocprofv3
kernel-trace CSV: the GPU-side cost between dependent launches of one forward.
Usage: python tools/trace_gaps.py <run_kernel_trace.csv> [--last N]"""
import argparse
import csv
import statistics
from collections import defaultdict


def main():
    p = argparse.ArgumentParser()
    p.add_argument("csv")
    p.add_argument("--last", type=int, default=200, help="kernels at the end of the trace to use")
    a = p.parse_args()
    rows = sorted(csv.DictReader(open(a.csv)), key=lambda r: int(r["Start_Timestamp"]))[-a.last:]
    dur, gap = defaultdict(list), defaultdict(list)
    prev_end = None
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        name = r["Kernel_Name"].split("(")[0][:48]
        dur[name].append((e - s) / 1e3)
        if prev_end is not None and s - prev_end < 50_000:  # gaps inside the timed loop only
            gap[name].append((s - prev_end) / 1e3)
        prev_end = e
    for name in sorted(dur, key=lambda n: -sum(dur[n])):
        g = gap.get(name) or [0.0]
        print(f"{name:48s} n={len(dur[name]):4d} dur {statistics.mean(dur[name]):8.1f} us  gap before "
              f"{statistics.mean(g):6.1f} us")


if __name__ == "__main__":
    main()
