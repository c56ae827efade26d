#!/usr/bin/env python3
"""Per-kernel median durations of a rocprofv3 kernel_trace.csv, and the timeline (start offset,
duration) of the launches between the Nth and N+1th launch of a marker kernel.
Usage: trace_summary.py TRACE.csv [MARKER_SUBSTRING N]"""
import csv
import re
import sys
from collections import defaultdict


def short(name):
    return re.sub(r"\(.*", "", name)[:50]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    d = defaultdict(list)
    for r in rows:
        d[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
    for k, v in d.items():
        if "omr" in k:
            print(f"{k:50s} n={len(v):4d} med {sorted(v)[len(v) // 2]:8.1f} us")
    if len(sys.argv) > 3:
        idx = [i for i, r in enumerate(rows) if sys.argv[2] in r["Kernel_Name"]]
        n = int(sys.argv[3])
        i0, i1 = idx[n], idx[n + 1]
        t0 = int(rows[i0]["Start_Timestamp"])
        for r in rows[i0:i1]:
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            print(f"  {short(r['Kernel_Name']):45s} start {(s - t0) / 1000:8.1f} dur {(e - s) / 1000:7.1f}")


if __name__ == "__main__":
    main()
