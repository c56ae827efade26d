#!/usr/bin/env python3
"""Per-(kernel, grid size) launch statistics of a rocprofv3 kernel_trace.csv, written as a small CSV
that the bench line's roofline fractions can be recomputed from (duration = End - Start, ns).

Usage: trace_kernels.py TRACE.csv OUT.csv
Columns: kernel, grid_size, workgroup_size, lds_bytes, launches, avg_ns, median_ns, min_ns, max_ns.
"""
import csv
import sys
from collections import defaultdict


def main():
    groups = defaultdict(list)
    meta = {}
    with open(sys.argv[1]) as fh:
        for r in csv.DictReader(fh):
            if "Grid_Size" in r:
                grid, wg = int(r["Grid_Size"]), r.get("Workgroup_Size", "")
            else:                                   # rocprofv3 (ROCm 7): per-dimension columns
                grid = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
                wg = int(r["Workgroup_Size_X"]) * int(r["Workgroup_Size_Y"]) * int(r["Workgroup_Size_Z"])
            key = (r["Kernel_Name"], grid)
            groups[key].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
            meta[key] = (wg, r.get("LDS_Block_Size", r.get("Lds_Size", "")))
    with open(sys.argv[2], "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["kernel", "grid_size", "workgroup_size", "lds_bytes", "launches", "avg_ns", "median_ns",
                    "min_ns", "max_ns"])
        for key in sorted(groups, key=lambda k: -sum(groups[k])):
            d = sorted(groups[key])
            w.writerow([key[0], key[1], meta[key][0], meta[key][1], len(d), round(sum(d) / len(d), 1),
                        d[len(d) // 2], d[0], d[-1]])


if __name__ == "__main__":
    main()
