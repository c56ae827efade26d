#!/usr/bin/env python3
"""Per-(kernel, grid size) launch statistics of a rocprofv3 kernel_trace.csv, written as a small CSV
that the bench line's roofline fractions can be recomputed from (duration = End - Start, ns).

Usage: trace_kernels.py TRACE.csv OUT.csv
Columns: kernel, grid_size, workgroup_size, lds_bytes, launches, avg_ns, median_ns, min_ns, max_ns.
Also writes OUT.json: the rows with the kernel-source build id (bench.kernel_build_id).
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
    # the same rows as JSON with the kernel-source fingerprint of this tree (bench.py reads the
    # committed all-sections trace through it: profile_provenance)
    import json
    import os
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    rows = []
    for key in sorted(groups, key=lambda k: -sum(groups[k])):
        d = sorted(groups[key])
        rows.append({"kernel": key[0], "grid_size": key[1], "launches": len(d), "avg_ns": round(sum(d) / len(d), 1),
                     "median_ns": d[len(d) // 2], "min_ns": d[0], "max_ns": d[-1]})
    with open(os.path.splitext(sys.argv[2])[0] + ".json", "w") as fh:
        json.dump({"build_id": bench.kernel_build_id(), "source_trace": os.path.basename(sys.argv[1]),
                   "kernels": rows}, fh, indent=0)


if __name__ == "__main__":
    main()
