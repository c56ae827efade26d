#!/usr/bin/env python3
"""HBM traffic per dispatch for every kernel in rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes.

Usage: pmc_traffic.py OUT.json pass1.csv [pass2.csv ...]

For each kernel name (template arguments kept) and grid size, averages FETCH_SIZE and WRITE_SIZE
(KiB per dispatch) over its dispatches and reports HBM read bytes = 2 x FETCH_SIZE x 1024 (the
gfx950 half-count of wide coalesced streaming reads, MI355X_MICROARCH.md "HBM [CDNA4]") and write
bytes = WRITE_SIZE x 1024.  The x2 is calibrated for 16-B-per-lane streaming loads only; kernels
whose reads are narrower carry "read_pattern_uncalibrated": the ratios between variants stay
valid, the absolute read figure is an estimate.
"""
import csv
import json
import sys
from collections import defaultdict


def main():
    out = sys.argv[1]
    vals = defaultdict(lambda: defaultdict(list))
    for path in sys.argv[2:]:
        with open(path) as fh:
            for row in csv.DictReader(fh):
                g = int(row["Grid_Size"])
                if g <= 0:
                    continue
                vals[(row["Kernel_Name"], g)][row["Counter_Name"]].append(float(row["Counter_Value"]))
    res = []
    for (name, g), cs in sorted(vals.items(), key=lambda kv: (kv[0][0], -kv[0][1])):
        rec = {"kernel": name, "grid_size": g}
        for c, v in cs.items():
            rec[c] = round(sum(v) / len(v), 3)
            rec[c + "_dispatches"] = len(v)
        if "FETCH_SIZE" in rec:
            rec["hbm_read_bytes"] = rec["FETCH_SIZE"] * 2 * 1024
        if "WRITE_SIZE" in rec:
            rec["hbm_write_bytes"] = rec["WRITE_SIZE"] * 1024
        res.append(rec)
    from build_id import build_id
    with open(out, "w") as fh:
        json.dump({"build_id": build_id(), "note": "per dispatch; read = FETCH_SIZE x 2 x 1024 (gfx950), write = WRITE_SIZE x 1024; "
                           "one counter per pass", "kernels": res}, fh, indent=1)
    for r in res:
        print(f'{r["kernel"][:90]:90s} grid {r["grid_size"]:>9d} rd {r.get("hbm_read_bytes", 0) / 1e6:10.3f} MB '
              f'wr {r.get("hbm_write_bytes", 0) / 1e6:10.3f} MB')


if __name__ == "__main__":
    main()
