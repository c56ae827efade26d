#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes for one kernel into profiles/pmc_*.json.

Usage: pmc_summary.py OUT.json KERNEL_SUBSTR TILES_PER_LAUNCH ALG_BYTES_PER_TILE pass1.csv [pass2.csv ...]

FETCH_SIZE/WRITE_SIZE are in KiB per dispatch.  On gfx950 FETCH_SIZE reports half the bytes of a
wide coalesced streaming read (MI355X_MICROARCH.md, HBM/rocprofv3 section), so HBM read bytes =
2 x FETCH_SIZE x 1024; WRITE_SIZE is exact for 16-B-per-lane streaming stores.
"""
import csv
import json
import sys
from collections import defaultdict


def main():
    out, kname, tiles, alg = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
    vals = defaultdict(list)
    for path in sys.argv[5:]:
        with open(path) as fh:
            for row in csv.DictReader(fh):
                if kname in row["Kernel_Name"] and int(row["Grid_Size"]) > 0:
                    vals[row["Counter_Name"]].append((int(row["Grid_Size"]), float(row["Counter_Value"])))
    # keep the batch launches only (the largest grid seen)
    gmax = max(g for v in vals.values() for g, _ in v)
    avg = {k: sum(x for g, x in v if g == gmax) / max(1, sum(1 for g, _ in v if g == gmax)) for k, v in vals.items()}
    res = {k: round(v, 3) for k, v in sorted(avg.items())}
    rd = 2 * avg.get("FETCH_SIZE", 0.0) * 1024
    wr = avg.get("WRITE_SIZE", 0.0) * 1024
    res.update({
        "kernel": kname, "grid_size": gmax, "tiles_per_launch": tiles,
        "hbm_read_bytes_per_launch": rd, "hbm_write_bytes_per_launch": wr,
        "hbm_bytes_per_tile": (rd + wr) / tiles,
        "algorithmic_bytes_per_tile": alg,
        "traffic_over_algorithmic": round((rd + wr) / tiles / alg, 4),
        "note": "FETCH_SIZE x2 (gfx950 half-count of wide streaming reads), KiB->B; one counter per pass",
    })
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
