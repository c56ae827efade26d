#!/usr/bin/env python3
"""Per-kernel averages of rocprofv3 --pmc counter CSVs (any number of passes).

Usage: pmc_kernels.py [--json OUT --case NAME --mcus N] pass1.csv [pass2.csv ...]
Prints, per kernel (largest grid only, i.e. the batch launches), the mean of every counter over
its dispatches, plus derived ratios: VALU instructions per wave, issue share of wave cycles.
With --json, the per-launch averages and the per-MCU instruction counts (N MCUs per launch) of
every kernel are merged into OUT under NAME (bench.py reads them for the JPEG VALU roofline).
"""
import csv
import json
import os
import sys
from collections import defaultdict


def main():
    args = sys.argv[1:]
    opt = {}
    while args and args[0].startswith("--"):
        opt[args[0][2:]] = args[1]
        args = args[2:]
    vals = defaultdict(lambda: defaultdict(list))
    grids = defaultdict(int)
    out = {}
    for path in args:
        with open(path) as fh:
            for row in csv.DictReader(fh):
                k = row["Kernel_Name"].split("(")[0]
                g = int(row["Grid_Size"])
                grids[k] = max(grids[k], g)
                vals[k][row["Counter_Name"]].append((g, float(row["Counter_Value"])))
    for k in sorted(vals):
        avg = {}
        for c, v in vals[k].items():
            sel = [x for g, x in v if g == grids[k]]
            avg[c] = sum(sel) / len(sel)
        out[k] = {"grid": grids[k], "counters": avg}
        if "mcus" in opt:
            n = int(opt["mcus"])
            out[k]["mcus_per_launch"] = n
            for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS"):
                if c in avg:
                    out[k][c + "_per_mcu"] = avg[c] / n
        print(f"== {k} (grid {grids[k]})")
        for c in sorted(avg):
            print(f"   {c:24s} {avg[c]:.4g}")
        w = avg.get("SQ_WAVES")
        if w:
            for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR"):
                if c in avg:
                    print(f"   {c + '/wave':24s} {avg[c] / w:.1f}")
        wc = avg.get("SQ_WAVE_CYCLES")
        if wc:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_WAIT_INST_LDS"):
                if c in avg:
                    print(f"   {c + '/wave_cycles':24s} {avg[c] / wc:.3f}")
    if "json" in opt:
        doc = {}
        if os.path.exists(opt["json"]):
            with open(opt["json"]) as fh:
                doc = json.load(fh)
        doc[opt.get("case", "default")] = out
        from build_id import build_id
        doc["build_id"] = build_id()
        with open(opt["json"], "w") as fh:
            json.dump(doc, fh, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
