#!/usr/bin/env python3
"""JSON form of a tools/pmc_kernels.py text summary (tools/gpu.sh sq=<probe> -> sq_<probe>.txt):
per kernel (its largest grid: the batch launches), the per-launch mean of every SQ counter.
bench.py reads these for the VALU-issue roofline of the batched PNG stages.

Usage: sq_json.py sq_png.txt OUT.json [source-tag]"""
import json
import re
import sys


def main():
    src, out = sys.argv[1], sys.argv[2]
    from build_id import build_id
    doc = {"source": sys.argv[3] if len(sys.argv) > 3 else src, "build_id": build_id(),
           "note": "per-launch means over the probe's dispatches of each kernel's largest grid", "kernels": {}}
    cur = None
    for line in open(src):
        m = re.match(r"== (\S.*) \(grid (\d+)\)", line)
        if m:
            cur = {"grid": int(m.group(2)), "counters": {}}
            doc["kernels"][m.group(1)] = cur
            continue
        m = re.match(r"\s+(SQ_\w+|GRBM_\w+)\s+([-+0-9.eE]+)$", line)
        if m and cur is not None:
            cur["counters"][m.group(1)] = float(m.group(2))
    json.dump(doc, open(out, "w"), indent=1, sort_keys=True)
    print(f"{len(doc['kernels'])} kernels -> {out}")


if __name__ == "__main__":
    main()
