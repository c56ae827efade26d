#!/usr/bin/env python3
"""profiles/pmc_render_c2.json (the headline's `traffic`, bench.py pmc_traffic) from a
tools/pmc_traffic.py summary of the headline leg (tools/gpu.sh pmc=c2): the K2 batch launch
(256 C2 tiles, the largest k_render grid), HBM bytes per tile against the algorithmic 12,582,912.

Usage: pmc_headline.py pmc_traffic_c2.json OUT.json [source-tag]"""
import json
import sys

ALG = 12582912
TILES = 256


def main():
    src, out = sys.argv[1], sys.argv[2]
    tag = sys.argv[3] if len(sys.argv) > 3 else ""
    d = json.load(open(src))
    ks = [k for k in d["kernels"] if k["kernel"].startswith("void omr::k_render<2, 8, true, false, 3, 4")
          and "FETCH_SIZE" in k and "WRITE_SIZE" in k]
    k = max(ks, key=lambda r: r["grid_size"])
    rd, wr = k["hbm_read_bytes"], k["hbm_write_bytes"]
    res = {"FETCH_SIZE": k["FETCH_SIZE"], "WRITE_SIZE": k["WRITE_SIZE"], "kernel": k["kernel"][:60],
           "grid_size": k["grid_size"], "tiles_per_launch": TILES, "dispatches": k.get("FETCH_SIZE_dispatches"),
           "hbm_read_bytes_per_launch": rd, "hbm_write_bytes_per_launch": wr,
           "hbm_bytes_per_tile": (rd + wr) / TILES, "algorithmic_bytes_per_tile": ALG,
           "traffic_over_algorithmic": round((rd + wr) / TILES / ALG, 4),
           "note": "FETCH_SIZE x2 (gfx950 half-count of wide streaming reads), KiB->B; one counter per pass",
           "source": tag, "build_id": d.get("build_id")}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
