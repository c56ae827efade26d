#!/usr/bin/env python3
"""Same-box A/B of batcher dispatch settings on the bench's serving legs (bench.serving_section:
the interactive leg -- one request in flight per client, batcher vs independent contexts -- and the
screenful leg, 8 tiles in flight per client, batcher and pool).  Settings are read by
omr_batcher_create, so each configuration sets the environment before its batchers are made:
    SERVING_AB="1:200 2:200 2:30"   lanes:lane_gap_us per configuration (default)
One JSON line per configuration and repeat."""
import json
import os
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "omero-ms-image-region_amd"))
sys.path.insert(0, REPO)


def main():
    import numpy as np
    import torch
    import bench
    import omr
    from omr import PixelBuffer, _lib, write_romio
    from omr.context import make_bindings, make_qdef
    from omr.synthetic import c2_channels
    dev = torch.device("cuda", 0)
    _, uniq, _ = bench.build_batch(torch, 8, 8, dev)
    host = uniq.cpu().numpy().view(np.uint16).byteswap()
    T, grid, C = bench.TILE, 4, bench.CHANNELS
    img = np.empty((1, C, 1, grid * T, grid * T), dtype=np.uint16)
    for ty in range(grid):
        for tx in range(grid):
            img[0, :, 0, ty * T:(ty + 1) * T, tx * T:(tx + 1) * T] = host[(ty * grid + tx) % host.shape[0]]
    fd, path = tempfile.mkstemp(prefix="omr_romio_", dir="/dev/shm")
    os.close(fd)
    try:
        write_romio(path, img, _lib.PIXELS_UINT16)
        pb = PixelBuffer(path, grid * T, grid * T, 1, C, 1, _lib.PIXELS_UINT16)
        qd, chans = make_qdef("rgb"), c2_channels(C)
        binds = make_bindings(chans)
        ctx = omr.Context(0, torch_order=False)
        for rep in range(int(os.environ.get("SERVING_AB_REPEATS", "2"))):
            for cfg in os.environ.get("SERVING_AB", "1:200 2:200 2:30").split():
                lanes, gap = cfg.split(":")
                os.environ["OMR_BATCH_LANES"], os.environ["OMR_BATCH_LANE_GAP_US"] = lanes, gap
                r = bench.serving_section(torch, ctx, pb, qd, chans, binds, grid, pool_devices=[0, 0])
                it = r["interactive"]
                bk = next(k for k in it if k.startswith("batcher"))
                out = {"cfg": cfg, "rep": rep,
                       "interactive": {"batcher": [it[bk]["tiles_per_s"], it[bk]["p50_ms"]],
                                       "independent": [it["independent_contexts"]["tiles_per_s"],
                                                       it["independent_contexts"]["p50_ms"]]},
                       "screenful": {k: [r[k]["tiles_per_s"], r[k]["p50_ms"], r[k]["rendered_per_s"]]
                                     for k in r if k.startswith(("batcher", "pool"))}}
                print(json.dumps(out), flush=True)
        ctx.close()
    finally:
        os.unlink(path)


if __name__ == "__main__":
    main()
