#!/usr/bin/env python3
"""PNG latency probe: one rendered C2 1024^2 tile -> device PNG (omr_encode_png_device) and the
1024^2 shape mask -> PNG (omr_render_shape_mask_png), p50 over 40 calls, sizes, and a decode
check of the tile PNG against the rendered pixels.  One JSON line."""
import io
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "omero-ms-image-region_amd"))


def main():
    import numpy as np
    import torch
    from PIL import Image
    import omr
    from omr import _lib
    from omr.context import make_qdef
    from omr.synthetic import c2_channels, tile_u16
    T = 1024
    ctx = omr.Context(0, torch_order=False)   # explicit syncs below, as the bench
    planes = [torch.from_numpy(np.ascontiguousarray(p.astype(">u2")).view(np.uint8).reshape(-1)).to("cuda")
              for p in tile_u16(7, 4, T, T)]
    out = torch.empty((T, T), dtype=torch.int32, device="cuda")
    ctx.render_packed_int_device(make_qdef("rgb"), c2_channels(4), planes, _lib.PIXELS_UINT16, T, T, out,
                                 big_endian=True)
    ctx.synchronize()
    lat = []
    for i in range(43):
        t0 = time.perf_counter()
        png = ctx.encode_png_device(out, T, T)
        if i >= 3:
            lat.append(time.perf_counter() - t0)
    a = out.cpu().numpy().view(np.uint32)
    rgb = np.stack([(a >> 16) & 0xFF, (a >> 8) & 0xFF, a & 0xFF], -1).astype(np.uint8)
    ok = bool(np.array_equal(np.asarray(Image.open(io.BytesIO(png)).convert("RGB")), rgb))
    rng = np.random.default_rng(3)
    yy, xx = np.mgrid[0:T, 0:T]
    m = np.zeros((T, T), bool)
    for _ in range(24):
        cy, cx, ry, rx = rng.uniform(0, T), rng.uniform(0, T), rng.uniform(10, 120), rng.uniform(10, 120)
        m |= ((yy - cy) / ry) ** 2 + ((xx - cx) / rx) ** 2 <= 1
    bits = np.packbits(m.reshape(-1)).tobytes()
    mlat = []
    ctx.set_semantics(_lib.SEM_MASK_PIXEL_FLIP)     # flip hv of a 1024-wide mask: pixel flip
    for i in range(43):
        t0 = time.perf_counter()
        mpng = ctx.render_shape_mask_png(bits, T, T, (255, 0, 0, 128), flip_h=True, flip_v=True)
        if i >= 3:
            mlat.append(time.perf_counter() - t0)
    print(json.dumps({"tile_png_p50_ms": round(1e3 * float(np.median(lat)), 4), "tile_png_bytes": len(png),
                      "tile_png_decodes_exact": ok, "mask_png_p50_ms": round(1e3 * float(np.median(mlat)), 4),
                      "mask_png_bytes": len(mpng)}))


if __name__ == "__main__":
    main()
