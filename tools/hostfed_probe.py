#!/usr/bin/env python3
"""Host-fed C2 render (omr_render_pixel_buffer_tiles, DMA from the registered ROMIO mapping or
staged through pinned memory) per copy mode, alternated over rounds of >= 0.5 s each on one box:
row bands (default: 64 MiB staging groups, file-adjacent bands as one copy), per-tile 2-D rects
(OMR_PIXBUF_BANDS=0), bands with 128 / 256 MiB groups (OMR_PIXBUF_GROUP_MB); 4096^2 4-channel uint16 file in /dev/shm, requests walking its 16
tiles in raster order.  One JSON line."""
import json
import os
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "omero-ms-image-region_amd"))


def main():
    import numpy as np
    import torch
    import omr
    from omr import PixelBuffer, _lib, write_romio
    from omr.context import make_bindings, make_qdef
    from omr.synthetic import c2_channels
    T, grid, C = 1024, 4, 4
    n_req = int(os.environ.get("HOSTFED_TILES", "64"))
    rng = np.random.default_rng(3)
    img = rng.integers(0, 65536, (1, C, 1, grid * T, grid * T), dtype=np.uint16)
    fd, path = tempfile.mkstemp(prefix="omr_hf_", dir="/dev/shm")
    os.close(fd)
    res = {"tiles_per_call": n_req}
    try:
        write_romio(path, img, _lib.PIXELS_UINT16)
        qd, chans = make_qdef("rgb"), c2_channels(C)
        binds = make_bindings(chans)
        reqs = [(0, 0, (i % grid) * T, ((i // grid) % grid) * T) for i in range(n_req)]
        pb = PixelBuffer(path, grid * T, grid * T, 1, C, 1, _lib.PIXELS_UINT16)
        out = torch.empty((n_req, T, T), dtype=torch.int32, device="cuda")
        ctxs = {}
        for name, env in (("bands", {}), ("tile_rects", {"OMR_PIXBUF_BANDS": "0"}),
                          ("bands_group_128mib", {"OMR_PIXBUF_GROUP_MB": "128"}),
                          ("bands_group_256mib", {"OMR_PIXBUF_GROUP_MB": "256"})):
            os.environ.update(env)
            ctxs[name] = omr.Context(0, torch_order=False)
            for k in env:
                del os.environ[k]
        legs = [(n, c, 1) for n, c in ctxs.items()] + [("bands_staged", ctxs["bands"], 0),
                                                       ("tile_rects_staged", ctxs["tile_rects"], 0)]
        for name, c, dma in legs:
            res[name] = []
        for rnd in range(3):
            for name, c, dma in legs:
                _lib.check(_lib.lib.omr_ctx_set_pixel_buffer_dma(c.h, dma))
                c.render_pixel_buffer_tiles(qd, chans, pb, reqs, T, T, out=out, bindings=binds)
                c.synchronize()
                n = 0
                t0 = time.perf_counter()
                while time.perf_counter() - t0 < 0.5:
                    c.render_pixel_buffer_tiles(qd, chans, pb, reqs, T, T, out=out, bindings=binds)
                    n += 1
                c.synchronize()
                el = time.perf_counter() - t0
                res[name].append(round(n * n_req / el, 1))
                _lib.lib.omr_ctx_set_pixel_buffer_dma(c.h, 1)
        for name, _, _ in legs:
            v = res[name]
            res[name] = {"tiles_per_s": v, "h2d_gbs_best": round(max(v) * C * T * T * 2 / 1e9, 2)}
        pb.close()
        for c in ctxs.values():
            c.close()
    finally:
        os.unlink(path)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
