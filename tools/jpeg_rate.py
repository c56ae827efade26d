#!/usr/bin/env python3
"""C2 (or C1 with JPEG_PROBE_CASE=c1) render -> JPEG throughput, fused path, 256 tiles per call:
tiles/s over >= 0.5 s of back-to-back calls after a 0.3 s prewarm, for the library and settings
of this process's environment (OMR_LIB, OMR_JPEG_*).  One JSON line; used for same-box A/B."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "omero-ms-image-region_amd"))
sys.path.insert(0, REPO)


def main():
    import torch
    import omr
    from omr import _lib
    from omr.context import make_bindings, make_qdef
    from omr.synthetic import c2_channels
    import bench
    B, T = int(os.environ.get("JPEG_PROBE_TILES", "256")), 1024
    dev = torch.device("cuda", 0)
    ctx = omr.Context(0, torch_order=False)
    if os.environ.get("JPEG_PROBE_CASE", "c2") == "c1":
        g = torch.Generator(device=dev)
        g.manual_seed(20261015)
        data = torch.randint(0, 256, (B, T, T), dtype=torch.uint8, device=dev, generator=g)
        q = make_qdef("greyscale")
        ch = [{"input_start": 0.0, "input_end": 255.0, "global_min": 0.0, "global_max": 255.0}]
        pt, pb, nc, be = _lib.PIXELS_UINT8, T * T, 1, False
    else:
        data, uniq, table = bench.build_batch(torch, B, 8, dev)
        q, ch = make_qdef("rgb"), c2_channels(4)
        pt, pb, nc, be = _lib.PIXELS_UINT16, T * T * 2, 4, True
    binds = make_bindings(ch)
    cap = B * T * T * 3
    d_out = torch.empty(cap, dtype=torch.uint8, device=dev)
    offs = torch.empty(B, dtype=torch.int64, device=dev)
    lens = torch.empty(B, dtype=torch.int32, device=dev)
    stat = torch.empty(B, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()

    def step():
        ctx.render_jpeg_batch_strided_device(q, ch, data, nc * pb, pb, B, pt, T, T, 0.9, d_out, offs, lens, stat,
                                             big_endian=be, bindings=binds)
    t_end = time.perf_counter() + 0.3
    while time.perf_counter() < t_end:
        step()
        ctx.synchronize()
    n = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.5:
        for _ in range(4):
            step()
        n += 4
    ctx.synchronize()
    el = time.perf_counter() - t0
    ln = lens.cpu()
    print(json.dumps({"case": os.environ.get("JPEG_PROBE_CASE", "c2"), "tiles_per_s": round(B * n / el, 1),
                      "ms_per_call": round(1e3 * el / n, 4), "calls": n,
                      "bytes_checksum": int(ln.sum().item()),
                      "env": {k: v for k, v in os.environ.items() if k.startswith("OMR_")}}))


if __name__ == "__main__":
    main()
