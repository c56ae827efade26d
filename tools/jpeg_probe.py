#!/usr/bin/env python3
"""C2 -> JPEG (or, with JPEG_PROBE_CASE=c1, C1: 1-channel uint8 greyscale) on 64 tiles (JPEG_PROBE_TILES), unfused
(K1+K2 then B1..B6) and fused (F1..B6), a few calls each: the program the JPEG PMC passes
(tools/gpu.sh sq=jpeg / pmc=jpeg / ab=jpeg:...) profile."""
import os
import sys

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
    B, T = int(os.environ.get("JPEG_PROBE_TILES", "64")), 1024
    dev = torch.device("cuda", 0)
    ctx = omr.Context(0, torch_order=False)   # explicit syncs below, as the bench
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
    argb = torch.empty((B, T, T), dtype=torch.int32, device=dev)
    d_out = torch.empty(B * T * T * 3, dtype=torch.uint8, device=dev)
    offs = torch.empty(B, dtype=torch.int64, device=dev)
    lens = torch.empty(B, dtype=torch.int32, device=dev)
    stat = torch.empty(B, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()                    # inputs made by torch kernels
    n = int(os.environ.get("JPEG_PROBE_ITERS", "5"))
    for _ in range(n):
        ctx.render_batch_strided_device(q, ch, data, nc * pb, pb, B, pt, T, T, argb, big_endian=be, bindings=binds)
        ctx.encode_jpeg_batch_device(argb, B, T, T, 0.9, d_out, offs, lens, stat)
    for _ in range(n):
        ctx.render_jpeg_batch_strided_device(q, ch, data, nc * pb, pb, B, pt, T, T, 0.9, d_out, offs, lens, stat,
                                             big_endian=be, bindings=binds)
    ctx.synchronize()
    print("ok")


if __name__ == "__main__":
    main()
