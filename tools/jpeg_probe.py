#!/usr/bin/env python3
"""C2 -> JPEG on 64 tiles, unfused (K1+K2 then B1..B6) and fused (F1..B6), a few calls each:
the program the JPEG PMC passes (tools/profile_jpeg_r02.sh) profile."""
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
    B, T = 64, 1024
    dev = torch.device("cuda", 0)
    data, uniq, table = bench.build_batch(torch, B, 8, dev)
    ctx = omr.Context(0)
    q, ch = make_qdef("rgb"), c2_channels(4)
    binds = make_bindings(ch)
    pb = T * T * 2
    argb = torch.empty((B, T, T), dtype=torch.int32, device=dev)
    d_out = torch.empty(B * T * T * 3, dtype=torch.uint8, device=dev)
    offs = torch.empty(B, dtype=torch.int64, device=dev)
    lens = torch.empty(B, dtype=torch.int32, device=dev)
    stat = torch.empty(B, dtype=torch.int32, device=dev)
    n = int(os.environ.get("JPEG_PROBE_ITERS", "5"))
    for _ in range(n):
        ctx.render_batch_strided_device(q, ch, data, 4 * pb, pb, B, _lib.PIXELS_UINT16, T, T, argb, big_endian=True,
                                        bindings=binds)
        ctx.encode_jpeg_batch_device(argb, B, T, T, 0.9, d_out, offs, lens, stat)
    for _ in range(n):
        ctx.render_jpeg_batch_strided_device(q, ch, data, 4 * pb, pb, B, _lib.PIXELS_UINT16, T, T, 0.9, d_out, offs,
                                             lens, stat, big_endian=True, bindings=binds)
    ctx.synchronize()
    print("ok")


if __name__ == "__main__":
    main()
