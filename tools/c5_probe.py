#!/usr/bin/env python3
"""C5 K2 (3-ch f32 1024^2, log / poly / poly+lut, windows p1/p99) on 32 tiles: per-launch K2 ms
under the context's current settings (OMR_K2_EVAL_CPT), one JSON line."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "omero-ms-image-region_amd"))
sys.path.insert(0, REPO)


def main():
    import numpy as np
    import torch
    import omr
    from omr import _lib
    from omr.context import make_bindings, make_qdef
    from omr.synthetic import c5_channels, c5_planes
    T, uniq = 1024, 4
    B = int(os.environ.get("C5_TILES", "32"))
    rng = np.random.default_rng(20261015 + 5)
    host = np.stack([np.stack(c5_planes(T, T, rng)) for _ in range(uniq)])
    chans = c5_channels(list(host[0]))       # the bench's C5 settings
    dev = torch.device("cuda", 0)
    src = torch.from_numpy(np.ascontiguousarray(host.astype(">f4")).view(np.uint8)).to(dev)
    data = torch.empty((B, 3 * T * T * 4), dtype=torch.uint8, device=dev)
    for t in range(B):
        data[t].copy_(src.view(uniq, -1)[t % uniq])
    out = torch.empty((B, T, T), dtype=torch.int32, device=dev)
    ctx = omr.Context(0, torch_order=False)   # explicit syncs below, as the bench
    torch.cuda.synchronize()                    # inputs made by torch kernels
    qd, binds, plane = make_qdef("rgb"), make_bindings(chans), T * T * 4

    def step():
        ctx.render_batch_strided_device(qd, chans, data, 3 * plane, plane, B, _lib.PIXELS_FLOAT, T, T, out,
                                        big_endian=True, bindings=binds)
    for _ in range(200):
        step()
    ctx.synchronize()
    ctx.kernel_timings()
    ctx.enable_kernel_timing(True)
    for _ in range(50):
        step()
    ctx.synchronize()
    k2 = sorted(ms for ms, k in ctx.kernel_timings() if k == 2)
    ref = out.cpu().numpy()
    print(json.dumps({"eval_cpt": os.environ.get("OMR_K2_EVAL_CPT", "4"), "k2_ms_median": k2[len(k2) // 2],
                      "k2_ms_min": k2[0], "frac": round(B * 16777216 / (k2[len(k2) // 2] * 1e-3) / 8e12, 4),
                      "checksum": int(ref.astype(np.int64).sum())}))


if __name__ == "__main__":
    main()
