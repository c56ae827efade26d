#!/usr/bin/env python3
"""Per-launch K2 durations on the C2 headline launch (256 strided BE tiles), to find where the
launch-to-launch spread comes from.  Phases: (a) the driver's shape — 5 warm-up steps then 20
timed launches, (b) ~1 s of back-to-back launches, (c) 20 timed launches again, (d) 20 timed
launches with a 50 ms idle gap before each (clock/power ramp after idle).  Prints one JSON line."""
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
    B = int(os.environ.get("K2_BATCH", "256"))
    dev = torch.device("cuda", 0)
    data, uniq, table = bench.build_batch(torch, B, 8, dev)
    out = torch.empty((B, 1024, 1024), dtype=torch.int32, device=dev)
    ctx = omr.Context(0)
    q, ch = make_qdef("rgb"), c2_channels(4)
    binds = make_bindings(ch)
    pb = 1024 * 1024 * 2

    def step():
        ctx.render_batch_strided_device(q, ch, data, 4 * pb, pb, B, _lib.PIXELS_UINT16, 1024, 1024, out,
                                        big_endian=True, bindings=binds)

    def timed(n, gap=0.0):
        ctx.kernel_timings()
        ctx.enable_kernel_timing(True)
        for _ in range(n):
            if gap:
                ctx.synchronize()
                time.sleep(gap)
            step()
        ctx.synchronize()
        ctx.enable_kernel_timing(False)
        return [round(ms, 4) for ms, k in ctx.kernel_timings() if k == 2]

    def stats(v):
        s = sorted(v)
        return {"n": len(v), "min": s[0], "med": s[len(s) // 2], "max": s[-1], "mean": round(sum(v) / len(v), 4),
                "series": v[:40]}
    res = {"batch": B, "nt_store": os.environ.get("OMR_K2_NT_STORE", "0")}
    for _ in range(5):
        step()
    ctx.synchronize()
    res["a_driver_shape"] = stats(timed(20))
    t0 = time.time()
    n = 0
    while time.time() - t0 < 1.0:
        step()
        n += 1
        if n % 50 == 0:
            ctx.synchronize()
    ctx.synchronize()
    res["b_sustained_launches"] = n
    res["c_after_sustained"] = stats(timed(20))
    res["d_after_idle_gap"] = stats(timed(20, gap=0.05))
    res["e_long"] = stats(timed(200))
    print(json.dumps(res), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
