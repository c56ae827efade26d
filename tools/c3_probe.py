#!/usr/bin/env python3
"""C3 probe: the projection glue on 3 x 512x512x64 u16 BE stacks (max and mean), per-launch K3
times from the context's HIP events after a 300 ms prewarm, and requests/s.  One JSON line."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "omero-ms-image-region_amd"))


def main():
    import torch
    import omr
    from omr import _lib
    from omr.context import make_bindings, make_qdef
    from omr.synthetic import c2_channels
    dev = torch.device("cuda", 0)
    S, Z, C = 512, 64, 3
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    n_sets = int(os.environ.get("C3_SETS", "4"))   # the bench's rotation (384 MiB > the Infinity Cache)
    sets = [[torch.randint(-32768, 32768, (Z, S, S), dtype=torch.int32, device=dev, generator=g).to(torch.int16)
             for _ in range(C)] for _ in range(n_sets)]
    turn = [0]
    chans = c2_channels(C)
    qd, binds = make_qdef("rgb"), make_bindings(c2_channels(C))
    out = torch.empty((S, S), dtype=torch.int32, device=dev)
    ctx = omr.Context(0, torch_order=False)   # explicit syncs below, as the bench
    torch.cuda.synchronize()                    # inputs made by torch kernels
    res = {}
    for name, alg in (("max", _lib.PROJECTION_MAX), ("mean", _lib.PROJECTION_MEAN)):
        def step():
            turn[0] += 1
            ctx.render_projected_device(qd, chans, sets[turn[0] % n_sets], _lib.PIXELS_UINT16, S, S, Z, alg, 0, Z - 1, out,
                                        big_endian=True, bindings=binds)
        t_end = time.perf_counter() + 0.3
        while time.perf_counter() < t_end:
            step()
        ctx.synchronize()
        t0 = time.perf_counter()
        for _ in range(200):
            step()
        ctx.synchronize()
        el = time.perf_counter() - t0
        ctx.kernel_timings()
        ctx.enable_kernel_timing(True)
        for _ in range(200):
            step()
        ctx.synchronize()
        ctx.enable_kernel_timing(False)
        k3 = sorted(ms for ms, k in ctx.kernel_timings() if k == 3)
        used = Z if alg == _lib.PROJECTION_MAX else Z - 1
        by = C * (used * S * S * 2 + S * S * 2)
        med = k3[len(k3) // 2]
        avg = sum(k3) / len(k3)
        res[name] = {"requests_per_s": round(200 / el, 1), "k3_ms_median": round(med, 5), "k3_ms_avg": round(avg, 5),
                     "frac": round(by / (avg * 1e-3) / 8e12, 4), "sets": n_sets, "checksum": int(out.sum().item())}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
