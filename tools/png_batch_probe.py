#!/usr/bin/env python3
"""Batched PNG probe: C2 tiles rendered on the GPU, then omr_encode_png_batch_device at 64 and 256
tiles per call (and the single-tile path for comparison); per-call ms, tiles/s, mean file size.
One JSON line.  PNG_PROBE_SIZES=64,256 overrides the batch sizes."""
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
    T = 1024
    sizes = [int(x) for x in os.environ.get("PNG_PROBE_SIZES", "64,256").split(",")]
    B = max(sizes)
    dev = torch.device("cuda", 0)
    ctx = omr.Context(0, torch_order=False)
    data, uniq, table = bench.build_batch(torch, B, 8, dev)
    q, ch = make_qdef("rgb"), c2_channels(4)
    binds = make_bindings(ch)
    argb = torch.empty((B, T, T), dtype=torch.int32, device=dev)
    pb = T * T * 2
    torch.cuda.synchronize()
    ctx.render_batch_strided_device(q, ch, data, 4 * pb, pb, B, _lib.PIXELS_UINT16, T, T, argb, big_endian=True,
                                    bindings=binds)
    ctx.synchronize()
    cap = _lib.lib.omr_png_batch_max_bytes(T, T, 3, B)
    out = torch.empty(cap, dtype=torch.uint8, device=dev)
    offs = torch.empty(B, dtype=torch.int64, device=dev)
    lens = torch.empty(B, dtype=torch.int32, device=dev)
    stat = torch.empty(B, dtype=torch.int32, device=dev)
    res = {}
    for n in sizes:
        def step():
            ctx.encode_png_batch_device(argb, n, T, T, out, offs, lens, stat)
        t_end = time.perf_counter() + 0.3
        while time.perf_counter() < t_end:
            step()
            ctx.synchronize()
        iters = max(3, int(2048 / n))
        t0 = time.perf_counter()
        for _ in range(iters):
            step()
        ctx.synchronize()
        el = time.perf_counter() - t0
        ln = lens[:n].cpu().numpy()
        res[f"batch{n}"] = {"ms_per_call": round(1e3 * el / iters, 4), "tiles_per_s": round(n * iters / el, 1),
                            "mean_file_bytes": int(ln.mean()), "status_ok": int((stat[:n] == 0).sum().item())}
        if os.environ.get("PNG_PROBE_HASH"):               # the files' bytes, for same-output A/Bs
            import hashlib
            ob, oo = out.cpu().numpy(), offs[:n].cpu().numpy()
            h = hashlib.sha256()
            for k in range(n):
                h.update(ob[oo[k]:oo[k] + ln[k].astype("uint32")].tobytes())
            res[f"batch{n}"]["sha256"] = h.hexdigest()
        ctx.kernel_timings()                            # per-stage HIP events (kinds 20-26)
        ctx.enable_kernel_timing(True)
        for _ in range(4):
            step()
        ctx.synchronize()
        ctx.enable_kernel_timing(False)
        acc = {}
        for ms, kind in ctx.kernel_timings():
            acc.setdefault(int(kind), []).append(ms)
        res[f"batch{n}"]["stage_ms"] = {k: round(sum(v) / len(v), 4) for k, v in sorted(acc.items())}
    if hasattr(_lib.lib, "omr_png_t3_probe"):            # a -DOMR_PNG_T3_PROBE build: P3 phase clocks
        import ctypes
        buf = (ctypes.c_ulonglong * 32)()
        if _lib.lib.omr_png_t3_probe(buf) == 0:
            t = list(buf)
            res["t3_phase_cycles"] = {f"{a}-{b}": int(t[b] - t[a]) for a, b in
                                      ((0, 1), (1, 2), (2, 3), (3, 4), (4, 5), (5, 6), (6, 7),
                                       (8, 9), (9, 10), (10, 11), (11, 12))}
            res["t4_phase_cycles"] = {f"{a}-{b}": int(t[16 + b] - t[16 + a]) for a, b in
                                      ((0, 1), (1, 2), (2, 3), (3, 4), (4, 5))}
    # single-tile path (host D3, one sync per tile)
    t0 = time.perf_counter()
    k = 32
    for i in range(k):
        ctx.encode_png_device(argb[i], T, T)
    el = time.perf_counter() - t0
    res["single"] = {"ms_per_tile": round(1e3 * el / k, 4), "tiles_per_s": round(k / el, 1)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
