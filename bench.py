#!/usr/bin/env python3
"""bench.py — BASELINE.json headline metric on the MI355X render path.

Workload (BASELINE.json configs[1], "C2"): 4-channel uint16 1024x1024 tiles (big-endian, as
ROMIO planes), per-channel window + colour composite to packed ARGB.  One step = one
omr_render_batch_device call over a batch of tiles already resident in HBM (K1 table build +
K2 quantize/composite).  Multi-GPU: one process per GPU, each rendering its own batch (tiles
are independent — no collective on the data path; barrier + max-over-ranks timing only).

Also reported: roofline of K2 (HIP events around every K2 launch on its stream), p50 tile
latency (device-resident and host-fed), and the reference-CPU proxy (oracle/liboracle.so,
per-request LUT rebuild + render, on the host cores) on a bounded sample.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "omero-ms-image-region_amd"))

METRIC = "1024² tiles/sec (whole node) at 1/2/4/8 GPUs; p50 tile latency; HBM GB/s"
TILE = 1024
CHANNELS = 4
BYTES_PER_TILE = TILE * TILE * CHANNELS * 2 + TILE * TILE * 4   # 12,582,912 algorithmic bytes
HBM_PEAK_GBS = 8000.0                                           # MI355X_MICROARCH.md: 8.0 TB/s spec


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def build_batch(torch, batch, unique, device):
    """[batch][4][1024][1024] big-endian uint16 tiles (int16 storage) + device pointer table."""
    from omr.synthetic import torch_tiles_u16
    uniq = torch_tiles_u16(unique, CHANNELS, TILE, TILE, device)
    uniq = uniq.view(torch.uint8).view(unique, CHANNELS, TILE, TILE, 2).flip(-1).contiguous().view(
        torch.int16).view(unique, CHANNELS, TILE, TILE)                          # -> big-endian bytes
    data = torch.empty((batch, CHANNELS, TILE, TILE), dtype=torch.int16, device=device)
    for t in range(batch):
        data[t].copy_(uniq[t % unique])
    plane_bytes = TILE * TILE * 2
    base = data.data_ptr()
    table = torch.tensor([[base + (t * CHANNELS + c) * plane_bytes for c in range(CHANNELS)]
                          for t in range(batch)], dtype=torch.int64, device=device)
    return data, uniq, table


def pmc_traffic(batch):
    """HBM bytes per K2 launch from the committed rocprofv3 PMC summary (profiles/), or None."""
    path = os.path.join(REPO, "profiles", "pmc_render_c2.json")
    if not os.path.exists(path):
        return None
    try:
        with open(path) as fh:
            d = json.load(fh)
        return d["hbm_bytes_per_tile"] * batch
    except Exception:
        return None


def host_cores():
    """(threads, nproc, quota): the CPUs this process may run on (what `nproc` prints), the
    cgroup CPU quota if one is set (cpu.max: quota/period CPUs' worth of time), and the thread
    count the CPU baseline uses — nproc, capped at the quota: on the GPU box nproc is the whole
    machine (256) while the job may use 16 CPUs' worth of time, and 256 threads time-sliced onto
    16 CPUs run the C2 baseline at 455 tiles/s against ~1000 with 16 (gpurun_out r02a)."""
    import math
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            q, p = fh.read().split()[:2]
            if q != "max":
                quota = round(int(q) / int(p), 2)
    except Exception:
        pass
    threads = min(n, max(1, math.ceil(quota))) if quota else n
    return threads, n, quota


def _oracle():
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_lib
    return oracle_lib


def cpu_baseline(torch, uniq, seconds, threads):
    """Reference-CPU proxy on a bounded sample: per-request LUT rebuild + render, on `threads`
    (= nproc) worker threads, and the same work on one thread."""
    import numpy as np
    oracle_lib = _oracle()
    from omr import _lib
    from omr.synthetic import c2_channels
    host = uniq.cpu().numpy().view(np.uint16)      # big-endian bytes in uint16 storage
    tiles = [[np.ascontiguousarray(host[t, c]) for c in range(CHANNELS)] for t in range(host.shape[0])]
    chans = c2_channels(CHANNELS)

    def run(nthreads, secs_target):
        n = nthreads
        secs, _ = oracle_lib.render_tiles_mt(chans, [tiles[t % len(tiles)] for t in range(n)], n,
                                             _lib.PIXELS_UINT16, TILE, TILE, big_endian=True,
                                             n_threads=nthreads, keep_output=False, fast=True)
        n = max(nthreads, int(n * secs_target / max(secs, 1e-3)) // nthreads * nthreads)
        secs, _ = oracle_lib.render_tiles_mt(chans, [tiles[t % len(tiles)] for t in range(n)], n,
                                             _lib.PIXELS_UINT16, TILE, TILE, big_endian=True,
                                             n_threads=nthreads, keep_output=False, fast=True)
        return n, secs
    n, secs = run(threads, seconds)
    n1, secs1 = run(1, min(4.0, seconds / 2))
    _, nproc, quota = host_cores()
    return {"value": round(n / secs, 3), "unit": "tiles/s", "cores": threads, "kind": "port",
            "nproc": nproc, "cgroup_cpu_quota": quota, "build": oracle_lib.FAST_BUILD,
            "single_thread": {"value": round(n1 / secs1, 3), "unit": "tiles/s", "cores": 1,
                              "sample": f"{n1} tiles in {secs1:.2f} s"},
            "sample": f"{n} C2 tiles (4ch uint16 1024^2 BE, per-request LUT rebuild + composite) "
                      f"in {secs:.2f} s on {threads} threads (nproc {nproc}, cgroup quota {quota} CPUs) "
                      f"(oracle/omr_oracle.c, "
                      f"{oracle_lib.FAST_BUILD})"}


def latencies(torch, omr, ctx, qdef, chans, data, iters=30):
    """p50 of one-tile requests: device-resident (HBM in/out) and host-fed (pinned H2D + D2H)."""
    import numpy as np
    from omr import _lib
    dev = data.device
    out1 = torch.empty((TILE, TILE), dtype=torch.int32, device=dev)
    planes = [data[0, c] for c in range(CHANNELS)]
    t_dev = []
    for i in range(iters + 3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ctx.render_packed_int_device(qdef, chans, planes, _lib.PIXELS_UINT16, TILE, TILE, out1, big_endian=True)
        ctx.synchronize()
        if i >= 3:
            t_dev.append(time.perf_counter() - t0)
    # the whole render_image_region request at its default format: render + one-tile JPEG
    # (q 0.9) copied back to the host (ImageRegionRequestHandler.java:559-582)
    t_jpg = []
    for i in range(iters + 3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ctx.render_packed_int_device(qdef, chans, planes, _lib.PIXELS_UINT16, TILE, TILE, out1, big_endian=True)
        ctx.encode_jpeg_device(out1, TILE, TILE, 0.9)
        if i >= 3:
            t_jpg.append(time.perf_counter() - t0)
    host = [np.ascontiguousarray(p.cpu().numpy()) for p in planes]
    t_host = []
    for i in range(iters + 3):
        t0 = time.perf_counter()
        ctx.render_packed_int(qdef, chans, host, _lib.PIXELS_UINT16, TILE, TILE, big_endian=True)
        if i >= 3:
            t_host.append(time.perf_counter() - t0)
    res = {"device_resident": round(1e3 * float(np.median(t_dev)), 4),
           "device_resident_to_jpeg_host": round(1e3 * float(np.median(t_jpg)), 4),
           "host_fed": round(1e3 * float(np.median(t_host)), 4)}
    # the same requests from C++ through the C ABI (tools/omr_latency.cpp, built by build()):
    # what a JNI / Panama caller sees without Python's marshalling
    exe = os.path.join(REPO, "tools", "omr_latency")
    if os.path.exists(exe):
        import subprocess
        try:
            r = subprocess.run([exe, "200", str(dev.index or 0)], capture_output=True, text=True, timeout=120)
            if r.returncode == 0:
                res["native_c_abi"] = json.loads(r.stdout.strip().splitlines()[-1])
            else:
                log(f"omr_latency failed ({r.returncode}): {r.stderr.strip()[-300:]}")
        except Exception as e:
            log(f"omr_latency failed: {e}")
    return res


def jpeg_section(torch, ctx, data, B, steps, warmup, cpu_seconds, threads, with_cpu):
    """render_image_region's default output (format=jpeg, ImageRegionRequestHandler.java:580-582)
    on whole batches: render batch -> batched JPEG (device-resident in, device JPEG files out).
    C2->JPEG on the C2 tiles, and BASELINE configs[0] (C1: 1-channel uint8 1024^2 greyscale,
    uniform [0,255], q=0.9).  Per-kernel HIP-event timings: K2 render (2), J1 FDCT (5),
    J3 Huffman (6), whole JPEG pipeline (4)."""
    import numpy as np
    from omr import _lib
    from omr.context import make_bindings, make_qdef
    from omr.synthetic import c2_channels
    dev = data.device
    q = 0.9
    res = {}
    g = torch.Generator(device=dev)
    g.manual_seed(20261015)
    u8 = torch.randint(0, 256, (B, TILE, TILE), dtype=torch.uint8, device=dev, generator=g)
    c1 = [{"input_start": 0.0, "input_end": 255.0, "global_min": 0.0, "global_max": 255.0}]
    cases = {
        "c2_u16_4ch_rgb_to_jpeg": (make_qdef("rgb"), c2_channels(CHANNELS), data, _lib.PIXELS_UINT16,
                                   CHANNELS * TILE * TILE * 2, TILE * TILE * 2, True),
        "c1_u8_grey_to_jpeg": (make_qdef("greyscale"), c1, u8, _lib.PIXELS_UINT8, TILE * TILE, TILE * TILE, False),
    }
    argb = torch.empty((B, TILE, TILE), dtype=torch.int32, device=dev)
    cap = B * (TILE * TILE * 3)
    d_out = torch.empty(cap, dtype=torch.uint8, device=dev)
    offs = torch.empty(B, dtype=torch.int64, device=dev)
    lens = torch.empty(B, dtype=torch.int32, device=dev)
    stat = torch.empty(B, dtype=torch.int32, device=dev)
    import omr
    ctx2 = omr.Context(ctx.device, torch_order=False)
    for name, (qd, chans, src, pt, tstride, cstride, be) in cases.items():
        binds = make_bindings(chans)

        def step():
            ctx.render_batch_strided_device(qd, chans, src, tstride, cstride, B, pt, TILE, TILE, argb,
                                            big_endian=be, bindings=binds)
            ctx.encode_jpeg_batch_device(argb, B, TILE, TILE, q, d_out, offs, lens, stat)
        el, avg = _timed(torch, ctx, step, steps, warmup)
        # Two contexts (two HIP streams) taking alternate batches, as two batcher dispatchers
        # would: one batch's HBM-bound render overlaps the other's VALU-bound JPEG kernels.
        bufs = [(argb, d_out, offs, lens, stat), tuple(torch.empty_like(t) for t in (argb, d_out, offs, lens, stat))]
        ctxs = [ctx, ctx2]
        k = [0]

        def step2():
            i = k[0] & 1
            k[0] += 1
            a, o, of, ln_, st_ = bufs[i]
            ctxs[i].render_batch_strided_device(qd, chans, src, tstride, cstride, B, pt, TILE, TILE, a,
                                                big_endian=be, bindings=binds)
            ctxs[i].encode_jpeg_batch_device(a, B, TILE, TILE, q, o, of, ln_, st_)
        for _ in range(warmup):
            step2()
        ctx.synchronize()
        ctx2.synchronize()
        t0 = time.perf_counter()
        for _ in range(2 * steps):
            step2()
        ctx.synchronize()
        ctx2.synchronize()
        el2 = time.perf_counter() - t0
        assert (bufs[1][4].cpu().numpy() == 0).all(), "JPEG batch did not fit its buffer"
        ln = lens.cpu().numpy().astype(np.int64)
        assert (stat.cpu().numpy() == 0).all(), "JPEG batch did not fit its buffer"
        ref_files = d_out.cpu().numpy()
        ref_offs = offs.cpu().numpy()

        # Fused: render + JPEG in one call (F1 = render + colour + FDCT in one kernel, the ARGB tile
        # never reaches HBM), omr_render_jpeg_batch_strided_device.
        def step_fused():
            ctx.render_jpeg_batch_strided_device(qd, chans, src, tstride, cstride, B, pt, TILE, TILE, q, d_out, offs,
                                                 lens, stat, big_endian=be, bindings=binds)
        el_f, avg_f = _timed(torch, ctx, step_fused, steps, warmup)
        fo, fl = offs.cpu().numpy(), lens.cpu().numpy()
        fb = d_out.cpu().numpy()
        assert all(fb[fo[i]:fo[i] + fl[i]].tobytes() == ref_files[ref_offs[i]:ref_offs[i] + ln[i]].tobytes()
                   for i in range(B)), "fused render->JPEG differs from render + JPEG"
        # fused, two contexts taking alternate batches: one batch's Huffman/stuffing tail overlaps
        # the other's F1
        k[0] = 0

        def step2_fused():
            i = k[0] & 1
            k[0] += 1
            _, o, of, ln_, st_ = bufs[i]
            ctxs[i].render_jpeg_batch_strided_device(qd, chans, src, tstride, cstride, B, pt, TILE, TILE, q, o, of,
                                                     ln_, st_, big_endian=be, bindings=binds)
        for _ in range(warmup):
            step2_fused()
        ctx.synchronize()
        ctx2.synchronize()
        t0 = time.perf_counter()
        for _ in range(2 * steps):
            step2_fused()
        ctx.synchronize()
        ctx2.synchronize()
        el2_f = time.perf_counter() - t0
        mcus = B * (TILE // 16) ** 2
        px = TILE * TILE
        nblk = (TILE // 16) ** 2 * 6
        res[name] = {
            "tiles_per_s": round(B * steps / el, 1),
            "ms_per_step": round(1e3 * el / steps, 4),
            "tiles_per_step": B,
            "tiles_per_s_two_streams": round(2 * B * steps / el2, 1),
            "quality": q,
            "mean_jpeg_bytes": int(ln.mean()),
            "kernel_ms": {"render_K2": round(avg.get(2, float("nan")), 5),
                          "jpeg_total": round(avg.get(4, float("nan")), 5),
                          "J1_fdct": round(avg.get(5, float("nan")), 5),
                          "J3_huffman": round(avg.get(6, float("nan")), 5)},
            "fused": {"tiles_per_s": round(B * steps / el_f, 1), "ms_per_step": round(1e3 * el_f / steps, 4),
                      "tiles_per_s_two_streams": round(2 * B * steps / el2_f, 1),
                      "kernel_ms": {"F1_render_fdct": round(avg_f.get(5, float("nan")), 5),
                                    "jpeg_total": round(avg_f.get(4, float("nan")), 5),
                                    "J3_huffman": round(avg_f.get(6, float("nan")), 5)},
                      "F1_plane_read_gbs": round(B * tstride / (avg_f.get(5, float("nan")) * 1e-3) / 1e9, 1),
                      "byte_identical_to_unfused": True},
            "mcus_per_step": mcus,
            "J1_ns_per_mcu": round(avg.get(5, float("nan")) * 1e6 / mcus, 4),
            "F1_ns_per_mcu": round(avg_f.get(5, float("nan")) * 1e6 / mcus, 4),
        }
        vr = jpeg_valu_roofline(name, mcus, avg.get(5), avg_f.get(5), avg.get(6))
        if vr:
            if name.startswith("c2") and B == 256:
                mt = jpeg_measured_traffic(B * tstride + int(ln.sum()))
                if mt:
                    vr["measured_traffic"] = mt
            res[name]["valu_roofline"] = vr
        if with_cpu:
            try:
                res[name]["cpu_baseline"] = jpeg_cpu_baseline(torch, name, src, chans, pt, be, q,
                                                              cpu_seconds, threads)
            except Exception as e:
                log(f"jpeg cpu baseline failed: {e}")
    ctx2.close()
    return res


def kernel_build_id():
    """Fingerprint of the kernel sources (csrc/*.hip and the device headers): a committed SQ / PMC
    profile carries the id of the build it was collected on (tools/sq_json.py, tools/pmc_traffic.py),
    and the bench marks a profile of another build as such instead of mixing it silently into this
    run's rooflines."""
    import hashlib
    d = os.path.join(os.path.dirname(os.path.abspath(__file__)), "omero-ms-image-region_amd", "csrc")
    h = hashlib.sha1()
    for f in sorted(os.listdir(d)):
        if f.endswith((".hip", ".h")):
            with open(os.path.join(d, f), "rb") as fh:
                h.update(f.encode() + b"\0" + fh.read())
    return h.hexdigest()[:12]


def profile_provenance(doc, path):
    """source / build fields for a roofline read from a committed profile file."""
    bid = doc.get("build_id") if isinstance(doc, dict) else None
    cur = kernel_build_id()
    out = {"source": os.path.relpath(path, os.path.dirname(os.path.abspath(__file__))),
           "profile_build_id": bid, "this_build_id": cur, "same_build": bid == cur}
    if bid != cur:
        out["note"] = "committed profile of another build: counters not measured this run"
    return out


VALU_PMC = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "r06", "jpeg_valu_pmc.json")
VALU_PEAK_ISSUE_CYCLES_PER_S = 256 * 4 * 2.4e9   # 1,024 SIMD-32s at 2.4 GHz
# issue cycles of one wave64 VALU instruction: 2 on a SIMD-32; f64 add / mul / fma issue at half
# the f32 rate and transcendentals (v_exp / v_log / v_sqrt / v_rcp ...) at half the issue rate
# (MI355X_MICROARCH.md, vector-instruction issue cost), so they are charged 4
VALU_CYCLES = 2.0
VALU_SLOW_COUNTERS = ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64",
                      "SQ_INSTS_VALU_TRANS_F64", "SQ_INSTS_VALU_TRANS_F32")


PNG_SQ = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "r06", "png_sq.json")
# batched PNG stages (omr_png.hip launch_png_batch timer kinds) -> the kernels they launch
# (direct mode, the default since round 6: P5b/P6 before P4, which codes into the files)
PNG_STAGE_KERNELS = {20: ("k_pngb_filter_wave<4, true>",), 21: ("k_pngb_parse", "k_pngb_hist"),
                     22: ("k_pngb_tables", "k_pngb_block_offsets"), 23: ("k_pngb_encode",),
                     24: ("k_pngb_meta", "k_pngb_offsets"), 25: ("k_pngb_fixup", "k_pngb_emit_direct"),
                     26: ("k_pngb_crc", "k_pngb_finish")}


def png_valu_roofline(stage_ms):
    """VALU issue of each batched PNG stage (256 C2 tiles per call): SQ_INSTS_VALU per launch from
    the committed SQ passes (tools/gpu.sh sq=png -> tools/sq_json.py -> profiles/r06/png_sq.json,
    the same probe workload) x 2 issue cycles, over the stage's measured time; peak = every SIMD
    issuing every cycle.  Next to the stage's HBM frac it says which bound the stage is nearer."""
    try:
        with open(PNG_SQ) as fh:
            doc = json.load(fh)
    except (OSError, ValueError):
        return None
    ks = doc.get("kernels", {})
    out = {"bound": "valu", "unit": "issue-cycles/s", "peak": VALU_PEAK_ISSUE_CYCLES_PER_S}
    out.update(profile_provenance(doc, PNG_SQ))
    for kind, names in PNG_STAGE_KERNELS.items():
        ms = stage_ms.get(kind)
        rows = [v for k, v in ks.items() if any(k.endswith("::" + nm) for nm in names)]
        if not ms or not rows:
            continue
        valu = sum(r["counters"].get("SQ_INSTS_VALU", 0.0) for r in rows)
        conf = sum(r["counters"].get("SQ_LDS_BANK_CONFLICT", 0.0) for r in rows)
        lds = sum(r["counters"].get("SQ_LDS_IDX_ACTIVE", 0.0) for r in rows)
        ach = VALU_CYCLES * valu / (ms * 1e-3)
        out[str(kind)] = {"kernels": list(names), "valu_instr_per_launch": valu,
                          "achieved": round(ach, 1), "frac": round(ach / VALU_PEAK_ISSUE_CYCLES_PER_S, 4),
                          "lds_bank_conflict_share": round(conf / lds, 3) if lds else None,
                          "avg_ms": round(ms, 5)}
    return out


PNG_PMC = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "r06", "pmc_traffic_png.json")


def png_measured_traffic(alg_bytes):
    """HBM bytes per batched-PNG call of 256 C2 tiles, per stage, from the committed PMC passes
    (tools/gpu.sh pmc=png: FETCH_SIZE x 2 read, WRITE_SIZE written, one counter per pass; each
    kernel's largest grid = the 256-tile launch), against this run's algorithmic bytes (ARGB in +
    files out)."""
    try:
        with open(PNG_PMC) as fh:
            doc = json.load(fh)
        ks = doc["kernels"]
    except (OSError, ValueError, KeyError):
        return None
    big = {}
    for k in ks:
        name = k["kernel"].split("(")[0].split("::")[-1]
        if "hbm_read_bytes" in k and (name not in big or k["grid_size"] > big[name]["grid_size"]):
            big[name] = k
    per = {}
    for kind, names in PNG_STAGE_KERNELS.items():
        rows = [big[n] for n in names if n in big]
        if rows:
            per[str(kind)] = {"kernels": list(names), "read_mb": round(sum(r["hbm_read_bytes"] for r in rows) / 1e6, 1),
                              "write_mb": round(sum(r["hbm_write_bytes"] for r in rows) / 1e6, 1)}
    tot = sum(v["read_mb"] + v["write_mb"] for v in per.values()) * 1e6
    out = profile_provenance(doc, PNG_PMC)
    out.update({"per_stage": per, "total_mb": round(tot / 1e6, 1), "algorithmic_mb": round(alg_bytes / 1e6, 1),
                "ratio": round(tot / alg_bytes, 3) if alg_bytes else None})
    return out


JPEG_PMC = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "r06", "pmc_traffic_jpeg.json")
JPEG_FUSED_KERNELS = ("k_jpeg_render_fdct", "k_jpeg_block_bits", "k_jpeg_group_scan", "k_jpeg_huff_thread",
                      "k_jpeg_tile_scan", "k_jpeg_stuff_count", "k_jpeg_stuff_batch")


def jpeg_measured_traffic(algo_bytes):
    """HBM bytes per fused C2 -> JPEG call of 256 tiles from the committed PMC passes
    (tools/pmc_traffic.py: FETCH_SIZE x 2 x 1 KiB read, WRITE_SIZE x 1 KiB written, one counter per
    pass), against this run's algorithmic bytes (planes in + JPEG files out)."""
    try:
        with open(JPEG_PMC) as fh:
            doc = json.load(fh)
        ks = doc["kernels"]
    except (OSError, ValueError, KeyError):
        return None
    per = {}
    for key in JPEG_FUSED_KERNELS:
        k = next((k for k in ks if key in k["kernel"]), None)
        if k is not None:
            per[key] = {"read_mb": round(k["hbm_read_bytes"] / 1e6, 1), "write_mb": round(k["hbm_write_bytes"] / 1e6, 1)}
    tot = sum(v["read_mb"] + v["write_mb"] for v in per.values()) * 1e6
    out = profile_provenance(doc, JPEG_PMC)
    out.update({"per_kernel": per, "total_mb": round(tot / 1e6, 1), "algorithmic_mb": round(algo_bytes / 1e6, 1),
                "ratio": round(tot / algo_bytes, 3)})
    return out


def jpeg_valu_roofline(name, mcus, j1_ms, f1_ms, j3_ms):
    """B1 / F1 / B3 are VALU-issue-bound: achieved = VALU issue cycles per launch
    (SQ_INSTS_VALU per MCU from the committed PMC passes, tools/gpu.sh sq=jpeg, at 2 cycles,
    plus 2 more for every f64 and transcendental instruction) x MCUs / the kernel's measured average
    duration; peak = every SIMD issuing every cycle at 2.4 GHz."""
    case = "c1" if name.startswith("c1") else "c2"
    try:
        with open(VALU_PMC) as fh:
            doc = json.load(fh)
        pmc = doc.get(case, {})
    except (OSError, ValueError):
        return None
    out = {"bound": "valu", "unit": "issue-cycles/s", "peak": VALU_PEAK_ISSUE_CYCLES_PER_S}
    out.update(profile_provenance(doc, VALU_PMC))
    out["source"] += f" [{case}]"
    for label, key, ms in (("B1_fdct", "k_jpeg_fdct_batch", j1_ms), ("F1_render_fdct", "k_jpeg_render_fdct", f1_ms),
                           ("B3_huffman", "k_jpeg_huff_thread", j3_ms)):
        k = next((k for k in pmc if key in k), None)
        if k is None or not ms:
            continue
        cnt, per = pmc[k]["counters"], pmc[k]["mcus_per_launch"]
        ipm = cnt["SQ_INSTS_VALU"] / per
        slow = sum(cnt.get(c, 0.0) for c in VALU_SLOW_COUNTERS) / per
        cyc = VALU_CYCLES * (ipm + slow)
        ach = cyc * mcus / (ms * 1e-3)
        out[label] = {"valu_instr_per_mcu": round(ipm, 1), "f64_and_transcendental_per_mcu": round(slow, 2),
                      "issue_cycles_per_mcu": round(cyc, 1), "achieved": round(ach, 1),
                      "frac": round(ach / VALU_PEAK_ISSUE_CYCLES_PER_S, 4), "avg_launch_ms": round(ms, 5)}
    return out


def jpeg_cpu_baseline(torch, name, src, chans, pt, be, q, seconds, threads):
    """Per request: CPU-restatement render (ISA-tuned build) + an IJG-grade JPEG encoder
    (PIL / libjpeg-turbo, SIMD islow FDCT + Huffman) at the Java ImageIO quality tables, 4:2:0 —
    the libjpeg lineage of the JDK writer behind compressToStream (ImageRegionRequestHandler.java:
    581).  Thread pool of nproc workers (ctypes and PIL's encoder release the GIL), and one thread."""
    import io
    import numpy as np
    from PIL import Image, features
    oracle_lib = _oracle()
    model = "greyscale" if len(chans) == 1 else "rgb"
    host = src[:4].cpu().numpy()
    if host.ndim == 4:
        tiles = [[np.ascontiguousarray(host[t, c]) for c in range(host.shape[1])] for t in range(host.shape[0])]
    else:
        tiles = [[np.ascontiguousarray(host[t])] for t in range(host.shape[0])]
    ql, qc = oracle_lib.quant_tables(q)
    qtables = [[int(v) for v in ql], [int(v) for v in qc]]

    def one(i):
        st, argb = oracle_lib.render(chans, tiles[i % len(tiles)], pt, TILE, TILE, model=model, big_endian=be,
                                     fast=True)
        # BGRA bytes -> RGB by PIL's C unpacker (ImageUtil.createBufferedImage drops alpha)
        img = Image.frombuffer("RGB", (TILE, TILE), argb, "raw", "BGRX", 0, 1)
        buf = io.BytesIO()
        img.save(buf, "JPEG", qtables=qtables, subsampling=2)
        return buf.tell()

    n, secs = _cpu_pool(one, seconds, threads)
    n1, secs1 = _cpu_pool(one, min(3.0, seconds / 2), 1)
    return {"value": round(n / secs, 3), "unit": "tiles/s", "cores": threads, "kind": "port",
            "single_thread": {"value": round(n1 / secs1, 3), "unit": "tiles/s", "cores": 1},
            "sample": f"{n} tiles ({name}: render + JPEG q={q}) in {secs:.2f} s on {threads} threads "
                      f"(render: oracle/omr_oracle.c {oracle_lib.FAST_BUILD}; JPEG: libjpeg-turbo "
                      f"{features.version('libjpeg_turbo')} via PIL)"}


SECTION_PREWARM_S = 0.2


def _timed(torch, ctx, step, steps, warmup):
    """Run prewarm + warmup + timed steps; returns (elapsed_s, {kind: avg_ms}).  Prewarm: the
    step back to back for SECTION_PREWARM_S (the GPU clocks drop while the CPU-baseline legs
    between sections keep it idle; the headline's --prewarm-ms).  The throughput
    pass runs with kernel timing off (per-launch HIP event records cost host and queue time that
    small per-request launches would otherwise carry); a second pass of the same steps collects
    the per-kernel averages from the context's HIP events."""
    t_end = time.perf_counter() + SECTION_PREWARM_S
    n = 0
    while time.perf_counter() < t_end:
        step()
        n += 1
        if n % 16 == 0:
            ctx.synchronize()
    for _ in range(warmup):
        step()
    ctx.synchronize()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    ctx.synchronize()
    el = time.perf_counter() - t0
    ctx.kernel_timings()
    ctx.enable_kernel_timing(True)
    for _ in range(steps):
        step()
    ctx.synchronize()
    ctx.enable_kernel_timing(False)
    tm = {}
    for ms, kind in ctx.kernel_timings():
        tm.setdefault(kind, []).append(ms)
    return el, {k: sum(v) / len(v) for k, v in tm.items()}


C3_WINDOWS, C3_WINDOW_S = 7, 0.05
SERVING_PASSES = 3     # timed passes of each serving leg (median): one pass is ~20-60 ms of requests
C3_SETS = 4            # distinct C3 request stack sets (96 MiB each) taken in turn


def _gated_burst_ms(torch, ctx, launch, n, gate_ms=30.0):
    """Average device time of `launch` over n back-to-back calls: the context stream is held by a
    spin kernel (torch.cuda._sleep) while the host queues all n, so no launch waits on the host and
    two events around the whole burst time only the kernels.  Per-launch HIP events on a ~17 us
    kernel read 1-3 us long (their own dispatch and completion signalling); around a
    burst of n launches that cost is paid once.  Returns None when torch has no _sleep."""
    sleep = getattr(torch.cuda, "_sleep", None)
    if sleep is None:
        return None
    s = ctx._ext_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    launch()                                                  # warm (tables, code objects)
    ctx.synchronize()
    with torch.cuda.stream(s):
        sleep(int(gate_ms * 1e-3 * 2.4e9))                    # >= gate_ms at <= 2.4 GHz
        e0.record(s)
    for _ in range(n):
        launch()
    e1.record(s)
    e1.synchronize()
    return e0.elapsed_time(e1) / n


def _windows(sync, step, n_windows, window_s):
    """Throughput of `step` over n_windows back-to-back windows of at least window_s each (steps
    issued back to back, one `sync` closing each window): the median window rate, and every
    window's.  Small per-request legs (C3: ~30-50 us each) measured over one short window swing
    with one host stall; the median of several >= 50 ms windows does not."""
    rates, total = [], 0
    sync()
    for _ in range(n_windows):
        t0 = time.perf_counter()
        n = 0
        while True:
            for _ in range(32):
                step()
            n += 32
            if time.perf_counter() - t0 >= window_s:
                break
        sync()
        el = time.perf_counter() - t0
        rates.append(n / el)
        total += n
    srt = sorted(rates)
    return {"median_per_s": round(srt[len(srt) // 2], 1), "min_per_s": round(srt[0], 1),
            "max_per_s": round(srt[-1], 1), "windows": len(rates), "requests": total}


def _cpu_pool(fn, seconds, threads):
    """fn(i) on a thread pool (ctypes releases the GIL): calibrate on one round, then time a
    bounded sample.  Returns (n, secs)."""
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(threads) as ex:
        t0 = time.perf_counter()
        list(ex.map(fn, range(threads)))
        first = time.perf_counter() - t0
        n = max(threads, int(threads * seconds / max(first, 1e-3)) // threads * threads)
        t0 = time.perf_counter()
        list(ex.map(fn, range(n)))
        return n, time.perf_counter() - t0


def c3_section(torch, ctx, steps, warmup, cpu_seconds, threads, with_cpu):
    """BASELINE configs[2] (C3): 3-channel uint16 512x512x64 Z-stack (big-endian, as ROMIO) ->
    max / mean intensity projection of every active channel -> composite of the projected full
    plane (ImageRegionRequestHandler.java:506-575): K1 (tables) + K3 (projection) + K2 (render);
    K3R (project + render fused) with OMR_K3R=1.
    One step = one render_image_region request with p=intmax|0:63 (or intmean)."""
    import numpy as np
    from omr import _lib
    from omr.context import make_bindings, make_qdef
    from omr.synthetic import c2_channels
    dev = torch.device("cuda", ctx.device)
    S, Z, C = 512, 64, 3
    g = torch.Generator(device=dev)
    g.manual_seed(20261015 + 3)
    # uniform uint16 values (every LUT entry, worst case for the window compares), stored big-endian.
    # C3_SETS distinct request stacks (3 x 32 MiB each) taken in turn: their 384 MiB exceed the
    # 256 MiB Infinity Cache, so every request reads its planes from HBM as a stream of distinct
    # requests does (round 5 re-read one 96 MiB set, partly a cache hit: its per-launch events read
    # 3 % faster than a rocprofv3 trace of the same kernel)
    def make_set():
        st = [torch.randint(0, 65536, (Z, S, S), dtype=torch.int32, device=dev, generator=g) for _ in range(C)]
        st = [(s & 0xFF) << 8 | (s >> 8) for s in st]                                   # -> BE bytes
        return [(s - 65536 * (s >= 32768).to(torch.int32)).to(torch.int16).contiguous() for s in st]
    sets = [make_set() for _ in range(C3_SETS)]
    stacks = sets[0]
    turn = [0]

    def next_set():
        turn[0] += 1
        return sets[turn[0] % C3_SETS]
    chans = c2_channels(C)
    qd = make_qdef("rgb")
    out = torch.empty((S, S), dtype=torch.int32, device=dev)
    binds = make_bindings(chans)   # marshalled once, as a Java caller would hold its Renderer state
    import omr
    ctx2 = omr.Context(ctx.device, torch_order=False)
    res = {}
    for name, alg, end in (("max", _lib.PROJECTION_MAX, Z - 1), ("mean", _lib.PROJECTION_MEAN, Z - 1)):
        def step():
            ctx.render_projected_device(qd, chans, next_set(), _lib.PIXELS_UINT16, S, S, Z, alg, 0, end, out,
                                        big_endian=True, bindings=binds)
        el, avg = _timed(torch, ctx, step, steps, warmup)
        one = _windows(ctx.synchronize, step, C3_WINDOWS, C3_WINDOW_S)
        # Two contexts (two HIP streams, as two Vert.x workers each holding one) taking alternate
        # requests: one request's K3 overlaps the other's launch gaps and small K1/K2 launches.
        outs = [out, torch.empty_like(out)]
        ctxs = [ctx, ctx2]
        k = [0]

        def step2():            # requests 2j and 2j + 1 (one per context) read stack set j
            i = k[0] & 1
            st = sets[(k[0] >> 1) % C3_SETS]
            k[0] += 1
            ctxs[i].render_projected_device(qd, chans, st, _lib.PIXELS_UINT16, S, S, Z, alg, 0, end, outs[i],
                                            big_endian=True, bindings=binds)

        def sync2():
            ctx.synchronize()
            ctx2.synchronize()
        for _ in range(2 * warmup):    # even: the last two requests read the same set
            step2()
        sync2()
        two = _windows(sync2, step2, C3_WINDOWS, C3_WINDOW_S)
        assert torch.equal(outs[0], outs[1]), "two-stream C3 renders differ"
        k3 = avg.get(3, float("nan"))          # per-launch HIP events: the kernel's duration (the frac)
        burst = None
        if os.environ.get("OMR_K3R", "0") in ("", "0"):
            # the glue's K3 (all three stacks in one launch), 200 launches back to back behind a gate
            outs3 = [torch.empty((S, S), dtype=torch.int16, device=dev) for _ in range(C)]

            def k3_launch():
                ctx.project_stacks_device(next_set(), _lib.PIXELS_UINT16, S, S, Z, alg, 0, end, outs3,
                                          big_endian_in=True)
            # back-to-back launches overlap one's tail with the next one's head: a throughput
            # figure, reported beside the roofline (which follows the kernel trace's duration)
            burst = _gated_burst_ms(torch, ctx, k3_launch, 200)
        used_z = Z if alg == _lib.PROJECTION_MAX else Z - 1
        if os.environ.get("OMR_K3R", "0") not in ("", "0"):
            # K3R (project + render fused): every used plane of the 3 stacks in, the ARGB plane out
            alg_bytes = C * used_z * S * S * 2 + S * S * 4
            kms = {"K3R_project_render": round(k3, 5)}
            kname = f"k_project_render<u16,BE,{name}> (K3R)"
        else:
            # K3 (all active channels in one launch): used planes in, one projected plane out each
            alg_bytes = C * (used_z * S * S * 2 + S * S * 2)
            kms = {"K3_project": round(k3, 5), "K3_project_gated_burst_per_launch": round(burst, 5) if burst else None,
                   "K2_render": round(avg.get(2, float("nan")), 5)}
            kname = f"k_project<u16,BE,{name}> (K3)"
        r = {"requests_per_s": one["median_per_s"], "ms_per_request": round(1e3 / one["median_per_s"], 4),
             "requests_per_s_two_streams": two["median_per_s"],
             "timing": {"one_stream": one, "two_streams": two,
                        "method": f"{C3_WINDOWS} back-to-back windows of >= {C3_WINDOW_S * 1e3:.0f} ms each "
                                  "(requests issued without a host sync, one sync per window); median window rate"},
             "kernel_ms": kms,
             "roofline": {"bound": "hbm", "kernel": kname,
                          "achieved": round(alg_bytes / (k3 * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBS,
                          "unit": "GB/s", "frac": round(alg_bytes / (k3 * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                          "algorithmic_bytes_per_launch": alg_bytes, "avg_launch_ms": round(k3, 5),
                          "timing": "per-launch HIP events around each launch on its stream (system fence "
                                    "off): the kernel duration a rocprofv3 trace reports",
                          "working_set": f"{C3_SETS} request stack sets x {C * Z * S * S * 2 >> 20} MiB in turn "
                                         "(beyond the 256 MiB Infinity Cache)"}}
        if os.environ.get("OMR_K3R", "0") in ("", "0"):
            tr = c3_trace_frac(0 if name == "max" else 1, alg_bytes)
            if tr:
                r["roofline"]["trace"] = tr
                r["roofline"]["trace_consistent_frac"] = tr["frac"]
        if burst:
            r["roofline"]["burst_throughput_frac"] = round(alg_bytes / (burst * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
            r["roofline"]["burst_timing"] = ("200 launches queued behind a spin kernel, two events around the "
                                             "burst: launch-to-launch throughput (tails overlap), not a duration")
        if with_cpu:
            try:
                oracle_lib = _oracle()
                host = [s.cpu().numpy().view(np.uint16) for s in stacks]

                def one(i):
                    planes = []
                    for c in range(C):
                        st, p = oracle_lib.project(host[c], _lib.PIXELS_UINT16, S, S, Z, alg, 0, end, be_in=True,
                                                   be_out=True, fast=True)
                        planes.append(p.view(np.uint16))
                    oracle_lib.render(chans, planes, _lib.PIXELS_UINT16, S, S, big_endian=True, fast=True)
                n, secs = _cpu_pool(one, cpu_seconds, threads)
                r["cpu_baseline"] = {"value": round(n / secs, 3), "unit": "requests/s", "cores": threads,
                                     "kind": "port",
                                     "sample": f"{n} C3 {name} requests (3x project 512x512x64 u16 + composite) "
                                               f"in {secs:.2f} s on {threads} threads (oracle/omr_oracle.c, "
                                               f"{oracle_lib.FAST_BUILD})"}
            except Exception as e:
                log(f"c3 cpu baseline failed: {e}")
        res[name] = r
    ctx2.close()
    return res


C3_TRACE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "r06", "all_sections_kernels.json")


def c3_trace_frac(alg, alg_bytes):
    """The C3 K3 roofline from the committed all-sections rocprofv3 trace (tools/gpu.sh trace ->
    tools/trace_kernels.py -> profiles/r06/all_sections_kernels.json): the median traced duration
    of the bench's K3 launches (k_project_v, this projection, three 512^2 x 64 stacks), beside the
    frac the bench's own per-launch events give."""
    try:
        with open(C3_TRACE) as fh:
            doc = json.load(fh)
    except (OSError, ValueError):
        return None
    rows = [r for r in doc.get("kernels", []) if f"k_project_v<unsigned short, true, false, {alg}," in r["kernel"]
            and r["grid_size"] == 393216]
    if not rows:
        return None
    r = max(rows, key=lambda r: r["launches"])
    out = profile_provenance(doc, C3_TRACE)
    out.update({"launches": r["launches"], "median_ns": r["median_ns"], "avg_ns": r["avg_ns"],
                "frac": round(alg_bytes / (r["median_ns"] * 1e-9) / 1e9 / HBM_PEAK_GBS, 4)})
    return out


def c5_section(torch, ctx, B, steps, warmup, cpu_seconds, threads, with_cpu):
    """BASELINE configs[4] (C5): 3-channel float32 1024^2 tiles, log (reverse) / poly k=0.5 /
    poly k=2 + .lut families, windows at p1/p99 (K2 eval mode: per-pixel double evaluation), plus
    render_shape_mask of a 1024x1024 bit mask (colour FF000080, flip hv)."""
    import numpy as np
    from omr import _lib
    from omr.context import make_bindings, make_qdef
    from omr.synthetic import c5_channels, c5_planes
    dev = torch.device("cuda", ctx.device)
    rng = np.random.default_rng(20261015 + 5)
    uniq = 4
    host = np.stack([np.stack(c5_planes(TILE, TILE, rng)) for _ in range(uniq)])
    chans = c5_channels(list(host[0]))      # p1/p99 windows; the x^0.5 window starts at >= 1.0
    be_host = host.astype(">f4")
    src = torch.from_numpy(np.ascontiguousarray(be_host).view(np.uint8)).to(dev)
    data = torch.empty((B, 3 * TILE * TILE * 4), dtype=torch.uint8, device=dev)
    for t in range(B):
        data[t].copy_(src.view(uniq, -1)[t % uniq])
    out = torch.empty((B, TILE, TILE), dtype=torch.int32, device=dev)
    qd = make_qdef("rgb")
    binds = make_bindings(chans)
    plane = TILE * TILE * 4

    def step():
        ctx.render_batch_strided_device(qd, chans, data, 3 * plane, plane, B, _lib.PIXELS_FLOAT, TILE, TILE, out,
                                        big_endian=True, bindings=binds)
    el, avg = _timed(torch, ctx, step, steps, warmup)
    k2 = avg.get(2, float("nan"))
    per_tile = 3 * plane + TILE * TILE * 4
    ach = per_tile * B / (k2 * 1e-3) / 1e9
    r = {"tiles_per_s": round(B * steps / el, 1), "ms_per_step": round(1e3 * el / steps, 4), "tiles_per_step": B,
         "roofline": {"bound": "hbm", "kernel": "k_render<f32,BE,3ch,eval> (K2)", "achieved": round(ach, 1),
                      "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
                      "algorithmic_bytes_per_launch": per_tile * B, "avg_launch_ms": round(k2, 5)}}
    if with_cpu:
        try:
            oracle_lib = _oracle()
            tiles = [[np.ascontiguousarray(be_host[t, c]) for c in range(3)] for t in range(uniq)]

            def one(i):
                oracle_lib.render(chans, tiles[i % uniq], _lib.PIXELS_FLOAT, TILE, TILE, big_endian=True, fast=True)
            n, secs = _cpu_pool(one, cpu_seconds, threads)
            r["cpu_baseline"] = {"value": round(n / secs, 3), "unit": "tiles/s", "cores": threads, "kind": "port",
                                 "sample": f"{n} C5 tiles (3ch f32 1024^2, log/poly/lut/reverse) in {secs:.2f} s "
                                           f"on {threads} threads (oracle/omr_oracle.c, {oracle_lib.FAST_BUILD})"}
        except Exception as e:
            log(f"c5 cpu baseline failed: {e}")
    # render_shape_mask: 1024x1024 mask of random ellipses, FF000080, flip hv (host API, p50).  A
    # 1024-wide mask with a flip is the reference's packed-buffer failure (404) by default, so the
    # leg runs the pixel flip (OMR_SEM_MASK_PIXEL_FLIP) it evidently intends.
    ctx.set_semantics(_lib.SEM_MASK_PIXEL_FLIP)
    yy, xx = np.mgrid[0:TILE, 0:TILE]
    m = np.zeros((TILE, TILE), bool)
    for _ in range(24):
        cy, cx, ry, rx = rng.uniform(0, TILE), rng.uniform(0, TILE), rng.uniform(10, 120), rng.uniform(10, 120)
        m |= ((yy - cy) / ry) ** 2 + ((xx - cx) / rx) ** 2 <= 1
    bits = np.packbits(m.reshape(-1)).tobytes()
    lat = []
    for i in range(23):
        t0 = time.perf_counter()
        png = ctx.render_shape_mask_png(bits, TILE, TILE, (255, 0, 0, 128), flip_h=True, flip_v=True)
        if i >= 3:
            lat.append(time.perf_counter() - t0)
    ctx.set_semantics(0)
    r["shape_mask_png"] = {"p50_ms": round(1e3 * float(np.median(lat)), 4), "png_bytes": len(png),
                           "size": "1024x1024 1-bit, flip hv", "semantics": "OMR_SEM_MASK_PIXEL_FLIP"}
    return r


def png_section(torch, ctx, data):
    """format=png (ImageRegionRequestHandler.java:583-600): one rendered C2 1024^2 tile -> device
    PNG (adaptive filters + dynamic-Huffman deflate, K5), p50 latency and size; PIL's zlib PNG
    writer on the host is timed beside it as a CPU reference point (ImageIO's writer cannot run
    here)."""
    import io
    import numpy as np
    from omr import _lib
    from omr.context import make_qdef
    from omr.synthetic import c2_channels
    out = torch.empty((TILE, TILE), dtype=torch.int32, device=data.device)
    ctx.render_packed_int_device(make_qdef("rgb"), c2_channels(CHANNELS), [data[0, c] for c in range(CHANNELS)],
                                 _lib.PIXELS_UINT16, TILE, TILE, out, big_endian=True)
    ctx.synchronize()
    lat = []
    for i in range(13):
        t0 = time.perf_counter()
        png = ctx.encode_png_device(out, TILE, TILE)
        if i >= 3:
            lat.append(time.perf_counter() - t0)
    res = {"p50_ms": round(1e3 * float(np.median(lat)), 4), "png_bytes": len(png),
           "raw_bytes": (3 * TILE + 1) * TILE, "ratio": round(len(png) / ((3 * TILE + 1) * TILE), 4),
           "single_tile_per_s": round(1.0 / float(np.median(lat)), 1)}
    # Batched (omr_encode_png_batch_device): the rendered C2 batch (all distinct tiles of `data`)
    # encoded at 64 and 256 tiles per call, one launch per stage, files packed in HBM.
    B = data.shape[0]
    argb = torch.empty((B, TILE, TILE), dtype=torch.int32, device=data.device)
    pb = TILE * TILE * 2
    ctx.render_batch_strided_device(make_qdef("rgb"), c2_channels(CHANNELS), data, CHANNELS * pb, pb, B,
                                    _lib.PIXELS_UINT16, TILE, TILE, argb, big_endian=True)
    cap = _lib.lib.omr_png_batch_max_bytes(TILE, TILE, 3, B)
    d_out = torch.empty(cap, dtype=torch.uint8, device=data.device)
    offs = torch.empty(B, dtype=torch.int64, device=data.device)
    lens = torch.empty(B, dtype=torch.int32, device=data.device)
    stat = torch.empty(B, dtype=torch.int32, device=data.device)
    ctx.synchronize()
    batched = {}
    raw = (3 * TILE + 1) * TILE                         # filtered stream bytes per tile
    for n in (64, 256):
        if n > B:
            continue
        def step():
            ctx.encode_png_batch_device(argb, n, TILE, TILE, d_out, offs, lens, stat)
        reps = max(4, 1024 // n)
        el, avg = _timed(torch, ctx, step, reps, 2)
        ln = lens[:n].cpu().numpy().astype(np.int64)
        assert int((stat[:n] != 0).sum().item()) == 0, "PNG batch status"
        files = int(ln.sum())
        ms = el * 1e3 / reps
        leg = {"tiles_per_s": round(n * reps / el, 1), "ms_per_call": round(ms, 4), "mean_png_bytes": int(ln.mean())}
        # Per-stage roofline from HIP events around each stage's launches (kinds 20-26,
        # omr_png.hip launch_png_batch; direct mode).  Algorithmic bytes per call: the filter reads
        # the ARGB tiles and writes the filtered streams; the parse and the encoder read the streams
        # (the encoder also writes the deflate stream into the files in place); P8 stores only the
        # bytes around the streams; CRC reads the files.  HBM-bound stages against 8 TB/s.
        stages = {20: ("filter (P1)", n * TILE * TILE * 4 + n * raw),
                  21: ("LZ77 parse + histograms (P2)", n * raw),
                  22: ("huffman tables + block offsets (P3, P3b)", 0),
                  23: ("encode (P4: codes from the parse traces, into the files)", n * raw + files),
                  24: ("meta + file offsets (P5b, P6)", 0),
                  25: ("fixup + bytes around the streams (P5, P8)", 0),
                  26: ("IDAT CRC (P9, P10)", files)}
        per = {}
        for k, (name, alg) in stages.items():
            if k not in avg:
                continue
            t = avg[k]
            e = {"stage": name, "avg_ms": round(t, 5)}
            if alg:
                gbs = alg / (t * 1e-3) / 1e9
                e.update({"algorithmic_bytes": alg, "achieved_gbs": round(gbs, 1),
                          "frac": round(gbs / HBM_PEAK_GBS, 4)})
            per[str(k)] = e
        alg_all = n * TILE * TILE * 4 + files
        stage_ms = sum(avg.get(k, 0.0) for k in stages)
        leg["roofline"] = {"bound": "hbm", "scope": "whole pipeline: ARGB tiles in + PNG files out per call",
                           "achieved": round(alg_all / (ms * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                           "frac": round(alg_all / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                           "algorithmic_bytes_per_call": alg_all, "sum_of_stage_ms": round(stage_ms, 5),
                           "stages": per}
        if n == 256:
            vr = png_valu_roofline(avg)
            if vr:
                leg["valu_roofline"] = vr
            mt = png_measured_traffic(alg_all)
            if mt:
                leg["roofline"]["measured_traffic"] = mt
        batched[f"tiles_per_call_{n}"] = leg
    # 256 per call on two contexts taking alternate batches (as the batcher's two dispatch lanes
    # do): one batch's latency-bound stages (P3: one workgroup per image; the small P5b/P6/P10
    # launches) overlap the other's filter / parse / encode
    if "tiles_per_call_256" in batched:
        import omr
        ctx2 = omr.Context(ctx.device, torch_order=False)
        try:
            n = 256
            bufs = [(d_out, offs, lens, stat),
                    (torch.empty(cap, dtype=torch.uint8, device=data.device),
                     torch.empty(B, dtype=torch.int64, device=data.device),
                     torch.empty(B, dtype=torch.int32, device=data.device),
                     torch.empty(B, dtype=torch.int32, device=data.device))]
            ctxs = [ctx, ctx2]
            reps = 8
            for k in range(4):
                ctxs[k & 1].encode_png_batch_device(argb, n, TILE, TILE, *bufs[k & 1])
            ctx.synchronize()
            ctx2.synchronize()
            t0 = time.perf_counter()
            for k in range(2 * reps):
                ctxs[k & 1].encode_png_batch_device(argb, n, TILE, TILE, *bufs[k & 1])
            ctx.synchronize()
            ctx2.synchronize()
            el2 = time.perf_counter() - t0
            ok = all(int((b[3][:n] != 0).sum().item()) == 0 for b in bufs)
            assert ok, "PNG batch status (two contexts)"
            assert torch.equal(bufs[0][2][:n], bufs[1][2][:n]), "two contexts' files differ in length"
            batched["tiles_per_call_256"]["tiles_per_s_two_streams"] = round(2 * reps * n / el2, 1)
        finally:
            ctx2.close()
    res["batched"] = batched
    if "tiles_per_call_256" in batched:
        res["batched_vs_single"] = round(batched["tiles_per_call_256"]["tiles_per_s"] / res["single_tile_per_s"], 2)
    try:
        from PIL import Image
        a = out.cpu().numpy().view(np.uint32)
        rgb = np.stack([(a >> 16) & 0xFF, (a >> 8) & 0xFF, a & 0xFF], -1).astype(np.uint8)
        im = Image.fromarray(rgb)
        t = []
        for i in range(4):
            b = io.BytesIO()
            t0 = time.perf_counter()
            im.save(b, format="PNG")
            t.append(time.perf_counter() - t0)
        res["cpu_pil_zlib"] = {"p50_ms": round(1e3 * float(np.median(t)), 3), "png_bytes": len(b.getvalue()),
                               "cores": 1}
    except Exception as e:   # PIL is a reference point only
        log(f"PIL PNG reference failed: {e}")
    return res


def serving_section(torch, ctx, pb, qd, chans, binds, grid, n_req=256, clients=8, pool_devices=None):
    """render_image_region JPEG tiles (q 0.9) served to concurrent clients from the ROMIO file:
    one request at a time on one context (the reference's shape: a Renderer per request) vs the
    batcher (omr_batcher_*: the dispatcher coalesces what the 8 client threads submit, 8 tiles
    per client at a time like a viewer filling a screen, into GPU batches).  Requests walk the 16 distinct tiles, so identical tiles in flight together are
    rendered once."""
    import threading
    import numpy as np
    from omr import Batcher, Pool
    reqs = [(0, 0, (i % grid) * TILE, ((i // grid) % grid) * TILE) for i in range(n_req)]
    dev = torch.empty((TILE, TILE), dtype=torch.int32, device="cuda")
    lat = []
    for warm in (True, False):       # a warm-up pass first (staging buffers, page cache, clocks)
        lat.clear()
        t0 = time.perf_counter()
        for r in reqs[:64]:
            a = time.perf_counter()
            ctx.render_pixel_buffer_tiles(qd, chans, pb, [r], TILE, TILE, out=dev, bindings=binds)
            ctx.encode_jpeg_device(dev, TILE, TILE, 0.9)
            lat.append(time.perf_counter() - a)
        el = time.perf_counter() - t0
    res = {"requests": n_req, "clients": clients,
           "one_at_a_time": {"tiles_per_s": round(64 / el, 1), "p50_ms": round(1e3 * float(np.median(lat)), 3)}}
    res["interactive"] = serving_interactive(torch, ctx, pb, qd, chans, binds, reqs, clients, res["one_at_a_time"])
    legs = [("batcher_max64_wait1000us", lambda: Batcher(ctx.device, max_batch=64, max_wait_us=1000))]
    if pool_devices:
        # omr_pool: one batcher per entry of pool_devices (the node's GPUs; on a one-GPU box the
        # entries share the card), each job to the least-queued one
        legs.append((f"pool_{len(pool_devices)}x_max64_wait1000us",
                     lambda: Pool(pool_devices, max_batch=64, max_wait_us=1000)))
    for name, make in legs:
        lats = []
        with make() as b:
            def client(k):          # a viewer asks for a screenful (8 tiles) at a time
                mine = list(range(k, n_req, clients))
                for s0 in range(0, len(mine), 8):
                    a = time.perf_counter()
                    ts = [b.submit(pb, qd, chans, *reqs[i], TILE, TILE, quality=0.9, bindings=binds)
                          for i in mine[s0:s0 + 8]]
                    for t in ts:
                        b.wait(t)
                        lats.append(time.perf_counter() - a)
            els = []
            for p in range(1 + SERVING_PASSES):    # a warm-up pass, then timed passes (median)
                if p == 1:
                    lats.clear()
                ths = [threading.Thread(target=client, args=(k,)) for k in range(clients)]
                t0 = time.perf_counter()
                for t in ths:
                    t.start()
                for t in ths:
                    t.join()
                if p:
                    els.append(time.perf_counter() - t0)
            el = float(np.median(els))
            st = b.stats()
        if isinstance(st, list):
            leg = {"devices": list(pool_devices), "jobs_per_device": [s["jobs"] for s in st],
                   "rendered": sum(s["rendered"] for s in st), "dedup": sum(s["dedup"] for s in st),
                   "rounds": sum(s["batches"] for s in st)}
        else:
            leg = {"rendered": st["rendered"], "dedup": st["dedup"], "rounds": st["batches"]}
        # stats cover the warm-up pass too: rendered / dedup per served request, and the rate of
        # distinct renders (what the GPU did) apart from requests answered by a sibling's render
        passes = 1 + SERVING_PASSES
        leg["rendered_per_s"] = round(leg["rendered"] / passes / el, 1)
        leg["dedup_share"] = round(leg["dedup"] / max(1, leg["rendered"] + leg["dedup"]), 3)
        res[name] = {"tiles_per_s": round(n_req / el, 1), "p50_ms": round(1e3 * float(np.median(lats)), 3), **leg}
    return res


def serving_interactive(torch, ctx, pb, qd, chans, binds, reqs, clients, single, per_client=32, passes=3):
    """The same tiles with ONE request in flight per client (a viewer asking for the next tile only
    when the last has arrived): `clients` threads each on its own context rendering its requests
    directly (the reference's shape: every worker renders its own request) against the batcher
    taking them all.  With k requests outstanding a request waits behind the others' PCIe
    transfers (8 MiB per tile in), so p50 grows with k whatever the dispatch; the leg reports both
    p50s beside the one-at-a-time p50 of a single client."""
    import threading
    import numpy as np
    import omr
    from omr import Batcher
    out = {"clients": clients, "requests_per_client": per_client, "in_flight_per_client": 1}
    ctxs = [omr.Context(ctx.device, torch_order=False) for _ in range(clients)]
    devs = [torch.empty((TILE, TILE), dtype=torch.int32, device="cuda") for _ in range(clients)]
    torch.cuda.synchronize()

    def run(job):
        lats = []

        def client(k):
            mine = [reqs[(k + clients * j) % len(reqs)] for j in range(per_client)]
            for r in mine:
                a = time.perf_counter()
                job(k, r)
                lats.append(time.perf_counter() - a)
        rates = []
        for p in range(passes + 1):        # a warm-up pass, then `passes` timed ones (median rate)
            if p == 1:
                lats.clear()
            ths = [threading.Thread(target=client, args=(k,)) for k in range(clients)]
            t0 = time.perf_counter()
            for t in ths:
                t.start()
            for t in ths:
                t.join()
            if p:
                rates.append(clients * per_client / (time.perf_counter() - t0))
        return {"tiles_per_s": round(float(np.median(rates)), 1), "p50_ms": round(1e3 * float(np.median(lats)), 3),
                "p90_ms": round(1e3 * float(np.percentile(lats, 90)), 3), "passes": passes,
                "requests_per_pass": clients * per_client}

    def direct(k, r):
        ctxs[k].render_pixel_buffer_tiles(qd, chans, pb, [r], TILE, TILE, out=devs[k], bindings=binds)
        ctxs[k].encode_jpeg_device(devs[k], TILE, TILE, 0.9)
    try:
        out["independent_contexts"] = run(direct)
        with Batcher(ctx.device, max_batch=64, max_wait_us=1000) as b:
            out["batcher_max64_wait1000us"] = run(
                lambda k, r: b.wait(b.submit(pb, qd, chans, *r, TILE, TILE, quality=0.9, bindings=binds)))
            st = b.stats()
            out["batcher_max64_wait1000us"].update({"rounds": st["batches"], "rendered": st["rendered"],
                                                    "dedup": st["dedup"]})
    finally:
        for c in ctxs:
            c.close()
    for k in ("independent_contexts", "batcher_max64_wait1000us"):
        out[k]["p50_vs_single_client"] = round(out[k]["p50_ms"] / single["p50_ms"], 2)
    return out


def _serve(b, submit_fns, clients):
    """Run submit_fns (each a callable returning a ticket) from `clients` threads, 8 in flight per
    client; returns (elapsed_s, per-request latencies)."""
    import threading
    lats = []

    def client(k):
        mine = submit_fns[k::clients]
        for s0 in range(0, len(mine), 8):
            a = time.perf_counter()
            ts = [f() for f in mine[s0:s0 + 8]]
            for t in ts:
                b.wait(t)
                lats.append(time.perf_counter() - a)
    ths = [threading.Thread(target=client, args=(k,)) for k in range(clients)]
    t0 = time.perf_counter()
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    return time.perf_counter() - t0, lats


def serving_projection_and_masks(torch, ctx, clients=8):
    """Serving legs for the other two request kinds the batcher now takes:
    - p=intmax|intmean requests (ImageRegionRequestHandler.java:506-558) on a C3-shaped image
      (3 x 512x512x64 u16 ROMIO stacks, 2 timepoints), JPEG out: 64 requests, all distinct
      (t x algorithm x z range), through the batcher with its HBM stack cache, then the same
      requests again (the cache warm: settings / range changes on an open image) -- and with the
      cache disabled (every request uploads its 96 MiB of stacks);
    - render_shape_mask (ShapeMaskRequestHandler.java:165-207): 1024^2 masks of random ellipses,
      colours and flips, 256 requests over 32 distinct masks, batched PNG vs one call at a time."""
    import tempfile
    import numpy as np
    from omr import Batcher, PixelBuffer, _lib, write_romio
    from omr.context import make_bindings, make_qdef
    from omr.synthetic import c2_channels
    res = {}
    S, Z, C, T = 512, 64, 3, 2
    rng = np.random.default_rng(33)
    img = rng.integers(0, 65536, (T, C, Z, S, S), dtype=np.uint16)
    d = "/dev/shm" if os.path.isdir("/dev/shm") else None
    fd, path = tempfile.mkstemp(prefix="omr_romio_z_", dir=d)
    os.close(fd)
    try:
        write_romio(path, img, _lib.PIXELS_UINT16)
        del img
        pb = PixelBuffer(path, S, S, Z, C, T, _lib.PIXELS_UINT16)
        qd, chans = make_qdef("rgb"), c2_channels(C)
        binds = make_bindings(chans)
        specs = [(t, p, z0) for t in range(T) for p in ("intmax", "intmean") for z0 in range(16)]   # 64 distinct
        proj = {"requests": len(specs), "clients": clients, "stack_bytes_per_request": C * Z * S * S * 2}
        for cache_mb, label in ((4096, "stack_cache"), (0, "no_stack_cache")):
            with Batcher(ctx.device, max_batch=64, max_wait_us=1000) as b:
                b.set_stack_cache(cache_mb << 20)
                fns = [(lambda t=t, p=p, z0=z0: b.submit(pb, qd, chans, 0, t, 0, 0, S, S, quality=0.9, bindings=binds,
                                                         projection=p, projection_start=z0, projection_end=Z - 1))
                       for t, p, z0 in specs]
                cold, _ = _serve(b, fns, clients)
                warm, lats = _serve(b, fns, clients)
                st, sc = b.stats(), b.stack_cache_stats()
            proj[label] = {"cold_requests_per_s": round(len(specs) / cold, 1),
                           "warm_requests_per_s": round(len(specs) / warm, 1),
                           "warm_p50_ms": round(1e3 * float(np.median(lats)), 3),
                           "rendered": st["rendered"], "dedup": st["dedup"], "stack_cache": sc}
        res["projection"] = proj
        pb.close()
    finally:
        os.unlink(path)
    # shape masks
    W = H = TILE
    yy, xx = np.mgrid[0:H, 0:W]
    masks = []
    for k in range(32):
        m = np.zeros((H, W), bool)
        for _ in range(12):
            cy, cx, ry, rx = rng.uniform(0, H), rng.uniform(0, W), rng.uniform(10, 150), rng.uniform(10, 150)
            m |= ((yy - cy) / ry) ** 2 + ((xx - cx) / rx) ** 2 <= 1
        masks.append((np.packbits(m.reshape(-1)).tobytes(), W, H,
                      tuple(int(v) for v in rng.integers(0, 256, 4)), bool(k & 1), bool(k & 2)))
    ctx.set_semantics(_lib.SEM_MASK_PIXEL_FLIP)     # 1024-wide + flip: the pixel flip the reference intends
    t0 = time.perf_counter()
    for mk in masks:
        ctx.render_shape_mask_png(*mk)
    one = time.perf_counter() - t0
    ctx.set_semantics(0)
    n_req = 256
    with Batcher(ctx.device, max_batch=64, max_wait_us=1000) as b:
        b.set_semantics(_lib.SEM_MASK_PIXEL_FLIP)
        fns = [(lambda mk=masks[i % len(masks)]: b.submit_mask(*mk)) for i in range(n_req)]
        _serve(b, fns, clients)
        el, lats = _serve(b, fns, clients)
        st = b.stats()
    res["shape_mask"] = {"one_at_a_time_per_s": round(len(masks) / one, 1), "requests": n_req,
                         "distinct_masks": len(masks), "batcher_requests_per_s": round(n_req / el, 1),
                         "batcher_p50_ms": round(1e3 * float(np.median(lats)), 3),
                         "rendered": st["rendered"], "dedup": st["dedup"],
                         "rendered_per_s": round(st["rendered"] / 2 / el, 1)}
    return res


def host_fed_section(torch, ctx, uniq, n_req, cpu_seconds, threads, with_cpu, pool_devices=None):
    """The step before the path: C2 tiles read from a ROMIO repository
    file (big-endian XYZCT planes, as pixelsService.getPixelBuffer opens, ImageRegionRequestHandler
    .java:302-309) by omr_render_pixel_buffer_tiles: pread into pinned staging, H2D on a copy
    stream, K1+K2, ARGB back to the host (pinned or pageable) or kept in HBM and JPEG-encoded
    there (only the JPEG files cross PCIe).  The file is a 4096x4096 4-channel uint16 image
    (128 MiB, page-cache resident after writing); requests walk its 16 tiles repeatedly."""
    import tempfile
    import numpy as np
    from omr import PixelBuffer, _lib, write_romio
    from omr.context import make_bindings, make_qdef
    from omr.synthetic import c2_channels
    host = uniq.cpu().numpy().view(np.uint16).byteswap()      # native values of the BE tiles
    grid = 4
    img = np.empty((1, CHANNELS, 1, grid * TILE, grid * TILE), dtype=np.uint16)
    for ty in range(grid):
        for tx in range(grid):
            img[0, :, 0, ty * TILE:(ty + 1) * TILE, tx * TILE:(tx + 1) * TILE] = host[(ty * grid + tx) % host.shape[0]]
    d = "/dev/shm" if os.path.isdir("/dev/shm") else None
    fd, path = tempfile.mkstemp(prefix="omr_romio_", dir=d)
    os.close(fd)
    res = {"file": f"4096x4096x4ch uint16 ROMIO ({img.nbytes >> 20} MiB, {'tmpfs' if d else 'tmp'})",
           "tiles_per_call": n_req, "pcie_bytes_per_tile_in": CHANNELS * TILE * TILE * 2}
    try:
        write_romio(path, img, _lib.PIXELS_UINT16)
        qd = make_qdef("rgb")
        chans = c2_channels(CHANNELS)
        binds = make_bindings(chans)
        reqs = [(0, 0, (i % grid) * TILE, ((i // grid) % grid) * TILE) for i in range(n_req)]
        pb = PixelBuffer(path, grid * TILE, grid * TILE, 1, CHANNELS, 1, _lib.PIXELS_UINT16)
        dev_out = torch.empty((n_req, TILE, TILE), dtype=torch.int32, device=uniq.device)
        pageable = np.empty((n_req, TILE, TILE), dtype=np.uint32)
        nbytes = n_req * TILE * TILE * 4
        pin = _lib.lib.omr_pinned_alloc(ctx.h, nbytes)
        import ctypes
        pinned = np.ctypeslib.as_array((ctypes.c_uint32 * (n_req * TILE * TILE)).from_address(pin)).reshape(
            n_req, TILE, TILE)
        jpeg_cap = n_req * (TILE * TILE * 3)
        d_jpg = torch.empty(jpeg_cap, dtype=torch.uint8, device=uniq.device)
        offs = torch.empty(n_req, dtype=torch.int64, device=uniq.device)
        lens = torch.empty(n_req, dtype=torch.int32, device=uniq.device)
        stat = torch.empty(n_req, dtype=torch.int32, device=uniq.device)

        def to_jpeg():
            ctx.render_pixel_buffer_tiles(qd, chans, pb, reqs, TILE, TILE, out=dev_out, bindings=binds)
            ctx.encode_jpeg_batch_device(dev_out, n_req, TILE, TILE, 0.9, d_jpg, offs, lens, stat)
            ln = lens.cpu()
            end = int((offs.cpu() + ln.to(torch.int64)).max())
            return d_jpg[:end].cpu()
        modes = {
            "device_out": lambda: ctx.render_pixel_buffer_tiles(qd, chans, pb, reqs, TILE, TILE, out=dev_out,
                                                                bindings=binds),
            "host_pinned_out": lambda: ctx.render_pixel_buffer_tiles(qd, chans, pb, reqs, TILE, TILE, out=pinned,
                                                                     bindings=binds),
            "host_pageable_out": lambda: ctx.render_pixel_buffer_tiles(qd, chans, pb, reqs, TILE, TILE,
                                                                       out=pageable, bindings=binds),
            "to_jpeg_host": to_jpeg,
            # the fallback when the driver refuses to register the file mapping: reader threads
            # memcpy rows into pinned slots (host-memcpy-bound on the box's CPU quota)
            "device_out_staged_fallback": None,
        }
        # the same device_out leg on a context whose pixel-buffer pipeline splits the tile copies
        # over two DMA queues (OMR_PIXBUF_COPY_STREAMS=2, read when its pipeline is created)
        import omr
        os.environ["OMR_PIXBUF_COPY_STREAMS"] = "2"
        ctx2 = omr.Context(ctx.device, torch_order=False)
        del os.environ["OMR_PIXBUF_COPY_STREAMS"]
        modes["device_out_2_copy_queues"] = lambda: ctx2.render_pixel_buffer_tiles(qd, chans, pb, reqs, TILE, TILE,
                                                                                   out=dev_out, bindings=binds)
        # and on one that copies each tile-channel plane as its own 2-D rect (OMR_PIXBUF_BANDS=0)
        # instead of one row band per plane for the tiles that share it (the default)
        os.environ["OMR_PIXBUF_BANDS"] = "0"
        ctx3 = omr.Context(ctx.device, torch_order=False)
        del os.environ["OMR_PIXBUF_BANDS"]
        modes["device_out_tile_rects"] = lambda: ctx3.render_pixel_buffer_tiles(qd, chans, pb, reqs, TILE, TILE,
                                                                                out=dev_out, bindings=binds)
        for name, fn in modes.items():
            if fn is None:          # reader threads -> pinned staging instead of DMA from the mapping
                _lib.lib.omr_ctx_set_pixel_buffer_dma(ctx.h, 0)
                fn = modes["device_out"]
            fn()
            ctx.synchronize()
            reps = 0                  # calls over >= 0.5 s (three calls read 10-15 % low on the first leg)
            t0 = time.perf_counter()
            while reps < 3 or time.perf_counter() - t0 < 0.5:
                fn()
                reps += 1
            ctx.synchronize()
            el = time.perf_counter() - t0
            res[name] = {"tiles_per_s": round(n_req * reps / el, 1), "ms_per_tile": round(1e3 * el / (n_req * reps), 4)}
        _lib.lib.omr_ctx_set_pixel_buffer_dma(ctx.h, 1)
        _lib.lib.omr_pinned_free(ctx.h, pin)
        ctx2.close()
        ctx3.close()
        res["pcie_probe"] = pcie_probe(torch, uniq.device)
        ceil = max(v["gbs"] for v in res["pcie_probe"].values() if isinstance(v, dict))
        best = max(res[k]["tiles_per_s"] for k in ("device_out", "device_out_2_copy_queues", "device_out_tile_rects"))
        res["device_out_h2d_gbs"] = round(best * res["pcie_bytes_per_tile_in"] / 1e9, 2)
        res["device_out_vs_pcie_probe"] = round(res["device_out_h2d_gbs"] / ceil, 3)
        res["serving"] = serving_section(torch, ctx, pb, qd, chans, binds, grid, pool_devices=pool_devices)
        pb.close()
        res["serving"].update(serving_projection_and_masks(torch, ctx))
    finally:
        os.unlink(path)
    return res


def pcie_probe(torch, device, mib=512):
    """The box's host -> HBM ceiling: pinned host memory copied to the device with hipMemcpyAsync
    (torch's copy_) in one contiguous transfer, and split over two streams (two DMA queues), timed
    with events after a warm-up copy.  The host-fed legs are judged against this."""
    n = mib << 20
    host = torch.empty(n, dtype=torch.uint8).pin_memory()
    dev = torch.empty(n, dtype=torch.uint8, device=device)
    res = {"bytes": n}
    streams = [torch.cuda.Stream(device=device), torch.cuda.Stream(device=device)]
    for name, k in (("one_stream", 1), ("two_streams", 2)):
        part = n // k
        for rep in range(2):                          # warm, then timed
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(k):
                with torch.cuda.stream(streams[i]):
                    dev[i * part:(i + 1) * part].copy_(host[i * part:(i + 1) * part], non_blocking=True)
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
        res[name] = {"gbs": round(n / el / 1e9, 2)}
    return res


def _get(d, *keys):
    for k in keys:
        if not isinstance(d, dict) or k not in d:
            return None
        d = d[k]
    return d


def sections_summary(line):
    """The headline figure of every section, as the LAST key of the JSON line: a driver record that
    keeps only the line's tail still shows them (the detail, with its sources, is earlier in the
    line).  Fracs are HBM (or VALU-issue) fractions of peak; ms are per-launch averages."""
    s = {"c2_render": {"tiles_per_s": line.get("value"), "hbm_frac": _get(line, "roofline", "frac"),
                       "k2_avg_ms": _get(line, "roofline", "avg_launch_ms"),
                       "traffic_ratio": (round(line["roofline"]["traffic"] / line["roofline"]["algorithmic_bytes_per_launch"], 4)
                                         if _get(line, "roofline", "traffic") else None)}}
    for case in ("c2_u16_4ch_rgb_to_jpeg", "c1_u8_grey_to_jpeg"):
        j = _get(line, "jpeg", case)
        if j:
            s["jpeg_" + case.split("_")[0]] = {
                "fused_tiles_per_s": _get(j, "fused", "tiles_per_s"), "unfused_tiles_per_s": j.get("tiles_per_s"),
                "f1_ms": _get(j, "fused", "kernel_ms", "F1_render_fdct"),
                "fused_total_ms": _get(j, "fused", "kernel_ms", "jpeg_total"),
                "f1_valu_frac": _get(j, "valu_roofline", "F1_render_fdct", "frac"),
                "traffic_ratio": _get(j, "valu_roofline", "measured_traffic", "ratio"),
                "byte_identical_to_unfused": _get(j, "fused", "byte_identical_to_unfused")}
    p = _get(line, "png", "batched", "tiles_per_call_256")
    if p:
        s["png_batched_256"] = {"tiles_per_s": p.get("tiles_per_s"), "ms_per_call": p.get("ms_per_call"),
                                "tiles_per_s_two_streams": p.get("tiles_per_s_two_streams"),
                                "hbm_frac": _get(p, "roofline", "frac"),
                                "traffic_ratio": _get(p, "roofline", "measured_traffic", "ratio")}
    for alg in ("max", "mean"):
        c = _get(line, "c3_projection", alg)
        if c:
            s["c3_" + alg] = {"hbm_frac": _get(c, "roofline", "frac"), "k3_avg_ms": _get(c, "roofline", "avg_launch_ms"),
                              "k3_trace_frac": _get(c, "roofline", "trace_consistent_frac"),
                              "requests_per_s": c.get("requests_per_s")}
    c5 = line.get("c5_float")
    if c5:
        s["c5_float"] = {"hbm_frac": _get(c5, "roofline", "frac"), "k2_avg_ms": _get(c5, "roofline", "avg_launch_ms"),
                         "tiles_per_s": c5.get("tiles_per_s")}
    h = line.get("host_fed")
    if h:
        s["host_fed"] = {"tiles_per_s": _get(h, "device_out", "tiles_per_s"),
                         "vs_pcie_probe": h.get("device_out_vs_pcie_probe")}
        it = _get(h, "serving", "interactive")
        if it:
            bk = next((k for k in it if k.startswith("batcher")), None)
            s["serving_one_in_flight"] = {
                "batcher_tiles_per_s": _get(it, bk, "tiles_per_s"), "batcher_p50_ms": _get(it, bk, "p50_ms"),
                "independent_tiles_per_s": _get(it, "independent_contexts", "tiles_per_s"),
                "independent_p50_ms": _get(it, "independent_contexts", "p50_ms")}
    lat = line.get("p50_tile_latency_ms")
    if lat:
        s["p50_ms"] = {"render_c_abi": _get(lat, "native_c_abi", "render_device_resident", "p50_ms"),
                       "render_jpeg_c_abi": _get(lat, "native_c_abi", "render_jpeg_one_call", "p50_ms")}
    if line.get("cpu_baseline"):
        s["cpu_baseline_tiles_per_s"] = line["cpu_baseline"].get("value")
        if line.get("value") and line["cpu_baseline"].get("value"):
            s["gpu_vs_cpu"] = round(line["value"] / line["cpu_baseline"]["value"], 1)
    return s


def spawn_ranks(n):
    """`bench.py --gpus N` without a launcher: start N rank processes (RANK/LOCAL_RANK/
    WORLD_SIZE/MASTER_* as torch.distributed.run sets them) and wait for them.  Called before
    this process touches the GPU (it never imports torch); only rank 0 prints the JSON line.
    Returns the exit code (first failing rank's, after the others are stopped)."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    import threading
    procs, pumps = [], []

    def pump(stream):       # the JSON line to stdout; anything else a rank prints (gloo banners) to stderr
        for line in iter(stream.readline, ""):
            (sys.stdout if line.startswith("{") else sys.stderr).write(line)
            (sys.stdout if line.startswith("{") else sys.stderr).flush()
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        p = subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__)] + sys.argv[1:], env=env,
                             stdout=subprocess.PIPE, text=True)
        procs.append(p)
        pumps.append(threading.Thread(target=pump, args=(p.stdout,), daemon=True))
        pumps[-1].start()
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            r = p.poll()
            if r is None:
                continue
            live.remove(p)
            if r != 0 and rc == 0:
                rc = r
                for q in live:          # a rank failed: stop the others (our own children)
                    q.terminate()
        time.sleep(0.05)
    for t in pumps:
        t.join(timeout=5)
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=256, help="tiles per GPU per step (weak scaling)")
    ap.add_argument("--total-tiles", type=int, default=0,
                    help="C4 mode: a fixed node-wide batch (e.g. 4096) sharded contiguously across "
                         "ranks (omr/shard.py; strong scaling); overrides --batch")
    ap.add_argument("--unique", type=int, default=8, help="distinct synthetic tiles per GPU")
    ap.add_argument("--addr", choices=["strided", "table"], default="strided",
                    help="batch descriptor: regular [tile][channel] layout or device pointer table")
    ap.add_argument("--cpu-seconds", type=float, default=8.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-jpeg", action="store_true", help="skip the render->JPEG batch section")
    ap.add_argument("--jpeg-batch", type=int, default=256, help="tiles per JPEG step (the headline step size)")
    ap.add_argument("--jpeg-steps", type=int, default=40)
    ap.add_argument("--no-configs", action="store_true",
                    help="skip the C3 (projection) and C5 (float32 families, shape mask) sections")
    ap.add_argument("--no-latency", action="store_true",
                    help="skip the single-tile latency probe (profiling runs: batch launches only)")
    ap.add_argument("--pool", type=int, default=0,
                    help="batchers of the serving-pool leg (omr_pool over cuda:i %% visible GPUs); "
                         "0 = one per visible GPU, at least 2")
    ap.add_argument("--prewarm-ms", type=float, default=300.0,
                    help="untimed device warm-up before the W warm-up steps: the first ~25 K2 launches "
                         "after idle run 0.77 -> 0.60 ms while the GPU clocks ramp (profiles/r02/"
                         "k2_series_*.json); 0 disables")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    import torch
    n_dev = torch.cuda.device_count()
    if n_dev < 1:
        raise SystemExit("bench.py: no GPU visible")
    dev_index = local_rank % n_dev          # more ranks than GPUs (a rehearsal): ranks share cards
    torch.cuda.set_device(dev_index)
    device = torch.device("cuda", dev_index)
    dist = None
    backend = None
    if world > 1:
        import torch.distributed as dist
        # RCCL needs one rank per GPU; ranks sharing a card meet over gloo (the only traffic is
        # the timing barrier and one max-reduction: no collective touches pixel data)
        backend = "nccl" if local_world <= n_dev else "gloo"
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group("gloo")

    import omr
    from omr import _lib
    from omr.context import make_bindings, make_qdef
    from omr.synthetic import c2_channels

    ctx = omr.Context(dev_index, torch_order=False)
    qdef = make_qdef("rgb")
    chans = c2_channels(CHANNELS)
    bindings = make_bindings(chans)
    from omr.shard import ShardPlan
    if args.total_tiles:
        plan = ShardPlan(args.total_tiles, world, rank)
        B = plan.count
    else:
        B = args.batch
    data, uniq, table = build_batch(torch, B, min(args.unique, B), device)
    out = torch.empty((B, TILE, TILE), dtype=torch.int32, device=device)

    plane_bytes = TILE * TILE * 2

    def step():
        if args.addr == "strided":
            ctx.render_batch_strided_device(qdef, chans, data, CHANNELS * plane_bytes, plane_bytes, B,
                                            _lib.PIXELS_UINT16, TILE, TILE, out, big_endian=True,
                                            bindings=bindings)
        else:
            ctx.render_batch_device(qdef, chans, table, B, _lib.PIXELS_UINT16, TILE, TILE, out,
                                    big_endian=True, bindings=bindings)

    def barrier():
        if dist:
            dist.barrier()

    # Device warm-up: the GPU leaves its idle clock state over the first ~15 ms of load (K2
    # launches after idle: 0.77, 0.74, 0.72, ... 0.60 ms, then 0.55 sustained; tools/k2_series.py).
    # A serving node under load runs at the sustained clocks, so the bench reaches them first:
    # back-to-back steps for --prewarm-ms, untimed, then the W warm-up steps, then the K timed steps.
    n_pre = 0
    if args.prewarm_ms > 0:
        t_end = time.perf_counter() + args.prewarm_ms / 1e3
        while time.perf_counter() < t_end:
            step()
            n_pre += 1
            if n_pre % 4 == 0:
                ctx.synchronize()
        ctx.synchronize()
    for _ in range(args.warmup):
        step()
    ctx.synchronize()

    # Timed region: K steps, kernel timing OFF (no per-launch event records).  Two HIP events on
    # the context's stream bracket the region as a device-side cross-check of the wall clock.
    ext = torch.cuda.ExternalStream(ctx.stream, device=device)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record(ext)
    for _ in range(args.steps):
        step()
    ev1.record(ext)
    ctx.synchronize()
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    region_ms = ev0.elapsed_time(ev1)

    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=device if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # Second pass, same K steps, kernel timing ON: per-launch K2 durations (HIP events around
    # each K2 launch on its stream) for the roofline.
    ctx.kernel_timings()
    ctx.enable_kernel_timing(True)
    for _ in range(args.steps):
        step()
    ctx.synchronize()
    ctx.enable_kernel_timing(False)
    k2 = sorted(ms for ms, kind in ctx.kernel_timings() if kind == 2)

    tiles = (args.total_tiles or world * B) * args.steps
    value = tiles / elapsed
    k2_ms = sum(k2) / len(k2) if k2 else float("nan")
    achieved = BYTES_PER_TILE * B / (k2_ms * 1e-3) / 1e9
    traffic = pmc_traffic(B)

    extra = {}
    if rank == 0 and world == 1:
        threads, _, _ = host_cores()
        if not args.no_latency:
            extra["p50_tile_latency_ms"] = latencies(torch, omr, ctx, qdef, chans, data)
        if not args.no_jpeg:
            extra["jpeg"] = jpeg_section(torch, ctx, data, min(args.jpeg_batch, B), args.jpeg_steps,
                                         2, args.cpu_seconds / 2, threads, not args.no_cpu_baseline)
        if not args.no_configs:
            try:
                extra["png"] = png_section(torch, ctx, data)
            except Exception as e:
                log(f"png section failed: {e}")
                raise
            try:
                n_pool = args.pool or max(2, n_dev)
                extra["host_fed"] = host_fed_section(torch, ctx, uniq, 64, args.cpu_seconds / 4, threads,
                                                     not args.no_cpu_baseline,
                                                     pool_devices=[i % n_dev for i in range(n_pool)])
            except Exception as e:
                log(f"host-fed section failed: {e}")
                raise
            try:
                extra["c3_projection"] = c3_section(torch, ctx, 20, 3, args.cpu_seconds / 4, threads,
                                                    not args.no_cpu_baseline)
            except Exception as e:
                log(f"c3 section failed: {e}")
                raise
            try:
                extra["c5_float"] = c5_section(torch, ctx, 64, 10, 2, args.cpu_seconds / 4, threads,
                                               not args.no_cpu_baseline)
            except Exception as e:
                log(f"c5 section failed: {e}")
                raise
        if not args.no_cpu_baseline:
            try:
                extra["cpu_baseline"] = cpu_baseline(torch, uniq, args.cpu_seconds, threads)
            except Exception as e:  # the baseline is reported, never the target
                log(f"cpu baseline failed: {e}")
                extra["cpu_baseline"] = None

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "tiles/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1e3 * elapsed / args.steps, 4),
            "higher_is_better": True,
            "scaling": "strong" if args.total_tiles else "weak",
            "vs_baseline": None,
            "dtype": "u16",
            "data": "synthetic (microscopy-like gamma background + gaussian blobs, seeded)",
            "config": {
                "workload": "C2: 4-channel uint16 1024x1024 big-endian tiles -> packed ARGB "
                            "(per-channel window + colour composite, rgb model), HBM-resident",
                "tiles_per_gpu_per_step": B,
                "tiles_per_node_per_step": args.total_tiles or world * B,
                "windows": "0:65535,1755:51199,3218:26623,100:4000",
                "colors": "0000FF,00FF00,FF0000,FFFFFF",
                "parallelism": f"dp{world} (independent tile batches per GPU, no collectives)",
                "batch_descriptor": args.addr,
                "ranks": world,
                "devices_visible": n_dev,
                "ranks_share_devices": world > n_dev,
                "control_backend": backend,
            },
            "roofline": {
                "bound": "hbm",
                "kernel": "k_render<u16,BE,4ch> (K2)",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "algorithmic_bytes_per_launch": BYTES_PER_TILE * B,
                "avg_launch_ms": round(k2_ms, 5),
                "min_launch_ms": round(k2[0], 5) if k2 else None,
                "median_launch_ms": round(k2[len(k2) // 2], 5) if k2 else None,
                "max_launch_ms": round(k2[-1], 5) if k2 else None,
                "launches": len(k2),
                "timing": "second pass of the same K steps with per-launch HIP events on the "
                          "K2 stream; the throughput pass runs with kernel timing off",
                "region_event_ms_per_step": round(region_ms / args.steps, 5),
            },
            "hbm_gbs": round(achieved, 1),
            "prewarm": {"ms": args.prewarm_ms, "steps": n_pre,
                        "why": "untimed, before the W warm-up steps: GPU clock ramp out of idle "
                               "(first ~25 K2 launches 0.77 -> 0.60 ms vs 0.55 sustained)"},
        }
        line.update(extra)
        if "cpu_baseline" not in line:
            line["cpu_baseline"] = None
        line["sections"] = sections_summary(line)      # last: the part of the line a tail keeps
        print(json.dumps(line), flush=True)
    ctx.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
