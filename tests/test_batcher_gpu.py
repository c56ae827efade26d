"""Request batching (omr_batcher_*): concurrent tile requests from several worker threads are
grouped by image + settings, rendered and encoded in GPU batches; every job must get exactly the
bytes the one-request path produces, and identical in-flight tiles are rendered once."""
import threading

import numpy as np
import pytest

import oracle_lib as O
from omr import Batcher, PixelBuffer, Pool, _lib, write_romio
from omr.synthetic import c2_channels

pytestmark = pytest.mark.gpu

X, Y, C, Z, T = 1024, 768, 3, 2, 1
TW, TH = 256, 256


@pytest.fixture(scope="module")
def romio(tmp_path_factory):
    rng = np.random.default_rng(44)
    px = rng.integers(0, 65536, (T, C, Z, Y, X), dtype=np.uint16)
    path = tmp_path_factory.mktemp("romio") / "pixels"
    write_romio(path, px, _lib.PIXELS_UINT16)
    return path, px


def one_request(ctx, pb, qdef, chans, z, x, y, flip_h, fmt, q):
    import torch
    out = torch.empty((TH, TW), dtype=torch.int32, device="cuda")
    ctx.render_pixel_buffer_tiles(qdef, chans, pb, [(z, 0, x, y)], TW, TH, out=out, flip_h=flip_h)
    if fmt == "jpeg":
        return ctx.encode_jpeg_device(out, TW, TH, q)
    if fmt == "png":
        return ctx.encode_png_device(out, TW, TH)
    return out.cpu().numpy().tobytes()


def test_concurrent_workers_match_single_requests(ctx, romio):
    path, px = romio
    pb = PixelBuffer(path, X, Y, Z, C, T, _lib.PIXELS_UINT16)
    settings = [(O.make_qdef("rgb"), c2_channels(3)), (O.make_qdef("greyscale"), c2_channels(3))]
    jobs = []
    rng = np.random.default_rng(1)
    for i in range(60):
        s = i % 2
        jobs.append(dict(s=s, z=int(rng.integers(0, Z)), x=int(rng.integers(0, X // TW)) * TW,
                         y=int(rng.integers(0, Y // TH)) * TH, flip=bool(i % 3 == 0),
                         fmt=["jpeg", "jpeg", "png", "argb"][i % 4], q=[0.9, 0.5][i % 2]))
    results = [None] * len(jobs)
    with Batcher(0, max_batch=32, max_wait_us=2000) as b:
        def worker(k):
            for i in range(k, len(jobs), 6):
                j = jobs[i]
                qd, ch = settings[j["s"]]
                t = b.submit(pb, qd, ch, j["z"], 0, j["x"], j["y"], TW, TH, flip_h=j["flip"], fmt=j["fmt"],
                             quality=j["q"])
                results[i] = b.wait(t)
        ths = [threading.Thread(target=worker, args=(k,)) for k in range(6)]
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        st = b.stats()
    assert st["jobs"] == len(jobs)
    for i, j in enumerate(jobs):
        qd, ch = settings[j["s"]]
        exp = one_request(ctx, pb, qd, ch, j["z"], j["x"], j["y"], j["flip"], j["fmt"], j["q"])
        assert results[i] == exp, f"job {i} {j}"
    argb_job = next(i for i, j in enumerate(jobs) if j["fmt"] == "argb")
    j = jobs[argb_job]
    qd, ch = settings[j["s"]]
    planes = [np.ascontiguousarray(px[0, c, j["z"], j["y"]:j["y"] + TH, j["x"]:j["x"] + TW]).astype(">u2")
              for c in range(C)]
    s, exp = O.render(ch, planes, _lib.PIXELS_UINT16, TW, TH, big_endian=True, flip_h=j["flip"],
                      model="rgb" if j["s"] == 0 else "greyscale")
    np.testing.assert_array_equal(np.frombuffer(results[argb_job], np.uint32).reshape(TH, TW), exp)
    pb.close()


def test_duplicates_rendered_once_and_errors(romio):
    path, px = romio
    pb = PixelBuffer(path, X, Y, Z, C, T, _lib.PIXELS_UINT16)
    qd, ch = O.make_qdef("rgb"), c2_channels(3)
    with Batcher(0, max_batch=64, max_wait_us=50000) as b:
        tickets = [b.submit(pb, qd, ch, 1, 0, 256, 512, TW, TH) for _ in range(5)]
        tickets.append(b.submit(pb, qd, ch, 0, 0, 0, 0, TW, TH))
        outs = [b.wait(t) for t in tickets]
        assert len(set(outs[:5])) == 1 and outs[5] != outs[0]
        st = b.stats()
        assert st["dedup"] >= 4 and st["rendered"] <= 2, st
        with pytest.raises(_lib.OmrError) as e:                       # unknown format -> 404
            b.submit(pb, qd, ch, 0, 0, 0, 0, TW, TH, fmt="gif")
        assert e.value.status == _lib.NOT_FOUND
        t = b.submit(pb, qd, ch, 0, 0, X - 100, 0, TW, TH)               # outside the image
        with pytest.raises(_lib.OmrError) as e:
            b.wait(t)
        assert e.value.status == _lib.INVALID_ARGUMENT
    pb.close()


def _oracle_argb(px, ch, model, z, x, y, flip):
    planes = [np.ascontiguousarray(px[0, c, z, y:y + TH, x:x + TW]).astype(">u2") for c in range(C)]
    s, exp = O.render(ch, planes, _lib.PIXELS_UINT16, TW, TH, big_endian=True, flip_h=flip, model=model)
    assert s == 0
    return exp


def test_every_format_against_the_oracle(romio):
    """Batched ARGB words, JPEG bytes and PNG pixels vs the CPU restatement (not vs the GPU's own
    one-request path)."""
    import io
    from PIL import Image
    path, px = romio
    pb = PixelBuffer(path, X, Y, Z, C, T, _lib.PIXELS_UINT16)
    jobs = [dict(model=m, z=z, x=x, y=y, flip=f, fmt=fmt, q=q)
            for i, (m, z, x, y, f, fmt, q) in enumerate([
                ("rgb", 0, 0, 0, False, "argb", 0.9), ("rgb", 1, 256, 256, True, "argb", 0.9),
                ("rgb", 0, 512, 0, False, "jpeg", 0.9), ("rgb", 1, 768, 512, True, "jpeg", 0.9),
                ("greyscale", 0, 256, 512, False, "jpeg", 0.5), ("rgb", 1, 0, 256, False, "png", 0.9),
                ("greyscale", 0, 512, 512, True, "png", 0.9), ("greyscale", 1, 768, 0, False, "argb", 0.9),
                ("rgb", 0, 256, 0, True, "tif", 0.9), ("greyscale", 1, 512, 256, False, "tif", 0.9)])]
    ch = c2_channels(3)
    with Batcher(0, max_batch=16, max_wait_us=20000) as b:
        tickets = [b.submit(pb, O.make_qdef(j["model"]), ch, j["z"], 0, j["x"], j["y"], TW, TH, flip_h=j["flip"],
                            fmt=j["fmt"], quality=j["q"]) for j in jobs]
        outs = [b.wait(t) for t in tickets]
    for j, got in zip(jobs, outs):
        exp = _oracle_argb(px, ch, j["model"], j["z"], j["x"], j["y"], j["flip"])
        if j["fmt"] == "argb":
            np.testing.assert_array_equal(np.frombuffer(got, np.uint32).reshape(TH, TW), exp)
        elif j["fmt"] == "jpeg":
            assert got == O.encode_jpeg(exp, TW, TH, j["q"]), j
        else:                                            # PNG / TIFF: decoded pixels
            im = Image.open(io.BytesIO(got))
            assert im.format == {"png": "PNG", "tif": "TIFF"}[j["fmt"]]
            rgb = np.asarray(im.convert("RGB"))
            np.testing.assert_array_equal(rgb, exp.view(np.uint8).reshape(TH, TW, 4)[..., 2::-1])
    pb.close()


def _check_against_oracle(px, jobs, outs, ch_of, flags_of=lambda j: 0):
    import io
    from PIL import Image
    for j, got in zip(jobs, outs):
        with O.semantics(flags_of(j)):
            planes = [np.ascontiguousarray(px[0, c, j["z"], j["y"]:j["y"] + TH, j["x"]:j["x"] + TW]).astype(">u2")
                      for c in range(C)]
            s, exp = O.render(ch_of(j), planes, _lib.PIXELS_UINT16, TW, TH, big_endian=True, flip_h=j["flip"],
                              model=j["model"])
            assert s == 0
            if j["fmt"] == "argb":
                np.testing.assert_array_equal(np.frombuffer(got, np.uint32).reshape(TH, TW), exp)
            elif j["fmt"] == "jpeg":
                assert got == O.encode_jpeg(exp, TW, TH, j["q"]), j
            else:
                rgb = np.asarray(Image.open(io.BytesIO(got)).convert("RGB"))
                np.testing.assert_array_equal(rgb, exp.view(np.uint8).reshape(TH, TW, 4)[..., 2::-1])


def _fractional_channels():
    ch = c2_channels(3)
    for c, (s, e) in enumerate([(100.5, 60000.25), (1755.5, 51199.5), (3218.75, 26623.25)]):
        ch[c]["input_start"], ch[c]["input_end"] = s, e
    return ch


def test_semantics_fixed_at_submit(romio):
    """Jobs keep the OMR_SEM_* flags they were submitted under: a set_semantics between two
    submits (while the first jobs are still queued) changes only the later jobs, and jobs with
    different flags never share a render (the dispatcher used to read the context's
    flags without a lock, mid-round)."""
    path, px = romio
    pb = PixelBuffer(path, X, Y, Z, C, T, _lib.PIXELS_UINT16)
    ch = c2_channels(3)
    for c, rgba in enumerate([(255, 129, 100, 101), (17, 200, 255, 250), (90, 90, 90, 3)]):
        ch[c]["rgba"] = rgba                   # translucent colours: OMR_SEM_ALPHA_SEPARATE changes pixels
    spots = [(0, 0), (256, 256), (512, 0), (768, 512)]
    jobs, tickets = [], []
    with Batcher(0, max_batch=64, max_wait_us=200000) as b:
        for flags in (0, _lib.SEM_ALPHA_SEPARATE, 0):
            b.set_semantics(flags)
            for x, y in spots:
                j = dict(model="rgb", z=1, x=x, y=y, flip=False, fmt="argb", q=0.9, flags=flags)
                jobs.append(j)
                tickets.append(b.submit(pb, O.make_qdef("rgb"), ch, 1, 0, x, y, TW, TH, fmt="argb"))
        outs = [b.wait(t) for t in tickets]
        st = b.stats()
    assert st["dedup"] == len(spots)          # the two flag-0 rounds share; the other flags never do
    _check_against_oracle(px, jobs, outs, lambda j: ch, lambda j: j["flags"])
    assert outs[0] != outs[len(spots)]
    with Batcher(0) as b2, pytest.raises(_lib.OmrError):
        b2.set_semantics(1 << 20)
    pb.close()


def test_pool_spreads_jobs_over_devices(romio):
    """omr_pool with two batchers (cuda:{i % device_count}: two contexts on one card when the
    box has one GPU): concurrent workers, every format, each output against the CPU restatement,
    and both batchers served jobs."""
    import torch
    path, px = romio
    pb = PixelBuffer(path, X, Y, Z, C, T, _lib.PIXELS_UINT16)
    devices = [i % torch.cuda.device_count() for i in range(2)]
    ch = c2_channels(3)
    rng = np.random.default_rng(17)
    jobs = [dict(model=["rgb", "greyscale"][i % 2], z=int(rng.integers(0, Z)), x=int(rng.integers(0, X // TW)) * TW,
                 y=int(rng.integers(0, Y // TH)) * TH, flip=bool(i % 3 == 0), fmt=["jpeg", "argb", "png", "tif"][i % 4],
                 q=[0.9, 0.6][i % 2]) for i in range(48)]
    outs, where = [None] * len(jobs), [None] * len(jobs)
    with Pool(devices, max_batch=16, max_wait_us=3000) as pool:
        import threading

        def worker(k):
            for i in range(k, len(jobs), 6):
                j = jobs[i]
                t = pool.submit(pb, O.make_qdef(j["model"]), ch, j["z"], 0, j["x"], j["y"], TW, TH,
                                flip_h=j["flip"], fmt=j["fmt"], quality=j["q"])
                where[i] = pool.device_index(t)
                outs[i] = pool.wait(t)
        ths = [threading.Thread(target=worker, args=(k,)) for k in range(6)]
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        stats = pool.stats()
    assert sorted(set(where)) == [0, 1]
    assert sum(s["jobs"] for s in stats) == len(jobs) and all(s["jobs"] > 0 for s in stats)
    _check_against_oracle(px, jobs, outs, lambda j: ch)
    pb.close()


def test_pool_per_tile_errors_and_semantics(tmp_path):
    import torch
    rng = np.random.default_rng(6)
    px = rng.integers(0, 50000, (T, C, 1, 512, 1024), dtype=np.uint16)
    px[0, 2, 0, 10, 20] = 65000                                     # inside tile (0, 0)
    path = tmp_path / "pixels"
    write_romio(path, px, _lib.PIXELS_UINT16)
    pb = PixelBuffer(path, 1024, 512, 1, C, T, _lib.PIXELS_UINT16)
    ch = _fractional_channels()
    for c in ch:
        c["global_max"] = 60000.0
    devices = [i % torch.cuda.device_count() for i in range(3)]
    tiles = [(x, y) for y in (0, 256) for x in (0, 256, 512, 768)]
    with Pool(devices, max_batch=4, max_wait_us=1000) as pool:
        pool.set_semantics(_lib.SEM_WINDOW_INT_BOUNDS)
        tickets = [pool.submit(pb, O.make_qdef("rgb"), ch, 0, 0, x, y, TW, TH, fmt="argb") for x, y in tiles]
        res = []
        for t in tickets:
            try:
                res.append(pool.wait(t))
            except _lib.OmrError as e:
                res.append(e.status)
        with pytest.raises(_lib.OmrError):
            pool.submit(pb, O.make_qdef("rgb"), ch, 0, 0, 0, 0, TW, TH, fmt="gif")
        with pytest.raises(_lib.OmrError):
            pool.set_semantics(1 << 20)
    for (x, y), r in zip(tiles, res):
        if (x, y) == (0, 0):
            assert r == _lib.QUANTIZATION
            continue
        planes = [np.ascontiguousarray(px[0, c, 0, y:y + TH, x:x + TW]).astype(">u2") for c in range(C)]
        with O.semantics(_lib.SEM_WINDOW_INT_BOUNDS):
            s, exp = O.render(ch, planes, _lib.PIXELS_UINT16, TW, TH, big_endian=True)
        np.testing.assert_array_equal(np.frombuffer(r, np.uint32).reshape(TH, TW), exp)
    pb.close()


def test_quantization_error_fails_only_its_tile(tmp_path):
    """One tile holds a pixel above the channel's LUT domain (globalMax): that request fails with
    QuantizationException (500); the tiles batched with it still render (each request has its own
    Renderer in the reference, ImageRegionRequestHandler.java:436-440, :479-480)."""
    rng = np.random.default_rng(5)
    px = rng.integers(0, 50000, (T, C, 1, 512, 1024), dtype=np.uint16)
    px[0, 1, 0, 300, 700] = 65000                                  # inside tile (x=512, y=256)
    path = tmp_path / "pixels"
    write_romio(path, px, _lib.PIXELS_UINT16)
    pb = PixelBuffer(path, 1024, 512, 1, C, T, _lib.PIXELS_UINT16)
    ch = c2_channels(3)
    for c in ch:
        c["global_max"] = 60000.0
    tiles = [(x, y) for y in (0, 256) for x in (0, 256, 512, 768)]
    with Batcher(0, max_batch=16, max_wait_us=20000) as b:
        tickets = [b.submit(pb, O.make_qdef("rgb"), ch, 0, 0, x, y, TW, TH, fmt="argb") for x, y in tiles]
        res = []
        for t in tickets:
            try:
                res.append(b.wait(t))
            except _lib.OmrError as e:
                res.append(e.status)
    for (x, y), r in zip(tiles, res):
        if (x, y) == (512, 256):
            assert r == _lib.QUANTIZATION
        else:
            planes = [np.ascontiguousarray(px[0, c, 0, y:y + TH, x:x + TW]).astype(">u2") for c in range(C)]
            s, exp = O.render(ch, planes, _lib.PIXELS_UINT16, TW, TH, big_endian=True)
            assert s == 0
            np.testing.assert_array_equal(np.frombuffer(r, np.uint32).reshape(TH, TW), exp)
    pb.close()


# ---- projection jobs (p=intmax|intmean|intsum, ImageRegionRequestHandler.java:506-558) ------------------
PX_, PY_, PZ_, PC_, PT_ = 256, 128, 6, 3, 2


@pytest.fixture(scope="module")
def romio_stack(tmp_path_factory):
    rng = np.random.default_rng(46)
    px = rng.integers(0, 65536, (PT_, PC_, PZ_, PY_, PX_), dtype=np.uint16)
    path = tmp_path_factory.mktemp("romio_z") / "pixels"
    write_romio(path, px, _lib.PIXELS_UINT16)
    return path, px


def _oracle_projected(px, ch, model, t, alg, start, end, flip_h=False, flip_v=False):
    """The glue on the CPU: every active channel's (c, t) stack projected, the full plane rendered."""
    planes = []
    for c in range(PC_):
        if not ch[c].get("active", True):
            planes.append(np.zeros(PX_ * PY_ * 2, np.uint8))
            continue
        stack = np.ascontiguousarray(px[t, c]).astype(">u2")
        st, p = O.project(stack, _lib.PIXELS_UINT16, PX_, PY_, PZ_, alg, start, end, 1, be_in=True, be_out=True)
        assert st == 0
        planes.append(p)
    st, exp = O.render(ch, planes, _lib.PIXELS_UINT16, PX_, PY_, big_endian=True, flip_h=flip_h, flip_v=flip_v,
                       model=model)
    return st, exp


def test_projection_jobs_against_the_oracle(romio_stack):
    """Projection requests through the batcher: every algorithm, default and explicit z ranges, both
    t, flips, every format; the full plane regardless of the tile fields; duplicates (same t,
    settings and projection) rendered once."""
    import io
    from PIL import Image
    path, px = romio_stack
    pb = PixelBuffer(path, PX_, PY_, PZ_, PC_, PT_, _lib.PIXELS_UINT16)
    ch = c2_channels(3)
    jobs = [dict(p="intmax", s=-1, e=-1, t=0, fh=False, fv=False, fmt="argb", model="rgb"),
            dict(p="intmax", s=-1, e=-1, t=1, fh=True, fv=False, fmt="argb", model="rgb"),
            dict(p="intmean", s=1, e=4, t=0, fh=False, fv=True, fmt="argb", model="greyscale"),
            dict(p="intsum", s=0, e=5, t=1, fh=False, fv=False, fmt="argb", model="rgb"),
            dict(p="intmax", s=2, e=3, t=1, fh=False, fv=False, fmt="jpeg", model="rgb"),
            dict(p="intmean", s=-1, e=-1, t=0, fh=True, fv=True, fmt="png", model="rgb"),
            dict(p="intmax", s=-1, e=-1, t=0, fh=False, fv=False, fmt="argb", model="rgb")]    # dup of job 0
    algs = {"intmax": _lib.PROJECTION_MAX, "intmean": _lib.PROJECTION_MEAN, "intsum": _lib.PROJECTION_SUM}
    with Batcher(0, max_batch=32, max_wait_us=50000) as b:
        tickets = [b.submit(pb, O.make_qdef(j["model"]), ch, 0, j["t"], 64, 32, 16, 16, flip_h=j["fh"], flip_v=j["fv"],
                            fmt=j["fmt"], quality=0.9, projection=j["p"], projection_start=j["s"],
                            projection_end=j["e"]) for j in jobs]
        outs = [b.wait(t) for t in tickets]
        st = b.stats()
    assert st["dedup"] >= 1
    assert outs[6] == outs[0]
    for j, got in zip(jobs, outs):
        s = 0 if j["s"] < 0 else j["s"]
        e = PZ_ - 1 if j["e"] < 0 else j["e"]
        stt, exp = _oracle_projected(px, ch, j["model"], j["t"], algs[j["p"]], s, e, j["fh"], j["fv"])
        assert stt == 0
        if j["fmt"] == "argb":
            np.testing.assert_array_equal(np.frombuffer(got, np.uint32).reshape(PY_, PX_), exp)
        elif j["fmt"] == "jpeg":
            assert got == O.encode_jpeg(exp, PX_, PY_, 0.9)
        else:
            rgb = np.asarray(Image.open(io.BytesIO(got)).convert("RGB"))
            np.testing.assert_array_equal(rgb, exp.view(np.uint8).reshape(PY_, PX_, 4)[..., 2::-1])
    pb.close()


def test_projection_job_errors_fail_alone(romio_stack):
    """The glue's quirk 3 (a rendered channel's index >= the number of active channels: OMR_INTERNAL,
    Appendix B) and a z range past sizeZ fail only their own job; a projection job in the same round
    still renders."""
    path, px = romio_stack
    pb = PixelBuffer(path, PX_, PY_, PZ_, PC_, PT_, _lib.PIXELS_UINT16)
    ch_bad = c2_channels(3)
    ch_bad[0]["active"] = False
    ch_bad[1]["active"] = False                  # only c=2 active: index 2 >= 1 active channel
    ch = c2_channels(3)
    with Batcher(0, max_batch=32, max_wait_us=50000) as b:
        t_bad = b.submit(pb, O.make_qdef("rgb"), ch_bad, 0, 0, 0, 0, 16, 16, fmt="argb", projection="intmax")
        t_range = b.submit(pb, O.make_qdef("rgb"), ch, 0, 1, 0, 0, 16, 16, fmt="argb", projection="intmax",
                           projection_start=0, projection_end=PZ_ + 3)
        t_ok = b.submit(pb, O.make_qdef("rgb"), ch, 0, 1, 0, 0, 16, 16, fmt="argb", projection="intmax")
        with pytest.raises(_lib.OmrError) as e:
            b.wait(t_bad)
        assert e.value.status == _lib.INTERNAL
        with pytest.raises(_lib.OmrError):
            b.wait(t_range)
        got = b.wait(t_ok)
        with pytest.raises(_lib.OmrError):                                 # unknown algorithm
            b.submit(pb, O.make_qdef("rgb"), ch, 0, 1, 0, 0, 16, 16, fmt="argb", projection=7)
    stt, exp = _oracle_projected(px, ch, "rgb", 1, _lib.PROJECTION_MAX, 0, PZ_ - 1)
    np.testing.assert_array_equal(np.frombuffer(got, np.uint32).reshape(PY_, PX_), exp)
    pb.close()


def test_projection_bad_t_never_cached(romio_stack):
    """A projection job at a t outside [0, sizeT) fails at wait in every round it is submitted:
    the stack cache never records a slot for a stack that was not uploaded (a second request for
    the same t must not read that slot as a hit), and a good job of the same image still renders."""
    path, px = romio_stack
    pb = PixelBuffer(path, PX_, PY_, PZ_, PC_, PT_, _lib.PIXELS_UINT16)
    ch = c2_channels(3)
    with Batcher(0, max_batch=8, max_wait_us=1000) as b:
        for _ in range(2):                                   # two separate dispatch rounds
            t_bad = b.submit(pb, O.make_qdef("rgb"), ch, 0, PT_ + 1, 0, 0, 16, 16, fmt="argb",
                             projection="intmax")
            with pytest.raises(_lib.OmrError) as e:
                b.wait(t_bad)
            assert e.value.status == _lib.INVALID_ARGUMENT
        got = b.wait(b.submit(pb, O.make_qdef("rgb"), ch, 0, 1, 0, 0, 16, 16, fmt="argb", projection="intmax"))
    stt, exp = _oracle_projected(px, ch, "rgb", 1, _lib.PROJECTION_MAX, 0, PZ_ - 1)
    np.testing.assert_array_equal(np.frombuffer(got, np.uint32).reshape(PY_, PX_), exp)
    pb.close()


def test_tile_outside_image_fails_alone(romio):
    """One out-of-bounds tile (x + width > sizeX, or z / t past the image) in a group fails only its
    own job; the group's other tiles render against the oracle."""
    path, px = romio
    pb = PixelBuffer(path, X, Y, Z, C, T, _lib.PIXELS_UINT16)
    qd, ch = O.make_qdef("rgb"), c2_channels(3)
    with Batcher(0, max_batch=64, max_wait_us=50000) as b:
        t_ok = b.submit(pb, qd, ch, 0, 0, 256, 0, TW, TH, fmt="argb")
        t_x = b.submit(pb, qd, ch, 0, 0, X - 100, 0, TW, TH, fmt="argb")
        t_z = b.submit(pb, qd, ch, Z, 0, 0, 0, TW, TH, fmt="argb")
        t_t = b.submit(pb, qd, ch, 0, T, 0, 0, TW, TH, fmt="argb")
        for t in (t_x, t_z, t_t):
            with pytest.raises(_lib.OmrError) as e:
                b.wait(t)
            assert e.value.status == _lib.INVALID_ARGUMENT
        got = b.wait(t_ok)
    np.testing.assert_array_equal(np.frombuffer(got, np.uint32).reshape(TH, TW),
                                  _oracle_argb(px, ch, "rgb", 0, 256, 0, False))
    pb.close()


def test_mask_jobs_bad_dims_empty_and_wide_fail_alone():
    """Masks the batch answers 404 take no output room (a 100000 x 100000 mask of 4 bytes must not
    size a 10 GB host buffer); an empty mask is not deduplicated with a 1-byte zero mask; a mask
    row too wide for the batched filter fails alone; the good masks of the round still encode."""
    import io
    from PIL import Image
    good = (bytes([0x55, 0xAA] * 8), 16, 8, (255, 0, 0, 255))
    with Batcher(0, max_batch=64, max_wait_us=50000) as b:
        b.set_semantics(_lib.SEM_MASK_PIXEL_FLIP)
        t_huge = b.submit_mask(b"\x01\x02\x03\x04", 100000, 100000, (255, 0, 0, 255))
        t_empty = b.submit_mask(b"", 8, 1, (255, 0, 0, 255))
        t_zero = b.submit_mask(b"\x00", 8, 1, (255, 0, 0, 255))
        t_wide = b.submit_mask(bytes((100001 + 7) // 8), 100001, 1, (0, 255, 0, 255))
        t_good = b.submit_mask(*good)
        with pytest.raises(_lib.OmrError) as e:
            b.wait(t_huge)
        assert e.value.status == _lib.NOT_FOUND
        with pytest.raises(_lib.OmrError) as e:
            b.wait(t_empty)
        assert e.value.status == _lib.NOT_FOUND
        zero = b.wait(t_zero)
        with pytest.raises(_lib.OmrError):
            b.wait(t_wide)
        png = b.wait(t_good)
    im = Image.open(io.BytesIO(zero))
    assert im.size == (8, 1) and list(im.getdata()) == [0] * 8
    im = Image.open(io.BytesIO(png))
    bits = np.unpackbits(np.frombuffer(good[0], np.uint8))[:16 * 8]
    np.testing.assert_array_equal(np.array(im).reshape(-1), bits)


def test_pool_projection_and_mask_jobs(romio_stack, romio):
    """A 2-entry pool serving tile, projection and shape-mask jobs from concurrent workers: every
    result against the CPU restatement, both batchers used."""
    import threading
    import torch
    path, px = romio_stack
    pb = PixelBuffer(path, PX_, PY_, PZ_, PC_, PT_, _lib.PIXELS_UINT16)
    ch = c2_channels(3)
    devices = [i % torch.cuda.device_count() for i in range(2)]
    rng = np.random.default_rng(8)
    masks = []
    for k in range(12):
        w, h = [(64, 32), (37, 21), (8, 8), (200, 100)][k % 4]
        masks.append((rng.integers(0, 256, (w * h + 7) // 8, dtype=np.uint8).tobytes(), w, h,
                      tuple(int(v) for v in rng.integers(0, 256, 4)), bool(k & 1), bool(k & 2)))
    outs_p, outs_m, where = [None] * 8, [None] * len(masks), []
    with Pool(devices, max_batch=16, max_wait_us=3000) as pool:
        pool.set_semantics(_lib.SEM_MASK_PIXEL_FLIP)

        def worker(k):
            for i in range(k, 8, 4):
                t = pool.submit(pb, O.make_qdef("rgb"), ch, 0, i % 2, 0, 0, 16, 16, fmt="argb",
                                projection=["intmax", "intmean"][i % 2])
                where.append(pool.device_index(t))
                outs_p[i] = pool.wait(t)
            for i in range(k, len(masks), 4):
                t = pool.submit_mask(*masks[i])
                where.append(pool.device_index(t))
                outs_m[i] = pool.wait(t)
        ths = [threading.Thread(target=worker, args=(k,)) for k in range(4)]
        for t in ths:
            t.start()
        for t in ths:
            t.join()
    assert sorted(set(where)) == [0, 1]
    for i in range(8):
        stt, exp = _oracle_projected(px, ch, "rgb", i % 2, [_lib.PROJECTION_MAX, _lib.PROJECTION_MEAN][i % 2], 0,
                                     PZ_ - 1)
        np.testing.assert_array_equal(np.frombuffer(outs_p[i], np.uint32).reshape(PY_, PX_), exp)
    import io
    from PIL import Image
    with O.semantics(_lib.SEM_MASK_PIXEL_FLIP):
        for (bits, w, h, rgba, fh, fv), png in zip(masks, outs_m):
            st, idx = O.mask_indices(bits, w, h, fh, fv)
            exp = np.zeros((h, w, 4), np.uint8)
            exp[idx == 1] = rgba
            np.testing.assert_array_equal(np.asarray(Image.open(io.BytesIO(png)).convert("RGBA")), exp)
    pb.close()


def test_mask_jobs_dedup_and_404(ctx):
    """Mask jobs of one round share one batch call; identical masks render once; every case the
    single call answers with 404 fails only its own job."""
    bits = bytes(range(32))
    with Batcher(0, max_batch=32, max_wait_us=50000) as b:
        b.set_semantics(_lib.SEM_MASK_PIXEL_FLIP)
        t = [b.submit_mask(bits, 16, 16, (255, 0, 0, 255)) for _ in range(3)]
        t.append(b.submit_mask(bits, 16, 16, (0, 255, 0, 255)))
        t.append(b.submit_mask(bytes(2), 16, 16, (0, 255, 0, 255)))           # short: 404
        t.append(b.submit_mask(None, 16, 16, (0, 255, 0, 255)))               # null: 404
        t.append(b.submit_mask(bits, 0, 16, (0, 255, 0, 255)))                # zero size: 404
        res = []
        for x in t:
            try:
                res.append(b.wait(x))
            except _lib.OmrError as e:
                res.append(e.status)
        st = b.stats()
    assert res[0] == res[1] == res[2] and res[3] != res[0]
    assert res[4:] == [_lib.NOT_FOUND] * 3
    assert st["dedup"] >= 2
    ctx.set_semantics(_lib.SEM_MASK_PIXEL_FLIP)
    try:
        assert res[0] == ctx.render_shape_mask_png(bits, 16, 16, (255, 0, 0, 255))
    finally:
        ctx.set_semantics(0)


def test_projection_stack_cache(romio_stack):
    """The HBM stack cache: a repeated projection (other algorithm / range / flips) on the same t hits
    the resident stacks, a tiny cache evicts and re-uploads, a disabled cache uploads every time --
    every result equal to the CPU restatement."""
    path, px = romio_stack
    pb = PixelBuffer(path, PX_, PY_, PZ_, PC_, PT_, _lib.PIXELS_UINT16)
    ch = c2_channels(3)
    stack_bytes = PX_ * PY_ * PZ_ * 2
    runs = [("intmax", 0, -1, -1, False), ("intmean", 0, 1, 4, True), ("intmax", 1, -1, -1, False),
            ("intsum", 0, 0, 5, False)]
    algs = {"intmax": _lib.PROJECTION_MAX, "intmean": _lib.PROJECTION_MEAN, "intsum": _lib.PROJECTION_SUM}
    for cap, expect_hits in [(1 << 30, True), (stack_bytes * 3, True), (stack_bytes, True), (0, False)]:
        with Batcher(0, max_batch=8, max_wait_us=100) as b:
            b.set_stack_cache(cap)
            for p, t, s, e, fh in runs:                                  # one job per round
                got = b.wait(b.submit(pb, O.make_qdef("rgb"), ch, 0, t, 0, 0, 16, 16, flip_h=fh, fmt="argb",
                                      projection=p, projection_start=s, projection_end=e))
                stt, exp = _oracle_projected(px, ch, "rgb", t, algs[p], 0 if s < 0 else s, PZ_ - 1 if e < 0 else e,
                                             fh)
                np.testing.assert_array_equal(np.frombuffer(got, np.uint32).reshape(PY_, PX_), exp)
            st = b.stack_cache_stats()
        assert (st["hits"] > 0) == expect_hits, (cap, st)
        assert st["resident_bytes"] <= cap
        if cap == 1 << 30:
            assert st["hits"] == 2 * 3 and st["misses"] == 2 * 3, st    # t=0 and t=1 uploaded once each
        elif cap == stack_bytes * 3:
            assert st["hits"] == 3 and st["misses"] == 9, st            # t=1 evicted t=0
    with Batcher(0) as b, pytest.raises(_lib.OmrError):
        b.set_stack_cache(-1)
    pb.close()
