"""Request batching (omr_batcher_*): concurrent tile requests from several worker threads are
grouped by image + settings, rendered and encoded in GPU batches; every job must get exactly the
bytes the one-request path produces, and identical in-flight tiles are rendered once."""
import threading

import numpy as np
import pytest

import oracle_lib as O
from omr import Batcher, PixelBuffer, _lib, write_romio
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
