"""Every OMR_SEM_* switch through libomr.so against the CPU restatement under the same switch
(include/omr/omr.h; tests/test_semantics.py pins what each switch means).  Each case also checks
that the switch changes the output on its input, so a switch that silently does nothing fails."""
import io

import numpy as np
import pytest

import oracle_lib as O
from omr import _lib
from omr.context import make_qdef
from omr.renderer import f32
from omr.synthetic import c2_channels, tile_u16

pytestmark = pytest.mark.gpu


@pytest.fixture
def sem_ctx(ctx):
    yield ctx
    ctx.set_semantics(0)


def _both(ctx, flags, channels, planes, pt, w, h, **kw):
    ctx.set_semantics(flags)
    q = make_qdef(kw.pop("model", "rgb"), **kw.pop("qdef", {}))
    got = ctx.render_packed_int(q, channels, planes, pt, w, h, **kw)
    with O.semantics(flags):
        st, exp = O.render(channels, planes, pt, w, h, qdef=q, **kw)
    assert st == 0
    np.testing.assert_array_equal(got, exp)
    return got


def _int_planes(pt, h, w, seed):
    rng = np.random.default_rng(seed)
    if pt == _lib.PIXELS_UINT16:
        return [rng.integers(0, 65536, (h, w)).astype(np.uint16) for _ in range(3)]
    if pt == _lib.PIXELS_INT16:
        return [rng.integers(-400, 400, (h, w)).astype(np.int16) for _ in range(3)]
    if pt == _lib.PIXELS_UINT8:
        return [rng.integers(0, 256, (h, w)).astype(np.uint8) for _ in range(3)]
    return [rng.integers(-128, 128, (h, w)).astype(np.int8) for _ in range(3)]


WINDOWS = {_lib.PIXELS_UINT16: [(100.5, 200.5), (1755.25, 51199.75), (3.5, 65534.5)],
           _lib.PIXELS_INT16: [(-100.5, 200.5), (-3.7, 50.2), (0.5, 399.5)],
           _lib.PIXELS_UINT8: [(10.5, 20.5), (0.5, 254.5), (99.9, 100.1)],
           _lib.PIXELS_INT8: [(-10.5, 20.5), (-127.5, 0.5), (5.25, 99.75)]}
RANGES = {_lib.PIXELS_UINT16: (0, 65535), _lib.PIXELS_INT16: (-32768, 32767), _lib.PIXELS_UINT8: (0, 255),
          _lib.PIXELS_INT8: (-128, 127)}


@pytest.mark.parametrize("pt", [_lib.PIXELS_UINT16, _lib.PIXELS_INT16, _lib.PIXELS_UINT8, _lib.PIXELS_INT8])
@pytest.mark.parametrize("variant", ["plain", "reverse", "codomain", "noise_reduction", "poly"])
def test_window_int_bounds(sem_ctx, pt, variant):
    h, w = 64, 256
    planes = _int_planes(pt, h, w, 11 + pt)
    if pt in (_lib.PIXELS_UINT16, _lib.PIXELS_INT16):   # every value near the window ends
        lo, hi = WINDOWS[pt][0]
        planes[0].reshape(-1)[:1024] = np.clip(np.arange(int(lo) - 500, int(lo) + 524), *RANGES[pt])
        planes[0].reshape(-1)[1024:2048] = np.clip(np.arange(int(hi) - 500, int(hi) + 524), *RANGES[pt])
    gmin, gmax = RANGES[pt]
    chans = []
    for c, (s, e) in enumerate(WINDOWS[pt]):
        d = {"input_start": f32(s), "input_end": f32(e), "global_min": float(gmin), "global_max": float(gmax),
             "rgba": [(255, 0, 0, 255), (0, 255, 0, 255), (0, 0, 255, 255)][c]}
        if variant == "reverse":
            d["reverse"] = c != 1
        if variant == "noise_reduction":
            d["noise_reduction"] = True
        if variant == "poly" and s > 0:
            d.update(family=_lib.FAMILY_POLYNOMIAL, coefficient=1.5)
        chans.append(d)
    kw = {"qdef": {"cd_start": 10, "cd_end": 200}} if variant == "codomain" else {}
    a = _both(sem_ctx, 0, chans, planes, pt, w, h, **kw)
    b = _both(sem_ctx, _lib.SEM_WINDOW_INT_BOUNDS, chans, planes, pt, w, h, **kw)
    if variant != "noise_reduction":     # NR clips both window ends before the bounds matter
        assert (a != b).any()


def test_window_int_bounds_batch_fast_path(sem_ctx):
    """The C2 batch launch with fractional windows: the switch takes K2 off its fast path."""
    import torch
    h, w, n = 128, 256, 6
    chans = c2_channels(4)
    for c, (s, e) in enumerate([(0.5, 65534.5), (1755.5, 51199.5), (3218.75, 26623.25), (100.5, 4000.5)]):
        chans[c]["input_start"], chans[c]["input_end"] = f32(s), f32(e)
    tiles = [[p.astype(">u2") for p in tile_u16(40 + t, 4, h, w, uniform=True)] for t in range(n)]
    be = np.stack([np.stack(t) for t in tiles]).astype(">u2")      # np.stack returns native order
    data = torch.from_numpy(be.view(np.uint8).copy()).to("cuda")
    out = torch.empty((n, h, w), dtype=torch.int32, device="cuda")
    plane = h * w * 2
    for flags in (0, _lib.SEM_WINDOW_INT_BOUNDS):
        sem_ctx.set_semantics(flags)
        torch.cuda.synchronize()
        sem_ctx.render_batch_strided_device(make_qdef("rgb"), chans, data, 4 * plane, plane, n, _lib.PIXELS_UINT16,
                                            w, h, out, big_endian=True)
        sem_ctx.synchronize()
        got = out.cpu().numpy().view(np.uint32)
        with O.semantics(flags):
            for t in range(n):
                st, exp = O.render(chans, tiles[t], _lib.PIXELS_UINT16, w, h, big_endian=True)
                np.testing.assert_array_equal(got[t], exp)


def test_alpha_separate(sem_ctx):
    h, w = 32, 256
    rng = np.random.default_rng(3)
    planes = [rng.integers(0, 256, (h, w)).astype(np.uint8) for _ in range(3)]
    planes[0][0] = np.arange(256)
    chans = [{"input_start": 0.0, "input_end": 255.0, "global_min": 0.0, "global_max": 255.0, "rgba": rgba}
             for rgba in [(255, 129, 100, 101), (17, 200, 255, 250), (90, 90, 90, 3)]]
    a = _both(sem_ctx, 0, chans, planes, _lib.PIXELS_UINT8, w, h)
    b = _both(sem_ctx, _lib.SEM_ALPHA_SEPARATE, chans, planes, _lib.PIXELS_UINT8, w, h)
    assert (a != b).any()
    u16 = [p.astype(np.uint16) * 257 for p in planes]
    for c in chans:
        c.update(input_end=65535.0, global_max=65535.0)
    _both(sem_ctx, _lib.SEM_ALPHA_SEPARATE, chans, u16, _lib.PIXELS_UINT16, w, h)


@pytest.mark.parametrize("pt", [_lib.PIXELS_UINT8, _lib.PIXELS_UINT16, _lib.PIXELS_FLOAT])
def test_greyscale_lut(sem_ctx, pt):
    h, w = 16, 256
    lut = np.concatenate([255 - np.arange(256), np.arange(256) // 3, np.full(256, 17)]).astype(np.uint8)
    rng = np.random.default_rng(9)
    if pt == _lib.PIXELS_UINT8:
        planes = [rng.integers(0, 256, (h, w)).astype(np.uint8) for _ in range(2)]
        hi = 255.0
    elif pt == _lib.PIXELS_UINT16:
        planes = [rng.integers(0, 65536, (h, w)).astype(np.uint16) for _ in range(2)]
        hi = 65535.0
    else:
        planes = [rng.uniform(-10, 300, (h, w)).astype(np.float32) for _ in range(2)]
        hi = 255.0
    chans = [{"input_start": 0.0, "input_end": hi, "global_min": 0.0, "global_max": hi, "lut": lut, "reverse": True},
             {"input_start": 0.0, "input_end": hi, "global_min": 0.0, "global_max": hi}]
    a = _both(sem_ctx, 0, chans, planes, pt, w, h, model="greyscale")
    b = _both(sem_ctx, _lib.SEM_GREYSCALE_LUT, chans, planes, pt, w, h, model="greyscale")
    assert (a != b).any()


@pytest.mark.parametrize("q", [0.3, 0.75, 0.9])
def test_jpeg_chroma_div2(sem_ctx, q):
    from PIL import Image
    import torch
    h, w = 200, 264
    planes = [p.astype(">u2") for p in tile_u16(12, 4, h, w)]
    st, argb = O.render(c2_channels(4), planes, _lib.PIXELS_UINT16, w, h, big_endian=True)
    outs = {}
    for flags in (0, _lib.SEM_JPEG_CHROMA_DIV2):
        sem_ctx.set_semantics(flags)
        got = sem_ctx.encode_jpeg(argb, w, h, q)
        d = torch.from_numpy(argb.view(np.int32).copy()).to("cuda")
        torch.cuda.synchronize()
        got_dev = sem_ctx.encode_jpeg_device(d, w, h, q)
        batch = sem_ctx.encode_jpeg_batch(torch.stack([d, d]), 2, w, h, q)
        with O.semantics(flags):
            exp = O.encode_jpeg(argb, w, h, q)
            ql, qc = O.quant_tables(q)
        assert got == exp and got_dev == exp and batch == [exp, exp]
        buf = io.BytesIO()
        rgb = np.ascontiguousarray(argb.view(np.uint8).reshape(h, w, 4)[..., 2::-1])
        Image.fromarray(rgb, "RGB").save(buf, "JPEG", qtables=[ql.tolist(), qc.tolist()], subsampling=2)
        assert got == buf.getvalue()
        outs[flags] = got
    assert outs[0] != outs[_lib.SEM_JPEG_CHROMA_DIV2]


def test_semantics_reject_unknown_flags(sem_ctx):
    with pytest.raises(_lib.OmrError):
        sem_ctx.set_semantics(1 << 20)
    sem_ctx.set_semantics(_lib.SEM_ALL)
    assert sem_ctx.semantics == _lib.SEM_ALL
