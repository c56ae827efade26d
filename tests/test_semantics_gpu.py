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


# ---- round 3: S2 log guard, S4 noise reduction, exp input normalisation, packed mask flip ----
# Every kernel path the switch can reach runs against the restatement under the same switch:
#   K1+K2 one-tile launch (K2 builds its tables in LDS), the full K2 batch launch (K1 tables,
#   2 chunks per lane), the fused render -> JPEG (F1; integer types: byte-identical to the unfused
#   GPU render + JPEG, and to the restatement's JPEG when the family is linear), and the
#   projection glue (K3 + K2 and K3R; integer types), plus the float threshold / Eval modes.
# Round 5: every quantization table (8/16-bit LUTs, the float / 32-bit code thresholds) is built on
# the host with the host libm, so integer types and threshold-mode float channels are bit-exact for
# every family; only Eval-mode channels (double pixels, or a q not provably monotone) evaluate
# log/pow/exp on the device and keep the +-1 code-value bar.

PRIMARY = [(255, 0, 0, 255), (0, 255, 0, 255), (0, 0, 255, 255)]


def _assert_close(got, exp, tol):
    if tol == 0:
        np.testing.assert_array_equal(got, exp)
        return
    for sh in (16, 8, 0):
        d = np.abs(((got >> sh) & 0xFF).astype(int) - ((exp >> sh) & 0xFF).astype(int))
        assert d.max() <= tol, f"component {sh}: max diff {d.max()}"


def _k3r_context():
    import os
    import omr
    os.environ["OMR_K3R"] = "1"
    try:
        return omr.Context(0)
    finally:
        del os.environ["OMR_K3R"]


def _every_path(ctx, flags, chans, planes, pt, w, h, tol, k3r_ctx=None, jpeg=True):
    """Renders `planes` (numpy, native order) under `flags` through every kernel path and checks
    each against the restatement.  Returns the one-tile ARGB.  8/16-bit integer types are held
    bit-exact whatever `tol` says: their quantization tables come from the host (round 5)."""
    import torch
    if _lib.BYTES_PER_PIXEL[pt] <= 2:
        tol = 0
    ctx.set_semantics(flags)
    q = make_qdef("rgb")
    with O.semantics(flags):
        st, exp = O.render(chans, planes, pt, w, h, qdef=q)
    assert st == 0
    got = ctx.render_packed_int(q, chans, planes, pt, w, h)                      # one-tile launch
    _assert_close(got, exp, tol)
    # full batch launch: enough tiles that K2 leaves its small-launch instantiation
    nb = max(2, -(-4_300_000 // (w * h)))
    plane_bytes = planes[0].nbytes
    one = np.concatenate([p.reshape(-1).view(np.uint8) for p in planes])
    data = torch.from_numpy(np.tile(one, nb)).to("cuda")
    out = torch.empty((nb, h, w), dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    ctx.render_batch_strided_device(q, chans, data, len(planes) * plane_bytes, plane_bytes, nb, pt, w, h, out)
    ctx.synchronize()
    allg = out.cpu().numpy().view(np.uint32)
    for t in (0, nb - 1):
        _assert_close(allg[t], exp, tol)
    assert (allg == allg[0]).all()
    if jpeg and _lib.BYTES_PER_PIXEL[pt] <= 2 and w % 16 == 0 and h % 16 == 0:
        n = 3
        cap = n * (lib_jpeg_max(w, h))
        d_out = torch.empty(cap, dtype=torch.uint8, device="cuda")
        offs = torch.empty(n, dtype=torch.int64, device="cuda")
        lens = torch.empty(n, dtype=torch.int32, device="cuda")
        ctx.render_jpeg_batch_strided_device(q, chans, data, len(planes) * plane_bytes, plane_bytes, n, pt, w, h,
                                             0.9, d_out, offs, lens)
        ctx.synchronize()
        fused = _files(d_out, offs, lens, n)
        unfused = ctx.encode_jpeg_batch(out[:n].contiguous(), n, w, h, 0.9)
        assert fused == unfused
        if tol == 0:
            with O.semantics(flags):
                assert fused[0] == O.encode_jpeg(exp, w, h, 0.9)
    ctx.set_semantics(0)
    return got


def lib_jpeg_max(w, h):
    return int(_lib.lib.omr_jpeg_max_bytes(w, h))


def _files(d_out, offs, lens, n):
    b = d_out.cpu().numpy()
    o = offs.cpu().numpy()
    ln = lens.cpu().numpy().view(np.uint32)
    return [b[o[i]:o[i] + ln[i]].tobytes() for i in range(n)]


def _glue_paths(ctx, k3r, flags, chans, stacks, pt, w, h, z, tol):
    import torch
    if _lib.BYTES_PER_PIXEL[pt] <= 2:
        tol = 0                                 # host-built quantization tables: exact
    for c in (ctx, k3r):
        c.set_semantics(flags)
        q = make_qdef("rgb")
        out = torch.empty((h, w), dtype=torch.int32, device="cuda")
        devs = [torch.from_numpy(s.reshape(-1).view(np.uint8).copy()).to("cuda") for s in stacks]
        torch.cuda.synchronize()
        c.render_projected_device(q, chans, devs, pt, w, h, z, _lib.PROJECTION_MAX, 0, z - 1, out)
        c.synchronize()
        got = out.cpu().numpy().view(np.uint32)
        planes = []
        for s in stacks:
            st, p = O.project(s, pt, w, h, z, _lib.PROJECTION_MAX, 0, z - 1)
            planes.append(p)
        with O.semantics(flags):
            st, exp = O.render(chans, planes, pt, w, h, qdef=q)
        _assert_close(got, exp, tol)
        c.set_semantics(0)


@pytest.fixture(scope="module")
def k3r_ctx():
    c = _k3r_context()
    yield c
    c.close()


def _u16_ramps(h, w, seed, hi=65536):
    rng = np.random.default_rng(seed)
    planes = [rng.integers(0, hi, (h, w)).astype(np.uint16) for _ in range(3)]
    planes[0].reshape(-1)[:4096] = np.arange(4096)
    return planes


def test_log_unguarded_integer_paths(sem_ctx, k3r_ctx):
    h, w = 64, 256
    planes = _u16_ramps(h, w, 31)
    chans = [{"input_start": 0.0, "input_end": 5000.0, "global_min": 0.0, "global_max": 65535.0,
              "family": _lib.FAMILY_LOGARITHMIC, "rgba": PRIMARY[0]},
             {"input_start": 300.0, "input_end": 40000.0, "global_min": 0.0, "global_max": 65535.0,
              "family": _lib.FAMILY_LOGARITHMIC, "rgba": PRIMARY[1]},
             {"input_start": 0.0, "input_end": 65535.0, "global_min": 0.0, "global_max": 65535.0,
              "rgba": PRIMARY[2]}]
    a = _every_path(sem_ctx, 0, chans, planes, _lib.PIXELS_UINT16, w, h, tol=1)
    b = _every_path(sem_ctx, _lib.SEM_LOG_UNGUARDED, chans, planes, _lib.PIXELS_UINT16, w, h, tol=1)
    assert (((a >> 16) & 0xFF) != ((b >> 16) & 0xFF)).any()      # window from 0: -inf start
    np.testing.assert_array_equal((a >> 8) & 0xFF, (b >> 8) & 0xFF)  # window inside x > 0: unchanged
    i16 = [(p.astype(np.int32) - 32768).astype(np.int16) for p in planes]
    ci = [dict(c, global_min=-32768.0, global_max=32767.0) for c in chans]
    ci[0].update(input_start=-100.0, input_end=3000.0)
    _every_path(sem_ctx, _lib.SEM_LOG_UNGUARDED, ci, i16, _lib.PIXELS_INT16, w, h, tol=1)
    u8 = [(p & 0xFF).astype(np.uint8) for p in planes]
    c8 = [dict(c, input_start=0.0, input_end=200.0, global_max=255.0) for c in chans]
    _every_path(sem_ctx, _lib.SEM_LOG_UNGUARDED, c8, u8, _lib.PIXELS_UINT8, w, h, tol=1)
    z = 5
    stacks = [np.stack([np.roll(p, k) for k in range(z)]) for p in planes]
    _glue_paths(sem_ctx, k3r_ctx, _lib.SEM_LOG_UNGUARDED, chans, stacks, _lib.PIXELS_UINT16, w, h, z, tol=1)


def test_log_unguarded_float_paths(sem_ctx):
    """Threshold mode (window above 0) and Eval mode (window from / below 0) under the switch."""
    h, w = 64, 256
    rng = np.random.default_rng(5)
    planes = [rng.uniform(-50, 6000, (h, w)).astype(np.float32) for _ in range(3)]
    planes[0].reshape(-1)[:8] = [0.0, -0.0, -1.0, 1e-30, np.inf, -np.inf, np.nan, 1.0]
    chans = [{"input_start": -10.0, "input_end": 100.0, "family": _lib.FAMILY_LOGARITHMIC, "rgba": PRIMARY[0]},
             {"input_start": 1.5, "input_end": 5000.0, "family": _lib.FAMILY_LOGARITHMIC, "rgba": PRIMARY[1]},
             {"input_start": 0.0, "input_end": 3000.0, "family": _lib.FAMILY_LOGARITHMIC, "rgba": PRIMARY[2]}]
    a = _every_path(sem_ctx, 0, chans, planes, _lib.PIXELS_FLOAT, w, h, tol=1)
    b = _every_path(sem_ctx, _lib.SEM_LOG_UNGUARDED, chans, planes, _lib.PIXELS_FLOAT, w, h, tol=1)
    assert (a != b).any()


@pytest.mark.parametrize("pt", [_lib.PIXELS_UINT16, _lib.PIXELS_INT16, _lib.PIXELS_UINT8, _lib.PIXELS_FLOAT])
def test_noise_reduction_off_paths(sem_ctx, k3r_ctx, pt):
    """Linear family with noise reduction: bit-exact on every path, with and without the switch."""
    h, w = 64, 256
    planes = _u16_ramps(h, w, 44)
    if pt == _lib.PIXELS_INT16:
        planes = [(p.astype(np.int32) - 32768).astype(np.int16) for p in planes]
        lo, hi = -32768.0, 32767.0
    elif pt == _lib.PIXELS_UINT8:
        planes = [(p & 0xFF).astype(np.uint8) for p in planes]
        lo, hi = 0.0, 255.0
    elif pt == _lib.PIXELS_FLOAT:
        planes = [p.astype(np.float32) * np.float32(0.37) for p in planes]
        lo, hi = 0.0, 0.0
    else:
        lo, hi = 0.0, 65535.0
    span = (hi - lo) if hi > lo else 24000.0
    chans = [{"input_start": lo + 0.1 * span, "input_end": lo + 0.6 * span, "global_min": lo, "global_max": hi,
              "noise_reduction": True, "rgba": PRIMARY[c]} for c in range(3)]
    chans[2]["noise_reduction"] = False
    chans[1]["reverse"] = True
    a = _every_path(sem_ctx, 0, chans, planes, pt, w, h, tol=0)
    b = _every_path(sem_ctx, _lib.SEM_NOISE_REDUCTION_OFF, chans, planes, pt, w, h, tol=0)
    assert (a != b).any()
    np.testing.assert_array_equal(a & 0xFF, b & 0xFF)    # channel without noise reduction unchanged
    if pt != _lib.PIXELS_FLOAT:
        z = 4
        stacks = [np.stack([np.roll(p, 3 * k) for k in range(z)]) for p in planes]
        _glue_paths(sem_ctx, k3r_ctx, _lib.SEM_NOISE_REDUCTION_OFF, chans, stacks, pt, w, h, z, tol=0)


@pytest.mark.parametrize("pt", [_lib.PIXELS_UINT16, _lib.PIXELS_FLOAT, _lib.PIXELS_UINT32])
def test_exp_normalized_paths(sem_ctx, k3r_ctx, pt):
    h, w = 64, 256
    planes = _u16_ramps(h, w, 71)
    if pt == _lib.PIXELS_FLOAT:
        planes = [p.astype(np.float32) / np.float32(600.0) - np.float32(5.0) for p in planes]
        wins = [(-5.0, 50.0), (1.0, 20.0), (0.0, 100.0)]
    elif pt == _lib.PIXELS_UINT32:
        planes = [p.astype(np.uint32) * np.uint32(3) for p in planes]
        wins = [(0.0, 196605.0), (1000.0, 9000.0), (50.0, 120000.0)]
    else:
        wins = [(0.0, 65535.0), (1000.0, 2000.0), (100.0, 30000.0)]
    ks = [1.0, 0.5, 2.0]
    chans = [{"input_start": s, "input_end": e, "global_min": 0.0, "global_max": 65535.0 if pt == _lib.PIXELS_UINT16 else 0.0,
              "family": _lib.FAMILY_EXPONENTIAL, "coefficient": k, "rgba": PRIMARY[c]}
             for c, ((s, e), k) in enumerate(zip(wins, ks))]
    a = _every_path(sem_ctx, 0, chans, planes, pt, w, h, tol=1)
    b = _every_path(sem_ctx, _lib.SEM_EXP_NORMALIZED, chans, planes, pt, w, h, tol=1)
    assert len(np.unique((b >> 16) & 0xFF)) > 100 and (a != b).any()
    if pt == _lib.PIXELS_UINT16:
        z = 3
        stacks = [np.stack([np.roll(p, 5 * k) for k in range(z)]) for p in planes]
        _glue_paths(sem_ctx, k3r_ctx, _lib.SEM_EXP_NORMALIZED, chans, stacks, pt, w, h, z, tol=1)


def _mask_png_indices(png):
    from PIL import Image
    im = Image.open(io.BytesIO(png))
    return (np.asarray(im.convert("RGBA"))[..., 3] > 0).astype(np.uint8)


@pytest.mark.parametrize("w,h", [(8, 2), (64, 33), (1024, 1024), (37, 21)])
@pytest.mark.parametrize("fh,fv", [(True, False), (False, True), (True, True)])
def test_mask_packed_flip(sem_ctx, w, h, fh, fv):
    """Default: the reference's packed-buffer flip (404 for a w*h/8-byte mask when w % 8 == 0);
    OMR_SEM_MASK_PIXEL_FLIP: pixel flip.  Width % 8 != 0 unpacks first: both settings agree."""
    rng = np.random.default_rng(w * 31 + h)
    bits = rng.integers(0, 256, (w * h + 7) // 8, dtype=np.uint8).tobytes()
    rgba = (255, 0, 0, 255)
    for flags in (0, _lib.SEM_MASK_PIXEL_FLIP):
        sem_ctx.set_semantics(flags)
        with O.semantics(flags):
            st, idx = O.mask_indices(bits, w, h, fh, fv)
        if st:
            assert st == _lib.NOT_FOUND and w % 8 == 0 and flags == 0
            with pytest.raises(_lib.OmrError) as e:
                sem_ctx.render_shape_mask_png(bits, w, h, rgba, fh, fv)
            assert e.value.status == _lib.NOT_FOUND
            continue
        png = sem_ctx.render_shape_mask_png(bits, w, h, rgba, fh, fv)
        np.testing.assert_array_equal(_mask_png_indices(png), idx)
    if w % 8 == 0 and w * h <= 4096:
        # a mask array of >= w*h bytes: the reference's byte flip succeeds and its first w*h/8
        # bytes render as packed bits
        big = rng.integers(0, 256, w * h + 3, dtype=np.uint8).tobytes()
        sem_ctx.set_semantics(0)
        st, idx = O.mask_indices(big, w, h, fh, fv)
        assert st == 0
        png = sem_ctx.render_shape_mask_png(big, w, h, rgba, fh, fv)
        np.testing.assert_array_equal(_mask_png_indices(png), idx)
    sem_ctx.set_semantics(0)


def test_mask_reference_failures_are_not_found(sem_ctx):
    for bits, w, h in ((bytes([0xFF]), 4, 4), (bytes([0xFF]), 0, 4), (b"", 8, 1)):
        with pytest.raises(_lib.OmrError) as e:
            sem_ctx.render_shape_mask_png(bits, w, h, (1, 2, 3, 4))
        assert e.value.status == _lib.NOT_FOUND
