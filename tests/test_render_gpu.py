"""Parity of the HIP render path (K1+K2 through the C ABI) against the CPU restatement.

Bar (BASELINE.json north_star): packed ARGB bit-exact for integer pixel types; float32 and
transcendental families (log/exp/poly LUTs built on the device) within +-1 code value per
channel contribution.
"""
import numpy as np
import pytest

import oracle_lib as O
from omr import _lib
from omr.renderer import f32
from omr.synthetic import C2_COLORS, C2_WINDOWS, c2_channels, c5_channels, c5_planes, tile_u16

pytestmark = pytest.mark.gpu


def dev(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1)).to("cuda")


def host_render(ctx, channels, planes, pt, w, h, **kw):
    q = O.make_qdef(kw.pop("model", "rgb"))
    return ctx.render_packed_int(q, channels, planes, pt, w, h, **kw)


def assert_argb_close(got, exp, tol):
    if tol == 0:
        np.testing.assert_array_equal(got, exp)
        return
    g = got.view(np.uint8).astype(int)
    e = exp.view(np.uint8).astype(int)
    assert np.abs(g - e).max() <= tol, f"max diff {np.abs(g - e).max()}"


@pytest.mark.parametrize("be", [False, True])
@pytest.mark.parametrize("flip", [(False, False), (True, False), (False, True), (True, True)])
def test_c2_u16_four_channel_bit_exact(ctx, be, flip):
    h, w = 96, 128
    planes = tile_u16(0, 4, h, w)
    src = [O.np.ascontiguousarray(p.astype(">u2") if be else p) for p in planes]
    chans = c2_channels(4)
    st, exp = O.render(chans, src, _lib.PIXELS_UINT16, w, h, big_endian=be, flip_h=flip[0], flip_v=flip[1])
    assert st == 0
    got = host_render(ctx, chans, src, _lib.PIXELS_UINT16, w, h, big_endian=be, flip_h=flip[0], flip_v=flip[1])
    np.testing.assert_array_equal(got, exp)


def test_u16_uniform_every_lut_entry(ctx):
    h, w = 256, 256   # 65536 pixels: every uint16 value once per channel
    rng = np.random.default_rng(7)
    planes = [rng.permutation(65536).astype(np.uint16).reshape(h, w) for _ in range(4)]
    chans = c2_channels(4)
    for c, (s, e) in enumerate([(0.0, 65535.0), (1755.0, 51199.0), (3218.5, 26623.25), (65534.0, 65535.0)]):
        chans[c]["input_start"], chans[c]["input_end"] = f32(s), f32(e)
    st, exp = O.render(chans, planes, _lib.PIXELS_UINT16, w, h)
    assert st == 0
    np.testing.assert_array_equal(host_render(ctx, chans, planes, _lib.PIXELS_UINT16, w, h), exp)


@pytest.mark.parametrize("pt", [_lib.PIXELS_UINT16, _lib.PIXELS_INT16])
@pytest.mark.parametrize("windows", [
    [(60000.3, 60010.7), (65000.5, 65001.25), (-5.0, 3.0), (0.0, 1.0)],          # steep: many skipped values
    [(12.25, 65535.0), (-70000.0, 70000.0), (30000.0, 30000.5), (1.0, 65536.0)],
    [(-32768.0, 32767.0), (-100.5, -99.75), (32000.0, 40000.0), (-40000.0, -32000.0)],
])
def test_16bit_every_index_fast_path_windows(ctx, pt, windows):
    """Every raw 16-bit value through windows that stress the fp32 estimate + exact-proof path."""
    h, w = 256, 256
    rng = np.random.default_rng(99)
    raw = [rng.permutation(65536).astype(np.uint16).reshape(h, w) for _ in range(4)]
    planes = [r.view(np.int16) if pt == _lib.PIXELS_INT16 else r for r in raw]
    lo, hi = (-32768, 32767) if pt == _lib.PIXELS_INT16 else (0, 65535)
    chans = c2_channels(4)
    for c, (s, e) in enumerate(windows):
        chans[c].update(input_start=f32(s), input_end=f32(e), global_min=lo, global_max=hi)
    for be in (False, True):
        src = [p.astype(p.dtype.newbyteorder(">")) if be else p for p in planes]
        st, exp = O.render(chans, src, pt, w, h, big_endian=be)
        assert st == 0
        np.testing.assert_array_equal(host_render(ctx, chans, src, pt, w, h, big_endian=be), exp)


@pytest.mark.parametrize("pt,dtype,lo,hi", [
    (_lib.PIXELS_UINT8, np.uint8, 0, 255), (_lib.PIXELS_INT8, np.int8, -128, 127),
    (_lib.PIXELS_INT16, np.int16, -32768, 32767), (_lib.PIXELS_UINT16, np.uint16, 0, 65535)])
@pytest.mark.parametrize("model", ["rgb", "greyscale"])
def test_integer_types_windows_reverse(ctx, pt, dtype, lo, hi, model):
    h, w = 40, 72
    rng = np.random.default_rng(11)
    planes = [rng.integers(lo, hi + 1, size=(h, w)).astype(dtype) for _ in range(3)]
    span = hi - lo
    chans = [
        {"input_start": f32(lo + 0.1 * span), "input_end": f32(lo + 0.8 * span), "global_min": lo,
         "global_max": hi, "rgba": (255, 128, 7, 255), "reverse": True},
        {"input_start": f32(lo), "input_end": f32(hi), "global_min": lo, "global_max": hi,
         "rgba": (0, 255, 0, 200)},
        {"input_start": f32(lo + 0.33 * span), "input_end": f32(lo + 0.34 * span), "global_min": lo,
         "global_max": hi, "rgba": (255, 255, 255, 255)},
    ]
    for be in (False, True):
        src = [p.astype(p.dtype.newbyteorder(">")) if be else p for p in planes]
        st, exp = O.render(chans, src, pt, w, h, model=model, big_endian=be)
        assert st == 0
        got = host_render(ctx, chans, src, pt, w, h, model=model, big_endian=be)
        np.testing.assert_array_equal(got, exp)


def test_lut_colour_inactive_and_ragged_width(ctx):
    h, w = 33, 37   # width % 8 != 0 -> scalar path
    planes = tile_u16(3, 3, h, w)
    lut = np.concatenate([np.arange(256), 255 - np.arange(256), (np.arange(256) * 7) % 256]).astype(np.uint8)
    chans = c2_channels(3)
    chans[1]["active"] = False
    chans[2]["lut"] = lut
    for flip in [(False, False), (True, True)]:
        st, exp = O.render(chans, planes, _lib.PIXELS_UINT16, w, h, flip_h=flip[0], flip_v=flip[1])
        got = host_render(ctx, chans, planes, _lib.PIXELS_UINT16, w, h, flip_h=flip[0], flip_v=flip[1])
        np.testing.assert_array_equal(got, exp)


def test_region_of_larger_plane_row_stride(ctx):
    H, W = 64, 100
    planes = tile_u16(5, 2, H, W)
    x0, y0, w, h = 12, 9, 64, 40
    chans = c2_channels(2)
    regions = [np.ascontiguousarray(p[y0:y0 + h, x0:x0 + w]) for p in planes]
    st, exp = O.render(chans, regions, _lib.PIXELS_UINT16, w, h)
    views = [p[y0:, x0:] for p in planes]   # base pointer at the region start
    import ctypes
    q = O.make_qdef("rgb")
    arr, keep = O.make_bindings(chans)
    ptrs = (ctypes.c_void_p * 2)(*[v.__array_interface__["data"][0] for v in views])
    out = np.empty((h, w), np.uint32)
    assert _lib.lib.omr_render_packed_int(ctx.h, ctypes.byref(q), arr, 2, ptrs, W, _lib.PIXELS_UINT16, 0,
                                          w, h, 0, 0, out.ctypes.data) == 0
    np.testing.assert_array_equal(out, exp)


@pytest.mark.parametrize("family,k", [(_lib.FAMILY_POLYNOMIAL, 2.0), (_lib.FAMILY_POLYNOMIAL, 0.5),
                                      (_lib.FAMILY_LOGARITHMIC, 1.0), (_lib.FAMILY_EXPONENTIAL, 0.25)])
def test_u16_nonlinear_families_lut_path(ctx, family, k):
    h, w = 64, 64
    planes = tile_u16(9, 2, h, w, uniform=True)
    chans = c2_channels(2)
    for c in chans:
        c["family"], c["coefficient"] = family, k
    st, exp = O.render(chans, planes, _lib.PIXELS_UINT16, w, h)
    got = host_render(ctx, chans, planes, _lib.PIXELS_UINT16, w, h)
    np.testing.assert_array_equal(got, exp)       # the byte LUT is built on the host: exact


def test_noise_reduction_linear_exact(ctx):
    h, w = 64, 64
    planes = tile_u16(10, 2, h, w, uniform=True)
    chans = c2_channels(2)
    chans[0]["noise_reduction"] = True
    st, exp = O.render(chans, planes, _lib.PIXELS_UINT16, w, h)
    np.testing.assert_array_equal(host_render(ctx, chans, planes, _lib.PIXELS_UINT16, w, h), exp)


def test_c5_float32_log_poly_reverse_lut(ctx):
    h, w = 64, 96
    rng = np.random.default_rng(20261015 + 5)
    planes = c5_planes(h, w, rng)
    chans = c5_channels(planes)
    for be in (False, True):
        src = [p.astype(">f4") if be else p for p in planes]
        st, exp = O.render(chans, src, _lib.PIXELS_FLOAT, w, h, big_endian=be)
        assert st == 0
        got = host_render(ctx, chans, src, _lib.PIXELS_FLOAT, w, h, big_endian=be)
        # every C5 channel is in threshold mode (monotone q) and its code thresholds come from the
        # host libm, as the restatement's q does: bit-exact, inside north_star's +-1 float bar
        np.testing.assert_array_equal(got, exp)
        for c in range(3):                           # each channel alone, greyscale -> its code value v
            solo = [dict(ch, active=(i == c)) for i, ch in enumerate(chans)]
            st, e1 = O.render(solo, src, _lib.PIXELS_FLOAT, w, h, big_endian=be, model="greyscale")
            g1 = host_render(ctx, solo, src, _lib.PIXELS_FLOAT, w, h, big_endian=be, model="greyscale")
            np.testing.assert_array_equal(g1, e1)


def test_c5_full_size_strided_batch(ctx):
    """C5 at BASELINE size (3ch float32 1024^2, BE) through the strided batch API the bench
    times: the composite and each channel alone (greyscale) bit-exact vs the restatement."""
    import torch
    h = w = 1024
    rng = np.random.default_rng(20261015 + 5)
    planes = c5_planes(h, w, rng)
    chans = c5_channels(planes)
    src = [p.astype(">f4") for p in planes]
    blob = np.concatenate([s.view(np.uint8).reshape(-1) for s in src])
    d = torch.from_numpy(np.concatenate([blob, blob])).to("cuda")          # 2 identical tiles
    plane = h * w * 4
    for model, cs in [("rgb", chans)] + [("greyscale", [dict(ch, active=(i == c)) for i, ch in enumerate(chans)])
                                           for c in range(3)]:
        out = torch.empty((2, h, w), dtype=torch.int32, device="cuda")
        ctx.render_batch_strided_device(O.make_qdef(model), cs, d, 3 * plane, plane, 2, _lib.PIXELS_FLOAT, w, h,
                                        out, big_endian=True)
        ctx.synchronize()
        got = out.cpu().numpy().view(np.uint32)
        st, exp = O.render(cs, src, _lib.PIXELS_FLOAT, w, h, big_endian=True, model=model)
        assert st == 0
        np.testing.assert_array_equal(got[0], got[1])
        # north_star's float32 bar is +-1 code value on the packed ARGB; the threshold mode is
        # exact (host-built code thresholds), so the measured maximum difference is 0
        diff = max(int(np.abs(((got[0] >> sh) & 0xFF).astype(int) - ((exp >> sh) & 0xFF).astype(int)).max())
                   for sh in (0, 8, 16))
        assert diff == 0, f"{model}: max ARGB component diff {diff}"
        if model == "greyscale":
            assert len(np.unique(exp & 0xFF)) > 200          # every channel spans the codomain


def test_float_linear_and_int32_double_exact(ctx):
    h, w = 32, 48
    rng = np.random.default_rng(3)
    cases = [(_lib.PIXELS_FLOAT, rng.normal(100, 50, (h, w)).astype(np.float32)),
             (_lib.PIXELS_DOUBLE, rng.normal(100, 50, (h, w))),
             (_lib.PIXELS_INT32, rng.integers(-1000, 1000, (h, w)).astype(np.int32)),
             (_lib.PIXELS_UINT32, rng.integers(0, 3_000_000_000, (h, w), dtype=np.uint64).astype(np.uint32))]
    for pt, p in cases:
        lo, hi = np.percentile(p, 5), np.percentile(p, 95)
        chans = [{"input_start": f32(lo), "input_end": f32(hi), "rgba": (10, 200, 255, 255), "reverse": True}]
        for be in (False, True):
            src = [p.astype(p.dtype.newbyteorder(">")) if be else p]
            st, exp = O.render(chans, src, pt, w, h, big_endian=be)
            np.testing.assert_array_equal(host_render(ctx, chans, src, pt, w, h, big_endian=be), exp)


def test_greyscale_first_active_only_and_no_active(ctx):
    h, w = 16, 24
    planes = tile_u16(2, 3, h, w)
    chans = c2_channels(3)
    chans[0]["active"] = False
    st, exp = O.render(chans, planes, _lib.PIXELS_UINT16, w, h, model="greyscale")
    np.testing.assert_array_equal(host_render(ctx, chans, planes, _lib.PIXELS_UINT16, w, h, model="greyscale"), exp)
    for c in chans:
        c["active"] = False
    for model in ("rgb", "greyscale"):
        st, exp = O.render(chans, planes, _lib.PIXELS_UINT16, w, h, model=model)
        got = host_render(ctx, chans, planes, _lib.PIXELS_UINT16, w, h, model=model)
        np.testing.assert_array_equal(got, exp)
        assert (got == 0xFF000000).all()


def test_quantization_exception_outside_lut_domain(ctx):
    h, w = 8, 16
    p = np.full((h, w), 1000, np.uint16)
    p[3, 5] = 60000
    chans = [{"input_start": 0.0, "input_end": 50000.0, "global_min": 0, "global_max": 50000, "rgba": (255, 0, 0, 255)}]
    st, _ = O.render(chans, [p], _lib.PIXELS_UINT16, w, h)
    assert st == _lib.QUANTIZATION
    with pytest.raises(_lib.OmrError) as ei:
        host_render(ctx, chans, [p], _lib.PIXELS_UINT16, w, h)
    assert ei.value.status == _lib.QUANTIZATION
    # context is usable again afterwards
    p[3, 5] = 7
    st, exp = O.render(chans, [p], _lib.PIXELS_UINT16, w, h)
    np.testing.assert_array_equal(host_render(ctx, chans, [p], _lib.PIXELS_UINT16, w, h), exp)


def test_batch_device_per_tile_status_and_results(ctx):
    import torch
    h, w, n = 64, 64, 5
    chans = c2_channels(4)
    for c in chans:
        c["global_max"] = 60000.0
    tiles = [[np.minimum(p, 50000) for p in tile_u16(100 + t, 4, h, w)] for t in range(n)]
    tiles[3][1][0, 0] = 65000          # outside [0, 60000] -> QuantizationException for tile 3
    big = [[p.astype(">u2") for p in t] for t in tiles]
    dbufs = [[dev(p) for p in t] for t in big]
    table = torch.tensor([[b.data_ptr() for b in t] for t in dbufs], dtype=torch.int64, device="cuda")
    out = torch.empty((n, h, w), dtype=torch.int32, device="cuda")
    status = torch.full((n,), -1, dtype=torch.int32, device="cuda")
    ctx.render_batch_device(O.make_qdef("rgb"), chans, table, n, _lib.PIXELS_UINT16, w, h, out, status,
                            big_endian=True, flip_h=True)
    with pytest.raises(_lib.OmrError):
        ctx.synchronize()
    st = status.cpu().numpy()
    assert list(st) == [0, 0, 0, _lib.QUANTIZATION, 0]
    got = out.cpu().numpy().view(np.uint32)
    for t in range(n):
        if t == 3:
            continue
        s, exp = O.render(chans, big[t], _lib.PIXELS_UINT16, w, h, big_endian=True, flip_h=True)
        np.testing.assert_array_equal(got[t], exp)


def test_batch_strided_matches_table(ctx):
    import torch
    h, w, n = 48, 64, 6
    chans = c2_channels(3)
    tiles = [[p.astype(">u2") for p in tile_u16(200 + t, 3, h, w)] for t in range(n)]
    raw = b"".join(p.tobytes() for t in tiles for p in t)             # big-endian bytes, [tile][chan]
    data = torch.frombuffer(bytearray(raw), dtype=torch.uint8).to("cuda")
    plane = h * w * 2
    out = torch.empty((n, h, w), dtype=torch.int32, device="cuda")
    ctx.render_batch_strided_device(O.make_qdef("rgb"), chans, data, 3 * plane, plane, n, _lib.PIXELS_UINT16, w, h,
                                    out, big_endian=True, flip_v=True)
    ctx.synchronize()
    got = out.cpu().numpy().view(np.uint32)
    for t in range(n):
        st, exp = O.render(chans, tiles[t], _lib.PIXELS_UINT16, w, h, big_endian=True, flip_v=True)
        np.testing.assert_array_equal(got[t], exp)


def test_device_api_matches_host_api(ctx):
    import torch
    h, w = 128, 256
    planes = [p.astype(">u2") for p in tile_u16(42, 4, h, w)]
    chans = c2_channels(4)
    out = torch.empty((h, w), dtype=torch.int32, device="cuda")
    ctx.render_packed_int_device(O.make_qdef("rgb"), chans, [dev(p) for p in planes], _lib.PIXELS_UINT16, w, h,
                                 out, big_endian=True, flip_v=True)
    ctx.synchronize()
    st, exp = O.render(chans, planes, _lib.PIXELS_UINT16, w, h, big_endian=True, flip_v=True)
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32), exp)


def test_invalid_arguments(ctx):
    chans = c2_channels(1)
    p = np.zeros((4, 4), np.uint16)
    with pytest.raises(_lib.OmrError) as ei:
        host_render(ctx, chans, [p], _lib.PIXELS_UINT16, 0, 4, flip_h=True)
    assert ei.value.status == _lib.INVALID_ARGUMENT
    with pytest.raises(_lib.OmrError):
        host_render(ctx, chans, [None], _lib.PIXELS_UINT16, 4, 4)
    with pytest.raises(_lib.OmrError):
        host_render(ctx, chans, [p], 99, 4, 4)
    # zero-size region without a flip renders nothing and succeeds (renderAsPackedInt -> int[0])
    assert host_render(ctx, chans, [p], _lib.PIXELS_UINT16, 0, 0).size == 0


def _edge_values(ch, pt, qd, n=65536):
    """Pixel values that pin every code boundary of q for one channel: the oracle's codes over
    a dense sweep of the window, every value where the code changes with its type neighbours,
    the window ends and the type's specials (NaN, +-inf, -0, extremes)."""
    ws, we = ch["input_start"], ch["input_end"]
    span = we - ws
    if pt == _lib.PIXELS_FLOAT:
        sweep = np.linspace(ws - 0.05 * span, we + 0.05 * span, 40000).astype(np.float32)
        dt = np.float32
    else:
        info = np.iinfo(np.int32 if pt == _lib.PIXELS_INT32 else np.uint32)
        sweep = np.unique(np.clip(np.linspace(ws - 0.05 * span, we + 0.05 * span, 40000),
                                  info.min, info.max).astype(np.int64)).astype(np.int32 if pt == _lib.PIXELS_INT32 else np.uint32)
        dt = sweep.dtype
    codes = np.array([O.quantize(float(x), ch) for x in sweep[:: max(1, len(sweep) // 4000)]])
    sub = sweep[:: max(1, len(sweep) // 4000)]
    edges = sub[1:][np.diff(codes) != 0]
    vals = [sweep, edges]
    if pt == _lib.PIXELS_FLOAT:
        for e in (edges, np.float32([ws, we])):
            vals += [np.nextafter(e, np.float32(np.inf)), np.nextafter(e, np.float32(-np.inf))]
        vals.append(np.float32([np.nan, -np.nan, np.inf, -np.inf, 0.0, -0.0, 3.4e38, -3.4e38, 1e-45]))
    else:
        info = np.iinfo(dt)
        vals += [(edges.astype(np.int64) + d).clip(info.min, info.max).astype(dt) for d in (-1, 1)]
        vals.append(np.array([info.min, info.max, 0, 1, info.max - 1], dtype=dt))
    v = np.concatenate([np.asarray(a, dtype=dt) for a in vals])
    return np.resize(v, n).astype(dt)


@pytest.mark.parametrize("case", [
    dict(pt=_lib.PIXELS_FLOAT, ws=-100.5, we=1000.25),
    dict(pt=_lib.PIXELS_FLOAT, ws=-100.5, we=1000.25, noise_reduction=True),
    dict(pt=_lib.PIXELS_FLOAT, ws=3.0, we=700.0, cd=(10, 200, 100)),
    # windows at / just above +0: the bucket origin lands at or next to key(+0), where K2 switches
    # between clamping the raw bits (origin >= key(+0)) and the key transform (round 6)
    dict(pt=_lib.PIXELS_FLOAT, ws=0.0, we=1.0),
    dict(pt=_lib.PIXELS_FLOAT, ws=1e-40, we=1e-38),
    dict(pt=_lib.PIXELS_FLOAT, ws=1e-30, we=3e-30, reverse=True),
    dict(pt=_lib.PIXELS_FLOAT, ws=1.5, we=5000.0, family=_lib.FAMILY_LOGARITHMIC),
    dict(pt=_lib.PIXELS_FLOAT, ws=0.1, we=900.0, family=_lib.FAMILY_POLYNOMIAL, coefficient=0.5),
    dict(pt=_lib.PIXELS_FLOAT, ws=2.0, we=300.0, family=_lib.FAMILY_POLYNOMIAL, coefficient=2.0),
    dict(pt=_lib.PIXELS_FLOAT, ws=0.5, we=50.0, family=_lib.FAMILY_EXPONENTIAL, coefficient=0.3),
    dict(pt=_lib.PIXELS_FLOAT, ws=-5.0, we=50.0, family=_lib.FAMILY_LOGARITHMIC, tol=1),   # Eval fallback
    dict(pt=_lib.PIXELS_FLOAT, ws=-700.0, we=650.0, family=_lib.FAMILY_POLYNOMIAL, coefficient=0.5),  # a0 NaN
    dict(pt=_lib.PIXELS_FLOAT, ws=-70.0, we=65.0, family=_lib.FAMILY_POLYNOMIAL, coefficient=2.0, tol=1),  # Eval
    dict(pt=_lib.PIXELS_INT32, ws=-1e9, we=2e9),
    dict(pt=_lib.PIXELS_INT32, ws=-7.0, we=250.0, reverse=True),
    dict(pt=_lib.PIXELS_UINT32, ws=1000.0, we=4e9),
    dict(pt=_lib.PIXELS_UINT32, ws=10.0, we=70000.0, family=_lib.FAMILY_LOGARITHMIC),
])
def test_threshold_mode_code_boundaries(ctx, case):
    """kModeThresh (monotone q through 255 LDS thresholds) against the CPU restatement at every
    code boundary, the window ends and NaN / inf / -0 / type extremes.  Threshold mode is
    bit-exact for every family (host-built thresholds, round 5); the Eval fallbacks (q not
    provably monotone: device log/pow) keep north_star's +-1 float bar, boundary flips only."""
    case = dict(case)
    pt, tol, cd = case.pop("pt"), case.pop("tol", 0), case.pop("cd", (0, 255, 255))
    ch = {"input_start": f32(case.pop("ws")), "input_end": f32(case.pop("we")), "rgba": (255, 255, 255, 255)}
    ch.update(case)
    qd = O.make_qdef("greyscale", cd[0], cd[1], cd[2])
    h, w = 64, 1024
    x = _edge_values(dict(ch), pt, qd, h * w).reshape(h, w)
    for be in (False, True):
        src = [x.astype(x.dtype.newbyteorder(">")) if be else x]
        st, exp = O.render([ch], src, pt, w, h, big_endian=be, qdef=qd)
        assert st == 0
        got = ctx.render_packed_int(qd, [ch], src, pt, w, h, big_endian=be)
        d = np.abs((got & 0xFF).astype(int) - (exp & 0xFF).astype(int))
        assert d.max() <= tol, f"max code diff {d.max()} at {x.reshape(-1)[np.argmax(d)]!r}"
        if tol:
            assert (d > 0).mean() < 0.01


def test_mixed_threshold_and_eval_channels(ctx):
    """One channel through thresholds (log, ws > 0), one through per-pixel double evaluation
    (x^2 over a window that crosses 0: not monotone) in the same launch; float and int32."""
    h, w = 64, 128
    rng = np.random.default_rng(31)
    for pt, dt in ((_lib.PIXELS_FLOAT, np.float32), (_lib.PIXELS_INT32, np.int32)):
        planes = [(rng.lognormal(4, 1.2, (h, w))).astype(dt), rng.normal(0, 50, (h, w)).astype(dt)]
        chans = [{"input_start": f32(5.0), "input_end": f32(900.0), "rgba": (255, 0, 0, 255),
                  "family": _lib.FAMILY_LOGARITHMIC},
                 {"input_start": f32(-60.0), "input_end": f32(70.0), "rgba": (0, 255, 255, 255),
                  "family": _lib.FAMILY_POLYNOMIAL, "coefficient": 2.0, "reverse": True}]
        for be in (False, True):
            src = [p.astype(p.dtype.newbyteorder(">")) if be else p for p in planes]
            st, exp = O.render(chans, src, pt, w, h, big_endian=be)
            got = host_render(ctx, chans, src, pt, w, h, big_endian=be)
            assert_argb_close(got, exp, tol=1)
            assert np.mean(got == exp) > 0.99


def test_back_to_back_settings_through_staging_ring(ctx):
    """More in-flight calls than the 8-slot parameter ring, each with its own windows, colours and
    flip, queued without a host sync: every output must carry its own call's settings (a reused
    slot must never feed a later call's plan to an earlier launch, or the reverse)."""
    import torch
    w, h = 96, 40
    planes = [p.astype(">u2") for p in tile_u16(11, 3, h, w)]
    dplanes = [dev(p) for p in planes]
    q = O.make_qdef("rgb")
    calls = []
    for i in range(21):
        chans = [{"active": True, "input_start": f32(100 * i + 50 * c), "input_end": f32(20000 + 1500 * i + 700 * c),
                  "global_min": 0.0, "global_max": 65535.0, "rgba": C2_COLORS[(i + c) % 4],
                  "reverse": (i + c) % 3 == 0} for c in range(3)]
        out = torch.empty((h, w), dtype=torch.int32, device="cuda")
        ctx.render_packed_int_device(q, chans, dplanes, _lib.PIXELS_UINT16, w, h, out, big_endian=True,
                                     flip_h=i % 2 == 1, flip_v=i % 5 == 0)
        calls.append((chans, out, i % 2 == 1, i % 5 == 0))
    ctx.synchronize()
    for i, (chans, out, fh, fv) in enumerate(calls):
        st, exp = O.render(chans, planes, _lib.PIXELS_UINT16, w, h, big_endian=True, flip_h=fh, flip_v=fv)
        assert st == 0
        np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32), exp, err_msg=f"call {i}")


@pytest.mark.parametrize("pt,na", [(_lib.PIXELS_UINT8, 1), (_lib.PIXELS_INT8, 2), (_lib.PIXELS_UINT16, 4),
                                   (_lib.PIXELS_INT16, 3)])
@pytest.mark.parametrize("n", [63, 64])
def test_small_and_full_launch_boundary(ctx, pt, na, n):
    """K2 runs one chunk per lane, with the contribution tables built in LDS instead of by K1,
    below 4 work blocks per CU (k2_small_launch: 256² 8/16-bit tiles give 8192 chunks, so 63
    tiles are small and 64 are not on a 256-CU part).  Both sides bit-exact against the oracle,
    with a reversed channel, a LUT channel and a flip."""
    import torch
    h = w = 256
    bpp = 1 if pt in (_lib.PIXELS_UINT8, _lib.PIXELS_INT8) else 2
    dt = {_lib.PIXELS_UINT8: np.uint8, _lib.PIXELS_INT8: np.int8, _lib.PIXELS_UINT16: np.uint16,
          _lib.PIXELS_INT16: np.int16}[pt]
    info = np.iinfo(dt)
    rng = np.random.default_rng(100 + pt * 10 + na)
    host = rng.integers(info.min, int(info.max) + 1, (n, na, h, w)).astype(dt)
    chans = c2_channels(na)
    for i, c in enumerate(chans):
        lo, hi = float(info.min), float(info.max)
        c["global_min"], c["global_max"] = lo, hi
        c["input_start"], c["input_end"] = f32(lo + (hi - lo) * 0.1 * (i + 1)), f32(hi - (hi - lo) * 0.05 * i)
    chans[0]["reverse"] = True
    if na > 1:
        chans[1]["lut"] = np.stack([np.arange(256), 255 - np.arange(256), np.arange(256) // 2], -1).astype(np.uint8)
    out = torch.empty((n, h, w), dtype=torch.int32, device="cuda")
    pb = h * w * bpp
    ctx.render_batch_strided_device(O.make_qdef("rgb"), chans, dev(host), na * pb, pb, n, pt, w, h, out,
                                    flip_h=True)
    got = out.cpu().numpy().view(np.uint32)
    for t in (0, n // 2, n - 1):
        st, exp = O.render(chans, [np.ascontiguousarray(host[t, c]) for c in range(na)], pt, w, h, flip_h=True)
        assert st == 0
        np.testing.assert_array_equal(got[t], exp, err_msg=f"tile {t}")


@pytest.mark.parametrize("pt,dtype,lo,hi", [(_lib.PIXELS_UINT8, np.uint8, 0, 256),
                                            (_lib.PIXELS_UINT16, np.uint16, 0, 65536),
                                            (_lib.PIXELS_INT16, np.int16, -32768, 32768),
                                            (_lib.PIXELS_FLOAT, np.float32, -100, 70000)])
def test_inverted_and_empty_windows(ctx, pt, dtype, lo, hi):
    """inputStart > inputEnd and inputStart == inputEnd: the lower end is tested first upstream,
    so below the start is cdStart even past the end, and the rest is cdEnd (a step at the start).
    Mixed with an ordinary window so every K2 mode path meets them (linear16 used to let the
    upper end win)."""
    w, h = 96, 40
    rng = np.random.default_rng(int(hi) & 0xFFFF)
    planes = [rng.integers(lo, hi, (h, w)).astype(dtype) for _ in range(3)]
    span = hi - lo
    for ws, we in [(lo + 0.8 * span, lo + 0.2 * span), (lo + 0.5 * span, lo + 0.5 * span),
                   (lo + 0.6 * span + 0.5, lo + 0.3 * span)]:
        chans = [{"input_start": f32(ws), "input_end": f32(we), "rgba": (255, 0, 0, 255)},
                 {"input_start": f32(lo + 0.1 * span), "input_end": f32(lo + 0.9 * span), "rgba": (0, 255, 0, 255)},
                 {"input_start": f32(we), "input_end": f32(ws), "rgba": (0, 0, 255, 255), "reverse": True}]
        if pt != _lib.PIXELS_FLOAT:
            for c in chans:
                c["global_min"], c["global_max"] = float(lo), float(hi - 1)
        got = host_render(ctx, chans, planes, pt, w, h)
        st, exp = O.render(chans, planes, pt, w, h)
        assert st == 0
        np.testing.assert_array_equal(got, exp, err_msg=f"window {ws}:{we}")


@pytest.mark.parametrize("lg,cpt", [("10", "-2"), ("11", "-1"), ("11", "-3"), ("10", "-3"), ("n1280", "-2"),
                                    ("n1792", "-2")])
def test_c5_bucket_and_pipe_variants_exact(lg, cpt, monkeypatch):
    """The measurement variants of the float threshold path (OMR_K2_BUCKETS_LG: buckets per
    channel, read per call; OMR_K2_EVAL_CPT: chunks per lane of the pipelined kernel, -3 two work
    blocks per workgroup, read at context creation) render the C5 composite bit-exact: coarser
    buckets only move keys between the one-read entries and the in-bucket searches."""
    import torch
    import omr
    h = w = 512
    rng = np.random.default_rng(20261015 + 7)
    planes = c5_planes(h, w, rng)
    chans = c5_channels(planes)
    src = [p.astype(">f4") for p in planes]
    blob = np.concatenate([s.view(np.uint8).reshape(-1) for s in src])
    n = 5                                                    # ragged against any work-block size
    d = torch.from_numpy(np.concatenate([blob] * n)).to("cuda")
    plane = h * w * 4
    st, exp = O.render(chans, src, _lib.PIXELS_FLOAT, w, h, big_endian=True, model="rgb")
    assert st == 0
    if lg.startswith("n"):
        monkeypatch.setenv("OMR_K2_BUCKETS", lg[1:])        # a bucket count, not a power of two
    else:
        monkeypatch.setenv("OMR_K2_BUCKETS_LG", lg)
    monkeypatch.setenv("OMR_K2_EVAL_CPT", cpt)
    c = omr.Context(0)
    try:
        out = torch.empty((n, h, w), dtype=torch.int32, device="cuda")
        c.render_batch_strided_device(O.make_qdef("rgb"), chans, d, 3 * plane, plane, n, _lib.PIXELS_FLOAT, w, h,
                                      out, big_endian=True)
        c.synchronize()
        got = out.cpu().numpy().view(np.uint32)
    finally:
        c.close()
    for t in range(n):
        np.testing.assert_array_equal(got[t], exp, err_msg=f"tile {t}")
