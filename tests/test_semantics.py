"""The OMR_SEM_* switches of the un-vendored upstream semantics, on the CPU restatement and the
host side of libomr.so (include/omr/omr.h).  Each switch is checked
against a hand-computed expectation, shown to change the output, and — for the JPEG tables —
pinned against PIL/libjpeg-turbo; plus the north-star JPEG bar: PSNR of the decoded JPEG vs the
source pixels within 0.1 dB of libjpeg-turbo at the same tables.
"""
import ctypes
import io

import numpy as np
import pytest

import oracle_lib as O
from omr import _lib
from omr.renderer import f32
from omr.synthetic import c2_channels, tile_u16

F = np.float32


def _ramp_u16(lo, n):
    return (np.arange(n, dtype=np.int64) + lo).astype(np.uint16).reshape(1, n)


def _chan(ws, we, **kw):
    d = {"input_start": f32(ws), "input_end": f32(we), "global_min": 0.0, "global_max": 65535.0,
         "rgba": (255, 255, 255, 255)}
    d.update(kw)
    return d


def _grey(argb):
    return (argb & 0xFF).astype(int)


def test_window_int_bounds_lut_types():
    """Window 100.5:200.5 on uint16: the default double compares quantize x=100 to cdStart and
    x=200 by the formula; (int)-cast bounds compute x=100 (round(2.55*-0.5) = -1 -> byte 255)
    and send x=200 to cdEnd."""
    px = _ramp_u16(95, 110)
    ch = [_chan(100.5, 200.5)]
    st, a = O.render(ch, [px], _lib.PIXELS_UINT16, 110, 1, model="greyscale")
    assert st == 0
    v = dict(zip(range(95, 205), _grey(a[0])))
    assert v[100] == 0 and v[101] == 1 and v[200] == 254 and v[201] == 255
    with O.semantics(_lib.SEM_WINDOW_INT_BOUNDS):
        st, b = O.render(ch, [px], _lib.PIXELS_UINT16, 110, 1, model="greyscale")
    w = dict(zip(range(95, 205), _grey(b[0])))
    assert w[99] == 0 and w[100] == 255 and w[101] == 1 and w[199] == 251 and w[200] == 255
    # integral windows: both rules agree
    ch2 = [_chan(100.0, 200.0)]
    st, c = O.render(ch2, [px], _lib.PIXELS_UINT16, 110, 1, model="greyscale")
    with O.semantics(_lib.SEM_WINDOW_INT_BOUNDS):
        st, d = O.render(ch2, [px], _lib.PIXELS_UINT16, 110, 1, model="greyscale")
    np.testing.assert_array_equal(c, d)


def test_window_int_bounds_leaves_float_types_alone():
    x = np.linspace(90, 210, 1000).astype(np.float32).reshape(1, -1)
    ch = [_chan(100.5, 200.5)]
    st, a = O.render(ch, [x], _lib.PIXELS_FLOAT, x.shape[1], 1, model="greyscale")
    with O.semantics(_lib.SEM_WINDOW_INT_BOUNDS):
        st, b = O.render(ch, [x], _lib.PIXELS_FLOAT, x.shape[1], 1, model="greyscale")
    np.testing.assert_array_equal(a, b)


def test_alpha_one_step_orders_agree_exhaustively():
    """(int)((c/255f * a/255f) * v) == (int)((c/255f * v) * a/255f) for every c, a, v in 0..255
    (float32): the multiply order inside one truncation needs no switch."""
    v = np.arange(256, dtype=F)
    for a in range(256):
        al = F(a) / F(255)
        ci = (np.arange(256, dtype=F) / F(255))[:, None]
        np.testing.assert_array_equal(((ci * al) * v).astype(np.int64), ((ci * v) * al).astype(np.int64))


def test_alpha_separate_truncation():
    """(int)((c/255f * a/255f) * v) vs (int)((int)(c/255f * v) * a/255f), float32 throughout."""
    px = np.arange(256, dtype=np.uint8).reshape(1, 256)
    rgba = (255, 129, 100, 101)
    ch = [{"input_start": 0.0, "input_end": 255.0, "global_min": 0.0, "global_max": 255.0, "rgba": rgba}]
    c = np.array(rgba[:3], F) / F(255)
    al = F(rgba[3]) / F(255)
    v = np.arange(256, dtype=F)
    exp_default = np.stack([((ci * al) * v).astype(np.int64) for ci in c], -1)
    exp_after = np.stack([((ci * v).astype(np.int32).astype(F) * al).astype(np.int64) for ci in c], -1)
    assert (exp_default != exp_after).any()
    for flags, exp in ((0, exp_default), (_lib.SEM_ALPHA_SEPARATE, exp_after)):
        with O.semantics(flags):
            st, a = O.render(ch, [px], _lib.PIXELS_UINT8, 256, 1)
        got = np.stack([(a[0] >> 16) & 0xFF, (a[0] >> 8) & 0xFF, a[0] & 0xFF], -1).astype(np.int64)
        np.testing.assert_array_equal(got, exp)


def test_greyscale_lut():
    px = np.arange(256, dtype=np.uint8).reshape(1, 256)
    lut = np.concatenate([255 - np.arange(256), np.arange(256) // 3, np.full(256, 17)]).astype(np.uint8)
    ch = [{"input_start": 0.0, "input_end": 255.0, "global_min": 0.0, "global_max": 255.0, "lut": lut}]
    st, a = O.render(ch, [px], _lib.PIXELS_UINT8, 256, 1, model="greyscale")
    assert ((a[0] >> 16) & 0xFF).tolist() == list(range(256))          # LUT ignored
    with O.semantics(_lib.SEM_GREYSCALE_LUT):
        st, b = O.render(ch, [px], _lib.PIXELS_UINT8, 256, 1, model="greyscale")
    assert ((b[0] >> 16) & 0xFF).tolist() == lut[:256].tolist()
    assert ((b[0] >> 8) & 0xFF).tolist() == lut[256:512].tolist()
    assert (b[0] & 0xFF).tolist() == lut[512:].tolist()


def _java_tables(q, div2):
    std_l = [16, 11, 10, 16, 24, 40, 51, 61, 12, 12, 14, 19, 26, 58, 60, 55, 14, 13, 16, 24, 40, 57, 69, 56,
             14, 17, 22, 29, 51, 87, 80, 62, 18, 22, 37, 56, 68, 109, 103, 77, 24, 35, 55, 64, 81, 104, 113, 92,
             49, 64, 78, 87, 103, 121, 120, 101, 72, 92, 95, 98, 112, 100, 103, 99]
    std_c = [17, 18, 24, 47] + [99] * 4 + [18, 21, 26, 66] + [99] * 4 + [24, 26, 56] + [99] * 5 + [47, 66] + [99] * 38
    qf = F(min(max(q, 0.01) if q > 0 else 0.01, 1.0))
    qf = F(0.5) / qf if qf < F(0.5) else F(2) - qf * F(2)
    sc = lambda t, s: [int(min(255, max(1, int(F(v) * F(s) + F(0.5))))) for v in t]   # noqa: E731
    base_c = sc(std_c, 0.5) if div2 else std_c
    return sc(std_l, qf), sc(base_c, qf)


@pytest.mark.parametrize("q", [0.05, 0.3, 0.75, 0.85, 0.9, 1.0])
def test_jpeg_chroma_table_switch(q):
    for div2, flags in ((False, 0), (True, _lib.SEM_JPEG_CHROMA_DIV2)):
        el, ec = _java_tables(q, div2)
        with O.semantics(flags):
            ol, oc = O.quant_tables(q)
        assert ol.tolist() == el and oc.tolist() == ec
        gl = (ctypes.c_uint8 * 64)()
        gc = (ctypes.c_uint8 * 64)()
        assert _lib.lib.omr_jpeg_quant_tables_sem(F(q), flags, gl, gc) == 0
        assert list(gl) == el and list(gc) == ec

def test_jpeg_q075_equals_the_writers_default_tables():
    """The JDK writer's MODE_DEFAULT tables are K1Div2Luminance / K2Div2Chrominance (the Annex K
    tables scaled by 0.5f).  An explicit q = 0.75 (linear scale 0.5) reproduces that pair under
    the default switch setting; under OMR_SEM_JPEG_CHROMA_DIV2 its chroma is halved twice."""
    half_l, _ = _java_tables(0.75, False)
    el, ec = _java_tables(0.75, False)
    dl, dc = _java_tables(0.75, True)
    k2div2 = _java_tables(0.75, True)[1]
    assert el == half_l
    assert ec != dc and dc == k2div2
    std_c = [17, 18, 24, 47]
    assert ec[:4] == [int(F(v) * F(0.5) + F(0.5)) for v in std_c]


def _psnr(a, b):
    mse = np.mean((a.astype(np.float64) - b.astype(np.float64)) ** 2)
    return np.inf if mse == 0 else 10 * np.log10(255.0 ** 2 / mse)


def _rgb(argb):
    return argb.view(np.uint8).reshape(argb.shape + (4,))[..., 2::-1]


@pytest.mark.parametrize("div2", [False, True])
@pytest.mark.parametrize("q", [0.5, 0.85, 0.95])
def test_jpeg_psnr_vs_libjpeg_turbo(q, div2):
    """North-star JPEG bar on a rendered C2 tile: the restatement's JPEG decodes to the same PSNR
    vs the source pixels as libjpeg-turbo's at the same tables (within 0.1 dB; here the files
    are byte-identical, so the difference is 0)."""
    from PIL import Image
    h, w = 192, 256
    planes = [p.astype(">u2") for p in tile_u16(5, 4, h, w)]
    st, argb = O.render(c2_channels(4), planes, _lib.PIXELS_UINT16, w, h, big_endian=True)
    src = np.ascontiguousarray(_rgb(argb))
    flags = _lib.SEM_JPEG_CHROMA_DIV2 if div2 else 0
    with O.semantics(flags):
        ours = O.encode_jpeg(argb, w, h, q)
    ql, qc = _java_tables(q, div2)
    buf = io.BytesIO()
    Image.fromarray(src, "RGB").save(buf, "JPEG", qtables=[ql, qc], subsampling=2)
    ref = buf.getvalue()
    d_ours = np.asarray(Image.open(io.BytesIO(ours)).convert("RGB"))
    d_ref = np.asarray(Image.open(io.BytesIO(ref)).convert("RGB"))
    assert abs(_psnr(src, d_ours) - _psnr(src, d_ref)) <= 0.1
    assert ours == ref
    assert _psnr(d_ours, d_ref) == np.inf or _psnr(d_ours, d_ref) >= 45.0


def test_ctx_semantics_flags_validated():
    assert _lib.lib.omr_ctx_set_semantics(None, 1) == _lib.INVALID_ARGUMENT
    assert _lib.lib.omr_ctx_get_semantics(None) == 0


# ---- round 3: the remaining [L] rules of the SEMANTICS TABLE (S2 log guard, S4 noise reduction,
# ---- the exponential input normalisation of Appendix C) and the packed-mask flip (S11)

def _grey_ramp(ch, lo, n, flags=0, pt=_lib.PIXELS_UINT16):
    px = _ramp_u16(lo, n)
    with O.semantics(flags):
        st, a = O.render(ch, [px], pt, n, 1, model="greyscale")
    assert st == 0
    return dict(zip(range(lo, lo + n), _grey(a[0])))


def test_log_guard_switch():
    """Window 0:100, log family.  Guarded (default): f(0) = 0, so the window maps
    round(255 ln x / ln 100).  Unguarded: f(0) = log(0) = -inf, a0 = 255/(ln 100 + inf) = 0 and
    0 * (f(x) + inf) = NaN, Math.round(NaN) = 0 -> every window pixel is cdStart."""
    import math
    ch = [_chan(0.0, 100.0, family=_lib.FAMILY_LOGARITHMIC)]
    a = _grey_ramp(ch, 0, 120)
    for x in (1, 2, 37, 50, 99):
        assert a[x] == int(math.floor(255 * math.log(x) / math.log(100) + 0.5)), x
    assert a[0] == 0 and a[100] == 255
    b = _grey_ramp(ch, 0, 120, _lib.SEM_LOG_UNGUARDED)
    assert all(b[x] == 0 for x in range(100)) and all(b[x] == 255 for x in range(100, 120))
    # a window inside x > 0: the guard never fires and both rules agree
    ch2 = [_chan(5.0, 90.0, family=_lib.FAMILY_LOGARITHMIC)]
    assert _grey_ramp(ch2, 0, 120) == _grey_ramp(ch2, 0, 120, _lib.SEM_LOG_UNGUARDED)


def test_log_guard_switch_float_negative_pixels():
    """float pixels below 0 inside a window that starts below 0: guarded f = 0 there; unguarded
    log(x < 0) = NaN -> round(NaN) = 0 (and f(ws) = NaN makes a0 NaN: the window is cdStart)."""
    x = np.linspace(-50, 150, 801).astype(np.float32).reshape(1, -1)
    ch = [{"input_start": -10.0, "input_end": 100.0, "family": _lib.FAMILY_LOGARITHMIC,
           "rgba": (255, 255, 255, 255)}]
    st, a = O.render(ch, [x], _lib.PIXELS_FLOAT, x.shape[1], 1, model="greyscale")
    with O.semantics(_lib.SEM_LOG_UNGUARDED):
        st2, b = O.render(ch, [x], _lib.PIXELS_FLOAT, x.shape[1], 1, model="greyscale")
    ga, gb = _grey(a[0]), _grey(b[0])
    inside = (x[0] >= -10) & (x[0] < 100)
    assert (ga[inside] > 0).any() and (gb[inside] == 0).all()
    assert (ga[x[0] >= 100] == 255).all() and (gb[x[0] >= 100] == 255).all()


def test_noise_reduction_switch():
    """Window 0:1000 with noise reduction: the default clips x < 100 and x >= 900 (the deciles);
    OMR_SEM_NOISE_REDUCTION_OFF renders the plain linear ramp round(0.255 x)."""
    ch = [_chan(0.0, 1000.0, noise_reduction=True)]
    a = _grey_ramp(ch, 0, 1100)
    assert a[50] == 0 and a[99] == 0 and a[100] == 26 and a[899] == 229 and a[900] == 255
    b = _grey_ramp(ch, 0, 1100, _lib.SEM_NOISE_REDUCTION_OFF)
    assert all(b[x] == int(np.floor(0.255 * x + 0.5)) for x in range(1000))
    assert b[50] == 13 and b[950] == 242
    plain = _grey_ramp([_chan(0.0, 1000.0)], 0, 1100)
    assert b == plain


def test_exp_normalized_switch():
    """Window 100:200, exponential k = 1.  Default exp(x): exp(200)/exp(150) ~ 5e21, so the window
    is cdStart up to x = 193 and rises only in its last pixels.  Normalised: f = exp((x-100)/100),
    f(ws) = 1, f(we) = e, q = round(255 (exp(t) - 1)/(e - 1))."""
    import math
    ch = [_chan(100.0, 200.0, family=_lib.FAMILY_EXPONENTIAL, coefficient=1.0)]
    a = _grey_ramp(ch, 90, 120)
    assert all(a[x] == 0 for x in range(90, 194))
    for x in range(194, 200):
        assert a[x] == int(math.floor(255 / (math.exp(200) - math.exp(100)) * (math.exp(x) - math.exp(100)) + 0.5))
    b = _grey_ramp(ch, 90, 120, _lib.SEM_EXP_NORMALIZED)
    for x in range(100, 200):
        t = (x - 100) / 100.0
        assert b[x] == int(math.floor(255.0 / (math.e - 1.0) * (math.exp(t) - 1.0) + 0.5)), x
    assert b[150] == 96 and b[99] == 0 and b[200] == 255


def test_exp_default_overflows_on_16bit_windows():
    """exp(65535) is +inf: with the default map a full 16-bit window renders cdStart below its end;
    the normalised map renders a curve."""
    ch = [_chan(0.0, 65535.0, family=_lib.FAMILY_EXPONENTIAL, coefficient=1.0)]
    a = _grey_ramp(ch, 0, 65536)
    assert all(a[x] == 0 for x in range(0, 65535, 97)) and a[65535] == 255
    b = _grey_ramp(ch, 0, 65536, _lib.SEM_EXP_NORMALIZED)
    assert len({b[x] for x in range(0, 65536, 7)}) > 200


@pytest.mark.parametrize("fh,fv", [(True, False), (False, True), (True, True)])
def test_mask_packed_flip_reproduced(fh, fv):
    """width % 8 == 0 with a flip: the reference flips the packed w*h/8-byte buffer as w*h bytes
    (ArrayIndexOutOfBoundsException -> 404); OMR_SEM_MASK_PIXEL_FLIP flips pixels."""
    w, h = 16, 3
    rng = np.random.default_rng(7)
    bits = rng.integers(0, 256, w * h // 8, dtype=np.uint8).tobytes()
    st, _ = O.mask_indices(bits, w, h, fh, fv)
    assert st == _lib.NOT_FOUND
    with O.semantics(_lib.SEM_MASK_PIXEL_FLIP):
        st, idx = O.mask_indices(bits, w, h, fh, fv)
    assert st == 0
    unpacked = np.unpackbits(np.frombuffer(bits, np.uint8)).reshape(h, w)
    exp = unpacked[::-1 if fv else 1, ::-1 if fh else 1]
    np.testing.assert_array_equal(idx, exp)
    # a buffer of >= w*h bytes: the byte flip succeeds and the first w*h/8 flipped bytes render
    big = rng.integers(0, 256, w * h + 5, dtype=np.uint8)
    st, idx = O.mask_indices(big.tobytes(), w, h, fh, fv)
    assert st == 0
    dest = np.zeros_like(big)
    dest[: w * h] = big[: w * h].reshape(h, w)[::-1 if fv else 1, ::-1 if fh else 1].reshape(-1)
    np.testing.assert_array_equal(idx, np.unpackbits(dest[: w * h // 8]).reshape(h, w))
    # no flip, or width % 8 != 0: the switch changes nothing
    for args in ((w, h, False, False), (12, 4, fh, fv)):
        st1, i1 = O.mask_indices(bits if args[0] == w else bits[:6], *args)
        with O.semantics(_lib.SEM_MASK_PIXEL_FLIP):
            st2, i2 = O.mask_indices(bits if args[0] == w else bits[:6], *args)
        assert st1 == st2 == 0
        np.testing.assert_array_equal(i1, i2)


def test_mask_reference_failures_are_404():
    """Exceptions inside renderShapeMask fail the future -> ShapeMaskVerticle answers 404."""
    assert O.mask_indices(bytes([0xFF]), 4, 4)[0] == _lib.NOT_FOUND      # IndexOutOfBounds (bits)
    assert O.mask_indices(bytes([0xFF]), 0, 4)[0] == _lib.NOT_FOUND      # zero size
    assert O.mask_indices(b"", 8, 1)[0] == _lib.NOT_FOUND                # null / empty mask


def test_semantics_flag_set_complete():
    assert _lib.SEM_ALL == sum(_lib.SEM_FLAGS.values()) == 0x1FF
    assert len(set(_lib.SEM_FLAGS.values())) == 9
