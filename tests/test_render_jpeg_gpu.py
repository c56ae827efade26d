"""Fused render -> JPEG (omr_render_jpeg_batch_*_device): render_image_region's default response
(renderAsPackedInt + flip + compressToStream, ImageRegionRequestHandler.java:559-582) for a batch
of HBM-resident tiles in one call.  Every file must be byte-identical to the CPU restatement's
render + JPEG of the same tile — through the fused F1 kernel (8/16-bit, 1..4 channels, sides
multiple of 16) and through the K2 + B1 fallback (ragged tiles, float pixels, > 4 channels)."""
import numpy as np
import pytest

import oracle_lib as O
from omr import _lib
from omr.context import make_qdef
from omr.renderer import f32
from omr.synthetic import c2_channels, tile_u16

pytestmark = pytest.mark.gpu


def _run(ctx, chans, tiles, pt, w, h, q=0.9, model="rgb", be=False, flip=(False, False), table=False,
         qd_kw=None):
    """tiles: [n][c] numpy planes (file byte order already applied).  Returns (files, status)."""
    import torch
    n, c = len(tiles), len(tiles[0])
    raw = np.stack([np.stack([np.ascontiguousarray(p).view(np.uint8).reshape(-1) for p in t]) for t in tiles])
    data = torch.from_numpy(raw.copy()).to("cuda")
    plane = raw.shape[2]
    cap = n * (w * h * 4 + 4096)
    d_out = torch.empty(cap, dtype=torch.uint8, device="cuda")
    offs = torch.empty(n, dtype=torch.int64, device="cuda")
    lens = torch.empty(n, dtype=torch.int32, device="cuda")
    stat = torch.full((n,), -7, dtype=torch.int32, device="cuda")
    qd = make_qdef(model, **(qd_kw or {}))
    torch.cuda.synchronize()
    if table:
        base = data.data_ptr()
        ptrs = torch.tensor([[base + (t * c + k) * plane for k in range(c)] for t in range(n)], dtype=torch.int64,
                            device="cuda")
        torch.cuda.synchronize()
        ctx.render_jpeg_batch_device(qd, chans, ptrs, n, pt, w, h, q, d_out, offs, lens, stat, big_endian=be,
                                     flip_h=flip[0], flip_v=flip[1])
    else:
        ctx.render_jpeg_batch_strided_device(qd, chans, data, c * plane, plane, n, pt, w, h, q, d_out, offs, lens,
                                             stat, big_endian=be, flip_h=flip[0], flip_v=flip[1])
    try:
        ctx.synchronize()
    except _lib.OmrError as e:
        if e.status != _lib.QUANTIZATION:
            raise
    o, ln, st = offs.cpu().numpy(), lens.cpu().numpy(), stat.cpu().numpy()
    buf = d_out.cpu().numpy()
    return [buf[o[i]:o[i] + ln[i]].tobytes() for i in range(n)], st


def _expect(chans, tiles, pt, w, h, q=0.9, model="rgb", be=False, flip=(False, False), qdef=None):
    out = []
    for t in tiles:
        st, argb = O.render(chans, t, pt, w, h, model=model, big_endian=be, flip_h=flip[0], flip_v=flip[1],
                            qdef=qdef)
        assert st == 0
        out.append(O.encode_jpeg(argb, w, h, q))
    return out


@pytest.mark.parametrize("table", [False, True])
def test_c2_full_size_fused_byte_identical(ctx, table):
    w = h = 1024
    tiles = [[p.astype(">u2") for p in tile_u16(60 + t, 4, h, w)] for t in range(3)]
    chans = c2_channels(4)
    files, st = _run(ctx, chans, tiles, _lib.PIXELS_UINT16, w, h, be=True, table=table)
    assert (st == 0).all()
    assert files == _expect(chans, tiles, _lib.PIXELS_UINT16, w, h, be=True)


@pytest.mark.parametrize("flip", [(True, False), (False, True), (True, True)])
@pytest.mark.parametrize("be", [False, True])
def test_flips_and_byte_order(ctx, flip, be):
    w, h = 256, 160
    tiles = [[(p.astype(">u2") if be else p) for p in tile_u16(70 + t, 3, h, w)] for t in range(2)]
    chans = c2_channels(3)
    files, st = _run(ctx, chans, tiles, _lib.PIXELS_UINT16, w, h, be=be, flip=flip, q=0.8)
    assert files == _expect(chans, tiles, _lib.PIXELS_UINT16, w, h, be=be, flip=flip, q=0.8)


@pytest.mark.parametrize("n_ch", [1, 2, 4])
def test_u8_greyscale_and_colour(ctx, n_ch):
    w, h = 128, 96
    rng = np.random.default_rng(n_ch)
    tiles = [[rng.integers(0, 256, (h, w)).astype(np.uint8) for _ in range(n_ch)] for _ in range(3)]
    chans = [{"input_start": f32(10.5), "input_end": f32(240.0), "global_min": 0.0, "global_max": 255.0,
              "rgba": [(255, 0, 0, 255), (0, 255, 0, 255), (0, 0, 255, 255), (200, 100, 50, 128)][k]}
             for k in range(n_ch)]
    for model in ("greyscale", "rgb"):
        files, st = _run(ctx, chans, tiles, _lib.PIXELS_UINT8, w, h, model=model, q=0.75)
        assert files == _expect(chans, tiles, _lib.PIXELS_UINT8, w, h, model=model, q=0.75)


def test_signed_reverse_lut_codomain_and_lut16(ctx):
    """int16 with reverse + a .lut channel (Linear16 with the second rounding stage under a
    non-default codomain), and a polynomial channel (byte-LUT gather, Mixed16)."""
    w, h = 192, 128
    rng = np.random.default_rng(4)
    tiles = [[rng.integers(-2000, 2000, (h, w)).astype(np.int16) for _ in range(3)] for _ in range(2)]
    lut = np.concatenate([np.arange(256), 255 - np.arange(256), (np.arange(256) * 3) % 256]).astype(np.uint8)
    chans = [{"input_start": f32(-1500.5), "input_end": f32(1800.0), "global_min": -32768.0, "global_max": 32767.0,
              "rgba": (0, 0, 255, 255), "reverse": True},
             {"input_start": f32(-100.0), "input_end": f32(1000.0), "global_min": -32768.0, "global_max": 32767.0,
              "lut": lut},
             {"input_start": f32(1.0), "input_end": f32(1900.0), "global_min": -32768.0, "global_max": 32767.0,
              "rgba": (255, 255, 0, 255), "family": _lib.FAMILY_POLYNOMIAL, "coefficient": 0.5}]
    for qd_kw in (None, {"cd_start": 20, "cd_end": 230}):
        files, st = _run(ctx, chans, tiles, _lib.PIXELS_INT16, w, h, qd_kw=qd_kw)
        assert files == _expect(chans, tiles, _lib.PIXELS_INT16, w, h, qdef=make_qdef("rgb", **(qd_kw or {})))


@pytest.mark.parametrize("shape", [(100, 60), (1024, 1000), (17, 16)])
def test_ragged_tiles_take_the_unfused_path(ctx, shape):
    w, h = shape
    tiles = [[p.astype(">u2") for p in tile_u16(80 + t, 4, h, w)] for t in range(2)]
    chans = c2_channels(4)
    files, st = _run(ctx, chans, tiles, _lib.PIXELS_UINT16, w, h, be=True, flip=(True, False))
    assert (st == 0).all()
    assert files == _expect(chans, tiles, _lib.PIXELS_UINT16, w, h, be=True, flip=(True, False))


def test_float_and_many_channels_unfused(ctx):
    w, h = 128, 64
    rng = np.random.default_rng(5)
    tiles = [[rng.uniform(-5, 300, (h, w)).astype(np.float32) for _ in range(2)] for _ in range(2)]
    chans = [{"input_start": 0.0, "input_end": 255.0, "rgba": (255, 0, 0, 255)},
             {"input_start": 10.0, "input_end": 200.0, "rgba": (0, 255, 0, 255)}]
    files, st = _run(ctx, chans, tiles, _lib.PIXELS_FLOAT, w, h)
    assert files == _expect(chans, tiles, _lib.PIXELS_FLOAT, w, h)
    tiles = [[p for p in tile_u16(90 + t, 6, h, w)] for t in range(2)]
    chans = c2_channels(4) + c2_channels(2)
    files, st = _run(ctx, chans, tiles, _lib.PIXELS_UINT16, w, h)
    assert files == _expect(chans, tiles, _lib.PIXELS_UINT16, w, h)


@pytest.mark.parametrize("fused", [True, False])
def test_quantization_error_flags_its_tile(ctx, fused):
    w, h = (128, 64) if fused else (120, 64)
    tiles = [[p.copy() for p in tile_u16(95 + t, 2, h, w)] for t in range(3)]
    for t in tiles:
        for p in t:
            np.minimum(p, 60000, out=p)
    tiles[1][1][5, 7] = 65000
    chans = c2_channels(2)
    for c in chans:
        c["global_max"] = 60000.0
    files, st = _run(ctx, chans, tiles, _lib.PIXELS_UINT16, w, h)
    assert st.tolist() == [0, _lib.QUANTIZATION, 0]
    exp = _expect(chans, [tiles[0], tiles[2]], _lib.PIXELS_UINT16, w, h)
    assert files[0] == exp[0] and files[2] == exp[1]


def test_quantization_error_signed_lower_and_upper_bounds(ctx):
    """Fused 16-bit domain check (packed per-lane min/max, folded once per lane): int16 planes,
    a pixel exactly at globalMin / globalMax is inside, one below / above flags only its tile."""
    w, h = 128, 64
    rng = np.random.default_rng(11)
    tiles = [[rng.integers(-900, 900, (h, w)).astype(np.int16) for _ in range(2)] for _ in range(4)]
    tiles[0][0][0, 0], tiles[0][1][63, 127] = -1000, 1000       # on the bounds: fine
    tiles[1][0][17, 33] = -1001                                 # below globalMin
    tiles[3][1][40, 2] = 1001                                   # above globalMax
    chans = [{"input_start": f32(-800.0), "input_end": f32(700.0), "global_min": -1000.0, "global_max": 1000.0,
              "rgba": (255, 0, 0, 255)},
             {"input_start": f32(-50.0), "input_end": f32(900.0), "global_min": -1000.0, "global_max": 1000.0,
              "rgba": (0, 255, 255, 255)}]
    files, st = _run(ctx, chans, tiles, _lib.PIXELS_INT16, w, h)
    assert st.tolist() == [0, _lib.QUANTIZATION, 0, _lib.QUANTIZATION]
    exp = _expect(chans, [tiles[0], tiles[2]], _lib.PIXELS_INT16, w, h)
    assert files[0] == exp[0] and files[2] == exp[1]


@pytest.mark.parametrize("gmin,gmax,bad", [(0.0, 2147483647.0, True), (-2147483648.0, 2147483647.0, False),
                                            (-2147483648.0, -1.0, True), (40000.0, 2147483647.0, True),
                                            (-2147483648.0, -40000.0, True)])
def test_int16_extreme_lut_domain(ctx, gmin, gmax, bad):
    """int16 channels whose LUT domain lies partly or wholly outside the type: the
    fused kernel moves the domain by the int16 bias after clamping it to the type, so gmax near
    INT32_MAX no longer wraps; the per-tile QuantizationException and every file agree with the
    restatement (tiles 0 and 2 hold pixels below 0 / inside, tile 1 only positives)."""
    w, h = 64, 48
    rng = np.random.default_rng(23)
    tiles = [[rng.integers(-3000, 3000, (h, w)).astype(np.int16) for _ in range(2)],
             [rng.integers(1, 3000, (h, w)).astype(np.int16) for _ in range(2)],
             [rng.integers(-3000, 3000, (h, w)).astype(np.int16) for _ in range(2)]]
    chans = [{"input_start": f32(-500.0), "input_end": f32(2500.0), "global_min": gmin, "global_max": gmax,
              "rgba": (255, 0, 0, 255)},
             {"input_start": f32(0.0), "input_end": f32(1000.0), "global_min": -32768.0, "global_max": 32767.0,
              "rgba": (0, 255, 0, 255)}]
    files, st = _run(ctx, chans, tiles, _lib.PIXELS_INT16, w, h)
    want = []
    for t in tiles:
        s_, _ = O.render(chans, t, _lib.PIXELS_INT16, w, h)
        want.append(s_)
    assert [int(x) != 0 for x in st.tolist()] == [x != 0 for x in want], (st.tolist(), want)
    ok = [i for i, x in enumerate(want) if x == 0]
    if ok:
        exp = _expect(chans, [tiles[i] for i in ok], _lib.PIXELS_INT16, w, h)
        assert [files[i] for i in ok] == exp
    if not bad:
        assert st.tolist() == [0, 0, 0]


def test_int16_window_start_inexact_after_bias_falls_back(ctx):
    """The fused kernel reads int16 pixels biased by 32768 and moves the window start with them;
    a window start for which ws + 32768 is not exact (1e-30) takes the K2 + B1 path instead.
    Both must give the oracle's files (a fused int16 case alongside for contrast)."""
    w, h = 64, 48
    rng = np.random.default_rng(19)
    tiles = [[rng.integers(-2000, 2000, (h, w)).astype(np.int16) for _ in range(2)] for _ in range(2)]
    for ws in (1e-30, -1000.25):
        chans = [{"input_start": f32(ws), "input_end": f32(1500.0), "global_min": -32768.0, "global_max": 32767.0,
                  "rgba": (255, 128, 0, 255)},
                 {"input_start": f32(-1500.0), "input_end": f32(20.0), "global_min": -32768.0,
                  "global_max": 32767.0, "rgba": (0, 64, 255, 255), "reverse": True}]
        files, st = _run(ctx, chans, tiles, _lib.PIXELS_INT16, w, h)
        assert st.tolist() == [0, 0]
        assert files == _expect(chans, tiles, _lib.PIXELS_INT16, w, h), ws


@pytest.mark.parametrize("starts", [(100.0, 0.0, 2000.0), (100.5, 0.0, 2000.25), (-3.0, 7.0, 65000.0)])
def test_fast16_integral_and_fractional_window_starts(ctx, starts):
    """Default-codomain linear u16 channels take F1's Fast16 mode; with every window start an
    integer the kernel subtracts in int32 (Fast16I), otherwise in f64: both byte-identical."""
    w, h = 128, 64
    tiles = [[p.astype(">u2") for p in tile_u16(120 + t, 3, h, w)] for t in range(2)]
    ends = (3000.0, 65535.0, 9000.75)
    chans = [{"input_start": f32(s), "input_end": f32(e), "global_min": 0.0, "global_max": 65535.0,
              "rgba": c} for s, e, c in zip(starts, ends, [(255, 0, 0, 255), (0, 255, 0, 255), (0, 0, 255, 255)])]
    files, st = _run(ctx, chans, tiles, _lib.PIXELS_UINT16, w, h, be=True, flip=(True, True))
    assert st.tolist() == [0, 0]
    assert files == _expect(chans, tiles, _lib.PIXELS_UINT16, w, h, be=True, flip=(True, True))


@pytest.mark.parametrize("pt,w,h", [(_lib.PIXELS_UINT16, 1024, 1024), (_lib.PIXELS_UINT16, 120, 72),
                                    (_lib.PIXELS_UINT8, 256, 128), (_lib.PIXELS_FLOAT, 64, 48)])
def test_render_jpeg_one_request(ctx, pt, w, h):
    """omr_render_jpeg (one request, default format): device planes -> host JPEG, fused for
    16-multiple 8/16-bit tiles, K2 + B1 otherwise; the restatement's render + JPEG file, with an
    inactive channel passed as a null plane, flips, and a QuantizationException."""
    import torch
    rng = np.random.default_rng(w + h)
    if pt == _lib.PIXELS_UINT16:
        planes = [p.astype(">u2") for p in tile_u16(150, 4, h, w)]
        chans = c2_channels(4)
        be = True
    elif pt == _lib.PIXELS_UINT8:
        planes = [rng.integers(0, 256, (h, w)).astype(np.uint8) for _ in range(4)]
        chans = [{"input_start": 10.0 * c, "input_end": 200.0 + c, "global_min": 0.0, "global_max": 255.0,
                  "rgba": (255 * (c & 1), 255 * (c >> 1 & 1), 128, 255)} for c in range(4)]
        be = False
    else:
        planes = [rng.uniform(-10, 300, (h, w)).astype(np.float32) for _ in range(4)]
        chans = [{"input_start": 0.0, "input_end": 255.0, "rgba": (255, 0, 0, 255)},
                 {"input_start": 5.0, "input_end": 200.0, "rgba": (0, 0, 255, 255)}] * 2
        be = False
    chans = [dict(c) for c in chans]
    chans[2]["active"] = False
    dev = [torch.from_numpy(np.ascontiguousarray(p).view(np.uint8).reshape(-1)).to("cuda") for p in planes]
    dev[2] = None
    q = make_qdef("rgb")
    for fh, fv in [(False, False), (True, True)]:
        got = ctx.render_jpeg_device(q, chans, dev, pt, w, h, 0.85, big_endian=be, flip_h=fh, flip_v=fv)
        st, argb = O.render(chans, planes, pt, w, h, big_endian=be, flip_h=fh, flip_v=fv)
        assert st == 0
        assert got == O.encode_jpeg(argb, w, h, 0.85), (fh, fv)
    if pt == _lib.PIXELS_UINT16:
        bad = [dict(c) for c in chans]
        bad[0]["global_max"] = 1000.0
        with pytest.raises(_lib.OmrError) as e:
            ctx.render_jpeg_device(q, bad, dev, pt, w, h, 0.85, big_endian=be)
        assert e.value.status == _lib.QUANTIZATION
        got = ctx.render_jpeg_device(q, chans, dev, pt, w, h, 0.85, big_endian=be)   # the flag was consumed
        st, argb = O.render(chans, planes, pt, w, h, big_endian=be)
        assert got == O.encode_jpeg(argb, w, h, 0.85)


def test_int16_fused_window_ends_at_the_int32_limits(ctx):
    """int16 through F1 moves the integer window ends by 32768; ends already clamped to the int32
    limits (a window end at 1e12 / -1e12, or beyond) must saturate, not wrap."""
    w, h = 64, 32
    rng = np.random.default_rng(23)
    tiles = [[rng.integers(-32768, 32768, (h, w)).astype(np.int16) for _ in range(2)] for _ in range(2)]
    chans = [{"input_start": f32(-1e12), "input_end": f32(1e12), "global_min": -32768.0, "global_max": 32767.0,
              "rgba": (255, 0, 0, 255)},
             {"input_start": f32(-100.0), "input_end": f32(3e9), "global_min": -32768.0, "global_max": 32767.0,
              "rgba": (0, 255, 0, 255), "reverse": True}]
    for qd_kw in (None, {"cd_start": 10, "cd_end": 240}):     # Fast16, then Linear16 (integer ends)
        files, st = _run(ctx, chans, tiles, _lib.PIXELS_INT16, w, h, qd_kw=qd_kw)
        assert st.tolist() == [0, 0]
        assert files == _expect(chans, tiles, _lib.PIXELS_INT16, w, h, qdef=make_qdef("rgb", **(qd_kw or {})))


@pytest.mark.parametrize("q", [1.0, 0.95])
def test_fused_int8_and_int16_blocks_in_one_wave(ctx, q):
    """F1's per-MCU int8 / int16 choice on rendered pixels: 16x16 patches of full-range noise in
    a smooth 8-bit plane, greyscale and colour, at qualities where the noisy MCUs need int16."""
    rng = np.random.default_rng(31)
    h, w, n = 128, 256, 2
    yy, xx = np.mgrid[0:h, 0:w]
    tiles = []
    for t in range(n):
        planes = []
        for c in range(2):
            p = ((xx * 255 // (w - 1) + yy + 40 * c + 7 * t) % 256).astype(np.uint8)
            noise = rng.integers(0, 256, (h, w), dtype=np.uint8)
            for y in range(0, h, 16):
                for x in range(0, w, 16):
                    if rng.random() < 0.3:
                        p[y:y + 16, x:x + 16] = noise[y:y + 16, x:x + 16]
            planes.append(p)
        tiles.append(planes)
    chans = [{"input_start": 0.0, "input_end": 255.0, "global_min": 0.0, "global_max": 255.0, "rgba": rgba}
             for rgba in ((255, 0, 0, 255), (0, 255, 255, 255))]
    for model in ("greyscale", "rgb"):
        got, st = _run(ctx, chans, tiles, _lib.PIXELS_UINT8, w, h, q=q, model=model)
        assert (st == 0).all()
        assert got == _expect(chans, tiles, _lib.PIXELS_UINT8, w, h, q=q, model=model), model
    # 16-bit planes (F1's fast16 modes), big-endian as ROMIO stores them
    tiles16 = [[(p.astype(np.uint16) * 257 + 3).astype(">u2") for p in t] for t in tiles]
    chans16 = [{"input_start": 300.0, "input_end": 64000.0, "global_min": 0.0, "global_max": 65535.0, "rgba": rgba}
               for rgba in ((255, 0, 0, 255), (0, 255, 255, 255))]
    got, st = _run(ctx, chans16, tiles16, _lib.PIXELS_UINT16, w, h, q=q, be=True)
    assert (st == 0).all()
    assert got == _expect(chans16, tiles16, _lib.PIXELS_UINT16, w, h, q=q, be=True)


@pytest.mark.parametrize("n_ch", [1, 3, 4])
@pytest.mark.parametrize("be", [False, True])
@pytest.mark.parametrize("pt", [_lib.PIXELS_UINT16, _lib.PIXELS_INT16])
def test_fast16_f32_pairs_byte_order_sign_and_domain_check(ctx, pt, be, n_ch):
    """F1's packed fast16-f32 render: each pixel pair becomes 2^23 + x by one v_perm per half
    (the big-endian swap folded into its selector), then one packed subtract and one packed fma.
    u16 and int16 (the sign bias on each half's first byte in file order), both byte orders,
    1 / 3 / 4 channels with integral window starts, channel 0 with a LUT domain narrower than the
    type (the domain check byte-swaps on its own), horizontal flip."""
    w, h = 128, 64
    rng = np.random.default_rng(41 + n_ch + 8 * be + 16 * (pt == _lib.PIXELS_INT16))
    if pt == _lib.PIXELS_INT16:
        lo, hi, dt = -32768, 32767, np.int16
        starts, ends = (-20000, -500, 100, 3000), (25000.0, 9000.0, 30000.0, 32000.0)
    else:
        lo, hi, dt = 0, 65535, np.uint16
        starts, ends = (0, 1000, 123, 40000), (65535.0, 20000.0, 5000.0, 65000.0)
    tiles = [[rng.integers(lo, hi + 1, (h, w)).astype(dt) for _ in range(n_ch)] for _ in range(2)]
    for t in tiles:                                   # channel 0 inside its narrower domain
        np.clip(t[0], lo + 100, hi - 101, out=t[0])
        t[0][3, 5], t[0][60, 127] = lo + 100, hi - 101
    if be:
        tiles = [[p.astype(p.dtype.newbyteorder(">")) for p in t] for t in tiles]
    colours = [(255, 0, 0, 255), (0, 255, 0, 255), (0, 0, 255, 255), (200, 100, 50, 255)]
    chans = [{"input_start": f32(float(starts[k])), "input_end": f32(ends[k]),
              "global_min": float(lo + 100 if k == 0 else lo), "global_max": float(hi - 101 if k == 0 else hi),
              "rgba": colours[k]} for k in range(n_ch)]
    files, st = _run(ctx, chans, tiles, pt, w, h, be=be, flip=(True, False))
    assert st.tolist() == [0, 0]
    assert files == _expect(chans, tiles, pt, w, h, be=be, flip=(True, False))
