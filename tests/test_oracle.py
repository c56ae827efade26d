"""Pin the CPU restatement (oracle/liboracle.so) before it is used as the checker.

* JPEG: entropy-coded data byte-identical to the committed PIL/libjpeg-turbo golden vectors.
* Flip: the reference's own index-oracle tests (ImageRegionRequestHandlerTest.java:69-200,
  ShapeMaskRequestHandlerTest.java:84-215), ported.
* Projection: hand-computed known answers of ProjectionService.java:176-291.
* Quantization: hand-computed known answers of the linear family and Java Math.round.
* Render: regression fixture (tests/golden/render_golden.npz).
"""
import io
import os

import numpy as np
import pytest

from omr import _lib

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def split_jpeg(d):
    """-> ({marker: [payloads]}, entropy-coded segment without EOI)."""
    i, segs = 2, {}
    while True:
        assert d[i] == 0xFF
        m, n = d[i + 1], (d[i + 2] << 8) | d[i + 3]
        segs.setdefault(m, []).append(bytes(d[i + 4:i + 2 + n]))
        i += 2 + n
        if m == 0xDA:
            end = len(d) - 2
            assert d[end] == 0xFF and d[end + 1] == 0xD9
            return segs, bytes(d[i:end])


def argb_of(rgb):
    rgb = rgb.astype(np.uint32)
    return (0xFF000000 | (rgb[..., 0] << 16) | (rgb[..., 1] << 8) | rgb[..., 2]).astype(np.uint32)


def jpeg_cases():
    g = np.load(os.path.join(GOLDEN, "jpeg_golden.npz"))
    n = len([k for k in g.files if k.startswith("rgb_")])
    return [(g[f"rgb_{i}"], g[f"jpeg_{i}"].tobytes(), g[f"meta_{i}"], g[f"qtab_{i}"]) for i in range(n)]


@pytest.mark.parametrize("case", range(9))
def test_oracle_jpeg_matches_libjpeg_turbo_golden(oracle, case):
    rgb, gold, meta, qtab = jpeg_cases()[case]
    w, h, q = int(meta[0]), int(meta[1]), float(meta[2])
    ql, qc = oracle.quant_tables(q)
    np.testing.assert_array_equal(np.concatenate([ql, qc]), qtab)
    mine = oracle.encode_jpeg(argb_of(rgb), w, h, q)
    sm, scan_m = split_jpeg(mine)
    sg, scan_g = split_jpeg(gold)
    assert scan_m == scan_g, "entropy-coded segment differs from libjpeg-turbo"
    assert b"".join(sm[0xDB]) == b"".join(sg[0xDB])
    assert b"".join(sm[0xC4]) == b"".join(sg[0xC4])
    from PIL import Image
    np.testing.assert_array_equal(np.asarray(Image.open(io.BytesIO(mine))), np.asarray(Image.open(io.BytesIO(gold))))


def test_java_quality_tables_known_values(oracle):
    ql, qc = oracle.quant_tables(0.9)          # linear 0.2 -> round(std * 0.2)
    assert list(ql[:8]) == [3, 2, 2, 3, 5, 8, 10, 12]
    assert list(qc[:4]) == [3, 4, 5, 9]
    ql, _ = oracle.quant_tables(1.0)
    assert (ql == 1).all()                     # linear 0 -> clamp to 1
    ql, _ = oracle.quant_tables(0.0)            # q <= 0 -> 0.01 -> scale 50 -> clamp 255
    assert ql.max() == 255


# ---- flips: ported index-oracle tests -------------------------------------------------
def _check_flip(oracle, w, h, fh, fv):
    src = np.arange(w * h, dtype=np.uint32)
    st, f = oracle.flip_int(src, w, h, fh, fv)
    assert st == 0
    for n in range(w * h):
        nc = w - 1 - n % w if fh else n % w
        nr = h - 1 - n // w if fv else n // w
        assert f[nr * w + nc] == n


@pytest.mark.parametrize("w,h", [(4, 4), (5, 5), (7, 4), (4, 7), (7, 1), (1, 7), (1, 1)])
def test_oracle_flip_index_oracle(oracle, w, h):
    for fh, fv in [(False, True), (True, False), (True, True)]:
        _check_flip(oracle, w, h, fh, fv)


def test_oracle_flip_errors(oracle):
    assert oracle.lib.oracle_flip_int(None, None, 4, 4, 1, 1) == _lib.INVALID_ARGUMENT   # testFlipNullImage
    src = np.array([1], np.uint32)
    assert oracle.flip_int(src, 0, 4, True, True)[0] == _lib.INVALID_ARGUMENT         # testFlipZeroXImage
    assert oracle.flip_int(src, 4, 0, True, True)[0] == _lib.INVALID_ARGUMENT         # testFlipZeroYImage


# ---- quantization KATs -------------------------------------------------------------------
def test_java_round(oracle):
    for x, e in [(0.5, 1), (1.5, 2), (2.5, 3), (-0.5, 0), (-2.5, -2), (0.49999999999999994, 0),
                 (127.5, 128), (float("nan"), 0), (254.9999, 255), (1e30, 2**63 - 1)]:
        assert oracle.java_round(x) == e, x


def lin(ws, we, **kw):
    d = {"input_start": ws, "input_end": we, "global_min": 0, "global_max": 65535, "rgba": (255, 255, 255, 255)}
    d.update(kw)
    return d


def test_linear_quantization_known_answers(oracle):
    ch = lin(0.0, 255.0)
    assert [oracle.quantize(x, ch) for x in (0, 1, 127, 254, 255, 300)] == [0, 1, 127, 254, 255, 255]
    ch = lin(0.0, 65535.0)                     # round(255 x / 65535) = round(x / 257)
    assert [oracle.quantize(x, ch) for x in (128, 129, 385, 386, 65534)] == [0, 1, 1, 2, 255]
    ch = lin(100.0, 4000.0)
    assert [oracle.quantize(x, ch) for x in (0, 99, 100, 3999, 4000, 65535)] == [0, 0, 0, 255, 255, 255]
    ch = lin(0.0, 2.0)                         # 127.5 -> 128 (Math.round is half-up)
    assert oracle.quantize(1, ch) == 128
    ch = lin(1755.0, 51199.0)
    assert oracle.quantize(26477, ch) == round(255 * (26477 - 1755) / (51199 - 1755) + 1e-12)
    lut = oracle.build_lut(lin(0.0, 65535.0), 65536)
    x = np.arange(65536)
    np.testing.assert_array_equal(lut, np.floor(255 * x / 65535 + 0.5).astype(np.uint8))


def test_reverse_and_colour_composite_known_answers(oracle):
    p = np.array([[0, 255, 128]], np.uint8)
    ch = [{"input_start": 0.0, "input_end": 255.0, "global_min": 0, "global_max": 255, "rgba": (255, 0, 0, 255)},
          {"input_start": 0.0, "input_end": 255.0, "global_min": 0, "global_max": 255, "rgba": (0, 0, 255, 255),
           "reverse": True}]
    st, out = oracle.render(ch, [p, p], _lib.PIXELS_UINT8, 3, 1)
    assert st == 0
    assert list(out[0]) == [0xFF0000FF, 0xFFFF0000, 0xFF80007F]
    st, out = oracle.render(ch, [p, p], _lib.PIXELS_UINT8, 3, 1, model="greyscale")
    assert list(out[0]) == [0xFF000000, 0xFFFFFFFF, 0xFF808080]


# ---- projection KATs (ProjectionService.java:176-291) ----------------------------------
def test_projection_known_answers(oracle):
    # 3 planes of a 2x1 uint16 image: pixel0 = [10, 30, 20], pixel1 = [65535, 65535, 1]
    stack = np.array([[10, 65535], [30, 65535], [20, 1]], np.uint16)
    st, out = oracle.project(stack, _lib.PIXELS_UINT16, 2, 1, 3, _lib.PROJECTION_MAX, 0, 2)
    assert st == 0 and list(out.view(np.uint16)) == [30, 65535]          # z <= end, inclusive
    st, out = oracle.project(stack, _lib.PIXELS_UINT16, 2, 1, 3, _lib.PROJECTION_MAX, 2, 2)
    assert list(out.view(np.uint16)) == [20, 1]
    st, out = oracle.project(stack, _lib.PIXELS_UINT16, 2, 1, 3, _lib.PROJECTION_MEAN, 0, 2)
    assert list(out.view(np.uint16)) == [20, 65535]                       # z < end: planes 0,1 only
    st, out = oracle.project(stack, _lib.PIXELS_UINT16, 2, 1, 3, _lib.PROJECTION_SUM, 0, 2)
    assert list(out.view(np.uint16)) == [40, 65535]                       # clamped to type max
    st, out = oracle.project(stack, _lib.PIXELS_UINT16, 2, 1, 3, _lib.PROJECTION_MEAN, 1, 1)
    assert list(out.view(np.uint16)) == [0, 0]                            # 0/0 -> NaN -> (int) 0
    st, out = oracle.project(stack, _lib.PIXELS_UINT16, 2, 1, 3, _lib.PROJECTION_SUM, 0, 2, stepping=2)
    assert list(out.view(np.uint16)) == [10, 65535]                       # z = 0 only (2 < 2 false)
    st, out = oracle.project(np.array([[7, 8], [8, 9]], np.uint16), _lib.PIXELS_UINT16, 2, 1, 2,
                             _lib.PROJECTION_MEAN, 0, 1)
    assert list(out.view(np.uint16)) == [7, 8]
    signed = np.array([[-5, -7], [-9, 3]], np.int16)                      # max starts from 0
    st, out = oracle.project(signed, _lib.PIXELS_INT16, 2, 1, 2, _lib.PROJECTION_MAX, 0, 1)
    assert list(out.view(np.int16)) == [0, 3]
    mean3 = np.array([[1], [2], [2], [0]], np.uint8)                      # 5/3 -> 1 (truncation)
    st, out = oracle.project(mean3, _lib.PIXELS_UINT8, 1, 1, 4, _lib.PROJECTION_MEAN, 0, 3)
    assert list(out) == [1]
    be = stack.astype(">u2")
    st, out = oracle.project(be, _lib.PIXELS_UINT16, 2, 1, 3, _lib.PROJECTION_MAX, 0, 2, be_in=True, be_out=True)
    assert list(out.view(">u2")) == [30, 65535]


def test_projection_validation(oracle):
    s = np.zeros((4, 2, 2), np.uint16)
    for start, end, step, alg in [(-1, 2, 1, 0), (0, 4, 1, 0), (4, 0, 1, 0), (0, 3, 0, 0), (0, 3, 1, 7)]:
        st, _ = oracle.project(s, _lib.PIXELS_UINT16, 2, 2, 4, alg, start, end, step)
        assert st == _lib.INVALID_ARGUMENT


# ---- shape mask ----------------------------------------------------------------------------
def test_mask_unpack_known_answers(oracle):
    st, idx = oracle.mask_indices(bytes([0x55, 0x55]), 8, 2)              # testRenderShapeMaskByteAligned
    assert st == 0 and idx.tolist() == [[0, 1] * 4] * 2
    st, idx = oracle.mask_indices(bytes([0x55, 0x55]), 4, 4)              # testRenderShapeMaskNotByteAligned
    assert idx.tolist() == [[0, 1, 0, 1]] * 4
    st, idx = oracle.mask_indices(bytes([0b10000000, 0b10000000]), 3, 3, fh=True)   # bits 0 and 8
    assert idx.tolist() == [[0, 0, 1], [0, 0, 0], [1, 0, 0]]
    assert oracle.mask_indices(bytes([0xFF]), 4, 4)[0] == _lib.NOT_FOUND   # too few bits: IOOBE -> 404


def test_render_golden_regression(oracle):
    from omr.synthetic import c2_channels
    g = np.load(os.path.join(GOLDEN, "render_golden.npz"))
    be = [p.astype(">u2") for p in g["planes"]]
    st, argb = oracle.render(c2_channels(4), be, _lib.PIXELS_UINT16, 64, 48, big_endian=True)
    np.testing.assert_array_equal(argb, g["argb"])
    st, argb = oracle.render(c2_channels(4), be, _lib.PIXELS_UINT16, 64, 48, big_endian=True, flip_h=True, flip_v=True)
    np.testing.assert_array_equal(argb, g["argb_flip_hv"])
