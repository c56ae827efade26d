"""K4 JPEG, K5 PNG and K6 shape-mask PNG on the GPU.

JPEG: the whole file byte-identical to the CPU restatement, which is itself pinned to
libjpeg-turbo (tests/test_oracle.py); PNG: decoded pixels identical;
shape mask: decoded RGBA identical to the unpacked/flipped mask through the 2-entry palette,
plus the reference's own dimension checks (ShapeMaskRequestHandlerTest.java:57-81).
"""
import io
import os

import numpy as np
import pytest

import oracle_lib as O
from omr import _lib
from omr.synthetic import c2_channels, tile_u16

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def argb_of(rgb):
    rgb = rgb.astype(np.uint32)
    return (0xFF000000 | (rgb[..., 0] << 16) | (rgb[..., 1] << 8) | rgb[..., 2]).astype(np.uint32)


def decode(b):
    from PIL import Image
    return Image.open(io.BytesIO(b))


def test_jpeg_golden_vectors_byte_identical(ctx):
    g = np.load(os.path.join(GOLDEN, "jpeg_golden.npz"))
    n = len([k for k in g.files if k.startswith("rgb_")])
    for i in range(n):
        rgb, meta = g[f"rgb_{i}"], g[f"meta_{i}"]
        w, h, q = int(meta[0]), int(meta[1]), float(meta[2])
        mine = ctx.encode_jpeg(argb_of(rgb), w, h, q)
        assert mine == O.encode_jpeg(argb_of(rgb), w, h, q), f"case {i}"
        np.testing.assert_array_equal(np.asarray(decode(mine)), np.asarray(decode(g[f"jpeg_{i}"].tobytes())))


@pytest.mark.parametrize("w,h,q", [(1024, 1024, 0.9), (1024, 1024, 0.85), (333, 77, 0.5), (15, 1000, 0.95),
                                   (1000, 15, 0.2), (2048, 17, 1.0)])
def test_jpeg_rendered_tiles_byte_identical(ctx, w, h, q):
    import torch
    planes = [p.astype(">u2") for p in tile_u16(7, 3, h, w)]
    chans = c2_channels(3)
    st, argb = O.render(chans, planes, _lib.PIXELS_UINT16, w, h, big_endian=True)
    d = torch.from_numpy(argb.view(np.int32)).to("cuda")
    mine = ctx.encode_jpeg_device(d, w, h, q)
    assert mine == O.encode_jpeg(argb, w, h, q)


def test_c1_greyscale_u8_tile_to_jpeg(ctx):
    """BASELINE config C1: 1-channel uint8 1024^2 greyscale linear tile -> JPEG."""
    import torch
    rng = np.random.default_rng(20261015)
    p = rng.integers(0, 256, (1024, 1024), dtype=np.uint8)
    chans = [{"input_start": 0.0, "input_end": 255.0, "global_min": 0, "global_max": 255}]
    out = torch.empty((1024, 1024), dtype=torch.int32, device="cuda")
    ctx.render_packed_int_device(O.make_qdef("greyscale"), chans, [torch.from_numpy(p).to("cuda")],
                                 _lib.PIXELS_UINT8, 1024, 1024, out)
    jpg = ctx.encode_jpeg_device(out, 1024, 1024, 0.9)
    st, argb = O.render(chans, [p], _lib.PIXELS_UINT8, 1024, 1024, model="greyscale")
    assert jpg == O.encode_jpeg(argb, 1024, 1024, 0.9)
    assert decode(jpg).size == (1024, 1024)


def test_jpeg_errors(ctx):
    with pytest.raises(_lib.OmrError):
        ctx.encode_jpeg(np.zeros((1, 1), np.uint32), 0, 1, 0.9)


@pytest.mark.parametrize("w,h", [(1024, 1024), (37, 53), (1, 1), (300, 230)])
def test_png_decodes_to_rgb(ctx, w, h):
    rng = np.random.default_rng(w * h)
    argb = rng.integers(0, 2**32, (h, w), dtype=np.uint64).astype(np.uint32)
    png = ctx.encode_png(argb, w, h)
    im = decode(png)
    assert im.mode == "RGB" and im.size == (w, h)
    rgb = np.asarray(im)
    exp = np.stack([(argb >> 16) & 0xFF, (argb >> 8) & 0xFF, argb & 0xFF], -1).astype(np.uint8)
    np.testing.assert_array_equal(rgb, exp)


def mask_rgba(png):
    im = decode(png)
    assert im.mode in ("P", "1", "L", "LA", "RGBA"), im.mode
    return np.asarray(im.convert("RGBA"))


@pytest.mark.parametrize("w,h", [(8, 2), (4, 4)])
def test_shape_mask_reference_dimensions(ctx, w, h):   # testRenderShapeMask{ByteAligned,NotByteAligned}
    png = ctx.render_shape_mask_png(bytes([0x55, 0x55]), w, h, (255, 0, 0, 255))
    assert decode(png).size == (w, h)


@pytest.mark.parametrize("w,h", [(8, 2), (4, 4), (64, 33), (37, 21), (1024, 1024)])
@pytest.mark.parametrize("fh,fv", [(False, False), (True, False), (False, True), (True, True)])
def test_shape_mask_pixels(ctx, w, h, fh, fv):
    rng = np.random.default_rng(w + 7 * h)
    bits = rng.integers(0, 256, (w * h + 7) // 8, dtype=np.uint8).tobytes()
    rgba = (255, 0, 0, 128)
    png = ctx.render_shape_mask_png(bits, w, h, rgba, fh, fv)
    st, idx = O.mask_indices(bits, w, h, fh, fv)
    assert st == 0
    exp = np.zeros((h, w, 4), np.uint8)
    exp[idx == 1] = rgba
    np.testing.assert_array_equal(mask_rgba(png), exp)


def test_shape_mask_errors(ctx):
    with pytest.raises(_lib.OmrError):
        ctx.render_shape_mask_png(bytes([0xFF]), 4, 4, (1, 2, 3, 4))   # too few bits
    with pytest.raises(_lib.OmrError):
        ctx.render_shape_mask_png(bytes([0xFF]), 0, 4, (1, 2, 3, 4))
