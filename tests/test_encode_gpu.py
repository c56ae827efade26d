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


@pytest.mark.parametrize("w,h,q", [(4096, 16, 0.9), (4100, 9, 0.9), (5000, 3, 0.5)])
def test_jpeg_single_tile_paths_around_batch_limit(ctx, w, h, q):
    """Up to 4096 px a single tile runs the batched B1-B6 pipeline with n = 1; wider images keep
    the legacy single-tile kernels.  Both, from host and from device memory, byte-identical."""
    import torch
    rng = np.random.default_rng(w * 7 + h)
    argb = argb_of(rng.integers(0, 256, (h, w, 3)))
    exp = O.encode_jpeg(argb, w, h, q)
    assert ctx.encode_jpeg(argb, w, h, q) == exp
    assert ctx.encode_jpeg_device(torch.from_numpy(argb.view(np.int32)).to("cuda"), w, h, q) == exp


def test_jpeg_undersized_output_reports_length(ctx):
    """A short caller buffer gives BUFFER_TOO_SMALL and still reports the needed length."""
    import ctypes
    import torch
    from omr.context import lib
    w, h = 64, 48
    argb = argb_of(np.random.default_rng(3).integers(0, 256, (h, w, 3)))
    exp = O.encode_jpeg(argb, w, h, 0.9)
    d = torch.from_numpy(argb.view(np.int32)).to("cuda")
    out = np.zeros(16, np.uint8)
    n = ctypes.c_size_t(0)
    st = lib.omr_encode_jpeg_device(ctx.h, ctypes.c_void_p(d.data_ptr()), w, h, ctypes.c_float(0.9),
                                    out.ctypes.data, out.size, ctypes.byref(n))
    assert st == _lib.BUFFER_TOO_SMALL and n.value == len(exp)
    assert ctx.encode_jpeg_device(d, w, h, 0.9) == exp      # the context recovers


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


@pytest.fixture
def pixel_flip(ctx):
    """Masks flipped at pixel level also when width % 8 == 0 (OMR_SEM_MASK_PIXEL_FLIP, in both
    libomr.so and the restatement); the default reproduction of the reference's packed-buffer
    flip is tested in test_semantics_gpu.py::test_mask_packed_flip."""
    ctx.set_semantics(_lib.SEM_MASK_PIXEL_FLIP)
    with O.semantics(_lib.SEM_MASK_PIXEL_FLIP):
        yield ctx
    ctx.set_semantics(0)


@pytest.mark.parametrize("w,h", [(8, 2), (4, 4), (64, 33), (37, 21), (1024, 1024)])
@pytest.mark.parametrize("fh,fv", [(False, False), (True, False), (False, True), (True, True)])
def test_shape_mask_pixels(pixel_flip, w, h, fh, fv):
    ctx = pixel_flip
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


def _idat_len(png):
    """Total IDAT payload bytes (zlib stream length)."""
    import struct
    i, n = 8, 0
    while i < len(png):
        ln, = struct.unpack(">I", png[i:i + 4])
        if png[i + 4:i + 8] == b"IDAT":
            n += ln
        i += 12 + ln
    return n


def _png_images():
    from omr.synthetic import c2_channels, tile_u16
    out = {}
    planes = tile_u16(3, 4, 512, 512)
    st, out["c2_render_512"] = O.render(c2_channels(4), planes, _lib.PIXELS_UINT16, 512, 512)
    yy, xx = np.mgrid[0:300, 0:400]
    rng = np.random.default_rng(1)
    g = ((xx * 255 // 399) << 16 | (yy * 255 // 299) << 8 | ((xx + yy) % 256)).astype(np.uint32) | 0xFF000000
    g[100:200, 50:350] = 0xFF102030                                    # flat block
    g[250:260] = g[240]                                                 # repeated rows
    g[:, 390:] ^= rng.integers(0, 4, (300, 10), dtype=np.uint32)        # a little noise
    out["gradient_400x300"] = g
    out["zeros_1024"] = np.zeros((1024, 1024), np.uint32)
    out["tiny_1x1"] = np.array([[0xFF123456]], np.uint32)
    return out


@pytest.mark.parametrize("name", ["c2_render_512", "gradient_400x300", "zeros_1024", "tiny_1x1"])
def test_png_deflate_decodes_and_compresses(ctx, name):
    """Dynamic-Huffman deflate of adaptively filtered rows: pixels identical after decoding
    (the PNG parity bar), and far smaller than stored blocks for image-like content."""
    import zlib
    argb = _png_images()[name]
    h, w = argb.shape
    png = ctx.encode_png(argb, w, h)
    rgb = np.asarray(decode(png))
    exp = np.stack([(argb >> 16) & 0xFF, (argb >> 8) & 0xFF, argb & 0xFF], -1).astype(np.uint8)
    np.testing.assert_array_equal(rgb, exp)
    stored = (3 * w + 1) * h
    z = _idat_len(png)
    if name != "tiny_1x1":
        assert z < 0.6 * stored, f"{name}: zlib {z} vs raw {stored}"
    # and the device-resident entry point gives the same file
    import torch
    d = torch.from_numpy(argb.view(np.int32)).to("cuda")
    assert ctx.encode_png_device(d, w, h) == png
    assert zlib.decompressobj() is not None


@pytest.mark.parametrize("w,h", [(1024, 1024), (333, 77)])
def test_shape_mask_png_compresses(pixel_flip, w, h):
    ctx = pixel_flip
    yy, xx = np.mgrid[0:h, 0:w]
    m = ((yy - h / 2) / (h / 3)) ** 2 + ((xx - w / 3) / (w / 4)) ** 2 <= 1
    m |= ((yy - h / 4) / (h / 6)) ** 2 + ((xx - 3 * w / 4) / (w / 8)) ** 2 <= 1
    bits = np.packbits(m.reshape(-1)).tobytes()
    rgba = (255, 0, 0, 128)
    png = ctx.render_shape_mask_png(bits, w, h, rgba, True, False)
    st, idx = O.mask_indices(bits, w, h, True, False)
    exp = np.zeros((h, w, 4), np.uint8)
    exp[idx == 1] = rgba
    np.testing.assert_array_equal(mask_rgba(png), exp)
    raw = ((w + 7) // 8 + 1) * h if w % 8 == 0 else (w + 1) * h
    assert _idat_len(png) < 0.25 * raw


def test_png_chunk_crcs_valid(ctx):
    """Every chunk's CRC-32 checks (zlib.crc32 over type + data), on the first encode of a size
    the context has not seen before as well as on repeats."""
    import struct
    import zlib
    for w, h in [(211, 97), (211, 97), (64, 64)]:
        rng = np.random.default_rng(w)
        argb = (rng.integers(0, 8, (h, w), dtype=np.uint32) * 0x010101) | 0xFF000000
        for png in (ctx.encode_png(argb, w, h), ctx.render_shape_mask_png(bytes(w * h // 8 + 1), w, h, (1, 2, 3, 4))):
            i = 8
            while i < len(png):
                ln, = struct.unpack(">I", png[i:i + 4])
                crc, = struct.unpack(">I", png[i + 8 + ln:i + 12 + ln])
                assert zlib.crc32(png[i + 4:i + 8 + ln]) == crc, png[i + 4:i + 8]
                i += 12 + ln


def test_png_wide_rows(ctx):
    """Rows wider than 64 KiB of LDS (2 x 3 x 12000 bytes): the filter kernel's LDS grows."""
    w, h = 12000, 3
    rng = np.random.default_rng(12)
    argb = (rng.integers(0, 4, (h, w), dtype=np.uint32) * 0x030507) | 0xFF000000
    png = ctx.encode_png(argb, w, h)
    exp = np.stack([(argb >> 16) & 0xFF, (argb >> 8) & 0xFF, argb & 0xFF], -1).astype(np.uint8)
    np.testing.assert_array_equal(np.asarray(decode(png)), exp)


def test_png_device_huffman_tables_match_host(monkeypatch):
    """D3 on the device (OMR_PNG_DEVICE_D3=1: one workgroup builds the length-limited codes and
    the run-length header) restates the host construction: every file byte-identical to the
    host-D3 encode, for images and masks, including noise (stored blocks) and a skewed
    (geometric) pixel distribution."""
    import omr
    rng = np.random.default_rng(77)
    imgs = dict(_png_images())
    imgs["noise_96"] = rng.integers(0, 2**32, (96, 96), dtype=np.uint32) | 0xFF000000
    v = np.concatenate([np.full(2 ** k, k, np.uint32) for k in range(18)])      # geometric counts
    imgs["skewed"] = (rng.permutation(v)[:128 * 1024].reshape(256, 512) * 0x010101) | 0xFF000000
    masks = [(w, h, np.packbits(rng.integers(0, 2, w * h)).tobytes()) for w, h in [(64, 48), (333, 77)]]
    with omr.Context(0) as host:
        want = {k: host.encode_png(a, a.shape[1], a.shape[0]) for k, a in imgs.items()}
        mwant = [host.render_shape_mask_png(b, w, h, (9, 8, 7, 6)) for w, h, b in masks]
    monkeypatch.setenv("OMR_PNG_DEVICE_D3", "1")
    with omr.Context(0) as dev:
        for k, a in imgs.items():
            assert dev.encode_png(a, a.shape[1], a.shape[0]) == want[k], k
        for (w, h, b), exp in zip(masks, mwant):
            assert dev.render_shape_mask_png(b, w, h, (9, 8, 7, 6)) == exp
