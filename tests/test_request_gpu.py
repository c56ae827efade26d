"""End-to-end request path on the GPU: query parameters -> ImageRegionCtx -> updateSettings ->
region geometry -> (projection) -> renderAsPackedInt + flip -> JPEG / PNG / TIFF bytes, against
the CPU restatement run on the same settings (ImageRegionRequestHandler.java:429-604).

The image is the reference tests' 768x768 plane with 512x512 tiles
(ImageRegionRequestHandlerTest.java:45-67), 3 channels, 2 z-sections, a 2-level pyramid.
"""
import ctypes
import io

import numpy as np
import pytest

import oracle_lib as O
from omr import _lib
from omr.request import (ImageRegionCtx, ImageRegionRequestHandler, InMemoryPixelBuffer,
                         LutProvider, RequestError, ShapeMaskCtx, ShapeMaskRequestHandler,
                         create_rendering_def, update_settings)
from omr.synthetic import microscopy_u16

pytestmark = pytest.mark.gpu

SIZE, TILE, C, Z = 768, 512, 3, 2


@pytest.fixture(scope="module")
def image():
    import torch
    rng = np.random.default_rng(20261015 + 77)
    full = np.stack([np.stack([microscopy_u16(SIZE, SIZE, rng) for _ in range(Z)]) for _ in range(C)])
    half = full[:, :, ::2, ::2].copy()                               # level 1: 384x384
    levels_np = [full[None], half[None]]                             # [T][C][Z][Y][X]
    dev = [torch.from_numpy(lv.astype(">u2").view(np.int16).copy()).to("cuda") for lv in levels_np]
    return levels_np, dev


def buffer(image):
    levels_np, dev = image
    return InMemoryPixelBuffer(dev, _lib.PIXELS_UINT16, big_endian=True, tile_size=(TILE, TILE))


def oracle_argb(irc, levels_np, luts=None):
    """The reference sequence on the CPU restatement with the same settings."""
    q, b = create_rendering_def(_lib.PIXELS_UINT16, C)
    update_settings(irc, C, q, b, luts)
    if irc.projection is not None:
        start = irc.projectionStart if irc.projectionStart is not None else 0
        end = irc.projectionEnd if irc.projectionEnd is not None else Z - 1
        planes = []
        for c in range(C):
            st, p = O.project(levels_np[0][0, c].astype(">u2"), _lib.PIXELS_UINT16, SIZE, SIZE, Z,
                              irc.projection, start, end, be_in=True, be_out=True)
            assert st == 0
            planes.append(p.view(">u2").reshape(SIZE, SIZE))
        x = y = 0
        w = h = SIZE
        lv = np.stack(planes)
    else:
        res = irc.resolution or 0
        lv = levels_np[res][0, :, irc.z]
        sy, sx = lv.shape[1:]
        if irc.tile is not None:
            tw = irc.tile.width or TILE
            th = irc.tile.height or TILE
            x, y, w, h = irc.tile.x * tw, irc.tile.y * th, tw, th
        elif irc.region is not None:
            x, y, w, h = irc.region.x, irc.region.y, irc.region.width, irc.region.height
        else:
            x, y, w, h = 0, 0, sx, sy
        w, h = min(w, sx - x), min(h, sy - y)
        if irc.flipHorizontal:
            x = sx - w - x
        if irc.flipVertical:
            y = sy - h - y
    planes = [np.ascontiguousarray(lv[c, y:y + h, x:x + w]).astype(">u2") for c in range(C)]
    ptrs = (ctypes.c_void_p * C)(*[p.ctypes.data for p in planes])
    out = np.zeros((h, w), np.uint32)
    st = O.lib.oracle_render_packed_int(ctypes.byref(q), b, C, ptrs, 0, _lib.PIXELS_UINT16, 1, w, h,
                                        out.ctypes.data)
    assert st == 0
    st, out = O.flip_int(out, w, h, irc.flipHorizontal, irc.flipVertical)
    return out


def params(**kw):
    p = [("imageId", "1"), ("theZ", "1"), ("theT", "0"), ("m", "c"),
         ("c", "1|0:65535$FF0000,2|1755:51199$00FF00,3|3218:26623$0000FF")]
    for k, v in kw.items():
        p = [(a, b) for a, b in p if a != k] + [(k, v)]
    return p


def rgb(argb):
    return np.stack([(argb >> 16) & 0xFF, (argb >> 8) & 0xFF, argb & 0xFF], -1).astype(np.uint8)


@pytest.mark.parametrize("kw", [
    dict(tile="0,0,0", format="png"),                                  # interior 512 tile
    dict(tile="0,1,1", format="png", flip="hv"),                       # edge tile 256x256, mirrored read
    dict(tile="0,1,0,300,200", format="tif", flip="h"),                # explicit tile size
    dict(region="100,50,333,77", format="png", flip="v", m="g"),       # region mode, greyscale
    dict(tile="1,0,0", format="png"),                                  # resolution 1: 384x384 level
    dict(format="png", maps='[{"reverse": {"enabled": true}}, null]'), # full plane, reverse ch 0
    dict(p="intmax", format="png"),                                    # projection: full plane
    dict(p="intmean|0:1", format="png", tile="0,1,1", flip="h"),       # projection drops the tile
])
def test_render_image_region_lossless_formats(ctx, image, kw):
    irc = ImageRegionCtx(params(**kw))
    got = ImageRegionRequestHandler(ctx, irc).render_image_region(buffer(image))
    exp = oracle_argb(irc, image[0])
    from PIL import Image
    img = Image.open(io.BytesIO(got))
    assert img.size == (exp.shape[1], exp.shape[0])
    np.testing.assert_array_equal(np.asarray(img.convert("RGB")), rgb(exp))


@pytest.mark.parametrize("q", [None, "0.9", "0.5"])
def test_render_image_region_jpeg_byte_identical(ctx, image, q):
    kw = dict(tile="0,0,1", flip="v")
    if q is not None:
        kw["q"] = q
    irc = ImageRegionCtx(params(**kw))
    got = ImageRegionRequestHandler(ctx, irc).render_image_region(buffer(image))
    exp = oracle_argb(irc, image[0])
    quality = float(np.float32(q)) if q is not None else 0.85
    assert got == O.encode_jpeg(exp, exp.shape[1], exp.shape[0], quality)


def test_render_image_region_lut_channel(ctx, image, tmp_path):
    ramp = np.concatenate([np.arange(256), np.arange(256)[::-1], (np.arange(256) * 7) % 256]).astype(np.uint8)
    (tmp_path / "fire.lut").write_bytes(ramp.tobytes())
    luts = LutProvider(str(tmp_path))
    irc = ImageRegionCtx(params(c="1|0:65535$fire.lut,-2|0:1$00FF00,3|3218:26623$0000FF", format="png"))
    got = ImageRegionRequestHandler(ctx, irc, luts).render_image_region(buffer(image))
    exp = oracle_argb(irc, image[0], luts)
    from PIL import Image
    np.testing.assert_array_equal(np.asarray(Image.open(io.BytesIO(got)).convert("RGB")), rgb(exp))


def test_projection_channel_index_quirk(ctx, image):
    """the projected buffer holds sizeC = #active channels but is read
    at the original channel index (ImageRegionRequestHandler.java:507-555).  With only channel 3
    active the reference's bounds check fails (500); OMR_SEM_PROJECTION_ALL_ACTIVE renders it."""
    from PIL import Image
    kw = dict(p="intmax", format="png", c="-1|0:65535$FF0000,-2|1755:51199$00FF00,3|3218:26623$0000FF")
    irc = ImageRegionCtx(params(**kw))
    with pytest.raises(_lib.OmrError) as e:
        ImageRegionRequestHandler(ctx, irc).render_image_region(buffer(image))
    assert e.value.status == _lib.INTERNAL and "DimensionsOutOfBounds" in ctx.last_error()
    ctx.set_semantics(_lib.SEM_PROJECTION_ALL_ACTIVE)
    try:
        got = ImageRegionRequestHandler(ctx, irc).render_image_region(buffer(image))
    finally:
        ctx.set_semantics(0)
    exp = oracle_argb(irc, image[0])
    np.testing.assert_array_equal(np.asarray(Image.open(io.BytesIO(got)).convert("RGB")), rgb(exp))
    # channel 1 alone (index 0 < sizeC 1) renders under both settings
    irc = ImageRegionCtx(params(p="intmax", format="png", c="1|0:65535$FF0000,-2|0:1$00FF00,-3|0:1$0000FF"))
    got = ImageRegionRequestHandler(ctx, irc).render_image_region(buffer(image))
    np.testing.assert_array_equal(np.asarray(Image.open(io.BytesIO(got)).convert("RGB")),
                                  rgb(oracle_argb(irc, image[0])))


def test_unknown_format_is_none_and_settings_errors(ctx, image):
    irc = ImageRegionCtx(params(format="gif"))
    assert ImageRegionRequestHandler(ctx, irc).render_image_region(buffer(image)) is None   # -> 404
    irc = ImageRegionCtx([(k, v) for k, v in params() if k != "m"])
    with pytest.raises(RequestError) as e:                                  # m null -> NPE -> 500
        ImageRegionRequestHandler(ctx, irc).render_image_region(buffer(image))
    assert e.value.http_status == 500


def test_shape_mask_handler(ctx):
    from PIL import Image
    w, h = 13, 5
    rng = np.random.default_rng(3)
    bits = rng.integers(0, 256, (w * h + 7) // 8, dtype=np.uint8).tobytes()
    smc = ShapeMaskCtx({"shapeId": "9", "color": "00FF0080", "flip": "v"})
    png = ShapeMaskRequestHandler(ctx, smc).render_shape_mask(bits, w, h, mask_fill_color=0x123456)
    st, idx = O.mask_indices(bits, w, h, False, True)
    img = Image.open(io.BytesIO(png))
    assert img.size == (w, h)
    np.testing.assert_array_equal(np.asarray(img), idx)
    assert img.getpalette()[3:6] == [0, 255, 0]
    with pytest.raises(RequestError) as e:
        ShapeMaskRequestHandler(ctx, smc).render_shape_mask(None, w, h)
    assert e.value.http_status == 404
    # an unparsable colour: splitHTMLColor -> null -> NPE inside renderShapeMask -> 404
    bad = ShapeMaskRequestHandler(ctx, ShapeMaskCtx({"shapeId": "9", "color": "nope"}))
    with pytest.raises(RequestError) as e:
        bad.render_shape_mask(bits, w, h)
    assert e.value.http_status == 404
    # width % 8 == 0 with a flip: the reference's flip of the packed buffer fails -> 404
    with pytest.raises(_lib.OmrError) as e:
        ShapeMaskRequestHandler(ctx, ShapeMaskCtx({"shapeId": "9", "flip": "h"})).render_shape_mask(
            bytes(2), 8, 2)
    assert e.value.status == _lib.NOT_FOUND and _lib.HTTP_STATUS[e.value.status] == 404


@pytest.mark.parametrize("kw", [
    dict(tile="0,1,0", format="png", flip="hv"),
    dict(region="100,50,333,77", format="png", m="g"),
    dict(p="intmax", format="png"),
    dict(tile="0,0,1", q="0.9"),                                     # default format: jpeg
])
def test_romio_pixel_buffer_matches_resident(ctx, image, tmp_path, kw):
    """The same request through a ROMIO repository file (getPixelBuffer, :302-309: pread into
    pinned staging) and through the HBM-resident buffer: identical encoded bytes."""
    from omr import PixelBuffer, write_romio
    levels_np, _ = image
    path = tmp_path / "pixels"
    write_romio(path, levels_np[0], _lib.PIXELS_UINT16)
    irc = ImageRegionCtx(params(**kw))
    resident = ImageRegionRequestHandler(ctx, irc).render_image_region(buffer(image))
    pb = PixelBuffer(path, SIZE, SIZE, Z, C, 1, _lib.PIXELS_UINT16)
    pb.getTileSize = lambda: (TILE, TILE)                            # the resident buffer's tiling
    from_file = ImageRegionRequestHandler(ctx, ImageRegionCtx(params(**kw))).render_image_region(pb)
    assert from_file == resident


@pytest.mark.parametrize("dma", [True, False])
def test_pipelined_pixel_buffer_tiles(ctx, tmp_path, dma):
    """omr_render_pixel_buffer_tiles over more tiles than one staging group (3 groups of <= 8
    1024^2 4-channel tiles), host pageable / host pinned / device outputs, vs the CPU restatement."""
    import torch
    from omr import PixelBuffer, write_romio
    from omr.synthetic import c2_channels
    X, Y, Zf, Cf, T = 2048, 1024, 2, 4, 2
    rng = np.random.default_rng(5)
    px = rng.integers(0, 65536, (T, Cf, Zf, Y, X), dtype=np.uint16)
    path = tmp_path / "big"
    write_romio(path, px, _lib.PIXELS_UINT16)
    chans = c2_channels(4)
    chans[2]["active"] = False
    q = O.make_qdef("rgb")
    reqs = [(i % Zf, (i // 2) % T, (i % 2) * 1024, 0) for i in range(19)]
    W = H = 1024
    _lib.check(_lib.lib.omr_ctx_set_pixel_buffer_dma(ctx.h, int(dma)))
    with PixelBuffer(path, X, Y, Zf, Cf, T, _lib.PIXELS_UINT16) as pb:
        host = ctx.render_pixel_buffer_tiles(q, chans, pb, reqs, W, H, flip_h=True)
        dev = torch.empty((len(reqs), H, W), dtype=torch.int32, device="cuda")
        ctx.render_pixel_buffer_tiles(q, chans, pb, reqs, W, H, out=dev, flip_h=True)
        nbytes = len(reqs) * H * W * 4
        p = _lib.lib.omr_pinned_alloc(ctx.h, nbytes)
        assert p
        try:
            pinned = np.ctypeslib.as_array((ctypes.c_uint32 * (len(reqs) * H * W)).from_address(p)).reshape(-1, H, W)
            ctx.render_pixel_buffer_tiles(q, chans, pb, reqs, W, H, out=pinned, flip_h=True)
            pinned_copy = pinned.copy()
        finally:
            _lib.lib.omr_pinned_free(ctx.h, p)
    _lib.lib.omr_ctx_set_pixel_buffer_dma(ctx.h, 1)
    dev_np = dev.cpu().numpy().view(np.uint32)
    for i, (z, t, x, y) in enumerate(reqs):
        planes = [np.ascontiguousarray(px[t, c, z, y:y + H, x:x + W]).astype(">u2") for c in range(Cf)]
        st, exp = O.render(chans, planes, _lib.PIXELS_UINT16, W, H, big_endian=True, flip_h=True)
        assert st == 0
        np.testing.assert_array_equal(host[i], exp, err_msg=f"host tile {i}")
        np.testing.assert_array_equal(dev_np[i], exp, err_msg=f"device tile {i}")
        np.testing.assert_array_equal(pinned_copy[i], exp, err_msg=f"pinned tile {i}")


@pytest.mark.parametrize("dma", [True, False])
@pytest.mark.parametrize("W,H,flip", [(512, 384, (False, True)), (300, 200, (True, False))])
def test_pixel_buffer_row_bands(ctx, tmp_path, W, H, flip, dma):
    """Band mode of omr_render_pixel_buffer_tiles (DMA): tiles that share a row band of a plane
    come in as one band at the image's row width -- a contiguous copy when they cover the whole
    row, a 2-D copy of their column span otherwise -- and render in place with the image's row
    stride.  Full rows, partial spans, overlapping bands, repeats and unaligned tile sizes against
    the CPU restatement; by DMA from the registered mapping and staged through pinned memory."""
    import torch
    from omr import PixelBuffer, write_romio
    from omr.synthetic import c2_channels
    X, Y, Zf, Cf, T = 4 * W, 4 * H, 2, 4, 1
    rng = np.random.default_rng(11)
    px = rng.integers(0, 65536, (T, Cf, Zf, Y, X), dtype=np.uint16)
    path = tmp_path / "bands"
    write_romio(path, px, _lib.PIXELS_UINT16)
    chans = c2_channels(4)
    chans[1]["active"] = False
    q = O.make_qdef("rgb")
    reqs = [(0, 0, k * W, 0) for k in range(4)]                      # a whole row: one contiguous band
    reqs += [(0, 0, W, H), (0, 0, 2 * W, H)]                         # a column span
    reqs += [(1, 0, 0, H // 2), (1, 0, 3 * W, H // 2)]               # overlapping band, wide span
    reqs += [(0, 0, 0, 0), (1, 0, W, 3 * H)]                         # a repeat; the last row
    fh, fv = flip
    _lib.check(_lib.lib.omr_ctx_set_pixel_buffer_dma(ctx.h, int(dma)))
    with PixelBuffer(path, X, Y, Zf, Cf, T, _lib.PIXELS_UINT16) as pb:
        host = ctx.render_pixel_buffer_tiles(q, chans, pb, reqs, W, H, flip_h=fh, flip_v=fv)
        dev = torch.empty((len(reqs), H, W), dtype=torch.int32, device="cuda")
        ctx.render_pixel_buffer_tiles(q, chans, pb, reqs, W, H, out=dev, flip_h=fh, flip_v=fv)
    _lib.lib.omr_ctx_set_pixel_buffer_dma(ctx.h, 1)
    dev_np = dev.cpu().numpy().view(np.uint32)
    for i, (z, t, x, y) in enumerate(reqs):
        planes = [np.ascontiguousarray(px[t, c, z, y:y + H, x:x + W]).astype(">u2") for c in range(Cf)]
        st, exp = O.render(chans, planes, _lib.PIXELS_UINT16, W, H, big_endian=True, flip_h=fh, flip_v=fv)
        assert st == 0
        np.testing.assert_array_equal(host[i], exp, err_msg=f"host tile {i}")
        np.testing.assert_array_equal(dev_np[i], exp, err_msg=f"device tile {i}")
