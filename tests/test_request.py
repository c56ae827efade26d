"""Request decode and renderer settings (CPU; no device work).

Ports ImageRegionCtxTest.java (reference src/test/.../ImageRegionCtxTest.java:121-394) onto the
C-ABI parser (omr_image_region_ctx_parse), plus updateSettings (ImageRegionRequestHandler.java
:689-741), ShapeMaskCtx, LutProviderImpl and the TIFF writer.  Test names carry the reference
test they port.
"""
import ctypes
import io
import os

import numpy as np
import pytest

from omr import _lib
from omr.request import (ImageRegionCtx, LutProvider, RequestError, ShapeMaskCtx,
                         create_rendering_def, update_settings)

# ImageRegionCtxTest.java:40-76
IMAGE_ID, Z, T, Q = 123, 1, 1, 0.8
RESOLUTION, TILE_X, TILE_Y = 0, 0, 1
TILE = f"{RESOLUTION},{TILE_X},{TILE_Y},1024,2048"
REGION = "1,2,3,4"
CH = [-1, 2, -3]
WIN = [(0.0, 65535.0), (1755.0, 51199.0), (3218.0, 26623.0)]
COL = ["0000FF", "00FF00", "FF0000"]
C = ",".join(f"{CH[i]}|{WIN[i][0]:f}:{WIN[i][1]:f}${COL[i]}" for i in range(3))   # Java "%d|%f:%f$%s"
MAPS = ('[{"reverse": {"enabled": false}}, {"reverse": {"enabled": false}}, '
        '{"reverse": {"enabled": false}}]')


def default_params():
    # MultiMap insertion order of setUpParams (:78-90)
    return [("imageId", str(IMAGE_ID)), ("theZ", str(Z)), ("theT", str(T)), ("q", str(Q)),
            ("tile", TILE), ("region", REGION), ("c", C), ("maps", MAPS)]


def set_param(params, key, value):
    out = [(k, v) for k, v in params if k.lower() != key.lower()]
    return out + [(key, value)]


def remove_param(params, key):
    return [(k, v) for k, v in params if k.lower() != key.lower()]


def assert_channel_info(ctx):   # assertChannelInfo (:92-114)
    assert ctx.compressionQuality == np.float32(Q)
    assert len(ctx.colors) == len(ctx.windows) == len(ctx.channels) == 3
    assert ctx.colors == COL
    assert ctx.channels == CH
    for i in range(3):
        assert ctx.windows[i] == [np.float32(WIN[i][0]), np.float32(WIN[i][1])]


def expect_iae(params):
    with pytest.raises(RequestError) as e:
        ImageRegionCtx(params)
    assert e.value.status == _lib.INVALID_ARGUMENT and e.value.http_status == 400


def test_missing_image_id():            # testMissingImageId
    expect_iae(remove_param(default_params(), "imageId"))


def test_image_id_format():             # testImageIdFormat
    expect_iae(set_param(default_params(), "imageId", "abc"))


def test_missing_the_z():               # testMissingTheZ
    expect_iae(remove_param(default_params(), "theZ"))


def test_the_z_format():                # testTheZFormat
    expect_iae(set_param(default_params(), "theZ", "abc"))


def test_missing_the_t():               # testMissingTheT
    expect_iae(remove_param(default_params(), "theT"))


def test_the_t_format():                # testTheTFormat
    expect_iae(set_param(default_params(), "theT", "abc"))


def test_region_format():               # testRegionFormat
    expect_iae(set_param(default_params(), "region", "1,2,3,abc"))


def test_channel_format():              # testChannelFormat / testChannelFormatActive
    expect_iae(set_param(default_params(), "c", "-1|0:65535$0000FF,a|1755:51199$00FF00,3|3218:26623$FF0000"))


def test_channel_format_range():        # testChannelFormatRange
    expect_iae(set_param(default_params(), "c", "-1|0:65535$0000FF,1|abc:51199$00FF00,3|3218:26623$FF0000"))


def test_quality_format():              # testQualityFormat
    expect_iae(set_param(default_params(), "q", "abc"))


def test_tile_short_parameters():       # testTileShortParameters
    p = set_param(remove_param(default_params(), "region"), "tile", f"{RESOLUTION},{TILE_X},{TILE_Y}")
    ctx = ImageRegionCtx(p)
    assert ctx.region is None and ctx.tile is not None
    assert (ctx.tile.getX(), ctx.tile.getY(), ctx.tile.getWidth(), ctx.tile.getHeight()) == (TILE_X, TILE_Y, 0, 0)
    assert ctx.resolution == RESOLUTION
    assert_channel_info(ctx)


def test_tile_parameters():             # testTileParameters
    p = remove_param(default_params(), "region") + [("m", "c")]
    ctx = ImageRegionCtx(p)
    assert ctx.m == "rgb"
    assert (ctx.tile.getX(), ctx.tile.getY(), ctx.tile.getWidth(), ctx.tile.getHeight()) == (TILE_X, TILE_Y, 1024, 2048)
    assert ctx.resolution == RESOLUTION
    assert_channel_info(ctx)


def test_region_parameters():           # testRegionParameters
    p = remove_param(default_params(), "tile") + [("m", "g")]
    ctx = ImageRegionCtx(p)
    assert ctx.tile is None and ctx.resolution is None
    assert ctx.m == "greyscale"
    assert (ctx.region.getX(), ctx.region.getY(), ctx.region.getWidth(), ctx.region.getHeight()) == (1, 2, 3, 4)
    assert_channel_info(ctx)


def test_codomain_maps():               # testCodomainMaps
    ctx = ImageRegionCtx(default_params())
    assert ctx.maps is not None and len(ctx.maps) == 3
    assert all(m == _lib.MAP_NONE for m in ctx.maps)
    assert not any(ctx.reverse_enabled(c) for c in range(3))


@pytest.mark.parametrize("p,proj", [("intmax", _lib.PROJECTION_MAX), ("intmean", _lib.PROJECTION_MEAN),
                                    ("intsum", _lib.PROJECTION_SUM), ("normal", None)])
def test_projection_modes(p, proj):     # testProjectionIntMax / IntMean / IntSum / Normal
    ctx = ImageRegionCtx(default_params() + [("p", p)])
    assert ctx.projection == proj
    assert ctx.projectionStart is None and ctx.projectionEnd is None


def test_projection_start_end():        # testProjectionIntMeanStartEnd
    ctx = ImageRegionCtx(default_params() + [("p", "intmax|0:1")])
    assert ctx.projection == _lib.PROJECTION_MAX
    assert (ctx.projectionStart, ctx.projectionEnd) == (0, 1)


def test_projection_start_end_invalid():   # testProjectionIntMeanStartEndInvalid
    ctx = ImageRegionCtx(default_params() + [("p", "intmax|a:b")])
    assert ctx.projection == _lib.PROJECTION_MAX
    assert ctx.projectionStart is None and ctx.projectionEnd is None


def test_create_cache_key_order_insensitivity():   # testCreateCacheKeyOrderInsensitivity
    p2 = list(reversed(default_params()))
    assert ImageRegionCtx(default_params()).cacheKey == ImageRegionCtx(p2).cacheKey
    assert ImageRegionCtx(default_params()).cacheKey != \
        ImageRegionCtx(set_param(default_params(), "q", "0.9")).cacheKey


# ---- beyond the reference's tests: Java parsing semantics the kernels depend on ----------------

def test_cache_key_is_guava_siphash24():
    """Guava Hashing.sipHash24() (k0=0x0706050403020100, k1=0x0f0e0d0c0b0a0908) over the UTF-8
    of "<class>:key=value..." with keys sorted; HashCode.toString() = little-endian hex."""
    def siphash24(data, k0=0x0706050403020100, k1=0x0F0E0D0C0B0A0908):
        M = (1 << 64) - 1
        rotl = lambda x, b: ((x << b) | (x >> (64 - b))) & M   # noqa: E731
        v = [0x736F6D6570736575 ^ k0, 0x646F72616E646F6D ^ k1, 0x6C7967656E657261 ^ k0,
             0x7465646279746573 ^ k1]

        def rnd():
            v[0] = (v[0] + v[1]) & M; v[1] = rotl(v[1], 13); v[1] ^= v[0]; v[0] = rotl(v[0], 32)
            v[2] = (v[2] + v[3]) & M; v[3] = rotl(v[3], 16); v[3] ^= v[2]
            v[0] = (v[0] + v[3]) & M; v[3] = rotl(v[3], 21); v[3] ^= v[0]
            v[2] = (v[2] + v[1]) & M; v[1] = rotl(v[1], 17); v[1] ^= v[2]; v[2] = rotl(v[2], 32)
        n = len(data)
        tail = data[n // 8 * 8:] + bytes(7 - n % 8) + bytes([n & 0xFF])
        for i in range(0, n // 8 * 8 + 8, 8):
            w = int.from_bytes((data[i:i + 8] if i < n // 8 * 8 else tail), "little")
            v[3] ^= w; rnd(); rnd(); v[0] ^= w
        v[2] ^= 0xFF
        for _ in range(4):
            rnd()
        return (v[0] ^ v[1] ^ v[2] ^ v[3]).to_bytes(8, "little").hex()
    # SipHash-2-4 reference vector (64-bit output, key 00..0f, message 00..0e)
    assert siphash24(bytes(range(15))) == "e545be4961ca29a1"
    p = default_params()
    sb = "com.glencoesoftware.omero.ms.image.region.ImageRegionCtx" + "".join(
        f":{k}={v}" for k, v in sorted(p))
    assert ImageRegionCtx(p).cacheKey == siphash24(sb.encode())


def test_float_windows_are_java_floats():
    c = "1|0.1:65535.7$FF0000,2|1e3:0x1.8p4$00FF00,3|  7  :8f$0000FF"
    ctx = ImageRegionCtx(set_param(default_params(), "c", c))
    assert ctx.windows[0] == [float(np.float32(0.1)), float(np.float32(65535.7))]
    assert ctx.windows[1] == [1000.0, 24.0]
    assert ctx.windows[2] == [7.0, 8.0]


@pytest.mark.parametrize("c,channels,windows,colors", [
    ("1$FF0000", [1], [[None, None]], ["FF0000"]),                  # colour on the active part
    ("1|0:$FF0000", [1], [[None, None]], ["FF0000"]),               # "0:".split(":") -> ["0"]
    ("1|$FF0000", [1], [[None, None]], ["FF0000"]),
    ("1|0:10:99$00FF00", [1], [[0.0, 10.0]], ["00FF00"]),
    ("-2|1:2$x.lut", [-2], [[1.0, 2.0]], ["x.lut"]),
])
def test_channel_entry_forms(c, channels, windows, colors):
    ctx = ImageRegionCtx(set_param(default_params(), "c", c))
    assert (ctx.channels, ctx.windows, ctx.colors) == (channels, windows, colors)


@pytest.mark.parametrize("c", ["1|0:255", "1|$", "1|0:255$", "", "+|0:1$FF0000", "99999999999|0:1$FF0000"])
def test_channel_entry_errors_are_400(c):
    expect_iae(set_param(default_params(), "c", c))


def test_tile_errors():
    expect_iae(set_param(default_params(), "tile", "0,a,1"))
    expect_iae(set_param(default_params(), "tile", "a,b"))          # NumberFormatException on tile[1] first
    with pytest.raises(RequestError) as e:                          # ArrayIndexOutOfBounds -> 500
        ImageRegionCtx(set_param(default_params(), "tile", "0,1"))
    assert e.value.http_status == 500
    ctx = ImageRegionCtx(set_param(default_params(), "tile", "0,1,2,3"))   # length 4: w/h ignored
    assert (ctx.tile.width, ctx.tile.height, ctx.resolution) == (0, 0, 0)


def test_projection_edge_forms():
    ctx = ImageRegionCtx(default_params() + [("p", "intsum|3:b")])
    assert (ctx.projection, ctx.projectionStart, ctx.projectionEnd) == (_lib.PROJECTION_SUM, 3, None)
    ctx = ImageRegionCtx(default_params() + [("p", "intmean|1:2|x")])     # 3 parts: bounds ignored
    assert (ctx.projectionStart, ctx.projectionEnd) == (None, None)
    for bad in ("intmax|:", "intmax|5"):                                 # AIOOBE is not caught
        with pytest.raises(RequestError) as e:
            ImageRegionCtx(default_params() + [("p", bad)])
        assert e.value.http_status == 500


def test_flip_format_quality_ia_defaults():
    ctx = ImageRegionCtx(default_params())
    assert ctx.format == "jpeg" and not ctx.flipHorizontal and not ctx.flipVertical
    assert ctx.invertedAxis is None and ctx.m is None
    ctx = ImageRegionCtx(default_params() + [("flip", "HV"), ("format", "png"), ("ia", "TRUE"),
                                             ("m", "x")])
    assert ctx.flipHorizontal and ctx.flipVertical and ctx.format == "png"
    assert ctx.invertedAxis is True and ctx.m is None


def test_multimap_is_case_insensitive_first_value_wins():
    p = [("IMAGEID", "5"), ("imageId", "6"), ("thez", "0"), ("THET", "2")]
    ctx = ImageRegionCtx(p)
    assert (ctx.imageId, ctx.z, ctx.t) == (5, 0, 2)


def test_maps_decode():
    m = '[null, {"reverse": {"enabled": true}}, {"x": 1}, {"reverse": null}, 5]'
    ctx = ImageRegionCtx(set_param(default_params(), "maps", m))
    assert ctx.maps == [_lib.MAP_NULL, _lib.MAP_REVERSE, _lib.MAP_NONE, _lib.MAP_NONE, _lib.MAP_BAD]
    ctx = ImageRegionCtx(set_param(default_params(), "maps", '[{"reverse": {"enabled": "true"}}]'))
    assert ctx.maps == [_lib.MAP_NONE]                              # Boolean.TRUE.equals("true") is false
    for bad in ('{"reverse": 1}', '[{"reverse": }]', "[1,", "abc"):
        with pytest.raises(RequestError) as e:                      # DecodeException -> 500
            ImageRegionCtx(set_param(default_params(), "maps", bad))
        assert e.value.http_status == 500


# ---- updateSettings (:689-741) ---------------------------------------------------------------

def settings(params, size_c=3, pixel_type=_lib.PIXELS_UINT16, luts=None):
    ctx = ImageRegionCtx(params)
    q, b = create_rendering_def(pixel_type, size_c)
    update_settings(ctx, size_c, q, b, luts)
    return q, b


def test_create_rendering_def_defaults():   # createRenderingDef (:258-300)
    q, b = create_rendering_def(_lib.PIXELS_UINT16, 4)
    assert (q.cd_start, q.cd_end, q.bit_resolution, q.model) == (0, 255, 255, _lib.MODEL_GREYSCALE)
    for c in range(4):
        assert b[c].active == (c < 3)
        assert (b[c].family, b[c].coefficient, b[c].noise_reduction) == (_lib.FAMILY_LINEAR, 1.0, 0)
        assert (b[c].input_start, b[c].input_end) == (0.0, 65535.0)
        assert list(b[c].rgba) == [255, 0, 0, 255]


def test_update_settings_reference_params():
    q, b = settings(default_params() + [("m", "c")])
    assert q.model == _lib.MODEL_RGB
    assert [b[c].active for c in range(3)] == [0, 1, 0]          # channels -1, 2, -3
    assert (b[1].input_start, b[1].input_end) == (1755.0, 51199.0)
    assert list(b[1].rgba) == [0, 255, 0, 255]
    assert (b[0].input_start, b[0].input_end) == (0.0, 65535.0)  # inactive: untouched defaults
    assert list(b[0].rgba) == [255, 0, 0, 255]


def test_update_settings_windows_indexed_by_channel_and_reverse():
    p = set_param(default_params(), "c", "1|10:20$FF000080,-2|0:1$00FF00,3|30:40$0000FF") + [("m", "g")]
    p = set_param(p, "maps", '[{"reverse": {"enabled": true}}, null, {"reverse": {"enabled": true}}]')
    q, b = settings(p)
    assert q.model == _lib.MODEL_GREYSCALE
    assert [b[c].active for c in range(3)] == [1, 0, 1]
    assert (b[2].input_start, b[2].input_end) == (30.0, 40.0)
    assert list(b[0].rgba) == [255, 0, 0, 128]
    assert (b[0].reverse, b[1].reverse, b[2].reverse) == (1, 0, 1)


@pytest.mark.parametrize("c,m", [
    (None, "c"),                                # channels null -> NPE
    ("1|0:1$FF0000", None),                     # m null -> NPE (:736)
    ("3|0:1$FF0000", "c"),                      # windows.get(2) on a 1-entry list -> IOOBE
    ("1$FF0000", "c"),                          # window {null,null} -> NPE (:700)
    ("1|0:1$abc", "c"),                         # splitHTMLColor -> null -> NPE (:712)
])
def test_update_settings_failures_are_500(c, m):
    p = remove_param(default_params(), "c")
    if c is not None:
        p = p + [("c", c)]
    if m is not None:
        p = p + [("m", m)]
    with pytest.raises(RequestError) as e:
        settings(p)
    assert e.value.status == _lib.INTERNAL and e.value.http_status == 500


def test_update_settings_bad_maps_entry_only_for_active_channel():
    p = set_param(default_params(), "maps", '[5, 5, 5]') + [("m", "c")]
    with pytest.raises(RequestError):           # channel 2 (index 1) active: ClassCastException
        settings(p)
    p = set_param(set_param(default_params(), "maps", "[5]"), "c", "-1|0:1$FF0000,2|0:1$FF0000") + [("m", "c")]
    settings(p)                                 # maps[0] bad but channel 1 inactive: never read


def test_lut_provider_and_lut_colour(tmp_path):
    ramp = np.concatenate([np.arange(256), 255 - np.arange(256), np.zeros(256)]).astype(np.uint8)
    (tmp_path / "sub").mkdir()
    (tmp_path / "sub" / "ramp.lut").write_bytes(ramp.tobytes())
    (tmp_path / "broken.lut").write_bytes(b"nope")           # logged and skipped (:52-55)
    (tmp_path / "notalut.txt").write_bytes(ramp.tobytes())
    luts = LutProvider(str(tmp_path))
    assert len(luts) == 1
    assert np.array_equal(luts.get("ramp.lut"), ramp)
    assert luts.get("missing.lut") is None
    p = set_param(default_params(), "c", "1|0:1$ramp.lut,2|0:1$missing.lut") + [("m", "c")]
    q, b = settings(p, size_c=2, luts=luts)
    assert bool(b[0].lut) and np.array_equal(np.ctypeslib.as_array(b[0].lut, (768,)), ramp)
    assert not bool(b[1].lut) and list(b[1].rgba) == [255, 0, 0, 255]   # missing LUT: colour stays


# ---- ShapeMaskCtx (ShapeMaskCtx.java:61-81) ----------------------------------------------------

def test_shape_mask_ctx():
    s = ShapeMaskCtx([("shapeId", "7"), ("color", "FF000080"), ("flip", "h")])
    assert (s.shapeId, s.color, s.flipHorizontal, s.flipVertical) == (7, "FF000080", True, False)
    assert s.cacheKey() == "ome.model.roi.Mask:7:FF000080"
    s = ShapeMaskCtx({"shapeId": "-3"})
    assert s.color is None and s.cacheKey() == "ome.model.roi.Mask:-3:null"
    for bad in ({}, {"shapeId": "x"}):
        with pytest.raises(RequestError) as e:
            ShapeMaskCtx(bad)
        assert e.value.http_status == 500


# ---- TIFF writer (host) ------------------------------------------------------------------------

@pytest.mark.parametrize("w,h", [(1, 1), (7, 5), (300, 40), (1024, 64)])
def test_tiff_decodes_to_rgb(w, h):
    from PIL import Image
    rng = np.random.default_rng(w * 1000 + h)
    argb = rng.integers(0, 2**32, size=(h, w), dtype=np.uint32)
    cap = _lib.lib.omr_tiff_max_bytes(w, h)
    out = np.empty(cap, np.uint8)
    n = ctypes.c_size_t()
    assert _lib.lib.omr_encode_tiff(None, argb.ctypes.data, w, h, out.ctypes.data, cap, ctypes.byref(n)) == 0
    img = Image.open(io.BytesIO(out[:n.value].tobytes()))
    assert img.mode == "RGB" and img.size == (w, h)
    got = np.asarray(img)
    exp = np.stack([(argb >> 16) & 0xFF, (argb >> 8) & 0xFF, argb & 0xFF], -1).astype(np.uint8)
    assert np.array_equal(got, exp)
