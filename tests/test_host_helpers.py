"""Host-side request helpers, ported known-answer tests of the reference.

getRegionDef / truncate / flip-region KATs:  ImageRegionRequestHandlerTest.java:202-618
splitHTMLColor:                               ImageRegionRequestHandler.java:865-890
Shape-mask fill colour:                       ShapeMaskRequestHandler.java:97-106
(reference paths relative to src/{main,test}/java/com/glencoesoftware/omero/ms/image/region/)
"""
import ctypes

import numpy as np
import pytest

from omr import _lib, split_html_color
from omr._lib import Region, lib
from omr.renderer import parse_lut

TILE, REGION, NONE = 0, 1, 2


def region_def(mode, req, levels, tile_size=(0, 0), resolution=-1, flip_h=False, flip_v=False, max_tile=1024):
    """reqHandler.getRegionDef(resolutionLevels, pixelBuffer) with maxTileLength 1024 (test setUp)."""
    lv = (ctypes.c_int32 * (2 * len(levels)))(*[v for l in levels for v in l])
    r = Region(*req) if req is not None else None
    out = Region()
    st = lib.omr_get_region_def(mode, ctypes.byref(r) if r else None, resolution, lv, len(levels),
                                tile_size[0], tile_size[1], max_tile, int(flip_h), int(flip_v), ctypes.byref(out))
    assert st == _lib.OK
    return out.x, out.y, out.width, out.height


L1024 = [(1024, 1024)]
L768 = [(768, 768)]


def test_ctx_tile():                                   # testGetRegionDefCtxTile
    assert region_def(TILE, (2, 2, 0, 0), L1024, (256, 256)) == (512, 512, 256, 256)


def test_ctx_tile_with_width_and_height():             # testGetRegionDefCtxTileWithWidthAndHeight
    assert region_def(TILE, (2, 2, 64, 128), L1024, (64, 128)) == (128, 256, 64, 128)


def test_ctx_region():                                 # testGetRegionDefCtxRegion
    assert region_def(REGION, (512, 512, 256, 256), L1024) == (512, 512, 256, 256)


def test_ctx_no_tile_or_region():                      # testGetRegionDefCtxNoTileOrRegion
    assert region_def(NONE, None, L1024) == (0, 0, 1024, 1024)


def test_tile_trunc_x():                               # testGetRegionDefCtxTileTruncX
    assert region_def(TILE, (1, 0, 0, 0), L1024, (800, 800)) == (800, 0, 224, 800)


def test_tile_trunc_y():                               # testGetRegionDefCtxTileTruncY
    assert region_def(TILE, (0, 1, 0, 0), L1024, (800, 800)) == (0, 800, 800, 224)


def test_tile_trunc_xy():                              # testGetRegionDefCtxTileTruncXY
    assert region_def(TILE, (1, 1, 0, 0), L1024, (800, 800)) == (800, 800, 224, 224)


def test_region_trunc_x():                             # testGetRegionDefCtxRegionTruncX
    assert region_def(REGION, (800, 100, 300, 400), L1024) == (800, 100, 224, 400)


def test_region_trunc_y():                             # testGetRegionDefCtxRegionTruncY
    assert region_def(REGION, (100, 800, 300, 400), L1024) == (100, 800, 300, 224)


def test_region_trunc_xy():                            # testGetRegionDefCtxRegionTruncXY
    assert region_def(REGION, (800, 800, 300, 400), L1024) == (800, 800, 224, 224)


@pytest.mark.parametrize("fh,fv,exp", [(True, False, (624, 200, 300, 400)),   # testFlipRegionDefFlipH
                                       (False, True, (100, 424, 300, 400)),   # testFlipRegionDefFlipV
                                       (True, True, (624, 424, 300, 400))])   # testFlipRegionDefFlipHV
def test_flip_region_def(fh, fv, exp):
    assert region_def(REGION, (100, 200, 300, 400), L1024, (256, 256), flip_h=fh, flip_v=fv) == exp


MIRROR_CASES = {   # testFlipRegionDefMirorXEdge / MirorYEdge / MirorXYEdge (768^2 image, 512^2 tiles)
    (True, False): [((0, 0, 1024, 1024), (0, 0, 768, 768)), ((512, 0, 512, 512), (0, 0, 256, 512)),
                    ((0, 512, 512, 512), (256, 512, 512, 256)), ((512, 512, 512, 512), (0, 512, 256, 256))],
    (False, True): [((0, 0, 512, 512), (0, 256, 512, 512)), ((512, 0, 512, 512), (512, 256, 256, 512)),
                    ((0, 512, 512, 512), (0, 0, 512, 256)), ((512, 512, 512, 512), (512, 0, 256, 256))],
    (True, True): [((0, 0, 512, 512), (256, 256, 512, 512)), ((512, 0, 512, 512), (0, 256, 256, 512)),
                   ((0, 512, 512, 512), (256, 0, 512, 256)), ((512, 512, 512, 512), (0, 0, 256, 256))],
}


@pytest.mark.parametrize("flips", list(MIRROR_CASES))
def test_flip_region_def_mirror_edges(flips):
    for req, exp in MIRROR_CASES[flips]:
        assert region_def(REGION, req, L768, (512, 512), flip_h=flips[0], flip_v=flips[1]) == exp


def test_select_resolution():                          # testSelectResolution
    levels = [(1024, 1024), (256, 512)]
    assert region_def(REGION, (100, 200, 400, 500), levels, (800, 800), resolution=1) == (100, 200, 156, 312)


def test_max_tile_length_clamps_tile_mode_only():      # :804-812 (tile) vs region unbounded
    assert region_def(TILE, (0, 0, 4096, 4096), [(8192, 8192)], max_tile=2048) == (0, 0, 2048, 2048)
    assert region_def(REGION, (0, 0, 4096, 4096), [(8192, 8192)], max_tile=2048) == (0, 0, 4096, 4096)


def test_resolution_level_and_check_plane_def():
    assert lib.omr_resolution_level(3, 0) == 2        # setResolutionLevel: nLevels - res - 1
    assert lib.omr_resolution_level(3, 2) == 0
    r = Region(900, 10, 300, 2000)
    lib.omr_check_plane_def(ctypes.byref(r), 1024, 1024)
    assert (r.x, r.y, r.width, r.height) == (900, 10, 124, 1014)


def test_region_arithmetic_wraps_like_java_int():
    # getRegionDef multiplies tile index by tile size in Java int (:803-804) and
    # truncate/flip subtract in int (:751-780): overflow wraps, it does not saturate.
    def wrap(v):
        return (v + 2**31) % 2**32 - 2**31
    x = region_def(TILE, (2**20 + 1, 0, 0, 0), L1024, (4096, 256), max_tile=4096)
    assert x[0] == wrap((2**20 + 1) * 4096) == 4096
    assert x[2] == min(4096, wrap(1024 - 4096)) == -3072
    big = region_def(REGION, (-2**31, 0, 100, 100), L1024, flip_h=True)
    w = min(100, wrap(1024 + 2**31))                                # Math.min(w, sizeX - x)
    assert big[2] == w == -2147482624 and big[0] == wrap(1024 - w + 2**31) == 0
    assert lib.omr_resolution_level(-2**31, 0) == 2**31 - 1
    r = Region(2**31 - 10, 0, 100, 50)
    lib.omr_check_plane_def(ctypes.byref(r), 1024, 1024)          # width + x wraps negative: untouched
    assert (r.x, r.width) == (2**31 - 10, 100)


@pytest.mark.parametrize("color,exp", [
    ("FF0000", [255, 0, 0, 255]), ("00FF00", [0, 255, 0, 255]), ("0000FF", [0, 0, 255, 255]),
    ("abbccd", [0xAB, 0xBC, 0xCD, 0xFF]), ("abbccdde", [0xAB, 0xBC, 0xCD, 0xDE]),
    ("FF000080", [255, 0, 0, 128]),
    # the 3/4-character path appends (ch + ch) as a decimal int (:873): '0'+'0' = 96
    ("000", [0x96, 0x96, 0x96, 0xFF]), ("0000", [0x96, 0x96, 0x96, 0x96]),
    ("abc", None), ("fff", None), ("", None), ("12345", None), ("GGGGGG", None), ("123456789", None),
    ("-1FFFF", [-1, 255, 255, 255]),
])
def test_split_html_color(color, exp):
    assert split_html_color(color) == exp


def test_shape_mask_fill_color():
    out = (ctypes.c_uint8 * 4)()
    assert lib.omr_shape_mask_fill_color(0, 0, None, out) == 0 and list(out) == [255, 255, 0, 255]  # yellow
    # java.awt.Color(int rgb): reads 0x??RRGGBB, alpha forced to 255
    assert lib.omr_shape_mask_fill_color(1, 0x11223344, None, out) == 0 and list(out) == [0x22, 0x33, 0x44, 255]
    assert lib.omr_shape_mask_fill_color(1, 0x11223344, b"FF000080", out) == 0 and list(out) == [255, 0, 0, 128]
    assert lib.omr_shape_mask_fill_color(0, 0, b"nope", out) == _lib.INVALID_ARGUMENT   # NPE -> 500
    assert lib.omr_shape_mask_fill_color(0, 0, b"-1FFFF", out) == _lib.INVALID_ARGUMENT  # Color IAE


def test_parse_lut_formats():
    raw = np.arange(768, dtype=np.uint16).astype(np.uint8)
    np.testing.assert_array_equal(parse_lut(raw.tobytes()), raw)
    hdr = b"ICOL" + bytes(28) + raw.tobytes()
    np.testing.assert_array_equal(parse_lut(hdr), raw)
    text = "Index\tRed\tGreen\tBlue\n" + "".join(f"{i}\t{i}\t{255 - i}\t{(3 * i) % 256}\n" for i in range(256))
    t = parse_lut(text.encode())
    np.testing.assert_array_equal(t[:256], np.arange(256))
    np.testing.assert_array_equal(t[256:512], 255 - np.arange(256))
    np.testing.assert_array_equal(t[512:], (3 * np.arange(256)) % 256)
    assert parse_lut(b"1 2 3\n") is None
