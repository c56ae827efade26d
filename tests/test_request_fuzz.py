"""Robustness of the host-side request parsers (no GPU): ImageRegionCtx / ShapeMaskCtx parsing,
splitHTMLColor and .lut parsing on randomised and hostile inputs (garbage, huge numbers, long
lists, unicode, separators in odd places, truncated JSON).  Every call must return a status the
reference maps (OK, 400, 500) — never crash, hang or write past its output."""
import ctypes
import os

import numpy as np
import pytest

from omr import _lib
from omr.request import ImageRegionCtx, RequestError, ShapeMaskCtx
from omr.renderer import split_html_color

N = int(os.environ.get("OMR_FUZZ_CASES", "400"))
KEYS = ["imageId", "theZ", "theT", "q", "tile", "region", "c", "maps", "m", "p", "ia", "flip", "format",
        "resolution", "shapeId", "color", "IMAGEID", "x"]
ATOMS = ["", "0", "1", "-1", "2147483647", "2147483648", "-2147483649", "1e40", "nan", "NaN", "inf", "0x10",
         "3.5", "-0", ",", ":", "|", "$", "[", "]", "{", "}", "\"", "'", "\\", "null", "true", "false",
         "FF0000", "#FFF", "00FF00FF", "abc", "é中", "\x7f", " ", "\t", "..", "-", "+", "intmax",
         "intmean", "intsum", "jpeg", "png", "tif", "h", "v", "hv", "c", "g", "reverse", "enabled"]


def _value(rng):
    k = int(rng.integers(0, 6))
    if k == 0:
        return "".join(rng.choice(ATOMS, int(rng.integers(0, 12))))
    if k == 1:   # channel-list like
        parts = []
        for _ in range(int(rng.integers(0, 40))):
            p = str(int(rng.integers(-5, 9)))
            if rng.integers(0, 2):
                p += "|" + str(float(rng.normal(0, 1e4))) + ":" + str(float(rng.normal(0, 1e4)))
            if rng.integers(0, 2):
                p += "$" + "".join(rng.choice(list("0123456789ABCDEFabcdefg#."), int(rng.integers(0, 9))))
            parts.append(p)
        return ",".join(parts)
    if k == 2:   # region / tile like
        return ",".join(str(int(rng.integers(-2**33, 2**33))) for _ in range(int(rng.integers(0, 7))))
    if k == 3:   # maps JSON, often truncated
        s = "[" + ",".join('{"reverse": {"enabled": %s}}' % rng.choice(["true", "false", "1", "null", '"x"'])
                           for _ in range(int(rng.integers(0, 6)))) + "]"
        return s[:int(rng.integers(0, len(s) + 1))]
    if k == 4:
        return "x" * int(rng.integers(0, 5000))
    return "".join(chr(int(c)) for c in rng.integers(1, 0x2FF, int(rng.integers(0, 30))))


def _params(rng):
    base = [("imageId", "1"), ("theZ", "0"), ("theT", "0")] if rng.integers(0, 3) else []
    extra = [(str(rng.choice(KEYS)), _value(rng)) for _ in range(int(rng.integers(0, 8)))]
    out = base + extra
    rng.shuffle(out)
    return out


@pytest.mark.parametrize("chunk", range(4))
def test_image_region_ctx_parse_fuzz(chunk):
    rng = np.random.default_rng(900 + chunk)
    for _ in range(N // 4):
        p = _params(rng)
        try:
            ImageRegionCtx(p)
        except RequestError as e:
            assert e.status in (_lib.INVALID_ARGUMENT, _lib.INTERNAL), (e.status, p)
        try:
            ShapeMaskCtx(p)
        except RequestError as e:
            assert e.status in (_lib.INVALID_ARGUMENT, _lib.INTERNAL, _lib.NOT_FOUND), (e.status, p)


def test_split_html_color_and_lut_parse_fuzz():
    rng = np.random.default_rng(77)
    for _ in range(N):
        v = _value(rng)
        r = split_html_color(v)
        # Integer.parseInt(s, 16) takes a sign (:880-883): "-F".."FF" -> -15..255
        assert r is None or (len(r) == 4 and all(-15 <= c <= 255 for c in r)), (v, r)
        data = bytes(int(b) for b in rng.integers(0, 256, int(rng.choice([0, 1, 767, 768, 769, 800, 1024, 3000]))))
        if rng.integers(0, 2):
            data = b"".join(rng.choice([b"1\t2\t3\n", b"Index\tRed\tGreen\tBlue\n", b"255 255 255\r\n", b"x\n"],
                                       int(rng.integers(0, 300))))
        out = (ctypes.c_uint8 * 800)(*([0xAB] * 800))
        buf = (ctypes.c_uint8 * max(len(data), 1)).from_buffer_copy(data or b"\0")
        st = _lib.lib.omr_parse_lut(buf, len(data), out)
        assert st in (_lib.OK, _lib.INVALID_ARGUMENT), st
        assert all(out[i] == 0xAB for i in range(768, 800))      # nothing written past 768 bytes
