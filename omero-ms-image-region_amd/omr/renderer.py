"""Renderer facade: the omeis Renderer surface the reference drives, backed by libomr.so.

Mirrors the calls of ImageRegionRequestHandler (reference paths relative to
src/main/java/com/glencoesoftware/omero/ms/image/region/):
  createRenderingDef            :258-300   -> create_rendering_def()
  new Renderer(...)             :436-440   -> Renderer(...)
  setActive / setChannelWindow / setChannelLookupTable / setRGBA /
  getCodomainChain(c).add(ReverseIntensityContext) / setModel      :689-741
  setResolutionLevel            :840-853
  renderAsPackedInt(planeDef, buffer)       :559   -> Renderer.render_as_packed_int[_device]
  flip                          :616-642   -> flip()
  splitHTMLColor                :865-890   -> split_html_color()
"""
import ctypes
import os

import numpy as np

from . import _lib
from ._lib import lib
from .context import make_qdef
from .request import LutProvider  # noqa: F401  (C-backed LutProviderImpl, omr_request.cpp)

# StatsFactory.initPixelsRange: the channel window defaults to the pixel-type range.
TYPE_RANGE = {
    _lib.PIXELS_INT8: (-128.0, 127.0), _lib.PIXELS_UINT8: (0.0, 255.0),
    _lib.PIXELS_INT16: (-32768.0, 32767.0), _lib.PIXELS_UINT16: (0.0, 65535.0),
    _lib.PIXELS_INT32: (-2147483648.0, 2147483647.0), _lib.PIXELS_UINT32: (0.0, 4294967295.0),
    _lib.PIXELS_FLOAT: (0.0, 1.0), _lib.PIXELS_DOUBLE: (0.0, 1.0),
}

FAMILIES = {"linear": _lib.FAMILY_LINEAR, "polynomial": _lib.FAMILY_POLYNOMIAL,
            "logarithmic": _lib.FAMILY_LOGARITHMIC, "exponential": _lib.FAMILY_EXPONENTIAL}


def f32(x):
    """Java Float widening: ImageRegionCtx parses windows as Float (ImageRegionCtx.java:313-314)."""
    return float(np.float32(x))


class ReverseIntensityContext:
    """omeis.providers.re.codomain.ReverseIntensityContext marker (:725-726)."""


class CodomainChain:
    def __init__(self):
        self.maps = []

    def add(self, ctx):
        self.maps.append(ctx)

    @property
    def reverse(self):
        return any(isinstance(m, ReverseIntensityContext) for m in self.maps)


class ChannelSettings:
    """One ChannelBinding (+ its QuantumStrategy settings)."""

    def __init__(self, pixel_type, active):
        lo, hi = TYPE_RANGE[pixel_type]
        self.active = active
        self.family = _lib.FAMILY_LINEAR
        self.coefficient = 1.0
        self.noise_reduction = False
        self.input_start, self.input_end = lo, hi
        self.global_min, self.global_max = lo, hi
        self.rgba = (255, 0, 0, 255)
        self.lut_name = None
        self.lut = None
        self.codomain = CodomainChain()

    def as_dict(self):
        return {"active": self.active, "family": self.family, "coefficient": self.coefficient,
                "noise_reduction": self.noise_reduction, "reverse": self.codomain.reverse,
                "input_start": self.input_start, "input_end": self.input_end,
                "global_min": self.global_min, "global_max": self.global_max,
                "rgba": self.rgba, "lut": self.lut}


class RenderingDef:
    def __init__(self, pixel_type, size_c):
        # QuantumDef defaults (:273-277) and greyscale model (:265-269)
        self.cd_start, self.cd_end, self.bit_resolution = 0, 255, 255
        self.model = "greyscale"
        # ChannelBinding defaults (:281-298): linear, k=1, no NR, type range, red, active c<3
        self.channels = [ChannelSettings(pixel_type, c < 3) for c in range(size_c)]


def create_rendering_def(pixel_type, size_c):
    return RenderingDef(pixel_type, size_c)


def parse_lut(data):
    data = bytes(data)
    buf = np.frombuffer(data, dtype=np.uint8) if data else np.zeros(1, np.uint8)
    out = np.empty(768, dtype=np.uint8)
    st = lib.omr_parse_lut(buf.ctypes.data, len(data), out.ctypes.data)
    return out if st == _lib.OK else None


class Renderer:
    """Per-request renderer state; rendering runs in libomr.so on the context's GPU."""

    def __init__(self, context, pixel_type, size_x, size_y, size_c, rendering_def=None,
                 lut_provider=None):
        self.ctx = context
        self.pixel_type = pixel_type
        self.size_x, self.size_y, self.size_c = size_x, size_y, size_c
        self.rdef = rendering_def or create_rendering_def(pixel_type, size_c)
        self.lut_provider = lut_provider or LutProvider()
        self.resolution_level = None

    # --- the omeis calls of updateSettings (:689-741) ---
    def setActive(self, c, active):
        self.rdef.channels[c].active = bool(active)

    def setChannelWindow(self, c, start, end):
        self.rdef.channels[c].input_start = float(start)
        self.rdef.channels[c].input_end = float(end)

    def setRGBA(self, c, r, g, b, a):
        ch = self.rdef.channels[c]
        ch.rgba = (r, g, b, a)
        ch.lut_name, ch.lut = None, None

    def setChannelLookupTable(self, c, name):
        ch = self.rdef.channels[c]
        ch.lut_name = name
        ch.lut = self.lut_provider.get(name)

    def getCodomainChain(self, c):
        return self.rdef.channels[c].codomain

    def setQuantumStrategy(self, c, family, coefficient=1.0, noise_reduction=False):
        ch = self.rdef.channels[c]
        ch.family = FAMILIES.get(family, family)
        ch.coefficient = float(coefficient)
        ch.noise_reduction = bool(noise_reduction)

    def setModel(self, model):
        self.rdef.model = "rgb" if model in ("rgb", _lib.MODEL_RGB) else "greyscale"

    def setResolutionLevel(self, level):
        self.resolution_level = level

    def getChannelBindings(self):
        return self.rdef.channels

    # --- rendering ---
    def qdef(self):
        return make_qdef(self.rdef.model, self.rdef.cd_start, self.rdef.cd_end,
                         self.rdef.bit_resolution)

    def render_as_packed_int(self, planes, width, height, big_endian=True, flip_h=False,
                             flip_v=False, row_stride=0):
        """renderAsPackedInt + flip on host arrays (planes[c] is the region of channel c)."""
        return self.ctx.render_packed_int(self.qdef(), self.rdef.channels, planes,
                                          self.pixel_type, width, height, big_endian, flip_h,
                                          flip_v, row_stride)

    def render_as_packed_int_device(self, planes, width, height, out, big_endian=True,
                                    flip_h=False, flip_v=False, row_stride=0):
        return self.ctx.render_packed_int_device(self.qdef(), self.rdef.channels, planes,
                                                 self.pixel_type, width, height, out, big_endian,
                                                 flip_h, flip_v, row_stride)


def flip(ctx, src, size_x, size_y, flip_h, flip_v):
    """ImageRegionRequestHandler.flip on a device ARGB tensor: returns src when not flipping,
    a new tensor otherwise; IllegalArgumentException -> ValueError."""
    if not flip_h and not flip_v:
        return src
    if src is None:
        raise ValueError("Attempted to flip null image")
    if size_x == 0 or size_y == 0:
        raise ValueError("Attempted to flip image with 0 size")
    dst = src.new_empty(src.shape)
    ctx.flip_argb_device(src, dst, size_x, size_y, flip_h, flip_v)
    return dst


def split_html_color(color):
    """splitHTMLColor (:865-890): [r, g, b, a] or None (bug-compatible 3/4-char path)."""
    if color is None:
        return None
    out = (ctypes.c_int32 * 4)()
    st = lib.omr_split_html_color(color.encode("latin-1", "replace"), out)
    return list(out) if st == _lib.OK else None
