"""Request layer: ImageRegionCtx / ShapeMaskCtx decode and the ImageRegionRequestHandler glue.

The parsing and the renderer settings run in libomr.so (csrc/omr_request.cpp, C ABI); this module
only marshals them and sequences the device calls the way the reference handler does
(reference paths relative to src/main/java/com/glencoesoftware/omero/ms/image/region/):

  ImageRegionCtx(params)               ImageRegionCtx.java:122-153   -> omr_image_region_ctx_parse
  ShapeMaskCtx(params)                 ShapeMaskCtx.java:61-72       -> omr_shape_mask_ctx_parse
  createRenderingDef                   ImageRegionRequestHandler.java:258-300 -> omr_create_rendering_def
  getRegion / getRegionDef / setResolutionLevel   :429-482, :789-853
  updateSettings                       :689-741                      -> omr_update_settings
  render (projection glue, renderAsPackedInt, flip, encode)          :496-604
  ShapeMaskRequestHandler.renderShapeMask                            ShapeMaskRequestHandler.java:96-221

Errors follow the reference: IllegalArgumentException -> RequestError(status INVALID_ARGUMENT,
HTTP 400); unchecked exceptions -> INTERNAL (500); QuantizationException -> QUANTIZATION (500);
an unknown format returns None (404, ImageRegionVerticle.java:179-182).
"""
import ctypes

import numpy as np

from . import _lib
from ._lib import lib, OmrError

MAX_TILE_LENGTH = 2048   # omero.pixeldata.max_tile_length default (beanRefContext.xml:63-66)


class RequestError(OmrError):
    """A reference exception surfaced by the request layer; .http_status is what the verticle answers."""

    @property
    def http_status(self):
        return _lib.HTTP_STATUS.get(self.status, 500)


def _entries(params):
    """MultiMap entries (insertion order) from a dict, a list of pairs or an object with .items()."""
    if params is None:
        return []
    if isinstance(params, (list, tuple)):
        return [(str(k), str(v)) for k, v in params]
    return [(str(k), str(v)) for k, v in params.items()]


def _marshal(params):
    ent = _entries(params)
    n = len(ent)
    names = (ctypes.c_char_p * max(n, 1))(*[k.encode("utf-8") for k, _ in ent])
    values = (ctypes.c_char_p * max(n, 1))(*[v.encode("utf-8") for _, v in ent])
    return names, values, n


def _err_buf():
    return ctypes.create_string_buffer(512)


class _Region:
    """omeis RegionDef view (getX/getY/getWidth/getHeight like the Java accessors)."""

    def __init__(self, x, y, width, height):
        self.x, self.y, self.width, self.height = x, y, width, height

    def getX(self):
        return self.x

    def getY(self):
        return self.y

    def getWidth(self):
        return self.width

    def getHeight(self):
        return self.height

    def __eq__(self, o):
        return isinstance(o, _Region) and (self.x, self.y, self.width, self.height) == \
            (o.x, o.y, o.width, o.height)

    def __repr__(self):
        return f"RegionDef(x={self.x}, y={self.y}, w={self.width}, h={self.height})"


class ImageRegionCtx:
    """ImageRegionCtx (ImageRegionCtx.java:39-403), fields named as in the reference."""

    def __init__(self, params, omero_session_key=""):
        names, values, n = _marshal(params)
        self._s = _lib.ImageRegionCtxStruct()
        err = _err_buf()
        st = lib.omr_image_region_ctx_parse(names, values, n, ctypes.byref(self._s), err, len(err))
        if st != _lib.OK:
            raise RequestError(st, err.value.decode("utf-8", "replace"))
        s = self._s
        self.omeroSessionKey = omero_session_key
        self.imageId = s.image_id
        self.z, self.t = s.z, s.t
        self.tile = _Region(s.tile.x, s.tile.y, s.tile.width, s.tile.height) if s.has_tile else None
        self.resolution = s.resolution if s.has_resolution else None
        self.region = _Region(s.region.x, s.region.y, s.region.width, s.region.height) \
            if s.has_region else None
        if s.n_channels < 0:
            self.channels = self.windows = self.colors = None
        else:
            k = s.n_channels
            self.channels = [s.channels[i] for i in range(k)]
            self.windows = [[float(s.windows[i][0]), float(s.windows[i][1])] if s.window_set[i]
                            else [None, None] for i in range(k)]
            self.colors = [s.colors[i].value.decode("utf-8") if s.color_set[i] else None for i in range(k)]
        self.m = {-1: None, _lib.MODEL_GREYSCALE: "greyscale", _lib.MODEL_RGB: "rgb"}[s.model]
        self.compressionQuality = float(s.quality) if s.has_quality else None
        self.invertedAxis = None if s.inverted_axis < 0 else bool(s.inverted_axis)
        self.projection = None if s.projection < 0 else s.projection
        self.projectionStart = s.projection_start if s.has_projection_start else None
        self.projectionEnd = s.projection_end if s.has_projection_end else None
        self.maps = None if s.n_maps < 0 else [s.map_reverse[i] for i in range(s.n_maps)]
        self.flipHorizontal, self.flipVertical = bool(s.flip_h), bool(s.flip_v)
        self.format = s.format.decode("utf-8")
        self.cacheKey = s.cache_key.decode("ascii")

    @property
    def struct(self):
        return self._s

    def reverse_enabled(self, c):
        """maps[c].reverse.enabled == Boolean.TRUE (ImageRegionRequestHandler.java:715-729)."""
        return self.maps is not None and c < len(self.maps) and self.maps[c] == _lib.MAP_REVERSE


class ShapeMaskCtx:
    """ShapeMaskCtx (ShapeMaskCtx.java:30-82)."""

    def __init__(self, params, omero_session_key=""):
        names, values, n = _marshal(params)
        s = _lib.ShapeMaskCtxStruct()
        err = _err_buf()
        st = lib.omr_shape_mask_ctx_parse(names, values, n, ctypes.byref(s), err, len(err))
        if st != _lib.OK:
            raise RequestError(st, err.value.decode("utf-8", "replace"))
        self.omeroSessionKey = omero_session_key
        self.shapeId = s.shape_id
        self.color = s.color.decode("utf-8") if s.has_color else None
        self.flipHorizontal, self.flipVertical = bool(s.flip_h), bool(s.flip_v)
        self._key = s.cache_key.decode("utf-8")

    def cacheKey(self):
        return self._key


class LutProvider:
    """LutProviderImpl (LutProviderImpl.java:29-75), backed by omr_lut_provider."""

    def __init__(self, root=None):
        h = ctypes.c_void_p()
        _lib.check(lib.omr_lut_provider_create(root.encode() if root else None, ctypes.byref(h)))
        self.h = h

    def __del__(self):
        try:
            if self.h:
                lib.omr_lut_provider_destroy(self.h)
                self.h = None
        except Exception:
            pass

    def __len__(self):
        return lib.omr_lut_provider_count(self.h)

    def add(self, name, table):
        t = np.ascontiguousarray(np.asarray(table, dtype=np.uint8).reshape(768))
        _lib.check(lib.omr_lut_provider_add(self.h, name.encode(), t.ctypes.data))

    def get(self, name):
        if name is None:
            return None
        p = lib.omr_lut_provider_get(self.h, name.encode())
        if not p:
            return None
        return np.ctypeslib.as_array((ctypes.c_uint8 * 768).from_address(p)).copy()

    def get_lut_readers(self, bindings):
        """Readers for ACTIVE channels only, None where a channel has no LUT (:63-73)."""
        return [self.get(getattr(b, "lut_name", None)) for b in bindings if b.active]


def create_rendering_def(pixel_type, size_c):
    """createRenderingDef (:258-300) -> (QuantumDef, ChannelBinding[size_c])."""
    q = _lib.QuantumDef()
    arr = (_lib.ChannelBinding * max(size_c, 1))()
    _lib.check(lib.omr_create_rendering_def(pixel_type, size_c, ctypes.byref(q), arr))
    return q, arr


def update_settings(ctx, size_c, qdef, bindings, lut_provider=None):
    """updateSettings (:689-741) on (QuantumDef, ChannelBinding[]) from create_rendering_def."""
    err = _err_buf()
    st = lib.omr_update_settings(ctypes.byref(ctx.struct), size_c, ctypes.byref(qdef), bindings,
                                 lut_provider.h if lut_provider is not None else None, err, len(err))
    if st != _lib.OK:
        raise RequestError(st, err.value.decode("utf-8", "replace"))
    return qdef, bindings


class InMemoryPixelBuffer:
    """A PixelBuffer whose planes are resident in device memory.

    levels[i] is a torch tensor [T][C][Z][Y][X] for resolution description i (0 = full
    resolution, as PixelBuffer.getResolutionDescriptions orders them); big_endian marks ROMIO
    byte order.  Reads return device pointers into the resident planes, so a render reads the
    region straight from HBM (the pinned-staging reader is SURVEY §8(f) row 1)."""

    def __init__(self, levels, pixel_type, big_endian=True, tile_size=(256, 256)):
        self.levels = levels
        self.pixel_type = pixel_type
        self.big_endian = big_endian
        self.tile_size = tile_size
        t, c, z, y, x = levels[0].shape
        self.size_t, self.size_c, self.size_z, self.size_y, self.size_x = t, c, z, y, x
        self.bpp = _lib.BYTES_PER_PIXEL[pixel_type]
        self.closed = 0

    def getResolutionLevels(self):
        return len(self.levels)

    def getResolutionDescriptions(self):
        return [[lv.shape[4], lv.shape[3]] for lv in self.levels]

    def getTileSize(self):
        return self.tile_size

    def plane_ptr(self, level_index, z, c, t, x=0, y=0):
        lv = self.levels[level_index]
        sx = lv.shape[4]
        return lv[t, c, z].data_ptr() + (y * sx + x) * self.bpp, sx

    def stack_ptr(self, c, t):
        return self.levels[0][t, c].data_ptr()

    def close(self):
        self.closed += 1


class ImageRegionRequestHandler:
    """The pixel path of ImageRegionRequestHandler (:159-604) over one omr Context."""

    def __init__(self, context, image_region_ctx, lut_provider=None, max_tile_length=MAX_TILE_LENGTH):
        self.ctx = context
        self.irc = image_region_ctx
        self.luts = lut_provider
        self.max_tile_length = max_tile_length

    def get_region_def(self, levels, tile_size):
        """getRegionDef (:789-832)."""
        irc = self.irc
        if irc.tile is not None:
            mode, req = 0, _lib.Region(irc.tile.x, irc.tile.y, irc.tile.width, irc.tile.height)
        elif irc.region is not None:
            mode, req = 1, _lib.Region(irc.region.x, irc.region.y, irc.region.width, irc.region.height)
        else:
            mode, req = 2, _lib.Region(0, 0, 0, 0)
        flat = (ctypes.c_int32 * (2 * len(levels)))(*[v for lv in levels for v in lv])
        out = _lib.Region()
        res = irc.resolution if irc.resolution is not None else -1
        st = lib.omr_get_region_def(mode, ctypes.byref(req), res, flat, len(levels), int(tile_size[0]),
                                    int(tile_size[1]), self.max_tile_length, int(irc.flipHorizontal),
                                    int(irc.flipVertical), ctypes.byref(out))
        if st != _lib.OK:
            raise RequestError(_lib.INTERNAL, "IndexOutOfBoundsException: resolution level")
        return out

    def render_image_region(self, pixel_buffer, out_argb=None):
        """getRegion (:429-482) + render (:496-604): encoded bytes, or None for an unknown format.
        out_argb (optional device int32 tensor) keeps the flipped ARGB for inspection."""
        import torch
        irc, pb = self.irc, pixel_buffer
        qdef, bindings = create_rendering_def(pb.pixel_type, pb.size_c)
        levels = pb.getResolutionDescriptions() if pb.getResolutionLevels() > 1 \
            else [[pb.size_x, pb.size_y]]
        rd = self.get_region_def(levels, pb.getTileSize())
        # setResolutionLevel (:840-853): Renderer level nLevels-res-1 == description index res
        level_index = irc.resolution if irc.resolution is not None else 0
        update_settings(irc, pb.size_c, qdef, bindings, self.luts)
        size_x, size_y = levels[level_index]
        lib.omr_check_plane_def(ctypes.byref(rd), size_x, size_y)         # checkPlaneDef (:651-681)
        dev = torch.device("cuda", self.ctx.device)
        if irc.projection is not None:
            # projection glue (:506-558): full plane at full resolution, region dropped
            start = irc.projectionStart if irc.projectionStart is not None else 0
            end = irc.projectionEnd if irc.projectionEnd is not None else pb.size_z - 1
            w, h = pb.size_x, pb.size_y
            keep = []
            if hasattr(pb, "stack_to_device"):            # ROMIO file: stage the stacks in HBM
                keep = [pb.stack_to_device(c, irc.t, dev) if bindings[c].active else None
                        for c in range(pb.size_c)]
                stacks = [k.data_ptr() if k is not None else None for k in keep]
            else:
                stacks = [pb.stack_ptr(c, irc.t) if bindings[c].active else None for c in range(pb.size_c)]
            out = out_argb if out_argb is not None else torch.empty((h, w), dtype=torch.int32, device=dev)
            _lib.check(lib.omr_render_projected_device(
                self.ctx.h, ctypes.byref(qdef), bindings, pb.size_c,
                (ctypes.c_void_p * pb.size_c)(*stacks), pb.pixel_type, int(pb.big_endian), w, h,
                pb.size_z, irc.projection, start, end, 1, int(irc.flipHorizontal),
                int(irc.flipVertical), out.data_ptr()), self.ctx.h)
            pb.close()
        elif hasattr(pb, "stack_to_device"):
            # ROMIO file: getTile reads straight into pinned staging, then K1+K2 (omr_pixbuf.cpp)
            w, h = rd.width, rd.height
            out = out_argb if out_argb is not None else torch.empty((h, w), dtype=torch.int32, device=dev)
            req = _lib.TileRequest(irc.z, irc.t, rd.x, rd.y)
            _lib.check(lib.omr_render_pixel_buffer_tiles(
                self.ctx.h, pb.h, ctypes.byref(qdef), bindings, pb.size_c, ctypes.byref(req), 1, w, h,
                int(irc.flipHorizontal), int(irc.flipVertical), out.data_ptr(), 1), self.ctx.h)
            pb.close()
        else:
            w, h = rd.width, rd.height
            ptrs, stride = [], 0
            for c in range(pb.size_c):
                if bindings[c].active:
                    p, stride = pb.plane_ptr(level_index, irc.z, c, irc.t, rd.x, rd.y)
                    ptrs.append(p)
                else:
                    ptrs.append(None)
            out = out_argb if out_argb is not None else torch.empty((h, w), dtype=torch.int32, device=dev)
            _lib.check(lib.omr_render_packed_int_device(
                self.ctx.h, ctypes.byref(qdef), bindings, pb.size_c,
                (ctypes.c_void_p * max(pb.size_c, 1))(*ptrs), stride, pb.pixel_type,
                int(pb.big_endian), w, h, int(irc.flipHorizontal), int(irc.flipVertical),
                out.data_ptr()), self.ctx.h)
            pb.close()
        fmt = irc.format
        if fmt == "jpeg":
            # compressionService.setCompressionLevel(q) is per call here (:457-460); the
            # CompressionServiceImpl default level applies when q is absent.
            q = irc.compressionQuality if irc.compressionQuality is not None else DEFAULT_JPEG_QUALITY
            return self.ctx.encode_jpeg_device(out, w, h, q)
        if fmt == "png":
            return self.ctx.encode_png_device(out, w, h)
        if fmt == "tif":
            return self.ctx.encode_tiff_device(out, w, h)
        return None


DEFAULT_JPEG_QUALITY = 0.85   # CompressionServiceImpl default compression level (SURVEY A-11)


class ShapeMaskRequestHandler:
    """ShapeMaskRequestHandler.renderShapeMask(Mask) (:96-116) over one omr Context."""

    def __init__(self, context, shape_mask_ctx):
        self.ctx = context
        self.smc = shape_mask_ctx

    def render_shape_mask(self, mask_bytes, width, height, mask_fill_color=None):
        if mask_bytes is None:
            raise RequestError(_lib.NOT_FOUND, "mask not found")
        rgba = (ctypes.c_uint8 * 4)()
        col = self.smc.color.encode() if self.smc.color is not None else None
        st = lib.omr_shape_mask_fill_color(int(mask_fill_color is not None),
                                           int(mask_fill_color or 0), col, rgba)
        if st != _lib.OK:   # NPE / IAE inside renderShapeMask: the future fails -> 404 (ShapeMaskVerticle:119-128)
            raise RequestError(_lib.NOT_FOUND, f"NullPointerException: colour '{self.smc.color}'")
        return self.ctx.render_shape_mask_png(mask_bytes, width, height, list(rgba),
                                              self.smc.flipHorizontal, self.smc.flipVertical)
