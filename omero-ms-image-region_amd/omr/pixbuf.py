"""PixelBuffer: the ROMIO repository pixel file the render path reads tiles from.

Mirrors upstream ome.io.nio.RomioPixelBuffer as used by
pixelsService.getPixelBuffer(pixels, false) (ImageRegionRequestHandler.java:302-309): one file of
big-endian planes in XYZCT order.  Reads go through libomr.so (pread; no numpy fallback).
"""
import ctypes

import numpy as np

from . import _lib
from ._lib import lib

_BE_DTYPES = {_lib.PIXELS_INT8: ">i1", _lib.PIXELS_UINT8: ">u1", _lib.PIXELS_INT16: ">i2",
              _lib.PIXELS_UINT16: ">u2", _lib.PIXELS_INT32: ">i4", _lib.PIXELS_UINT32: ">u4",
              _lib.PIXELS_FLOAT: ">f4", _lib.PIXELS_DOUBLE: ">f8"}


def write_romio(path, pixels, pixel_type):
    """Write a [t][c][z][y][x] array as a ROMIO pixel file (big-endian, XYZCT plane order)."""
    a = np.ascontiguousarray(np.asarray(pixels).astype(_BE_DTYPES[pixel_type]))
    assert a.ndim == 5, "pixels must be [t][c][z][y][x]"
    a.tofile(path)


class PixelBuffer:
    def __init__(self, path, size_x, size_y, size_z, size_c, size_t, pixel_type):
        h = ctypes.c_void_p()
        st = lib.omr_pixel_buffer_open(str(path).encode(), size_x, size_y, size_z, size_c, size_t, pixel_type,
                                       ctypes.byref(h))
        if st != _lib.OK:
            raise _lib.OmrError(st, f"cannot open pixel buffer {path}")
        self.h = h
        self.size_x, self.size_y, self.size_z, self.size_c, self.size_t = size_x, size_y, size_z, size_c, size_t
        self.pixel_type = pixel_type

    def close(self):
        if self.h:
            lib.omr_pixel_buffer_close(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # PixelBuffer interface the handler uses (ImageRegionRequestHandler.java:446-454): a ROMIO
    # buffer has one resolution level.
    big_endian = True

    def getResolutionLevels(self):
        return 1

    def getResolutionDescriptions(self):
        return [[self.size_x, self.size_y]]

    def getTileSize(self):
        return (min(self.size_x, 256), min(self.size_y, 256))

    def stack_to_device(self, c, t, device):
        """The Z-stack of (c, t) — contiguous in XYZCT order — as a device byte tensor
        (ProjectionService.projectStack reads whole stacks, ProjectionService.java:46-120)."""
        import torch
        host = np.empty((self.size_z, self.size_y, self.size_x), dtype=_BE_DTYPES[self.pixel_type])
        for z in range(self.size_z):
            _lib.check(lib.omr_pixel_buffer_get_tile(self.h, z, c, t, 0, 0, self.size_x, self.size_y,
                                                     host[z].ctypes.data, host[z].nbytes))
        return torch.from_numpy(host.view(np.uint8).reshape(-1)).to(device)

    def plane_offset(self, z, c, t):
        return lib.omr_pixel_buffer_plane_offset(self.h, z, c, t)

    def get_tile(self, z, c, t, x, y, w, h):
        """PixelBuffer.getTile: [h][w] array in file (big-endian) byte order."""
        if w < 0 or h < 0:   # DimensionsOutOfBoundsException, as the C bounds check
            raise _lib.OmrError(_lib.INVALID_ARGUMENT, f"tile {w}x{h} out of bounds")
        out = np.empty((h, w), dtype=_BE_DTYPES[self.pixel_type])
        _lib.check(lib.omr_pixel_buffer_get_tile(self.h, z, c, t, x, y, w, h, out.ctypes.data, out.nbytes))
        return out
