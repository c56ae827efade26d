"""ROMIO PixelBuffer reader (omr_pixel_buffer_*): host-only, no GPU needed.

Layout of upstream ome.io.nio.RomioPixelBuffer (the file pixelsService.getPixelBuffer opens,
ImageRegionRequestHandler.java:302-309): big-endian planes in XYZCT order.
"""
import numpy as np
import pytest

from omr import PixelBuffer, _lib, write_romio

TYPES = [(_lib.PIXELS_UINT8, np.uint8), (_lib.PIXELS_INT8, np.int8), (_lib.PIXELS_UINT16, np.uint16),
         (_lib.PIXELS_INT16, np.int16), (_lib.PIXELS_UINT32, np.uint32), (_lib.PIXELS_INT32, np.int32),
         (_lib.PIXELS_FLOAT, np.float32), (_lib.PIXELS_DOUBLE, np.float64)]


def rand_pixels(dtype, shape, seed):
    rng = np.random.default_rng(seed)
    if np.issubdtype(dtype, np.floating):
        return rng.normal(0, 1000, shape).astype(dtype)
    info = np.iinfo(dtype)
    return rng.integers(info.min, info.max, shape, endpoint=True, dtype=np.int64).astype(dtype)


@pytest.mark.parametrize("pt,dtype", TYPES)
def test_get_tile_matches_layout(tmp_path, pt, dtype):
    T, C, Z, Y, X = 2, 3, 4, 37, 53
    px = rand_pixels(dtype, (T, C, Z, Y, X), 7 + pt)
    path = tmp_path / "pixels"
    write_romio(path, px, pt)
    with PixelBuffer(path, X, Y, Z, C, T, pt) as pb:
        bpp = _lib.BYTES_PER_PIXEL[pt]
        for (z, c, t) in [(0, 0, 0), (3, 2, 1), (1, 1, 0)]:
            assert pb.plane_offset(z, c, t) == (((t * C + c) * Z + z) * Y * X) * bpp
        for (z, c, t, x, y, w, h) in [(0, 0, 0, 0, 0, X, Y), (3, 2, 1, 5, 7, 20, 11), (1, 1, 0, 0, 30, X, 7),
                                      (2, 0, 1, 52, 36, 1, 1), (0, 2, 0, 10, 0, 0, 5)]:
            got = pb.get_tile(z, c, t, x, y, w, h)
            exp = px[t, c, z, y:y + h, x:x + w].astype(np.dtype(dtype).newbyteorder(">"))
            assert got.dtype == exp.dtype
            np.testing.assert_array_equal(got.view(np.uint8), np.ascontiguousarray(exp).view(np.uint8))


def test_bounds_and_open_errors(tmp_path):
    px = rand_pixels(np.uint16, (1, 2, 2, 16, 24), 1)
    path = tmp_path / "p"
    write_romio(path, px, _lib.PIXELS_UINT16)
    with PixelBuffer(path, 24, 16, 2, 2, 1, _lib.PIXELS_UINT16) as pb:
        for args in [(2, 0, 0, 0, 0, 1, 1), (0, 2, 0, 0, 0, 1, 1), (0, 0, 1, 0, 0, 1, 1), (0, 0, 0, 20, 0, 5, 1),
                     (0, 0, 0, 0, 10, 1, 7), (0, 0, 0, -1, 0, 1, 1)]:
            with pytest.raises(_lib.OmrError) as ei:
                pb.get_tile(*args)
            assert ei.value.status == _lib.INVALID_ARGUMENT
        assert pb.plane_offset(5, 0, 0) == -1
    with pytest.raises(_lib.OmrError) as ei:                  # file shorter than the dimensions
        PixelBuffer(path, 24, 16, 3, 2, 1, _lib.PIXELS_UINT16)
    assert ei.value.status == _lib.INVALID_ARGUMENT
    with pytest.raises(_lib.OmrError) as ei:
        PixelBuffer(tmp_path / "missing", 24, 16, 2, 2, 1, _lib.PIXELS_UINT16)
    assert ei.value.status == _lib.NOT_FOUND
    with pytest.raises(_lib.OmrError):
        PixelBuffer(path, 24, 16, 2, 2, 1, 99)


def test_render_without_gpu_fails_loudly(tmp_path):
    """The pipelined render needs a context; there is no CPU fallback."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    import ctypes
    h = ctypes.c_void_p()
    assert _lib.lib.omr_ctx_create(0, ctypes.byref(h)) == _lib.DEVICE
    assert _lib.lib.omr_render_pixel_buffer_tiles(None, None, None, None, 0, None, 0, 8, 8, 0, 0, None, 0) \
        == _lib.INVALID_ARGUMENT


def test_batcher_without_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    import ctypes
    h = ctypes.c_void_p()
    assert _lib.lib.omr_batcher_create(0, 8, 100, ctypes.byref(h)) == _lib.DEVICE
    assert _lib.lib.omr_batcher_create(0, 0, 100, ctypes.byref(h)) == _lib.INVALID_ARGUMENT
