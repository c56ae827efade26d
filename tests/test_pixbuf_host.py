"""ROMIO pixel buffer on the host (no GPU): RomioPixelBuffer's size check, getTile bounds
(DimensionsOutOfBoundsException -> 400) and byte order, and dimensions whose file size
overflows int64 (rejected, never wrapped past the size check)."""
import numpy as np
import pytest

from omr import PixelBuffer, _lib, write_romio


@pytest.fixture
def romio(tmp_path):
    rng = np.random.default_rng(5)
    px = rng.integers(0, 65536, (2, 3, 2, 40, 56), dtype=np.uint16)   # [t][c][z][y][x]
    path = tmp_path / "pixels"
    write_romio(path, px, _lib.PIXELS_UINT16)
    return path, px


def test_get_tile_matches_file(romio):
    path, px = romio
    pb = PixelBuffer(path, 56, 40, 2, 3, 2, _lib.PIXELS_UINT16)
    for (z, c, t, x, y, w, h) in [(0, 0, 0, 0, 0, 56, 40), (1, 2, 1, 5, 7, 13, 11), (1, 1, 0, 55, 39, 1, 1),
                                  (0, 2, 1, 0, 3, 56, 2), (1, 0, 1, 10, 10, 0, 0)]:
        tile = pb.get_tile(z, c, t, x, y, w, h)
        assert np.array_equal(tile.astype(np.uint16), px[t, c, z, y:y + h, x:x + w])


@pytest.mark.parametrize("bad", [(-1, 0, 0, 0, 0, 1, 1), (2, 0, 0, 0, 0, 1, 1), (0, 3, 0, 0, 0, 1, 1),
                                 (0, 0, 2, 0, 0, 1, 1), (0, 0, 0, 50, 0, 7, 1), (0, 0, 0, 0, 35, 1, 6),
                                 (0, 0, 0, -1, 0, 1, 1), (0, 0, 0, 0, 0, -1, 1), (0, 0, 0, 2**31 - 1, 0, 1, 1)])
def test_get_tile_out_of_bounds(romio, bad):
    path, _ = romio
    pb = PixelBuffer(path, 56, 40, 2, 3, 2, _lib.PIXELS_UINT16)
    with pytest.raises(_lib.OmrError) as e:
        pb.get_tile(*bad)
    assert e.value.status == _lib.INVALID_ARGUMENT


@pytest.mark.parametrize("dims", [(56, 40, 2, 3, 3), (2**31 - 1, 2**31 - 1, 2**31 - 1, 2**31 - 1, 2**31 - 1),
                                  (2**31 - 1, 2**31 - 1, 2**31 - 1, 1, 1), (65536, 65536, 65536, 65536, 1),
                                  (0, 40, 2, 3, 2), (56, 40, 2, -3, 2)])
def test_open_rejects_short_file_and_overflowing_dims(romio, dims):
    path, _ = romio
    with pytest.raises(_lib.OmrError) as e:
        PixelBuffer(path, *dims, _lib.PIXELS_UINT16)
    assert e.value.status == _lib.INVALID_ARGUMENT


def test_open_missing_file(tmp_path):
    with pytest.raises(_lib.OmrError) as e:
        PixelBuffer(tmp_path / "none", 4, 4, 1, 1, 1, _lib.PIXELS_UINT16)
    assert e.value.status == _lib.NOT_FOUND
