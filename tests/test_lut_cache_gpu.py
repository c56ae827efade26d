"""The context's device cache of kModeLut16 byte LUTs (non-linear 16-bit families and noise
reduction, omr_render.hip device_quant_lut): every request is still bit-exact against the CPU
restatement when settings repeat (hits), when more settings pass through one context than the
cache holds (LRU eviction, kDevLutEntries = 64), and for LUT domains wider than the pixel type
(globalMin / globalMax beyond 0..65535: up to 2^24 entries, built once per setting)."""
import numpy as np
import pytest

import oracle_lib as O
from omr import _lib
from omr.synthetic import c2_channels, tile_u16

pytestmark = pytest.mark.gpu


def _render(ctx, chans, planes, w, h):
    return ctx.render_packed_int(O.make_qdef("rgb"), chans, planes, _lib.PIXELS_UINT16, w, h)


def test_lut_cache_hits_and_eviction(ctx):
    h, w = 32, 48
    planes = tile_u16(21, 2, h, w, uniform=True)
    base = c2_channels(2)
    settings = []
    for i in range(80):                       # > kDevLutEntries distinct non-linear settings
        chans = [dict(c) for c in base]
        chans[0]["family"] = _lib.FAMILY_POLYNOMIAL
        chans[0]["coefficient"] = 0.5 + i / 40.0
        chans[1]["family"] = _lib.FAMILY_LOGARITHMIC if i % 2 else _lib.FAMILY_EXPONENTIAL
        chans[1]["coefficient"] = 0.25 + (i % 7) / 10.0
        chans[1]["input_start"], chans[1]["input_end"] = 1.0 + i, 3000.0 + 97 * i
        settings.append(chans)
    exp = []
    for chans in settings:
        st, e = O.render(chans, planes, _lib.PIXELS_UINT16, w, h)
        assert st == 0
        exp.append(e)
    for rep in range(2):                      # first pass fills and evicts; second re-builds / hits
        for i in (list(range(80)) if rep == 0 else [79, 78, 0, 1, 40, 79, 0]):
            np.testing.assert_array_equal(_render(ctx, settings[i], planes, w, h), exp[i], err_msg=f"setting {i}")


@pytest.mark.parametrize("gmin,gmax", [(-100000.0, 100000.0), (-5.0, 70000.0), (0.0, 65535.0)])
def test_lut_wide_domains(ctx, gmin, gmax):
    h, w = 24, 40
    planes = tile_u16(22, 2, h, w, uniform=True)
    chans = c2_channels(2)
    for c in chans:
        c["global_min"], c["global_max"] = gmin, gmax
    chans[0]["family"] = _lib.FAMILY_POLYNOMIAL
    chans[0]["coefficient"] = 1.7
    chans[1]["noise_reduction"] = True
    for _ in range(2):                        # miss, then hit
        st, exp = O.render(chans, planes, _lib.PIXELS_UINT16, w, h)
        assert st == 0
        np.testing.assert_array_equal(_render(ctx, chans, planes, w, h), exp)
