"""F1's single-precision Fast16 quantize (omr_k2.h fast16f) against the double-precision rule.

For a linear channel with the default codomain and an integral window start, the LUT entry is
round(a0 * (x - ws)) clamped to [0, 255] (Java Math.round on doubles; ImageRegionRequestHandler
renders through the Renderer).  The fused render -> JPEG kernel replaces the four
f64 operations per channel-pixel with trunc(clamp(fma(x - ws, fa, fb), 0, 255)) in f32 when the
host's search (fast16_f32_params in csrc/omr_render.hip) proves the two step at the same 255 pixel
values.  This test checks every 16-bit pixel value exhaustively for the parameters the library
returns, so an accepted (fa, fb) can never change a pixel; the f64 rule itself is pinned to the
oracle's quantize for a few windows.
"""
import ctypes

import numpy as np
import pytest

from omr import _lib

_hook = _lib.lib.omr_debug_fast16_f32_params
_hook.restype = ctypes.c_int32
_hook.argtypes = [ctypes.c_double, ctypes.c_int64, ctypes.c_int32,
                  ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_float)]

X = np.arange(65536, dtype=np.int64)


def params(a0, wsi):
    fa, fb = ctypes.c_float(), ctypes.c_float()
    ok = _hook(a0, wsi, 65535, ctypes.byref(fa), ctypes.byref(fb))
    return bool(ok), np.float32(fa.value), np.float32(fb.value)


def rule_f64(a0, wsi):
    """fast16i: trunc(a0 * (x - ws) + 0.5) clamped, in IEEE double (numpy does not fuse)."""
    e = np.float64(a0) * (X - wsi).astype(np.float64) + 0.5
    return np.clip(np.where(e < 256.0, e, 255.0), 0.0, 255.0).astype(np.int64)


def rule_f32(fa, fb, wsi):
    """fast16f: fma(x - ws, fa, 1.5 * 2^23) rounds the exact (x - ws) * fa to the nearest integer,
    ties to even (ulp 1 in [2^23, 2^24)); the bits minus 0x4B400000 clamped to [0, 255].  Exact
    in Python integers: fa = m * 2^e with an integer m, so (x - ws) * fa = (x - ws) * m / 2^-e."""
    assert fb == np.float32(12582912.0)
    m, e = np.frexp(np.float64(fa))                 # fa = m * 2^e, 0.5 <= m < 1
    mi, s = int(m * 2 ** 24), 24 - int(e)           # fa = mi / 2^s exactly (f32: 24-bit significand)
    t = (X - wsi) * mi
    if s <= 0:
        n = t << -s
    else:
        q, r = np.divmod(t, 1 << s)                 # floor division, 0 <= r < 2^s
        half = 1 << (s - 1)
        n = q + ((r > half) | ((r == half) & ((q & 1) == 1)))
    return np.clip(n, 0, 255).astype(np.int64)


def windows(seed, n):
    rng = np.random.default_rng(seed)
    out = [(0, 65535.0), (1755, 51199.0), (3218, 26623.0), (100, 4000.0)]   # the C2 bench windows
    for _ in range(n):
        ws = int(rng.integers(-40000, 65535))
        kind = rng.integers(0, 4)
        width = {0: rng.integers(1, 256), 1: rng.integers(256, 4096), 2: rng.integers(4096, 70000),
                 3: rng.uniform(0.5, 3000.0)}[int(kind)]
        out.append((ws, float(np.float32(ws + width))))
    return out


def test_accepted_parameters_are_exact_on_every_pixel_value():
    accepted = 0
    ws_list = windows(7, 300)
    for i, (ws, we) in enumerate(ws_list):
        a0 = 255.0 / (we - ws)
        ok, fa, fb = params(a0, ws)
        if i < 4:
            assert ok, f"C2 window {ws}:{we} should take the f32 path"
        if not ok:
            continue
        accepted += 1
        want, got = rule_f64(a0, ws), rule_f32(fa, fb, ws)
        bad = np.nonzero(want != got)[0]
        assert bad.size == 0, (ws, we, fa, fb, bad[:5], want[bad[:5]], got[bad[:5]])
    assert accepted >= 0.85 * len(ws_list), accepted


def test_f64_rule_is_the_oracle_quantize(oracle):
    for ws, we in [(0, 65535.0), (1755, 51199.0), (100, 4000.0), (30000, 30017.0)]:
        ch = {"active": True, "input_start": float(ws), "input_end": we, "global_min": 0.0,
              "global_max": 65535.0, "rgba": (255, 255, 255, 255)}
        a0 = 255.0 / (we - ws)
        want = rule_f64(a0, ws)
        xs = np.concatenate([np.arange(0, 65536, 97), np.arange(max(0, ws - 300), min(65536, int(we) + 300))])
        got = np.array([oracle.quantize(float(x), ch) for x in xs])
        assert np.array_equal(got, want[xs]), (ws, we)


def test_rejects_degenerate_slopes():
    assert not params(0.0, 0)[0]
    assert not params(-1.0, 0)[0]
    assert not params(float("nan"), 0)[0]
    assert not params(1.0, 1 << 24)[0]
