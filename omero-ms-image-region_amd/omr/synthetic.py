"""Synthetic inputs of the BASELINE.json configs; no datasets exist offline.

seed = 20261015 + tile_index.  "Microscopy" channels: gamma(k=2, theta=300) background plus
32 Gaussian blobs of amplitude U(2000, 40000), clipped to [0, 65535].
"""
import numpy as np

SEED = 20261015

# C2 render settings: windows and colours of ImageRegionCtxTest.java:62-67 plus a white
# fourth channel (forces the non-primary additive path).
C2_WINDOWS = [(0.0, 65535.0), (1755.0, 51199.0), (3218.0, 26623.0), (100.0, 4000.0)]
C2_COLORS = [(0, 0, 255, 255), (0, 255, 0, 255), (255, 0, 0, 255), (255, 255, 255, 255)]


def microscopy_u16(h, w, rng, blobs=32):
    img = rng.gamma(2.0, 300.0, size=(h, w))
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float32)
    for _ in range(blobs):
        cy, cx = rng.uniform(0, h), rng.uniform(0, w)
        s = rng.uniform(3, max(4.0, min(h, w) / 16))
        a = rng.uniform(2000, 40000)
        img += a * np.exp(-((yy - cy) ** 2 + (xx - cx) ** 2) / (2 * s * s))
    return np.clip(img, 0, 65535).astype(np.uint16)


def tile_u16(tile_index, channels, h, w, uniform=False):
    rng = np.random.default_rng(SEED + tile_index)
    if uniform:
        return [rng.integers(0, 65536, size=(h, w), dtype=np.uint16) for _ in range(channels)]
    return [microscopy_u16(h, w, rng) for _ in range(channels)]


def to_big_endian(a):
    return a.astype(a.dtype.newbyteorder(">"))


def c2_channels(n=4):
    from .renderer import f32
    return [{"active": True, "input_start": f32(C2_WINDOWS[i][0]), "input_end": f32(C2_WINDOWS[i][1]),
             "global_min": 0.0, "global_max": 65535.0, "rgba": C2_COLORS[i]} for i in range(n)]


def torch_tiles_u16(n_tiles, channels, h, w, device, seed=SEED):
    """Device-resident batch [n_tiles][channels][h][w] uint16 (stored as int16 bits) with the
    microscopy distribution, generated on the GPU (torch is only the allocator/RNG here)."""
    import torch
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    torch.manual_seed(seed)                 # the Gamma background samples from the global RNG
    out = torch.empty((n_tiles, channels, h, w), dtype=torch.int16, device=device)
    yy = torch.arange(h, device=device, dtype=torch.float32).view(h, 1)
    xx = torch.arange(w, device=device, dtype=torch.float32).view(1, w)
    for t in range(n_tiles):
        for c in range(channels):
            k = torch.distributions.Gamma(torch.tensor(2.0, device=device), torch.tensor(1 / 300.0, device=device))
            img = k.sample((h, w))
            p = torch.rand((32, 4), generator=g, device=device)
            for b in range(32):
                cy, cx = p[b, 0] * h, p[b, 1] * w
                s = 3 + p[b, 2] * (min(h, w) / 16 - 3)
                a = 2000 + p[b, 3] * 38000
                img += a * torch.exp(-((yy - cy) ** 2 + (xx - cx) ** 2) / (2 * s * s))
            u = img.clamp(0, 65535).to(torch.int32)
            out[t, c] = (u - 65536 * (u >= 32768).to(torch.int32)).to(torch.int16)
    return out


C5_LUT = np.concatenate([np.arange(256), np.arange(256) // 2, 255 - np.arange(256)]).astype(np.uint8)
# x^0.5 needs a window start above 0: on the +-normal channel p1 is about -700, where pow(ws, 0.5)
# is NaN, a0 is NaN and the whole channel would quantize to cdStart (a constant that never
# exercises the +-1 float bar).  The window start is held at 1.0 there.
C5_POLY_MIN_START = 1.0


def c5_planes(h, w, rng):
    """C5 (BASELINE configs[4]): 3-channel float32, lognormal(5, 1.5) / normal(0, 300) / lognormal."""
    return [rng.lognormal(5, 1.5, size=(h, w)).astype(np.float32),
            rng.normal(0, 300, size=(h, w)).astype(np.float32),
            rng.lognormal(5, 1.5, size=(h, w)).astype(np.float32)]


def c5_channels(planes):
    """C5 render settings: windows at p1/p99 of each channel; log (reverse) / poly k = 0.5 (window
    start >= C5_POLY_MIN_START) / poly k = 2 + .lut."""
    from . import _lib
    from .renderer import f32
    chans = []
    for i, p in enumerate(planes):
        lo, hi = float(np.percentile(p, 1)), float(np.percentile(p, 99))
        if i == 1:
            lo = max(lo, C5_POLY_MIN_START)
        chans.append({"input_start": f32(lo), "input_end": f32(hi), "rgba": C2_COLORS[i]})
    chans[0].update(family=_lib.FAMILY_LOGARITHMIC, reverse=True)
    chans[1].update(family=_lib.FAMILY_POLYNOMIAL, coefficient=0.5)
    chans[2].update(family=_lib.FAMILY_POLYNOMIAL, coefficient=2.0, lut=C5_LUT)
    return chans
