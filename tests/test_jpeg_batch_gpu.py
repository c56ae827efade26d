"""Batched JPEG (omr_encode_jpeg_batch[_device]) on the GPU: every tile's file byte-identical to
the CPU restatement (itself pinned to libjpeg-turbo, tests/test_oracle.py), across ragged sizes,
qualities, content that exercises ZRL/EOB/long symbols, tile strides and undersized outputs.
"""
import os

import numpy as np
import pytest

import oracle_lib as O
from omr import _lib
from omr.synthetic import c2_channels, tile_u16

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def argb_of(rgb):
    rgb = rgb.astype(np.uint32)
    return (0xFF000000 | (rgb[..., 0] << 16) | (rgb[..., 1] << 8) | rgb[..., 2]).astype(np.uint32)


def content(kind, h, w, seed):
    rng = np.random.default_rng(seed)
    if kind == "noise":                      # dense high-frequency blocks: long lanes, big values
        return rng.integers(0, 2**32, (h, w), dtype=np.uint32)
    if kind == "sparse":                     # isolated dots: long zero runs -> ZRL codes
        img = np.zeros((h, w, 3), np.uint8)
        n = max(1, h * w // 200)
        img[rng.integers(0, h, n), rng.integers(0, w, n)] = rng.integers(0, 256, (n, 3))
        return argb_of(img)
    if kind == "flat":                       # all-zero AC: EOB-only blocks, DC-only
        return np.full((h, w), 0xFF336699, np.uint32)
    if kind == "grey":                       # r == g == b (greyscale model): B1's grey-MCU path,
        v = rng.integers(0, 256, (h, w))     # with a few colour pixels so some MCUs are mixed
        img = np.stack([v, v, v], -1)
        img[rng.integers(0, h, 3), rng.integers(0, w, 3), 0] ^= 1
        return argb_of(img)
    yy, xx = np.mgrid[0:h, 0:w]               # smooth gradient + mild noise
    rgb = np.stack([(xx * 255 // max(w - 1, 1)), (yy * 255 // max(h - 1, 1)), (xx + yy) % 256], -1)
    rgb = np.clip(rgb + rng.integers(-3, 4, rgb.shape), 0, 255)
    return argb_of(rgb)


def run_batch(ctx, tiles, w, h, q, stride=None):
    import torch
    n = len(tiles)
    stride = stride or w * h
    buf = np.zeros(n * stride, np.uint32)
    for i, t in enumerate(tiles):
        buf[i * stride:i * stride + w * h] = t.reshape(-1)
    d = torch.from_numpy(buf.view(np.int32)).to("cuda")
    # room for noise at q 1.0 (over 1 B/px): the default cap assumes typical content
    return ctx.encode_jpeg_batch(d, n, w, h, q, cap=n * (4 * w * h + 4096),
                                 tile_stride=stride if stride != w * h else 0)


@pytest.mark.parametrize("w,h", [(1, 1), (8, 8), (17, 9), (16, 16), (333, 77), (15, 200), (256, 256)])
@pytest.mark.parametrize("q", [0.85, 1.0, 0.05])
def test_batch_byte_identical_mixed_content(ctx, w, h, q):
    kinds = ["noise", "sparse", "flat", "smooth", "grey"]
    tiles = [content(kinds[i % 5], h, w, 1000 * w + h + i) for i in range(6)]
    got = run_batch(ctx, tiles, w, h, q)
    for i, t in enumerate(tiles):
        assert got[i] == O.encode_jpeg(t, w, h, q), f"tile {i} ({kinds[i % 5]})"


def test_batch_golden_vectors(ctx):
    g = np.load(os.path.join(GOLDEN, "jpeg_golden.npz"))
    n = len([k for k in g.files if k.startswith("rgb_")])
    for i in range(n):
        rgb, meta = g[f"rgb_{i}"], g[f"meta_{i}"]
        w, h, q = int(meta[0]), int(meta[1]), float(meta[2])
        a = argb_of(rgb)
        got = run_batch(ctx, [a, a[::-1].copy()], w, h, q)
        assert got[0] == O.encode_jpeg(a, w, h, q), f"case {i}"
        assert got[1] == O.encode_jpeg(a[::-1].copy(), w, h, q)


def test_batch_rendered_c2_tiles_1024(ctx):
    """C2 tiles rendered by the batch renderer, then batch-encoded: the render_image_region
    default (format=jpeg) on a whole batch."""
    import torch
    n, w, h = 4, 1024, 1024
    planes = [[p.astype(">u2") for p in tile_u16(t, 4, h, w)] for t in range(n)]
    raw = b"".join(p.tobytes() for t in planes for p in t)   # big-endian bytes (np.stack would go native)
    data = torch.from_numpy(np.frombuffer(raw, np.int16).copy()).to("cuda")
    out = torch.empty((n, h, w), dtype=torch.int32, device="cuda")
    pb = w * h * 2
    ctx.render_batch_strided_device(O.make_qdef("rgb"), c2_channels(4), data, 4 * pb, pb, n,
                                    _lib.PIXELS_UINT16, w, h, out, big_endian=True)
    got = ctx.encode_jpeg_batch(out, n, w, h, 0.9)
    for t in range(n):
        st, argb = O.render(c2_channels(4), planes[t], _lib.PIXELS_UINT16, w, h, big_endian=True)
        assert got[t] == O.encode_jpeg(argb, w, h, 0.9), f"tile {t}"


def test_batch_tile_stride_and_device_api(ctx):
    import torch
    w, h, n = 40, 24, 5
    tiles = [content("smooth", h, w, 7 + i) for i in range(n)]
    got = run_batch(ctx, tiles, w, h, 0.7, stride=w * h + 123)
    assert all(got[i] == O.encode_jpeg(tiles[i], w, h, 0.7) for i in range(n))
    # device API: files packed back to back, status per tile
    d = torch.from_numpy(np.stack(tiles).view(np.int32)).to("cuda")
    exp = [O.encode_jpeg(t, w, h, 0.7) for t in tiles]
    cap = sum(len(e) for e in exp[:3]) + 10          # room for the first three only
    d_out = torch.zeros(cap, dtype=torch.uint8, device="cuda")
    offs = torch.zeros(n, dtype=torch.int64, device="cuda")
    lens = torch.zeros(n, dtype=torch.int32, device="cuda")
    stat = torch.full((n,), -1, dtype=torch.int32, device="cuda")
    ctx.encode_jpeg_batch_device(d, n, w, h, 0.7, d_out, offs, lens, stat)
    ctx.synchronize()
    o, ln, s = offs.cpu().numpy(), lens.cpu().numpy(), stat.cpu().numpy()
    host = d_out.cpu().numpy().tobytes()
    for i in range(3):
        assert s[i] == _lib.OK and host[o[i]:o[i] + ln[i]] == exp[i]
    assert list(s[3:]) == [_lib.BUFFER_TOO_SMALL] * 2 and list(ln[3:]) == [0, 0]


def test_batch_errors(ctx):
    import torch
    d = torch.zeros(64, dtype=torch.int32, device="cuda")
    for n, w, h in [(0, 8, 8), (1, 0, 8), (1, 8, 5000)]:
        with pytest.raises(_lib.OmrError) as e:
            ctx.encode_jpeg_batch(d, n, w, h, 0.9)
        assert e.value.status == _lib.INVALID_ARGUMENT
    with pytest.raises(_lib.OmrError) as e:
        ctx.encode_jpeg_batch(d, 1, 8, 8, 0.9, cap=100)   # a 8x8 file is > 100 bytes
    assert e.value.status == _lib.BUFFER_TOO_SMALL


@pytest.mark.parametrize("seed", list(range(int(os.environ.get("OMR_SWEEP_SEEDS", "24")))))
def test_jpeg_sweep_sizes_qualities(ctx, seed):
    """Random tile sizes (1..300 per side, any remainder mod 16), qualities in (0, 1] and content
    kinds through the batched encoder and the single-tile entry point: byte-identical to the
    restatement."""
    import torch
    rng = np.random.default_rng(500 + seed)
    w, h = int(rng.integers(1, 301)), int(rng.integers(1, 301))
    q = float(rng.choice([0.01, 0.3, 0.75, 0.9, 1.0, float(rng.uniform(0.02, 1.0))]))
    kinds = ["noise", "sparse", "flat", "smooth", "grey"]
    tiles = [content(kinds[int(rng.integers(0, 5))], h, w, 40 * seed + i) for i in range(3)]
    got = run_batch(ctx, tiles, w, h, q)
    for i, t in enumerate(tiles):
        exp = O.encode_jpeg(t, w, h, q)
        assert got[i] == exp, f"batch tile {i} {w}x{h} q={q}"
    d = torch.from_numpy(tiles[0].reshape(-1).view(np.int32).copy()).to("cuda")
    assert ctx.encode_jpeg_device(d, w, h, q) == O.encode_jpeg(tiles[0], w, h, q), f"single {w}x{h} q={q}"


def patchwork(h, w, seed, p_noise=0.3):
    """16x16 patches of full-range noise among smooth ones: at high quality the noisy MCUs hold
    ACs outside int8 (their blocks go out in the int16 form) next to int8 MCUs in the same wave."""
    rng = np.random.default_rng(seed)
    img = content("smooth", h, w, seed)
    noise = content("noise", h, w, seed + 1)
    for y in range(0, h, 16):
        for x in range(0, w, 16):
            if rng.random() < p_noise:
                img[y:y + 16, x:x + 16] = noise[y:y + 16, x:x + 16]
    return img


@pytest.mark.parametrize("q", [1.0, 0.97, 0.9])
@pytest.mark.parametrize("p_noise", [0.05, 0.3])
def test_batch_int8_and_int16_blocks_in_one_wave(ctx, q, p_noise):
    """B1 stores an MCU's blocks as int8 when every AC fits and as int16 otherwise; B2a walks each
    form and B3 widens int8 blocks in waves that also hold int16 ones: files byte-identical."""
    w, h = 256, 128
    tiles = [patchwork(h, w, 77 + i, p_noise) for i in range(3)]
    got = run_batch(ctx, tiles, w, h, q)
    for i, t in enumerate(tiles):
        assert got[i] == O.encode_jpeg(t, w, h, q), f"tile {i}"
