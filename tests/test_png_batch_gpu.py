"""Batched PNG (omr_encode_png_batch_device) and the shape-mask batch (omr_render_shape_mask_png_batch)
on the GPU.

The parity bar of PNG is decoded pixels: every file decodes (PIL) to the
tile's RGB / the mask's palette image, every chunk CRC and the zlib Adler-32 check (PIL and zlib
verify them).  Where the batch chose the dynamic-Huffman stream the file is also byte-identical to
the single-tile encoder's (same filters, parse and code), so the batch is pinned to the path the
round-1..3 PNG tests already cover; noise takes stored blocks (of the filtered rows) in the batch.
Masks are checked against the CPU restatement's unpack/flip (oracle mask_indices), including the
reference's 404 cases and its packed-buffer flip (ShapeMaskRequestHandler.java:165-207).
"""
import io
import struct
import zlib

import numpy as np
import pytest

import oracle_lib as O
from omr import _lib

pytestmark = pytest.mark.gpu


def decode(b):
    from PIL import Image
    return Image.open(io.BytesIO(b))


def rgb_of(argb):
    return np.stack([(argb >> 16) & 0xFF, (argb >> 8) & 0xFF, argb & 0xFF], -1).astype(np.uint8)


def chunks(png):
    assert png[:8] == b"\x89PNG\r\n\x1a\n"
    i, out = 8, []
    while i < len(png):
        ln, = struct.unpack(">I", png[i:i + 4])
        typ, data = png[i + 4:i + 8], png[i + 8:i + 8 + ln]
        crc, = struct.unpack(">I", png[i + 8 + ln:i + 12 + ln])
        assert zlib.crc32(png[i + 4:i + 8 + ln]) == crc, typ
        out.append((typ, data))
        i += 12 + ln
    assert i == len(png) and out[-1][0] == b"IEND"
    return out


def idat_is_stored(png):
    z = b"".join(d for t, d in chunks(png) if t == b"IDAT")
    return (z[2] >> 1) & 3 == 0


def tiles(kind, n, w, h, seed):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        if kind == "noise":
            a = rng.integers(0, 2**32, (h, w), dtype=np.uint64).astype(np.uint32)
        elif kind == "flat":
            a = np.full((h, w), 0xFF000000 | (i * 0x010203), np.uint32)
        else:                                   # image-like: gradients, blocks, a little noise
            yy, xx = np.mgrid[0:h, 0:w]
            a = ((xx * 255 // max(w - 1, 1)) << 16 | (yy * 255 // max(h - 1, 1)) << 8 | ((xx + yy + i) % 256))
            a = a.astype(np.uint32) | 0xFF000000
            a[h // 4:h // 2, w // 5:w // 2] = 0xFF102030 + i
            a ^= rng.integers(0, 3, (h, w), dtype=np.uint32)
        out.append(a)
    return np.stack(out)


def encode_batch(ctx, argb, cap=None, stride=0):
    import torch
    n, h, w = argb.shape
    d = torch.from_numpy(argb.view(np.int32).copy()).to("cuda")
    if cap is None:
        cap = _lib.lib.omr_png_batch_max_bytes(w, h, 3, n)
    out = torch.empty(max(cap, 1), dtype=torch.uint8, device="cuda")
    offs = torch.full((n,), -1, dtype=torch.int64, device="cuda")
    lens = torch.full((n,), -1, dtype=torch.int32, device="cuda")
    stat = torch.full((n,), -1, dtype=torch.int32, device="cuda")
    ctx.encode_png_batch_device(d, n, w, h, out[:cap] if cap else out[:0], offs, lens, stat, tile_stride=stride)
    torch.cuda.synchronize()
    o, l, s, b = offs.cpu().numpy(), lens.cpu().numpy(), stat.cpu().numpy(), out.cpu().numpy()
    return [(int(s[i]), int(o[i]), b[int(o[i]):int(o[i]) + int(l[i])].tobytes()) for i in range(n)]


@pytest.mark.parametrize("kind,n,w,h", [("image", 1, 1024, 1024), ("image", 16, 256, 256), ("image", 3, 37, 53),
                                        ("flat", 5, 64, 8), ("image", 7, 1, 1), ("noise", 4, 300, 230),
                                        ("image", 2, 4096, 17)])
def test_png_batch_decodes_and_matches_single(ctx, kind, n, w, h):
    argb = tiles(kind, n, w, h, n * w + h)
    res = encode_batch(ctx, argb)
    for i, (st, off, png) in enumerate(res):
        assert st == 0 and off % 16 == 0
        chunks(png)
        np.testing.assert_array_equal(np.asarray(decode(png)), rgb_of(argb[i]))
        if kind == "noise":
            assert idat_is_stored(png)
        assert png == ctx.encode_png(argb[i], w, h), f"tile {i}: file differs from the single-tile encoder's"
    offs = [r[1] for r in res]
    assert offs == sorted(offs) and len(set(offs)) == n


def test_png_batch_mixed_content_and_stride(ctx):
    """Flat, image-like and noise tiles in one launch (each picks dynamic or stored on its own), and
    a tile stride larger than the tile."""
    import torch
    w, h = 128, 96
    argb = np.concatenate([tiles("flat", 2, w, h, 1), tiles("noise", 2, w, h, 2), tiles("image", 2, w, h, 3)])
    n = len(argb)
    pad = np.zeros((n, h + 3, w), np.uint32)
    pad[:, :h] = argb
    res = encode_batch(ctx, argb)
    for i, (st, _, png) in enumerate(res):
        assert st == 0
        np.testing.assert_array_equal(np.asarray(decode(png)), rgb_of(argb[i]))
    # strided: tile i at i * (h + 3) * w pixels
    d = torch.from_numpy(pad.view(np.int32).reshape(-1)).to("cuda")
    cap = _lib.lib.omr_png_batch_max_bytes(w, h, 3, n)
    out = torch.empty(cap, dtype=torch.uint8, device="cuda")
    offs = torch.zeros(n, dtype=torch.int64, device="cuda")
    lens = torch.zeros(n, dtype=torch.int32, device="cuda")
    ctx.encode_png_batch_device(d, n, w, h, out, offs, lens, None, tile_stride=(h + 3) * w)
    b, o, ln = out.cpu().numpy(), offs.cpu().numpy(), lens.cpu().numpy()
    for i in range(n):
        assert b[o[i]:o[i] + ln[i]].tobytes() == res[i][2]


def test_png_batch_output_too_small(ctx):
    """Files that do not fit report OMR_BUFFER_TOO_SMALL with length 0; the ones before still land."""
    argb = tiles("image", 4, 64, 64, 9)
    full = encode_batch(ctx, argb)
    need = full[1][1] + (len(full[1][2]) + 15) // 16 * 16   # room for exactly the first two 16-byte slots
    res = encode_batch(ctx, argb, cap=need)
    assert [r[0] for r in res] == [0, 0, _lib.BUFFER_TOO_SMALL, _lib.BUFFER_TOO_SMALL]
    assert res[0][2] == full[0][2] and res[1][2] == full[1][2]
    assert res[2][2] == b"" and res[3][2] == b""


def test_png_batch_rendered_c2_tiles(ctx):
    """The bench's workload: C2 tiles rendered on the GPU, batch-encoded, decoded == the oracle's ARGB."""
    import torch
    from omr.context import make_qdef
    from omr.synthetic import c2_channels, tile_u16
    n, t = 6, 256
    chans = c2_channels(4)
    planes = [[p.astype(">u2") for p in tile_u16(k, 4, t, t)] for k in range(n)]
    # np.stack of '>u2' arrays yields native uint16: store big-endian explicitly
    host = np.stack([np.stack(p) for p in planes]).astype(">u2")
    base = torch.from_numpy(host.view(np.uint8).reshape(-1).copy()).to("cuda")
    argb = torch.empty((n, t, t), dtype=torch.int32, device="cuda")
    plane = t * t * 2
    ctx.render_batch_strided_device(make_qdef("rgb"), chans, base, 4 * plane, plane, n, _lib.PIXELS_UINT16, t, t,
                                    argb, big_endian=True)
    cap = _lib.lib.omr_png_batch_max_bytes(t, t, 3, n)
    out = torch.empty(cap, dtype=torch.uint8, device="cuda")
    offs = torch.zeros(n, dtype=torch.int64, device="cuda")
    lens = torch.zeros(n, dtype=torch.int32, device="cuda")
    stat = torch.full((n,), -1, dtype=torch.int32, device="cuda")
    ctx.encode_png_batch_device(argb, n, t, t, out, offs, lens, stat)
    b, o, ln, s = out.cpu().numpy(), offs.cpu().numpy(), lens.cpu().numpy(), stat.cpu().numpy()
    for k in range(n):
        assert s[k] == 0
        st, exp = O.render(chans, planes[k], _lib.PIXELS_UINT16, t, t, big_endian=True)
        assert st == 0
        np.testing.assert_array_equal(np.asarray(decode(b[o[k]:o[k] + ln[k]].tobytes())), rgb_of(exp))


def test_png_batch_errors(ctx):
    import torch
    d = torch.zeros(16, dtype=torch.int32, device="cuda")
    out = torch.empty(4096, dtype=torch.uint8, device="cuda")
    for w, h in [(0, 4), (4, 0), (4097, 1), (1, 4097)]:
        with pytest.raises(_lib.OmrError):
            ctx.encode_png_batch_device(d, 1, w, h, out)
    ctx.encode_png_batch_device(d, 0, 4, 4, out)                      # nothing to do


def mask_rgba(png):
    return np.asarray(decode(png).convert("RGBA"))


def expect_mask(bits, w, h, fh, fv, rgba):
    st, idx = O.mask_indices(bits, w, h, fh, fv)
    assert st == 0
    exp = np.zeros((h, w, 4), np.uint8)
    exp[idx == 1] = rgba
    return exp


@pytest.fixture
def pixel_flip(ctx):
    ctx.set_semantics(_lib.SEM_MASK_PIXEL_FLIP)
    with O.semantics(_lib.SEM_MASK_PIXEL_FLIP):
        yield ctx
    ctx.set_semantics(0)


def test_mask_batch_mixed_sizes_colours_flips(pixel_flip):
    ctx = pixel_flip
    rng = np.random.default_rng(77)
    masks = []
    for k, (w, h) in enumerate([(8, 2), (4, 4), (64, 33), (37, 21), (1024, 1024), (1, 1), (333, 77), (16, 1)]):
        bits = rng.integers(0, 256, (w * h + 7) // 8, dtype=np.uint8).tobytes()
        rgba = tuple(int(v) for v in rng.integers(0, 256, 4))
        masks.append((bits, w, h, rgba, bool(k & 1), bool(k & 2)))
    res = ctx.render_shape_mask_png_batch(masks)
    for (bits, w, h, rgba, fh, fv), (st, png) in zip(masks, res):
        assert st == 0
        chunks(png)
        assert decode(png).size == (w, h)
        np.testing.assert_array_equal(mask_rgba(png), expect_mask(bits, w, h, fh, fv, rgba))
        assert png == ctx.render_shape_mask_png(bits, w, h, rgba, fh, fv)


def test_mask_batch_404_cases_and_packed_flip(ctx):
    """Each mask fails alone, with the single call's outcome: short masks, zero sizes, a null mask
    and (default semantics) the packed-buffer flip of a w % 8 == 0 mask: 404 when the buffer holds
    fewer than w*h bytes, else the byte-flipped buffer rendered as packed bits."""
    w, h = 16, 4
    good = bytes(range(8))
    big = bytes((i * 37) & 0xFF for i in range(w * h))        # w*h bytes: the packed flip succeeds
    col = (255, 0, 0, 255)
    masks = [(good, w, h, col, False, False), (bytes(2), w, h, col, False, False), (good, 0, h, col, False, False),
             (None, w, h, col, False, False), (good, w, h, col, True, False), (big, w, h, col, True, True),
             (good, 9, 3, col, True, False)]
    res = ctx.render_shape_mask_png_batch(masks)
    st = [r[0] for r in res]
    assert st == [0, _lib.NOT_FOUND, _lib.NOT_FOUND, _lib.NOT_FOUND, _lib.NOT_FOUND, 0, 0], st
    for m, (s, png) in zip(masks, res):
        if m[0] is None:
            continue
        if s:
            with pytest.raises(_lib.OmrError) as e:
                ctx.render_shape_mask_png(*m)
            assert e.value.status == s
        else:
            np.testing.assert_array_equal(mask_rgba(png), mask_rgba(ctx.render_shape_mask_png(*m)))


def test_mask_batch_capacity(pixel_flip):
    ctx = pixel_flip
    masks = [(bytes([0x5A] * 128), 32, 32, (1, 2, 3, 4), False, False) for _ in range(3)]
    full = ctx.render_shape_mask_png_batch(masks)
    one = len(full[0][1])
    res = ctx.render_shape_mask_png_batch(masks, cap=2 * ((one + 15) // 16 * 16) + 15)
    assert [r[0] for r in res] == [0, 0, _lib.BUFFER_TOO_SMALL]
    assert res[0][1] == full[0][1] and res[1][1] == full[1][1]


@pytest.mark.parametrize("kind,n,w,h", [("image", 3, 1024, 40), ("noise", 2, 1024, 9), ("image", 5, 512, 33),
                                        ("image", 4, 100, 17), ("image", 2, 764, 21), ("flat", 3, 8, 5),
                                        ("noise", 3, 256, 19), ("image", 2, 768, 26), ("noise", 2, 768, 11),
                                        ("image", 2, 260, 9)])
def test_png_batch_wave_filter_matches_workgroup_filter(ctx, kind, n, w, h, monkeypatch):
    """D1's wave form (uniform RGB batches, W % 4 == 0, W <= 1024) writes the same filtered rows,
    the same filter bytes and the same Adler partials as the workgroup form: the files are
    byte-identical (OMR_PNG_FILTER_WAVE=0 selects the workgroup form, read per call).  Widths
    256 / 512 / 768 / 1024 run the guard-free FULL instantiations (M = 1..4), the others the
    guarded ones."""
    argb = tiles(kind, n, w, h, 7 * w + h + n)
    monkeypatch.setenv("OMR_PNG_FILTER_WAVE", "0")
    ref = encode_batch(ctx, argb)
    monkeypatch.setenv("OMR_PNG_FILTER_WAVE", "1")
    got = encode_batch(ctx, argb)
    for i in range(n):
        assert got[i][0] == 0 and ref[i][0] == 0
        assert got[i][2] == ref[i][2], f"tile {i}: wave-form file differs"
        np.testing.assert_array_equal(np.asarray(decode(got[i][2])), rgb_of(argb[i]))


def test_png_batch_wave_filter_rendered_c2(ctx, monkeypatch):
    """The bench's tiles (C2 rendered on the GPU, 1024^2): wave-form and workgroup-form D1 give
    byte-identical files."""
    import torch
    from omr.synthetic import c2_channels, tile_u16
    import oracle_lib as O
    w = h = 1024
    outs = []
    for t in range(2):
        planes = [p.astype(">u2") for p in tile_u16(t, 4, h, w)]
        st, argb = O.render(c2_channels(4), planes, _lib.PIXELS_UINT16, w, h, big_endian=True)
        outs.append(argb)
    argb = np.stack(outs)
    monkeypatch.setenv("OMR_PNG_FILTER_WAVE", "0")
    ref = encode_batch(ctx, argb)
    monkeypatch.setenv("OMR_PNG_FILTER_WAVE", "1")
    got = encode_batch(ctx, argb)
    for i in range(2):
        assert got[i][2] == ref[i][2], f"tile {i}: wave-form file differs"


def test_single_request_paths_batched_and_legacy(monkeypatch):
    """Single PNG / mask requests run the batched pipeline with n = 1 (round 5); the legacy
    single-image pipeline (OMR_PNG_SINGLE_BATCHED=0, read at context creation; still the path
    for images beyond 4096 px) gives the same pixels."""
    import omr
    argb = tiles("image", 1, 300, 77, 5)[0]
    rng = np.random.default_rng(3)
    bits = rng.integers(0, 256, (37 * 21 + 7) // 8, dtype=np.uint8).tobytes()
    outs = {}
    for flag in ("1", "0"):
        monkeypatch.setenv("OMR_PNG_SINGLE_BATCHED", flag)
        c = omr.Context(0)
        try:
            outs[flag] = (c.encode_png(argb, 300, 77), c.render_shape_mask_png(bits, 37, 21, (9, 8, 7, 200), True, False))
        finally:
            c.close()
    for k in (0, 1):
        np.testing.assert_array_equal(np.asarray(decode(outs["1"][k]).convert("RGBA")),
                                      np.asarray(decode(outs["0"][k]).convert("RGBA")))
    np.testing.assert_array_equal(np.asarray(decode(outs["1"][0])), rgb_of(argb))


def test_png_batch_high_entropy_groups_in_a_dynamic_stream(ctx):
    """A compressible image with a band of noise: the dynamic stream wins overall, while the noise
    groups need more than 8 bits per byte -- P4's slow path (interior words ORed in memory).  The
    files decode to the pixels, their IDAT is dynamic, and a stored-winning image (all noise)
    skips P4 entirely."""
    rng = np.random.default_rng(77)
    w, h = 1024, 96
    a = np.full((h, w), 0xFF204060, np.uint32)
    a[40:56] = rng.integers(0, 2**32, (16, w), dtype=np.uint64).astype(np.uint32) | 0xFF000000
    noise = rng.integers(0, 2**32, (h, w), dtype=np.uint64).astype(np.uint32)
    argb = np.stack([a, noise, a])
    res = encode_batch(ctx, argb)
    for i, (st, off, png) in enumerate(res):
        assert st == 0
        chunks(png)
        np.testing.assert_array_equal(np.asarray(decode(png)), rgb_of(argb[i]))
    assert not idat_is_stored(res[0][2]) and idat_is_stored(res[1][2])
    assert res[0][2] == res[2][2]


def test_png_batch_sparse_noisy_segments(ctx):
    """A flat image with a short run of noisy pixels in every row: the stream as a whole codes far
    below 8 bits per byte, but the noisy segments' literals take long codes (> 256 bits per
    32-byte segment), so P4 codes those lanes again from their stashed bytes inside an LDS-staged
    group.  Files decode to the pixels and match the single-request path."""
    rng = np.random.default_rng(11)
    w, h = 1024, 64
    a = np.full((h, w), 0xFF204060, np.uint32)
    for y in range(h):
        x0 = int(rng.integers(0, w - 16))
        a[y, x0:x0 + 11] = rng.integers(0, 2**32, 11, dtype=np.uint64).astype(np.uint32) | 0xFF000000
    b = a.copy()
    b[::7] = 0xFF000000 | (np.arange(w, dtype=np.uint32) * 2654435761 % 2**24)
    argb = np.stack([a, b])
    res = encode_batch(ctx, argb)
    for i, (st, off, png) in enumerate(res):
        assert st == 0
        chunks(png)
        assert not idat_is_stored(png)
        np.testing.assert_array_equal(np.asarray(decode(png)), rgb_of(argb[i]))
        assert png == ctx.encode_png(argb[i], w, h)


_MODES_SCRIPT = r"""
import hashlib, os, sys
import numpy as np
sys.path.insert(0, os.path.join(os.environ["OMR_REPO"], "omero-ms-image-region_amd"))
sys.path.insert(0, os.path.join(os.environ["OMR_REPO"], "tests"))
import omr, torch
from test_png_batch_gpu import tiles, encode_batch
h = hashlib.sha256()
with omr.Context(0) as ctx:
    for kind, n, w, h_, seed in (("image", 5, 256, 200, 1), ("noise", 3, 130, 70, 2), ("flat", 2, 64, 8, 3),
                                 ("image", 3, 1, 1, 4), ("image", 2, 1023, 33, 5)):
        for st, off, png in encode_batch(ctx, tiles(kind, n, w, h_, seed)):
            assert st == 0
            h.update(png)
        h.update(ctx.encode_png(tiles(kind, 1, w, h_, seed + 7)[0], w, h_))
    rng = np.random.default_rng(6)
    for w, h_ in ((333, 77), (64, 48)):
        h.update(ctx.render_shape_mask_png(np.packbits(rng.integers(0, 2, w * h_)).tobytes(), w, h_, (9, 8, 7, 6)))
print(h.hexdigest())
"""


def test_png_direct_mode_matches_words_buffer_forms():
    """Direct mode (the default since round 6: P4 codes into the files in place, P8 stores only the
    bytes around the streams) writes the same bytes as the words-buffer forms it replaced -- P8
    with the CRC fused (OMR_PNG_DIRECT=0) and P8 + a separate P9 (OMR_PNG_CRC_P9=1).  The modes
    are read once per process, so each runs in a child process, one after another."""
    import os
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    digests = {}
    for name, env in (("direct", {}), ("fused", {"OMR_PNG_DIRECT": "0"}),
                      ("separate", {"OMR_PNG_DIRECT": "0", "OMR_PNG_CRC_P9": "1"})):
        e = dict(os.environ, OMR_REPO=repo, **env)
        r = subprocess.run([sys.executable, "-c", _MODES_SCRIPT], env=e, capture_output=True, text=True, timeout=110)
        assert r.returncode == 0, f"{name}: {r.stderr[-2000:]}"
        digests[name] = r.stdout.strip().splitlines()[-1]
    assert digests["direct"] == digests["fused"] == digests["separate"], digests
