"""JPEG pinned at BASELINE config size against PIL / libjpeg-turbo itself (not the CPU
restatement): C1 (1-channel uint8 1024^2 greyscale, q 0.9) and C2 (4-channel uint16 1024^2 colour
composite, q 0.9), encoded on the box by PIL at ImageIO's quality tables (tests/golden/make_golden.py
java_quant_tables, an independent Python restatement of javax.imageio's table scaling) and 4:2:0.
The GPU file must be byte-identical -- headers and entropy-coded segment -- on the single-tile
path, the batched encoder and the fused render -> JPEG kernel.

The ImageIO encoder (LocalCompress.compressToStream, ImageRegionRequestHandler.java:576-582) is the
IJG islow lineage libjpeg-turbo implements; jpeg is the default format (ImageRegionCtx.java:146)."""
import importlib.util
import io
import os

import numpy as np
import pytest

import oracle_lib as O
from omr import _lib
from omr.synthetic import c2_channels, tile_u16

pytestmark = pytest.mark.gpu

_spec = importlib.util.spec_from_file_location(
    "make_golden", os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "make_golden.py"))
_mg = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(_mg)

W = H = 1024
Q = 0.9


def _pil_jpeg(argb, q):
    from PIL import Image
    rgb = np.ascontiguousarray(argb.view(np.uint8).reshape(H, W, 4)[..., 2::-1])
    ql, qc = _mg.java_quant_tables(q)
    buf = io.BytesIO()
    Image.fromarray(rgb, "RGB").save(buf, "JPEG", qtables=[ql, qc], subsampling=2)
    return buf.getvalue()


def _scan(b):
    """The entropy-coded segment: from after the SOS header to the EOI marker."""
    sos = b.index(b"\xff\xda")
    n = int.from_bytes(b[sos + 2:sos + 4], "big")
    return b[sos + 2 + n:-2]


def _check(files, ref, what):
    for i, f in enumerate(files):
        assert _scan(f) == _scan(ref), f"{what} tile {i}: entropy-coded segment differs from PIL"
        assert f == ref, f"{what} tile {i}: headers differ from PIL"


def _paths(ctx, qdef, chans, raw_tiles, pt, big_endian, argb):
    """Single-tile, batched and fused JPEG of identical tiles; returns (single, batch, fused)."""
    import torch
    n = len(raw_tiles)
    data = torch.from_numpy(np.stack(raw_tiles)).to("cuda")
    plane = raw_tiles[0].size // len(chans)
    out = torch.empty((n, H, W), dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    ctx.render_batch_strided_device(qdef, chans, data, len(chans) * plane, plane, n, pt, W, H, out,
                                    big_endian=big_endian)
    ctx.synchronize()
    np.testing.assert_array_equal(out[0].cpu().numpy().view(np.uint32), argb)     # render exact first
    single = [ctx.encode_jpeg_device(out[i], W, H, Q) for i in range(n)]
    batch = ctx.encode_jpeg_batch(out, n, W, H, Q)
    cap = n * int(_lib.lib.omr_jpeg_max_bytes(W, H))
    d_out = torch.empty(cap, dtype=torch.uint8, device="cuda")
    offs = torch.empty(n, dtype=torch.int64, device="cuda")
    lens = torch.empty(n, dtype=torch.int32, device="cuda")
    ctx.render_jpeg_batch_strided_device(qdef, chans, data, len(chans) * plane, plane, n, pt, W, H, Q, d_out, offs,
                                         lens, big_endian=big_endian)
    ctx.synchronize()
    b, o, ln = d_out.cpu().numpy(), offs.cpu().numpy(), lens.cpu().numpy().view(np.uint32)
    fused = [b[o[i]:o[i] + ln[i]].tobytes() for i in range(n)]
    return single, batch, fused


def test_c1_u8_greyscale_1024_matches_pil(ctx):
    rng = np.random.default_rng(20261015)
    p = rng.integers(0, 256, (H, W), dtype=np.uint8)
    chans = [{"input_start": 0.0, "input_end": 255.0, "global_min": 0, "global_max": 255}]
    qd = O.make_qdef("greyscale")
    st, argb = O.render(chans, [p], _lib.PIXELS_UINT8, W, H, model="greyscale")
    assert st == 0
    ref = _pil_jpeg(argb, Q)
    single, batch, fused = _paths(ctx, qd, chans, [p.reshape(-1)] * 2, _lib.PIXELS_UINT8, False, argb)
    _check(single, ref, "C1 single")
    _check(batch, ref, "C1 batch")
    _check(fused, ref, "C1 fused")


@pytest.mark.parametrize("uniform", [False, True])
def test_c2_u16_4ch_1024_matches_pil(ctx, uniform):
    planes = [p.astype(">u2") for p in tile_u16(0, 4, H, W, uniform=uniform)]
    chans = c2_channels(4)
    qd = O.make_qdef("rgb")
    st, argb = O.render(chans, planes, _lib.PIXELS_UINT16, W, H, big_endian=True)
    assert st == 0
    ref = _pil_jpeg(argb, Q)
    raw = np.concatenate([p.view(np.uint8).reshape(-1) for p in planes])
    single, batch, fused = _paths(ctx, qd, chans, [raw] * 2, _lib.PIXELS_UINT16, True, argb)
    _check(single, ref, "C2 single")
    _check(batch, ref, "C2 batch")
    _check(fused, ref, "C2 fused")
