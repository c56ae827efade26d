"""The sizes the reference actually serves, end to end on the GPU.

- `tile=0,x,y,2048,2048`: maxTileLength defaults to 2048 (beanRefContext.xml:63-65) and tile mode
  is clamped to it (ImageRegionRequestHandler.java:804-812), so a 2048^2 tile is the largest tile a
  viewer receives.  A C2 tile (4-channel big-endian uint16) goes through the render (bit-exact vs
  the CPU restatement), JPEG on the single-tile, batched and fused render -> JPEG paths (byte-
  identical to PIL / libjpeg-turbo at the Java tables) and PNG (single request and batched: decoded
  pixels equal the render).
- Region mode is unbounded apart from the image (:817-827): a 6000 x 2500 full-plane region goes
  through the render, the one-request render -> JPEG call (omr_render_jpeg, whose regions past
  4096 a side take the whole-image J1-J6 encoder), the device JPEG encoder and the whole-image PNG
  path (past the batched encoder's 4096-a-side limit).
- Shape masks wider than 4096 (ShapeMaskRequestHandler.java:165-221: 1-bit rows when
  width % 8 == 0, 8-bit rows otherwise), single and batched, decoded against the restatement's
  unpack / flip.
"""
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

Q = 0.9


def _pil_jpeg(argb, w, h, q):
    from PIL import Image
    rgb = np.ascontiguousarray(argb.view(np.uint8).reshape(h, w, 4)[..., 2::-1])
    ql, qc = _mg.java_quant_tables(q)
    buf = io.BytesIO()
    Image.fromarray(rgb, "RGB").save(buf, "JPEG", qtables=[ql, qc], subsampling=2)
    return buf.getvalue()


def _png_rgb(b):
    from PIL import Image
    return np.asarray(Image.open(io.BytesIO(b)).convert("RGB"))


def _rgb(argb, w, h):
    return np.ascontiguousarray(argb.view(np.uint8).reshape(h, w, 4)[..., 2::-1])


def _c2(w, h, seed=0):
    planes = [p.astype(">u2") for p in tile_u16(seed, 4, h, w)]
    chans = c2_channels(4)
    st, argb = O.render(chans, planes, _lib.PIXELS_UINT16, w, h, big_endian=True)
    assert st == 0
    return planes, chans, argb


def test_max_tile_2048_c2_render_jpeg_png(ctx):
    import torch
    W = H = 2048
    planes, chans, argb = _c2(W, H)
    qd = O.make_qdef("rgb")
    raw = np.concatenate([p.view(np.uint8).reshape(-1) for p in planes])
    n = 2
    data = torch.from_numpy(np.stack([raw] * n)).to("cuda")
    plane = W * H * 2
    out = torch.empty((n, H, W), dtype=torch.int32, device="cuda")
    ctx.render_batch_strided_device(qd, chans, data, 4 * plane, plane, n, _lib.PIXELS_UINT16, W, H, out,
                                    big_endian=True)
    ctx.synchronize()
    for i in range(n):
        np.testing.assert_array_equal(out[i].cpu().numpy().view(np.uint32), argb)
    ref = _pil_jpeg(argb, W, H, Q)
    assert ctx.encode_jpeg_device(out[0], W, H, Q) == ref, "single-tile JPEG differs from PIL"
    for i, f in enumerate(ctx.encode_jpeg_batch(out, n, W, H, Q)):
        assert f == ref, f"batched JPEG tile {i} differs from PIL"
    cap = n * int(_lib.lib.omr_jpeg_max_bytes(W, H))
    d_out = torch.empty(cap, dtype=torch.uint8, device="cuda")
    offs = torch.empty(n, dtype=torch.int64, device="cuda")
    lens = torch.empty(n, dtype=torch.int32, device="cuda")
    stat = torch.empty(n, dtype=torch.int32, device="cuda")
    ctx.render_jpeg_batch_strided_device(qd, chans, data, 4 * plane, plane, n, _lib.PIXELS_UINT16, W, H, Q, d_out,
                                         offs, lens, stat, big_endian=True)
    ctx.synchronize()
    b, o, ln = d_out.cpu().numpy(), offs.cpu().numpy(), lens.cpu().numpy().view(np.uint32)
    assert (stat.cpu().numpy() == 0).all()
    for i in range(n):
        assert b[o[i]:o[i] + ln[i]].tobytes() == ref, f"fused render -> JPEG tile {i} differs from PIL"
    dev = [data[0, c * plane:(c + 1) * plane] for c in range(4)]
    assert ctx.render_jpeg_device(qd, chans, dev, _lib.PIXELS_UINT16, W, H, Q, big_endian=True) == ref
    # PNG: the single request (a batch of one) and the batched encoder decode to the render
    rgb = _rgb(argb, W, H)
    np.testing.assert_array_equal(_png_rgb(ctx.encode_png_device(out[0], W, H)), rgb)
    pcap = n * int(_lib.lib.omr_png_batch_max_bytes(W, H, 3, 1))
    p_out = torch.empty(pcap, dtype=torch.uint8, device="cuda")
    p_offs = torch.empty(n, dtype=torch.int64, device="cuda")
    p_lens = torch.empty(n, dtype=torch.int32, device="cuda")
    p_stat = torch.empty(n, dtype=torch.int32, device="cuda")
    ctx.encode_png_batch_device(out, n, W, H, p_out, p_offs, p_lens, p_stat)
    ctx.synchronize()
    assert (p_stat.cpu().numpy() == 0).all()
    pb, po, pl = p_out.cpu().numpy(), p_offs.cpu().numpy(), p_lens.cpu().numpy().view(np.uint32)
    for i in range(n):
        np.testing.assert_array_equal(_png_rgb(pb[po[i]:po[i] + pl[i]].tobytes()), rgb)


def test_region_6000x2500_render_jpeg_png(ctx):
    """A full-plane region wider than 4096 (region mode: no maxTileLength clamp)."""
    import torch
    W, H = 6000, 2500
    planes, chans, argb = _c2(W, H, seed=3)
    qd = O.make_qdef("rgb")
    dev = [torch.from_numpy(np.ascontiguousarray(p).view(np.uint8).reshape(-1)).to("cuda") for p in planes]
    out = torch.empty((H, W), dtype=torch.int32, device="cuda")
    ctx.render_packed_int_device(qd, chans, dev, _lib.PIXELS_UINT16, W, H, out, big_endian=True)
    ctx.synchronize()
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32), argb)
    ref = _pil_jpeg(argb, W, H, Q)
    assert ctx.encode_jpeg_device(out, W, H, Q) == ref, "whole-image JPEG differs from PIL"
    assert ctx.render_jpeg_device(qd, chans, dev, _lib.PIXELS_UINT16, W, H, Q, big_endian=True) == ref, \
        "render -> JPEG request past 4096 differs from PIL"
    np.testing.assert_array_equal(_png_rgb(ctx.encode_png_device(out, W, H)), _rgb(argb, W, H))
    # the batched JPEG / PNG encoders take tiles up to 4096 a side and say so
    with pytest.raises(_lib.OmrError) as e:
        ctx.encode_jpeg_batch(out, 1, W, H, Q)
    assert e.value.status == _lib.INVALID_ARGUMENT


def test_region_flipped_past_4096(ctx):
    """Flips on the wide region (the reference flips the rendered buffer, :574-575, :616-642)."""
    import torch
    W, H = 4104, 40
    planes, chans, _ = _c2(W, H, seed=5)
    qd = O.make_qdef("rgb")
    dev = [torch.from_numpy(np.ascontiguousarray(p).view(np.uint8).reshape(-1)).to("cuda") for p in planes]
    for fh, fv in ((True, False), (False, True), (True, True)):
        st, exp = O.render(chans, planes, _lib.PIXELS_UINT16, W, H, big_endian=True, flip_h=fh, flip_v=fv)
        assert st == 0
        out = torch.empty((H, W), dtype=torch.int32, device="cuda")
        ctx.render_packed_int_device(qd, chans, dev, _lib.PIXELS_UINT16, W, H, out, big_endian=True, flip_h=fh,
                                     flip_v=fv)
        ctx.synchronize()
        np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32), exp)
        assert ctx.render_jpeg_device(qd, chans, dev, _lib.PIXELS_UINT16, W, H, Q, big_endian=True, flip_h=fh,
                                      flip_v=fv) == _pil_jpeg(exp, W, H, Q)


@pytest.fixture
def pixel_flip(ctx):
    ctx.set_semantics(_lib.SEM_MASK_PIXEL_FLIP)
    with O.semantics(_lib.SEM_MASK_PIXEL_FLIP):
        yield ctx
    ctx.set_semantics(0)


def _mask_rgba(png):
    from PIL import Image
    return np.asarray(Image.open(io.BytesIO(png)).convert("RGBA"))


def _expect_mask(bits, w, h, fh, fv, rgba):
    st, idx = O.mask_indices(bits, w, h, fh, fv)
    assert st == 0
    exp = np.zeros((h, w, 4), np.uint8)
    exp[idx == 1] = rgba
    return exp


@pytest.mark.parametrize("w,h", [(5000, 64), (4999, 37), (8192, 8)])
def test_shape_mask_wider_than_4096(pixel_flip, w, h):
    ctx = pixel_flip
    rng = np.random.default_rng(w + h)
    bits = rng.integers(0, 256, (w * h + 7) // 8, dtype=np.uint8).tobytes()
    rgba = (255, 0, 0, 128)
    masks = [(bits, w, h, rgba, fh, fv) for fh, fv in ((False, False), (True, False), (False, True), (True, True))]
    res = ctx.render_shape_mask_png_batch(masks)
    for (b, mw, mh, col, fh, fv), (st, png) in zip(masks, res):
        assert st == 0
        exp = _expect_mask(b, mw, mh, fh, fv, col)
        np.testing.assert_array_equal(_mask_rgba(png), exp)
        np.testing.assert_array_equal(_mask_rgba(ctx.render_shape_mask_png(b, mw, mh, col, fh, fv)), exp)
