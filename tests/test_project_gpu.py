"""K3 Z-projection and the flip kernels on the GPU vs the CPU restatement.

Projection: ProjectionService.java:46-317 (bit-exact for every pixel type: integer sums are
exact, float sums keep the reference's z order in double).  Flips: the reference's index-oracle
tests (ImageRegionRequestHandlerTest.java:69-200, ShapeMaskRequestHandlerTest.java:84-215).
"""
import os

import numpy as np
import pytest

import oracle_lib as O
from omr import _lib, flip
from omr.synthetic import c2_channels, microscopy_u16

pytestmark = pytest.mark.gpu

TYPES = [(_lib.PIXELS_UINT8, np.uint8), (_lib.PIXELS_INT8, np.int8), (_lib.PIXELS_UINT16, np.uint16),
         (_lib.PIXELS_INT16, np.int16), (_lib.PIXELS_UINT32, np.uint32), (_lib.PIXELS_INT32, np.int32),
         (_lib.PIXELS_FLOAT, np.float32), (_lib.PIXELS_DOUBLE, np.float64)]


def dev(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1)).to("cuda")


def rand_stack(dtype, z, h, w, seed):
    rng = np.random.default_rng(seed)
    if np.issubdtype(dtype, np.floating):
        return (rng.normal(0, 1e4, (z, h, w))).astype(dtype)
    info = np.iinfo(dtype)
    return rng.integers(info.min, info.max, (z, h, w), endpoint=True, dtype=np.int64).astype(dtype)


@pytest.mark.parametrize("pt,dtype", TYPES)
@pytest.mark.parametrize("alg", [_lib.PROJECTION_MAX, _lib.PROJECTION_MEAN, _lib.PROJECTION_SUM])
def test_projection_bit_exact_all_types(ctx, pt, dtype, alg):
    z, h, w = 7, 9, 13                                     # ragged plane (117 px)
    stack = rand_stack(dtype, z, h, w, 100 + pt)
    for (start, end, step, bi, bo) in [(0, 6, 1, False, False), (1, 5, 2, True, True), (3, 3, 1, True, False),
                                       (0, 6, 3, False, True)]:
        src = stack.astype(stack.dtype.newbyteorder(">")) if bi else stack
        st, exp = O.project(src, pt, w, h, z, alg, start, end, step, be_in=bi, be_out=bo)
        assert st == 0
        got = ctx.project_stack(src, pt, w, h, z, alg, start, end, step, big_endian_in=bi, big_endian_out=bo)
        np.testing.assert_array_equal(got, exp, err_msg=f"{start},{end},{step},{bi},{bo}")


@pytest.mark.parametrize("pt,dtype", TYPES)
@pytest.mark.parametrize("alg", [_lib.PROJECTION_MAX, _lib.PROJECTION_MEAN, _lib.PROJECTION_SUM])
def test_projection_vector_path_all_types(ctx, pt, dtype, alg):
    """16-B vector K3 (plane = whole 16-B chunks): z split over 4 waves for max and integer
    sums, uneven quarters, unroll tails, start > end, stepping."""
    z, h, w = 37, 16, 24
    stack = rand_stack(dtype, z, h, w, 300 + pt)
    for (start, end, step, bi, bo) in [(0, 36, 1, False, False), (2, 30, 3, True, True), (5, 5, 1, True, False),
                                       (9, 4, 1, False, True), (0, 36, 7, True, True), (1, 34, 1, False, False)]:
        src = stack.astype(stack.dtype.newbyteorder(">")) if bi else stack
        st, exp = O.project(src, pt, w, h, z, alg, start, end, step, be_in=bi, be_out=bo)
        assert st == 0
        got = ctx.project_stack(src, pt, w, h, z, alg, start, end, step, big_endian_in=bi, big_endian_out=bo)
        np.testing.assert_array_equal(got, exp, err_msg=f"{start},{end},{step},{bi},{bo}")


def test_projection_device_api_and_validation(ctx):
    import torch
    z, h, w = 64, 128, 256
    stack = rand_stack(np.uint16, z, h, w, 5)
    d = dev(stack.astype(">u2"))
    out = torch.empty(h * w * 2, dtype=torch.uint8, device="cuda")
    ctx.project_stack_device(d, _lib.PIXELS_UINT16, w, h, z, _lib.PROJECTION_MEAN, 0, z - 1, out,
                             big_endian_in=True)
    ctx.synchronize()
    st, exp = O.project(stack.astype(">u2"), _lib.PIXELS_UINT16, w, h, z, _lib.PROJECTION_MEAN, 0, z - 1, be_in=True)
    np.testing.assert_array_equal(out.cpu().numpy(), exp)
    for start, end, step, alg in [(-1, 2, 1, 0), (0, z, 1, 0), (z, 0, 1, 0), (0, 3, 0, 0), (0, 3, 1, 9)]:
        with pytest.raises(_lib.OmrError) as ei:
            ctx.project_stack(stack, _lib.PIXELS_UINT16, w, h, z, alg, start, end, step)
        assert ei.value.status == _lib.INVALID_ARGUMENT


@pytest.mark.parametrize("alg", [_lib.PROJECTION_MAX, _lib.PROJECTION_MEAN, _lib.PROJECTION_SUM])
def test_project_stacks_device_one_launch(ctx, alg):
    """omr_project_stacks_device: three stacks in one launch (the glue's K3), each == the oracle."""
    import torch
    z, h, w = 20, 64, 96
    stacks = [rand_stack(np.uint16, z, h, w, 40 + c).astype(">u2") for c in range(3)]
    outs = [torch.empty(h * w * 2, dtype=torch.uint8, device="cuda") for _ in range(3)]
    ctx.project_stacks_device([dev(s) for s in stacks], _lib.PIXELS_UINT16, w, h, z, alg, 2, z - 3, outs,
                              big_endian_in=True)
    ctx.synchronize()
    for s, o in zip(stacks, outs):
        st, exp = O.project(s, _lib.PIXELS_UINT16, w, h, z, alg, 2, z - 3, be_in=True)
        assert st == 0
        np.testing.assert_array_equal(o.cpu().numpy(), exp)
    with pytest.raises(_lib.OmrError):
        ctx.project_stacks_device([dev(stacks[0])] * 33, _lib.PIXELS_UINT16, w, h, z, alg, 0, 1, outs * 11)


@pytest.mark.parametrize("alg", [_lib.PROJECTION_MAX, _lib.PROJECTION_MEAN])
def test_c3_projection_then_composite_full_size(ctx, alg):
    """BASELINE config C3: 3-channel uint16 512x512x64 Z-stack -> max/mean projection -> composite.
    Default bounds 0..63 (ImageRegionRequestHandler.java:511-516): mean skips the last plane."""
    import torch
    z, h, w = 64, 512, 512
    rng = np.random.default_rng(20261015 + 3)
    base = [microscopy_u16(h, w, rng) for _ in range(3)]
    stacks = [np.stack([np.clip(b.astype(np.int64) + rng.integers(-500, 500, (h, w)), 0, 65535).astype(np.uint16)
                        for _ in range(z)]) for b in base]
    be = [s.astype(">u2") for s in stacks]
    chans = c2_channels(3)
    projected = []
    for s in be:
        st, p = O.project(s, _lib.PIXELS_UINT16, w, h, z, alg, 0, z - 1, be_in=True, be_out=True)
        assert st == 0
        projected.append(p.view(">u2").reshape(h, w))
    st, exp = O.render(chans, projected, _lib.PIXELS_UINT16, w, h, big_endian=True)
    out = torch.empty((h, w), dtype=torch.int32, device="cuda")
    ctx.render_projected_device(O.make_qdef("rgb"), chans, [dev(s) for s in be], _lib.PIXELS_UINT16, w, h, z,
                                alg, 0, z - 1, out, big_endian=True)
    ctx.synchronize()
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32), exp)


# ---- flips: ported index-oracle tests on the device kernels ------------------------------
@pytest.mark.parametrize("w,h", [(4, 4), (5, 5), (7, 4), (4, 7), (7, 1), (1, 7), (1, 1)])
def test_flip_argb_index_oracle(ctx, w, h):
    import torch
    src = torch.arange(w * h, dtype=torch.int32, device="cuda")
    for fh, fv in [(False, True), (True, False), (True, True)]:
        f = flip(ctx, src, w, h, fh, fv).cpu().numpy()
        for n in range(w * h):
            nc = w - 1 - n % w if fh else n % w
            nr = h - 1 - n // w if fv else n // w
            assert f[nr * w + nc] == n
    assert flip(ctx, src, w, h, False, False) is src           # no flip returns src


@pytest.mark.parametrize("w,h", [(4, 4), (5, 5), (7, 4), (4, 7), (7, 1), (1, 7), (1, 1)])
def test_flip_mask_index_oracle(ctx, w, h):
    import torch
    src = torch.arange(w * h, dtype=torch.uint8, device="cuda")
    dst = torch.empty_like(src)
    for fh, fv in [(False, True), (True, False), (True, True)]:
        ctx.flip_mask_device(src, dst, w, h, fh, fv)
        f = dst.cpu().numpy()
        for n in range(w * h):
            nc = w - 1 - n % w if fh else n % w
            nr = h - 1 - n // w if fv else n // w
            assert f[nr * w + nc] == n


def test_flip_errors(ctx):
    import torch
    with pytest.raises(ValueError):
        flip(ctx, None, 4, 4, True, True)                          # testFlipNullImage
    src = torch.ones(1, dtype=torch.int32, device="cuda")
    with pytest.raises(ValueError):
        flip(ctx, src, 0, 4, True, True)                           # testFlipZeroXImage
    with pytest.raises(ValueError):
        flip(ctx, src, 4, 0, True, True)                           # testFlipZeroYImage
    with pytest.raises(_lib.OmrError):
        ctx.flip_argb_device(None, src, 4, 4, True, True)


# ---- projection glue: project every active channel + render (K3 + K2, or the fused K3R) ----
@pytest.fixture(scope="module")
def k3r_ctx():
    import os
    import omr
    os.environ["OMR_K3R"] = "1"                 # read at context creation
    try:
        c = omr.Context(0)
    finally:
        del os.environ["OMR_K3R"]
    yield c
    c.close()


@pytest.fixture(params=["k3_k2", "k3r"])
def glue_ctx(request, ctx, k3r_ctx):
    return ctx if request.param == "k3_k2" else k3r_ctx


def _glue(ctx, chans, stacks, pt, w, h, z, alg, start, end, stepping=1, be=False, flip=(False, False),
          model="rgb", qd_kw=None):
    import torch
    q = O.make_qdef(model, **(qd_kw or {}))
    out = torch.empty((h, w), dtype=torch.int32, device="cuda")
    devs = [dev(s) if s is not None else None for s in stacks]
    torch.cuda.synchronize()
    ctx.render_projected_device(q, chans, devs, pt, w, h, z, alg, start, end, out, stepping=stepping,
                                big_endian=be, flip_h=flip[0], flip_v=flip[1])
    ctx.synchronize()
    got = out.cpu().numpy().view(np.uint32)
    planes = []
    for c, s in enumerate(stacks):
        if s is None or not chans[c].get("active", True):
            planes.append(None)
            continue
        st, p = O.project(s, pt, w, h, z, alg, start, end, stepping, be_in=be, be_out=be)
        assert st == 0
        planes.append(p)
    planes = [p if p is not None else np.zeros(w * h * np.dtype(stacks[0].dtype).itemsize, np.uint8) for p in planes]
    st, exp = O.render(chans, planes, pt, w, h, big_endian=be, flip_h=flip[0], flip_v=flip[1], qdef=q)
    assert st == 0
    np.testing.assert_array_equal(got, exp)


GLUE_TYPES = [(_lib.PIXELS_UINT16, np.uint16, (0.0, 65535.0)), (_lib.PIXELS_INT16, np.int16, (-32768.0, 32767.0)),
              (_lib.PIXELS_UINT8, np.uint8, (0.0, 255.0)), (_lib.PIXELS_INT8, np.int8, (-128.0, 127.0))]


@pytest.mark.parametrize("pt,dtype,rng_", GLUE_TYPES)
@pytest.mark.parametrize("alg", [_lib.PROJECTION_MAX, _lib.PROJECTION_MEAN, _lib.PROJECTION_SUM])
@pytest.mark.parametrize("be", [False, True])
def test_projection_glue_types_and_algorithms(glue_ctx, pt, dtype, rng_, alg, be):
    ctx = glue_ctx
    z, h, w = 13, 48, 64
    stacks = [rand_stack(dtype, z, h, w, 300 + c) for c in range(3)]
    if be:
        stacks = [s.astype(s.dtype.newbyteorder(">")) for s in stacks]
    lo, hi = rng_
    span = hi - lo
    chans = [{"input_start": lo + span * f0, "input_end": lo + span * f1, "global_min": lo, "global_max": hi,
              "rgba": col} for (f0, f1), col in zip([(0.0, 1.0), (0.1, 0.7), (0.3, 0.4)],
                                                    [(255, 0, 0, 255), (0, 255, 0, 255), (0, 0, 255, 255)])]
    _glue(ctx, chans, stacks, pt, w, h, z, alg, 1, z - 2, be=be, flip=(True, False))


@pytest.mark.parametrize("n_ch", [1, 2, 4])
@pytest.mark.parametrize("flip", [(False, False), (False, True), (True, True)])
def test_projection_glue_channels_flips_modes(glue_ctx, n_ch, flip):
    ctx = glue_ctx
    z, h, w = 64, 64, 128
    rng = np.random.default_rng(n_ch)
    stacks = [np.clip(microscopy_u16(h, w, rng).astype(np.int64) + rng.integers(-300, 300, (z, h, w)), 0,
                      65535).astype(np.uint16) for _ in range(n_ch)]
    chans = c2_channels(4)[:n_ch]
    lut = np.concatenate([np.arange(256), 255 - np.arange(256), np.arange(256) // 2]).astype(np.uint8)
    variants = [{}, {"reverse": True}, {"lut": lut}, {"family": _lib.FAMILY_LOGARITHMIC}]
    for c in range(n_ch):
        chans[c].update(variants[c])
    for alg, stepping in ((_lib.PROJECTION_MAX, 1), (_lib.PROJECTION_MEAN, 2), (_lib.PROJECTION_SUM, 3)):
        _glue(ctx, chans, stacks, _lib.PIXELS_UINT16, w, h, z, alg, 2, z - 1, stepping=stepping, flip=flip)
    _glue(ctx, chans, stacks, _lib.PIXELS_UINT16, w, h, z, _lib.PROJECTION_MEAN, 0, z - 1,
          qd_kw={"cd_start": 30, "cd_end": 220})


def test_projection_glue_unfused_cases(glue_ctx):
    ctx = glue_ctx
    """Odd width, five channels, 8-bit mean, float: the K3 + K2 path, same results."""
    rng = np.random.default_rng(9)
    z = 9
    s16 = [rng.integers(0, 65536, (z, 8, 33)).astype(np.uint16) for _ in range(5)]
    chans = c2_channels(4) + c2_channels(1)
    _glue(ctx, chans[:2], s16[:2], _lib.PIXELS_UINT16, 33, 8, z, _lib.PROJECTION_MEAN, 0, z - 1)
    s16 = [rng.integers(0, 65536, (z, 8, 32)).astype(np.uint16) for _ in range(5)]
    _glue(ctx, chans, s16, _lib.PIXELS_UINT16, 32, 8, z, _lib.PROJECTION_MAX, 0, z - 1)
    s8 = [rng.integers(0, 256, (z, 16, 32)).astype(np.uint8) for _ in range(2)]
    c8 = [{"input_start": 0.0, "input_end": 255.0, "global_min": 0.0, "global_max": 255.0, "rgba": (255, 9, 0, 255)},
          {"input_start": 20.0, "input_end": 90.0, "global_min": 0.0, "global_max": 255.0, "rgba": (0, 99, 255, 255)}]
    _glue(ctx, c8, s8, _lib.PIXELS_UINT8, 32, 16, z, _lib.PROJECTION_MEAN, 0, z - 1)
    sf = [rng.uniform(-10, 300, (z, 16, 32)).astype(np.float32) for _ in range(2)]
    cf = [{"input_start": 0.0, "input_end": 255.0, "rgba": (255, 0, 0, 255)},
          {"input_start": 5.0, "input_end": 200.0, "rgba": (0, 0, 255, 255)}]
    _glue(ctx, cf, sf, _lib.PIXELS_FLOAT, 32, 16, z, _lib.PROJECTION_MAX, 0, z - 1)


def test_projection_glue_quantization_error(glue_ctx):
    ctx = glue_ctx
    import torch
    z, h, w = 4, 16, 32
    stacks = [np.full((z, h, w), 100, np.uint16) for _ in range(2)]
    stacks[1][2, 3, 4] = 65000
    chans = c2_channels(2)
    for c in chans:
        c["global_max"] = 60000.0
    out = torch.empty((h, w), dtype=torch.int32, device="cuda")
    ctx.render_projected_device(O.make_qdef("rgb"), chans, [dev(s) for s in stacks], _lib.PIXELS_UINT16, w, h, z,
                                _lib.PROJECTION_MAX, 0, z - 1, out)
    with pytest.raises(_lib.OmrError) as e:
        ctx.synchronize()
    assert e.value.status == _lib.QUANTIZATION


@pytest.mark.parametrize("seed", list(range(int(os.environ.get("OMR_SWEEP_SEEDS", "40")))))
def test_projection_glue_sweep(glue_ctx, seed):
    """Random projection requests through the glue (K3 + K2, and K3R): type, byte order, active
    channels, windows (inverted / empty / fractional), reverse, .lut, codomain, algorithm,
    z range and stepping, flips — against the restatement's project + render."""
    rng = np.random.default_rng(7000 + seed)
    pt, dtype, (lo, hi) = GLUE_TYPES[seed % len(GLUE_TYPES)]
    n = int(rng.integers(1, 5))
    z, h, w = int(rng.integers(2, 20)), 16, 32 * int(rng.integers(1, 3))
    stacks = [rand_stack(dtype, z, h, w, 9000 + 10 * seed + c) for c in range(n)]
    be = bool(rng.integers(0, 2))
    if be:
        stacks = [s.astype(s.dtype.newbyteorder(">")) for s in stacks]
    chans = []
    for c in range(n):
        a, b = sorted(rng.uniform(lo, hi, 2))
        kind = rng.integers(0, 5)
        ws, we = (b, a) if kind == 0 else (a, a) if kind == 1 else (a + 0.5, b) if kind == 2 else (a, b)
        d = {"input_start": float(ws), "input_end": float(we), "global_min": lo, "global_max": hi,
             "rgba": tuple(int(v) for v in rng.integers(0, 256, 4)), "reverse": bool(rng.integers(0, 3) == 0)}
        if rng.integers(0, 5) == 0:
            d["lut"] = rng.integers(0, 256, 768).astype(np.uint8)
        chans.append(d)
    alg = int(rng.choice([_lib.PROJECTION_MAX, _lib.PROJECTION_MEAN, _lib.PROJECTION_SUM]))
    start = int(rng.integers(0, z))
    end = int(rng.integers(start, z))
    if alg != _lib.PROJECTION_MAX and end == start:
        end = min(z - 1, start + 1)
        if end == start:
            start = max(0, start - 1)
    qd_kw = {"cd_start": 20, "cd_end": 230} if rng.integers(0, 4) == 0 else None
    _glue(glue_ctx, chans, stacks, pt, w, h, z, alg, start, end, stepping=int(rng.integers(1, 4)), be=be,
          flip=(bool(rng.integers(0, 2)), bool(rng.integers(0, 2))), qd_kw=qd_kw)
