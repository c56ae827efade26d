"""Every native method of OmrNative.java executed on the GPU through the JNI shim
(jni/omr_jni.c compiled against the mock JVM, tests/jni_mock.py) and compared with the CPU
restatement: the Java-side marshalling (13-double channel pack, LUT arrays, plane copies into
pinned staging, Set<T>ArrayRegion results, status -> OmrException) runs end to end, with the JNI
rules the mock checks kept on every call."""
import io

import numpy as np
import pytest

import jni_mock as M
import oracle_lib as O
from omr import _lib, write_romio
from omr.synthetic import c2_channels, tile_u16

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def jctx():
    h = M.call("create", 0)
    assert h
    yield h
    M.call("destroy", h)
    M.lib.mock_reset()


def _render(h, chans, planes, pt, w, ht, model=1, be=False, fh=False, fv=False):
    s, luts = M.pack_channels(chans)
    jp = M.jobjects([M.jbytes(np.ascontiguousarray(p).view(np.uint8).reshape(-1)) if p is not None else None
                     for p in planes])
    out = M.jints(np.zeros(w * ht, np.int32))
    M.call("renderPackedInt", h, model, s, luts, jp, pt, int(be), w, ht, int(fh), int(fv), out)
    return M.to_ints(out).view(np.uint32).reshape(ht, w)


@pytest.mark.parametrize("fh,fv", [(False, False), (True, False), (True, True)])
def test_render_packed_int_c2(jctx, fh, fv):
    w, h = 256, 96
    planes = [p.astype(">u2") for p in tile_u16(3, 4, h, w)]
    chans = c2_channels(4)
    chans[1]["reverse"] = True
    chans[2]["lut"] = (np.arange(768) * 7 % 256).astype(np.uint8)
    got = _render(jctx, chans, planes, _lib.PIXELS_UINT16, w, h, be=True, fh=fh, fv=fv)
    st, exp = O.render(chans, planes, _lib.PIXELS_UINT16, w, h, big_endian=True, flip_h=fh, flip_v=fv)
    assert st == 0
    np.testing.assert_array_equal(got, exp)


def test_render_greyscale_inactive_null_plane_and_many_channels(jctx):
    w, h = 64, 32
    rng = np.random.default_rng(8)
    planes = [rng.integers(0, 256, (h, w)).astype(np.uint8) for _ in range(3)]
    chans = [{"input_start": 10.0, "input_end": 200.5, "global_min": 0.0, "global_max": 255.0, "rgba": (0, 255, 0, 255)}
             for _ in range(3)]
    chans[0]["active"] = False
    got = _render(jctx, chans, [None, planes[1], planes[2]], _lib.PIXELS_UINT8, w, h, model=0)
    st, exp = O.render(chans, [np.zeros_like(planes[0]), planes[1], planes[2]], _lib.PIXELS_UINT8, w, h,
                       model="greyscale")
    np.testing.assert_array_equal(got, exp)
    # 24 active channels with LUTs: the plane and LUT loops keep the local references bounded
    lut = (np.arange(768) % 251).astype(np.uint8)
    many = [dict(chans[1], rgba=tuple(int(v) for v in rng.integers(0, 256, 4)), lut=lut if i % 2 else None)
            for i in range(24)]
    ps = [rng.integers(0, 256, (h, w)).astype(np.uint8) for _ in range(24)]
    got = _render(jctx, many, ps, _lib.PIXELS_UINT8, w, h)
    st, exp = O.render(many, ps, _lib.PIXELS_UINT8, w, h)
    np.testing.assert_array_equal(got, exp)


def test_render_quantization_exception(jctx):
    w, h = 32, 8
    planes = [np.full((h, w), 100, np.uint16) for _ in range(2)]
    planes[1][3, 4] = 65000
    chans = c2_channels(2)
    for c in chans:
        c["global_max"] = 60000.0
    with pytest.raises(M.JavaException) as e:
        _render(jctx, chans, planes, _lib.PIXELS_UINT16, w, h)
    assert e.value.status == _lib.QUANTIZATION and "OmrException" in e.value.cls


@pytest.mark.parametrize("alg", [_lib.PROJECTION_MAX, _lib.PROJECTION_MEAN, _lib.PROJECTION_SUM])
def test_project_stack(jctx, alg):
    sx, sy, sz = 96, 40, 9
    rng = np.random.default_rng(alg)
    stack = rng.integers(0, 65536, (sz, sy, sx)).astype(">u2")
    out = M.jbytes(np.zeros(sx * sy * 2, np.uint8))
    M.call("projectStack", jctx, M.jbytes(stack.view(np.uint8).reshape(-1)), _lib.PIXELS_UINT16, 1, sx, sy, sz, alg,
           1, sz - 1, 2, out, 1)
    st, exp = O.project(stack, _lib.PIXELS_UINT16, sx, sy, sz, alg, 1, sz - 1, 2, be_in=True, be_out=True)
    assert st == 0 and M.to_bytes(out) == exp.tobytes()
    with pytest.raises(M.JavaException) as e:     # zIntervalBoundsCheck: start >= sizeZ (ValidationException)
        M.call("projectStack", jctx, M.jbytes(stack.view(np.uint8).reshape(-1)), _lib.PIXELS_UINT16, 1, sx, sy, sz,
               alg, sz, 2, 1, out, 1)
    assert e.value.status == _lib.INVALID_ARGUMENT


def test_encoders(jctx):
    from PIL import Image
    w, h = 200, 120
    planes = [p.astype(">u2") for p in tile_u16(9, 4, h, w)]
    st, argb = O.render(c2_channels(4), planes, _lib.PIXELS_UINT16, w, h, big_endian=True)
    ja = M.jints(argb.view(np.int32))
    jpg = M.to_bytes(M.call("encodeJpeg", jctx, ja, w, h, np.float32(0.85)))
    assert jpg == O.encode_jpeg(argb, w, h, 0.85)
    rgb = argb.view(np.uint8).reshape(h, w, 4)[..., 2::-1]
    for name, fmt in (("encodePng", "PNG"), ("encodeTiff", "TIFF")):
        data = M.to_bytes(M.call(name, jctx, ja, w, h))
        im = Image.open(io.BytesIO(data))
        assert im.format == fmt
        np.testing.assert_array_equal(np.asarray(im.convert("RGB")), rgb)


def test_shape_mask(jctx):
    from PIL import Image
    w, h = 37, 21
    rng = np.random.default_rng(2)
    bits = rng.integers(0, 256, (w * h + 7) // 8, dtype=np.uint8).tobytes()
    png = M.to_bytes(M.call("renderShapeMaskPng", jctx, M.jbytes(bits), w, h, M.jbytes(bytes([255, 0, 0, 128])), 1, 0))
    st, idx = O.mask_indices(bits, w, h, True, False)
    np.testing.assert_array_equal(np.asarray(Image.open(io.BytesIO(png))), idx)
    # width % 8 == 0 with a flip: the reference's packed-buffer flip -> 404; the switch flips pixels
    b8 = bytes(rng.integers(0, 256, 64 * 8 // 8, dtype=np.uint8))
    with pytest.raises(M.JavaException) as e:
        M.call("renderShapeMaskPng", jctx, M.jbytes(b8), 64, 8, M.jbytes(bytes(4)), 0, 1)
    assert e.value.status == _lib.NOT_FOUND
    M.call("setSemantics", jctx, _lib.SEM_MASK_PIXEL_FLIP)
    try:
        png = M.to_bytes(M.call("renderShapeMaskPng", jctx, M.jbytes(b8), 64, 8, M.jbytes(bytes([1, 2, 3, 255])), 0, 1))
        with O.semantics(_lib.SEM_MASK_PIXEL_FLIP):
            st, idx = O.mask_indices(b8, 64, 8, False, True)
        np.testing.assert_array_equal((np.asarray(Image.open(io.BytesIO(png)).convert("RGBA"))[..., 3] > 0), idx == 1)
    finally:
        M.call("setSemantics", jctx, 0)
    with pytest.raises(M.JavaException) as e:                   # a null mask: 404 as the reference
        M.call("renderShapeMaskPng", jctx, None, 8, 8, M.jbytes(bytes(4)), 0, 0)
    assert e.value.status == _lib.NOT_FOUND
    with pytest.raises(M.JavaException) as e:
        M.call("setSemantics", jctx, 1 << 20)
    assert e.value.status == _lib.INVALID_ARGUMENT


@pytest.fixture(scope="module")
def romio(tmp_path_factory):
    rng = np.random.default_rng(12)
    px = rng.integers(0, 65536, (1, 3, 1, 512, 512), dtype=np.uint16)
    path = tmp_path_factory.mktemp("jni_romio") / "pixels"
    write_romio(path, px, _lib.PIXELS_UINT16)
    pb = M.call("pixelBufferOpen", M.jstring(str(path)), 512, 512, 1, 3, 1, _lib.PIXELS_UINT16)
    yield pb, px
    M.call("pixelBufferClose", pb)


def _oracle_tile(px, chans, x, y, n, fh=False):
    planes = [np.ascontiguousarray(px[0, c, 0, y:y + n, x:x + n]).astype(">u2") for c in range(3)]
    st, exp = O.render(chans, planes, _lib.PIXELS_UINT16, n, n, big_endian=True, flip_h=fh)
    assert st == 0
    return exp


@pytest.mark.parametrize("kind", ["batcher", "pool"])
def test_batcher_and_pool(romio, kind):
    import torch
    from PIL import Image
    pb, px = romio
    chans = c2_channels(3)
    chans[0]["lut"] = (255 - np.arange(768) % 256).astype(np.uint8)
    n = 128
    if kind == "batcher":
        q = M.call("batcherCreate", 0, 16, 2000)
        submit, wait, destroy, sem = "batcherSubmit", "batcherWait", "batcherDestroy", "batcherSetSemantics"
    else:
        devs = [i % torch.cuda.device_count() for i in range(2)]
        q = M.call("poolCreate", M.jints(np.array(devs, np.int32)), 16, 2000)
        submit, wait, destroy, sem = "poolSubmit", "poolWait", "poolDestroy", "poolSetSemantics"
    try:
        s, luts = M.pack_channels(chans)
        jobs = [(x, y, fmt, fh) for (x, y), fmt, fh in zip([(0, 0), (128, 0), (256, 384), (384, 128), (0, 256)],
                                                          [_lib.FORMAT_ARGB, _lib.FORMAT_JPEG, _lib.FORMAT_PNG,
                                                           _lib.FORMAT_TIFF, _lib.FORMAT_ARGB],
                                                          [False, True, False, True, False])]
        tickets = [M.call(submit, q, pb, 1, s, luts, 0, 0, x, y, n, n, int(fh), 0, fmt, np.float32(0.9))
                   for x, y, fmt, fh in jobs]
        for (x, y, fmt, fh), t in zip(jobs, tickets):
            got = M.to_bytes(M.call(wait, q, t))
            exp = _oracle_tile(px, chans, x, y, n, fh)
            if fmt == _lib.FORMAT_ARGB:
                np.testing.assert_array_equal(np.frombuffer(got, np.uint32).reshape(n, n), exp)
            elif fmt == _lib.FORMAT_JPEG:
                assert got == O.encode_jpeg(exp, n, n, 0.9)
            else:
                rgb = np.asarray(Image.open(io.BytesIO(got)).convert("RGB"))
                np.testing.assert_array_equal(rgb, exp.view(np.uint8).reshape(n, n, 4)[..., 2::-1])
        with pytest.raises(M.JavaException) as e:               # unknown format -> 404
            M.call(submit, q, pb, 1, s, luts, 0, 0, 0, 0, n, n, 0, 0, 99, np.float32(0.9))
        assert e.value.status == _lib.NOT_FOUND
        t = M.call(submit, q, pb, 1, s, luts, 0, 0, 500, 0, n, n, 0, 0, _lib.FORMAT_ARGB, np.float32(0.9))
        with pytest.raises(M.JavaException) as e:               # outside the image
            M.call(wait, q, t)
        assert e.value.status == _lib.INVALID_ARGUMENT
        M.call(sem, q, _lib.SEM_ALPHA_SEPARATE)
        with pytest.raises(M.JavaException):
            M.call(sem, q, 1 << 20)
    finally:
        M.call(destroy, q)


@pytest.mark.parametrize("kind", ["batcher", "pool"])
def test_projected_and_mask_jobs(romio, kind):
    """batcherSubmitProjected / poolSubmitProjected (the full plane, p=intmax over the one z of the
    fixture = the plane itself) and batcherSubmitMask / poolSubmitMask (PNG; a short mask throws 404
    at wait)."""
    import torch
    from PIL import Image
    pb, px = romio
    chans = c2_channels(3)
    if kind == "batcher":
        q = M.call("batcherCreate", 0, 16, 2000)
        sp, sm, wait, destroy = "batcherSubmitProjected", "batcherSubmitMask", "batcherWait", "batcherDestroy"
    else:
        devs = [i % torch.cuda.device_count() for i in range(2)]
        q = M.call("poolCreate", M.jints(np.array(devs, np.int32)), 16, 2000)
        sp, sm, wait, destroy = "poolSubmitProjected", "poolSubmitMask", "poolWait", "poolDestroy"
    try:
        s, luts = M.pack_channels(chans)
        t = M.call(sp, q, pb, 1, s, luts, 0, _lib.PROJECTION_MAX, -1, -1, 1, 0, _lib.FORMAT_ARGB, np.float32(0.9))
        got = np.frombuffer(M.to_bytes(M.call(wait, q, t)), np.uint32).reshape(512, 512)
        np.testing.assert_array_equal(got, _oracle_tile(px, chans, 0, 0, 512, fh=True))
        rng = np.random.default_rng(3)
        bits = rng.integers(0, 256, 37 * 21 // 8 + 1, dtype=np.uint8).tobytes()
        t = M.call(sm, q, M.jbytes(bits), 37, 21, M.jbytes(bytes([255, 0, 0, 128])), 1, 0)
        png = M.to_bytes(M.call(wait, q, t))
        st, idx = O.mask_indices(bits, 37, 21, True, False)
        exp = np.zeros((21, 37, 4), np.uint8)
        exp[idx == 1] = (255, 0, 0, 128)
        np.testing.assert_array_equal(np.asarray(Image.open(io.BytesIO(png)).convert("RGBA")), exp)
        t = M.call(sm, q, M.jbytes(bytes(2)), 37, 21, M.jbytes(bytes(4)), 0, 0)
        with pytest.raises(M.JavaException) as e:
            M.call(wait, q, t)
        assert e.value.status == _lib.NOT_FOUND
        with pytest.raises(M.JavaException) as e:                  # 3-byte colour
            M.call(sm, q, M.jbytes(bits), 37, 21, M.jbytes(bytes(3)), 0, 0)
        assert e.value.status == _lib.INVALID_ARGUMENT
    finally:
        M.call(destroy, q)
