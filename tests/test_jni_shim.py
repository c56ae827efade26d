"""The JNI shim (jni/omr_jni.c) executed on the CPU through the mock JVM (tests/jni/): the JNI
function table of the test-only jni.h in specification order, every native method of
OmrNative.java exported, and every validation path — null or short Java arrays, bad settings and
LUTs, null handles — throwing OmrException(INVALID_ARGUMENT) before the shim touches the GPU,
with the JNI rules the mock counts kept on every path (tests/jni_mock.py).  The GPU half is
tests/test_jni_shim_gpu.py."""
import ctypes
import filecmp
import os
import shutil
import subprocess
import sys

import numpy as np
import pytest

import jni_mock as M
from omr import _lib

IA = _lib.INVALID_ARGUMENT


def test_jni_header_table_is_in_specification_order(tmp_path):
    sys.path.insert(0, M.JNI_DIR)
    import gen_jni_h
    names = gen_jni_h.table()
    assert len(names) == 234
    for n, i in gen_jni_h.SPEC_INDEX.items():
        assert names[i] == n
    # the committed header is the generator's output
    for f in ("gen_jni_h.py", "jni.h.in"):
        shutil.copy(os.path.join(M.JNI_DIR, f), tmp_path / f)
    subprocess.run([sys.executable, str(tmp_path / "gen_jni_h.py")], check=True)
    assert filecmp.cmp(tmp_path / "jni.h", os.path.join(M.JNI_DIR, "jni.h"), shallow=False)


def test_struct_offsets_follow_the_table():
    """The compiled table: each used slot sits at index * sizeof(void*) (no padding, no reorder)."""
    src = os.path.join(M.JNI_DIR, "jni.h")
    import re
    body = open(src).read()
    slots = re.findall(r"/\* (\d+) \*/", body)
    assert [int(s) for s in slots] == list(range(234))


def test_every_native_method_is_exported():
    natives = M.native_methods()
    assert natives and natives == set(M.SIGS), (natives ^ set(M.SIGS))
    for n in natives:
        assert hasattr(M.lib, M.PREFIX + n), n


@pytest.fixture
def fake():
    dummy = ctypes.create_string_buffer(64)
    h = M.FakeContext(ctypes.addressof(dummy), None, 0)
    yield ctypes.addressof(h)
    M.lib.mock_reset()
    del dummy, h


def _raises(status, name, *args, cls="OmrException"):
    with pytest.raises(M.JavaException) as e:
        M.call(name, *args)
    assert cls in e.value.cls and e.value.status == status, e.value
    return e.value


def _c2(n=4):
    from omr.synthetic import c2_channels
    return c2_channels(n)


def test_render_packed_int_validation(fake):
    w, h = 32, 8
    s, luts = M.pack_channels(_c2())
    planes = M.jobjects([M.jbytes(np.zeros(w * h * 2, np.uint8)) for _ in range(4)])
    out = M.jints(np.zeros(w * h, np.int32))
    pt = _lib.PIXELS_UINT16
    args = lambda **k: [k.get("h", fake), 1, k.get("s", s), k.get("luts", luts), k.get("planes", planes),   # noqa
                        k.get("pt", pt), 1, k.get("w", w), k.get("ht", h), 0, 0, k.get("out", out)]
    _raises(IA, "renderPackedInt", *args(h=0))                                # null context
    _raises(IA, "renderPackedInt", *args(s=None))                             # null settings
    _raises(IA, "renderPackedInt", *args(s=M.jdoubles(np.zeros(14))))         # not 13 per channel
    _raises(IA, "renderPackedInt", *args(s=M.jdoubles(np.zeros(13 * 65))))    # > 64 channels
    _raises(IA, "renderPackedInt", *args(pt=9))                               # unknown pixel type
    _raises(IA, "renderPackedInt", *args(w=-1))
    _raises(IA, "renderPackedInt", *args(planes=None))
    _raises(IA, "renderPackedInt", *args(planes=M.jobjects([M.jbytes(np.zeros(w * h * 2, np.uint8))] * 3)))
    short = M.jobjects([M.jbytes(np.zeros(w * h * 2, np.uint8))] * 3 + [M.jbytes(np.zeros(w * h * 2 - 1, np.uint8))])
    _raises(IA, "renderPackedInt", *args(planes=short))                        # one plane 1 byte short
    nulls = M.jobjects([M.jbytes(np.zeros(w * h * 2, np.uint8))] * 3 + [None])
    _raises(IA, "renderPackedInt", *args(planes=nulls))                        # active channel without a plane
    _raises(IA, "renderPackedInt", *args(out=M.jints(np.zeros(w * h - 1, np.int32))))
    _raises(IA, "renderPackedInt", *args(out=None))
    _raises(IA, "renderPackedInt", *args(w=1 << 16, ht=1 << 15))              # plane > a Java array
    bad_lut = _c2()
    bad_lut[1]["lut"] = np.zeros(700, np.uint8)
    s2, l2 = M.pack_channels(bad_lut)
    _raises(IA, "renderPackedInt", *args(s=s2, luts=l2))                        # LUT not 768 bytes
    _raises(IA, "renderPackedInt", *args(luts=M.jobjects([None, None])))       # LUT array too short


def test_render_packed_int_inactive_null_plane_passes_validation(fake):
    """An inactive channel may have a null plane: validation passes and the shim reaches its
    pinned staging, which the dummy context cannot provide (OOM, still no JNI rule broken)."""
    w, h = 16, 4
    ch = _c2()
    ch[2]["active"] = False
    s, luts = M.pack_channels(ch)
    planes = M.jobjects([M.jbytes(np.zeros(w * h * 2, np.uint8))] * 2 + [None] + [M.jbytes(np.zeros(w * h * 2, np.uint8))])
    e = _raises(_lib.OOM, "renderPackedInt", fake, 1, s, luts, planes, _lib.PIXELS_UINT16, 1, w, h, 0, 0,
                M.jints(np.zeros(w * h, np.int32)))
    assert "pinned" in e.message


def test_local_references_stay_bounded_with_many_lut_channels(fake):
    """64 channels, each with a LUT: the settings loop deletes each element's local reference
    (a leak would peak at 64 live references; the JVM guarantees 16)."""
    ch = [dict(c, lut=np.arange(768) % 256) for c in _c2(1) * 64]
    s, luts = M.pack_channels(ch)
    w, h = 8, 2
    planes = M.jobjects([M.jbytes(np.zeros(w * h * 2, np.uint8))] * 63)      # one short: fails after the loop
    _raises(IA, "renderPackedInt", fake, 1, s, luts, planes, _lib.PIXELS_UINT16, 1, w, h, 0, 0,
            M.jints(np.zeros(w * h, np.int32)))


def test_project_stack_validation(fake):
    sx, sy, sz = 8, 4, 3
    st, out = M.jbytes(np.zeros(sx * sy * sz * 2, np.uint8)), M.jbytes(np.zeros(sx * sy * 2, np.uint8))
    a = lambda **k: [k.get("h", fake), k.get("st", st), k.get("pt", _lib.PIXELS_UINT16), 0, sx, sy,   # noqa
                     k.get("sz", sz), 0, 0, sz - 1, 1, k.get("out", out), 0]
    _raises(IA, "projectStack", *a(h=0))
    _raises(IA, "projectStack", *a(st=None))
    _raises(IA, "projectStack", *a(st=M.jbytes(np.zeros(sx * sy * sz * 2 - 2, np.uint8))))
    _raises(IA, "projectStack", *a(out=M.jbytes(np.zeros(sx * sy * 2 - 1, np.uint8))))
    _raises(IA, "projectStack", *a(pt=42))
    _raises(IA, "projectStack", *a(sz=0))


@pytest.mark.parametrize("name", ["encodeJpeg", "encodePng", "encodeTiff"])
def test_encode_validation(fake, name):
    w, h = 16, 16
    extra = [np.float32(0.9)] if name == "encodeJpeg" else []
    _raises(IA, name, 0, M.jints(np.zeros(w * h, np.int32)), w, h, *extra)
    _raises(IA, name, fake, None, w, h, *extra)
    _raises(IA, name, fake, M.jints(np.zeros(w * h - 1, np.int32)), w, h, *extra)
    _raises(IA, name, fake, M.jints(np.zeros(w * h, np.int32)), 0, h, *extra)


def test_shape_mask_validation(fake):
    bits = M.jbytes(bytes(8))
    _raises(IA, "renderShapeMaskPng", 0, bits, 8, 8, M.jbytes(bytes(4)), 0, 0)
    _raises(IA, "renderShapeMaskPng", fake, bits, 8, 8, None, 0, 0)               # null colour
    _raises(IA, "renderShapeMaskPng", fake, bits, 8, 8, M.jbytes(bytes(3)), 0, 0)  # 3-byte colour
    # The library's 404 cases are caught before any staging is pinned (the fake context has no
    # library state behind it, so reaching omr_pinned_alloc would fail differently): huge sizes,
    # w*h past a Java int, a mask shorter than w*h bits, a null mask, a zero size.
    NF, col = _lib.NOT_FOUND, M.jbytes(bytes(4))
    _raises(NF, "renderShapeMaskPng", fake, bits, 1 << 30, 1 << 30, col, 0, 0)
    _raises(NF, "renderShapeMaskPng", fake, bits, 65536, 32768, col, 0, 0)        # 2^31 pixels
    _raises(NF, "renderShapeMaskPng", fake, bits, 9, 8, col, 0, 0)                # 72 bits > 64
    _raises(NF, "renderShapeMaskPng", fake, None, 8, 8, col, 0, 0)
    _raises(NF, "renderShapeMaskPng", fake, bits, 0, 8, col, 0, 0)
    _raises(NF, "renderShapeMaskPng", fake, bits, 8, -1, col, 1, 1)


def test_batcher_and_pool_validation(fake):
    s, luts = M.pack_channels(_c2(3))
    args = [1, 1, s, luts, 0, 0, 0, 0, 64, 64, 0, 0, 0, np.float32(0.9)]
    _raises(IA, "batcherSubmit", 0, *args)                 # null batcher
    _raises(IA, "poolSubmit", 0, *args)
    _raises(IA, "batcherWait", 0, 1)
    _raises(IA, "batcherSubmitProjected", 0, 1, 1, s, luts, 0, 0, -1, -1, 0, 0, 0, np.float32(0.9))
    _raises(IA, "poolSubmitProjected", 0, 1, 1, s, luts, 0, 0, -1, -1, 0, 0, 0, np.float32(0.9))
    _raises(IA, "batcherSubmitMask", 0, M.jbytes(bytes(8)), 8, 8, M.jbytes(bytes(4)), 0, 0)
    _raises(IA, "poolSubmitMask", 0, M.jbytes(bytes(8)), 8, 8, M.jbytes(bytes(4)), 0, 0)
    _raises(IA, "poolWait", 0, 1)
    _raises(IA, "poolCreate", M.jints(np.zeros(0, np.int32)), 8, 100)              # no devices
    _raises(IA, "poolCreate", None, 8, 100)
    _raises(IA, "pixelBufferOpen", None, 1, 1, 1, 1, 1, 1)
    _raises(_lib.NOT_FOUND, "pixelBufferOpen", M.jstring("/nonexistent/pixels"), 4, 4, 1, 1, 1, _lib.PIXELS_UINT8)
    for name in ("batcherSetSemantics", "poolSetSemantics"):
        _raises(IA, name, 0, 1)
    _raises(IA, "setSemantics", 0, 1)
    M.call("destroy", 0)            # null handles are ignored
    M.call("batcherDestroy", 0)
    M.call("poolDestroy", 0)
    M.call("pixelBufferClose", 0)


def test_mock_counts_breaches():
    """The rule checks are live: a short region read throws AIOOBE and an array call on null
    counts as a breach."""
    M.lib.mock_begin_call()
    a = M.jbytes(bytes(4))
    buf = (ctypes.c_uint8 * 8)()
    tbl = ctypes.cast(ctypes.cast(M.ENV, ctypes.POINTER(ctypes.c_void_p))[0], ctypes.POINTER(ctypes.c_void_p))
    get_region = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32,
                                  ctypes.c_void_p)(tbl[200])
    get_region(M.ENV, a, 0, 8, buf)
    assert M.lib.mock_exception_class() == b"java/lang/ArrayIndexOutOfBoundsException"
    get_len = ctypes.CFUNCTYPE(ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p)(tbl[171])
    M.lib.mock_begin_call()
    get_len(M.ENV, None)
    assert M.lib.mock_counter(4) == 1
    M.lib.mock_reset()
