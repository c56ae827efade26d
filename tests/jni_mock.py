"""ctypes driver of tests/jni/libomr_jni_mock.so: jni/omr_jni.c (the product JNI shim) compiled
against a mock JVM (tests/jni/mock_jni.c).  TEST INFRASTRUCTURE.

`OmrNative` mirrors java/.../gpu/OmrNative.java: each method builds the Java arguments as mock
objects, calls the JNIEXPORT function the JVM would call, checks the JNI rules the mock counts
(no call inside a critical region, none with an exception pending, no null / mistyped array,
no critical array left held, local references bounded) and raises `JavaException` for a pending
exception, as the JVM would on return from the native method."""
import ctypes
import os
import re
import subprocess

import numpy as np

from omr import _lib   # noqa: F401  (loads torch's HIP runtime, then libomr.so, before the mock)

HERE = os.path.dirname(os.path.abspath(__file__))
JNI_DIR = os.path.join(HERE, "jni")
PATH = os.path.join(JNI_DIR, "libomr_jni_mock.so")
REPO = os.path.dirname(HERE)
JAVA = os.path.join(REPO, "java/src/main/java/com/glencoesoftware/omero/ms/image/region/gpu/OmrNative.java")
PREFIX = "Java_com_glencoesoftware_omero_ms_image_region_gpu_OmrNative_"
CHANNEL_FIELDS = 13
MAX_LOCAL_REFS = 4      # peak live local references a native call may hold (FindClass + string + throwable + 1)


def build():
    """CPU-side build (gcc): the mock library must exist before any GPU run loads it."""
    subprocess.run(["make", "-s", "-C", JNI_DIR], check=True)


if not os.path.exists(PATH):
    build()
lib = ctypes.CDLL(PATH)
_vp, _i32, _i64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64
for _name, _res, _args in [
        ("mock_env", _vp, []), ("mock_bytes", _vp, [_vp, _i32]), ("mock_ints", _vp, [_vp, _i32]),
        ("mock_doubles", _vp, [_vp, _i32]), ("mock_objects", _vp, [_i32]), ("mock_set", None, [_vp, _i32, _vp]),
        ("mock_string", _vp, [ctypes.c_char_p]), ("mock_len", _i32, [_vp]), ("mock_data", _vp, [_vp]),
        ("mock_exception_status", _i32, []), ("mock_exception_class", ctypes.c_char_p, []),
        ("mock_exception_message", ctypes.c_char_p, []), ("mock_counter", _i64, [_i32]),
        ("mock_begin_call", None, []), ("mock_reset", None, [])]:
    _f = getattr(lib, _name)
    _f.restype, _f.argtypes = _res, _args
ENV = lib.mock_env()


class JavaException(Exception):
    def __init__(self, cls, status, message):
        self.cls, self.status, self.message = cls, status, message
        super().__init__(f"{cls}({status}): {message}")


def native_methods():
    """`native` method names of OmrNative.java."""
    with open(JAVA) as f:
        return set(re.findall(r"\bnative\s+[\w\[\]]+\s+(\w+)\s*\(", f.read()))


def _sig(name, res, args):
    f = getattr(lib, PREFIX + name)
    f.restype = res
    f.argtypes = [_vp, _vp] + args       # JNIEnv*, jclass (static methods)
    return f


_b = ctypes.c_uint8
_f32 = ctypes.c_float
SIGS = {
    "create": (_i64, [_i32]),
    "destroy": (None, [_i64]),
    "setSemantics": (None, [_i64, _i32]),
    "renderPackedInt": (None, [_i64, _i32, _vp, _vp, _vp, _i32, _b, _i32, _i32, _b, _b, _vp]),
    "projectStack": (None, [_i64, _vp, _i32, _b, _i32, _i32, _i32, _i32, _i32, _i32, _i32, _vp, _b]),
    "encodeJpeg": (_vp, [_i64, _vp, _i32, _i32, _f32]),
    "encodePng": (_vp, [_i64, _vp, _i32, _i32]),
    "encodeTiff": (_vp, [_i64, _vp, _i32, _i32]),
    "renderShapeMaskPng": (_vp, [_i64, _vp, _i32, _i32, _vp, _b, _b]),
    "pixelBufferOpen": (_i64, [_vp, _i32, _i32, _i32, _i32, _i32, _i32]),
    "pixelBufferClose": (None, [_i64]),
    "batcherCreate": (_i64, [_i32, _i32, _i32]),
    "batcherDestroy": (None, [_i64]),
    "batcherSetSemantics": (None, [_i64, _i32]),
    "batcherSubmit": (_i64, [_i64, _i64, _i32, _vp, _vp, _i32, _i32, _i32, _i32, _i32, _i32, _b, _b, _i32, _f32]),
    "batcherSubmitProjected": (_i64, [_i64, _i64, _i32, _vp, _vp, _i32, _i32, _i32, _i32, _b, _b, _i32, _f32]),
    "batcherSubmitMask": (_i64, [_i64, _vp, _i32, _i32, _vp, _b, _b]),
    "batcherWait": (_vp, [_i64, _i64]),
    "poolCreate": (_i64, [_vp, _i32, _i32]),
    "poolDestroy": (None, [_i64]),
    "poolSetSemantics": (None, [_i64, _i32]),
    "poolSubmit": (_i64, [_i64, _i64, _i32, _vp, _vp, _i32, _i32, _i32, _i32, _i32, _i32, _b, _b, _i32, _f32]),
    "poolSubmitProjected": (_i64, [_i64, _i64, _i32, _vp, _vp, _i32, _i32, _i32, _i32, _b, _b, _i32, _f32]),
    "poolSubmitMask": (_i64, [_i64, _vp, _i32, _i32, _vp, _b, _b]),
    "poolWait": (_vp, [_i64, _i64]),
}
FN = {n: _sig(n, r, a) for n, (r, a) in SIGS.items()}


def call(name, *args):
    """One native call as the JVM makes it; returns its result, raises JavaException."""
    lib.mock_begin_call()
    res = FN[name](ENV, None, *args)
    counters = {k: lib.mock_counter(i) for i, k in enumerate(
        ["local_live", "local_peak", "critical_breach", "exception_breach", "argument_breach", "critical_held"])}
    assert counters["critical_breach"] == 0, (name, counters)
    assert counters["exception_breach"] == 0, (name, counters)
    assert counters["argument_breach"] == 0, (name, counters)
    assert counters["critical_held"] == 0, (name, counters)
    assert counters["local_live"] <= 1, (name, counters)            # at most the returned array
    assert counters["local_peak"] <= MAX_LOCAL_REFS, (name, counters)
    st = lib.mock_exception_status()
    if st != -2:
        raise JavaException(lib.mock_exception_class().decode(), st, lib.mock_exception_message().decode())
    return res


# ---- Java values ----------------------------------------------------------------------------
def jbytes(a):
    b = np.ascontiguousarray(np.frombuffer(bytes(a), np.uint8) if isinstance(a, (bytes, bytearray)) else a).view(np.uint8)
    return lib.mock_bytes(b.ctypes.data if b.size else None, b.size)


def jints(a):
    a = np.ascontiguousarray(a).view(np.int32).reshape(-1)
    return lib.mock_ints(a.ctypes.data if a.size else None, a.size)


def jdoubles(a):
    a = np.ascontiguousarray(a, dtype=np.float64).reshape(-1)
    return lib.mock_doubles(a.ctypes.data if a.size else None, a.size)


def jobjects(items):
    arr = lib.mock_objects(len(items))
    for i, o in enumerate(items):
        lib.mock_set(arr, i, o)
    return arr


def jstring(s):
    return lib.mock_string(s.encode())


def to_bytes(obj):
    if not obj:
        return None
    n = lib.mock_len(obj)
    return ctypes.string_at(lib.mock_data(obj), n)


def to_ints(obj):
    n = lib.mock_len(obj)
    return np.ctypeslib.as_array((ctypes.c_int32 * n).from_address(lib.mock_data(obj))).copy()


def pack_channels(channels):
    """OmrNative.packChannel for every channel dict -> (settings double[], luts byte[][] or None)."""
    s = np.zeros(len(channels) * CHANNEL_FIELDS)
    luts = []
    for c, d in enumerate(channels):
        o = c * CHANNEL_FIELDS
        s[o:o + 13] = [1.0 if d.get("active", True) else 0.0, d.get("family", 0), d.get("coefficient", 1.0),
                       1.0 if d.get("noise_reduction") else 0.0, 1.0 if d.get("reverse") else 0.0,
                       d["input_start"], d["input_end"], d.get("global_min", 0.0), d.get("global_max", 0.0),
                       *d.get("rgba", (255, 0, 0, 255))]
        lut = d.get("lut")
        luts.append(jbytes(np.asarray(lut, np.uint8)) if lut is not None else None)
    return jdoubles(s), (jobjects(luts) if any(x is not None for x in luts) else None)


class FakeContext(ctypes.Structure):
    """A jctx handle whose omr_ctx is a dummy (CPU tests of the validation paths only: every one
    of them must throw before the shim touches the library context)."""
    _fields_ = [("ctx", ctypes.c_void_p), ("pin", ctypes.c_void_p), ("pin_cap", ctypes.c_size_t)]
