"""ctypes binding of oracle/liboracle.so — the CPU restatement used as the parity checker.

Test infrastructure only (see oracle/omr_oracle.c header).
"""
import ctypes
import os

import numpy as np

from omr import _lib
from omr.context import make_bindings, make_qdef

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PATH = os.path.join(REPO, "oracle", "liboracle.so")
if not os.path.exists(PATH):
    raise ImportError(f"{PATH} missing: run `make -C oracle`")
lib = ctypes.CDLL(PATH)


def _cpu_flags():
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("flags"):
                    return set(line.split(":", 1)[1].split())
    except OSError:
        pass
    return set()


# The timed CPU baseline (bench.py cpu_baseline legs) runs an ISA-tuned build of the same
# source: -O3 -march=x86-64-v4 (AVX-512) when this host has it, else x86-64-v3 (AVX2/FMA;
# -ffp-contract=off keeps the arithmetic identical).  Parity checks use the portable build.
_V4 = {"avx512f", "avx512bw", "avx512cd", "avx512dq", "avx512vl"}
_flags = _cpu_flags()
FAST_BUILD = "-O3 (portable)"
fast_lib = lib
for _tag, _need in (("v4", _V4), ("v3", {"avx2", "fma", "bmi2"})):
    _p_fast = os.path.join(REPO, "oracle", f"liboracle_{_tag}.so")
    if _need <= _flags and os.path.exists(_p_fast):
        fast_lib = ctypes.CDLL(_p_fast)
        FAST_BUILD = f"-O3 -march=x86-64-{_tag}"
        break

_vp, _i32, _i64, _sz, _f32 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_size_t, ctypes.c_float
_QD = ctypes.POINTER(_lib.QuantumDef)
_CB = ctypes.POINTER(_lib.ChannelBinding)
for name, res, args in [
    ("oracle_java_round", _i64, [ctypes.c_double]),
    ("oracle_quantize", _i32, [ctypes.c_double, _CB, _QD]),
    ("oracle_build_lut", _i32, [_CB, _QD, _vp, _i64]),
    ("oracle_render_packed_int", _i32, [_QD, _CB, _i32, _vp, _i64, _i32, _i32, _i32, _i32, _vp]),
    ("oracle_flip_int", _i32, [_vp, _vp, _i32, _i32, _i32, _i32]),
    ("oracle_flip_byte", _i32, [_vp, _vp, _i32, _i32, _i32, _i32]),
    ("oracle_project_stack", _i32, [_vp, _i32, _i32, _i32, _i32, _i32, _i32, _i32, _i32, _i32, _vp, _i32]),
    ("oracle_mask_indices", _i32, [_vp, _sz, _i32, _i32, _i32, _i32, _vp]),
    ("oracle_jpeg_quant_tables", None, [_f32, _vp, _vp]),
    ("oracle_set_semantics", None, [ctypes.c_uint32]),
    ("oracle_get_semantics", ctypes.c_uint32, []),
    ("oracle_encode_jpeg", _sz, [_vp, _i32, _i32, _f32, _vp, _sz]),
    ("oracle_jpeg_coefficients", _i64, [_vp, _i32, _i32, _f32, _vp, _i64]),
    ("oracle_render_tiles_mt", ctypes.c_double, [_QD, _CB, _i32, _vp, _i32, _i32, _i32, _i32, _i32,
                                                 _i32, _i32, _vp, _i32]),
]:
    for _l in {id(lib): lib, id(fast_lib): fast_lib}.values():
        fn = getattr(_l, name)
        fn.restype = res
        fn.argtypes = args


def _p(a):
    return None if a is None else a.ctypes.data


class semantics:
    """with oracle_lib.semantics(flags): ... — OMR_SEM_* switches of the restatement."""

    def __init__(self, flags):
        self.flags = int(flags)

    def __enter__(self):
        self.prev = lib.oracle_get_semantics()
        lib.oracle_set_semantics(self.flags)
        return self

    def __exit__(self, *exc):
        lib.oracle_set_semantics(self.prev)


def java_round(x):
    return lib.oracle_java_round(float(x))


def quantize(x, channel, model="rgb"):
    arr, keep = make_bindings([channel])
    q = make_qdef(model)
    return lib.oracle_quantize(float(x), arr, ctypes.byref(q))


def build_lut(channel, n):
    arr, keep = make_bindings([channel])
    q = make_qdef("rgb")
    out = np.empty(n, dtype=np.uint8)
    lib.oracle_build_lut(arr, ctypes.byref(q), out.ctypes.data, n)
    return out


def render(channels, planes, pixel_type, width, height, model="rgb", big_endian=False,
           flip_h=False, flip_v=False, row_stride=0, qdef=None, fast=False):
    """renderAsPackedInt + flip on the CPU. Returns (status, argb[h, w])."""
    arr, keep = make_bindings(channels)
    q = qdef or make_qdef(model)
    ptrs = (ctypes.c_void_p * max(len(planes), 1))(*[_p(p) for p in planes])
    out = np.zeros((height, width), dtype=np.uint32)
    st = (fast_lib if fast else lib).oracle_render_packed_int(ctypes.byref(q), arr, len(channels), ptrs, row_stride,
                                      pixel_type, int(big_endian), width, height, out.ctypes.data)
    if st == 0 and (flip_h or flip_v):
        f = np.empty_like(out)
        st = lib.oracle_flip_int(out.ctypes.data, f.ctypes.data, width, height, int(flip_h), int(flip_v))
        out = f
    return st, out


def flip_int(src, w, h, fh, fv):
    src = np.ascontiguousarray(src, dtype=np.uint32)
    out = np.zeros_like(src)
    st = lib.oracle_flip_int(_p(src), out.ctypes.data, w, h, int(fh), int(fv))
    return st, out


def project(stack, pixel_type, sx, sy, sz, alg, start, end, stepping=1, be_in=False, be_out=False,
            fast=False):
    bpp = _lib.BYTES_PER_PIXEL[pixel_type]
    out = np.zeros(sx * sy * bpp, dtype=np.uint8)
    st = (fast_lib if fast else lib).oracle_project_stack(_p(stack), pixel_type, int(be_in), sx, sy, sz, alg, start, end,
                                  stepping, out.ctypes.data, int(be_out))
    return st, out


def mask_indices(bits, w, h, fh=False, fv=False):
    bits = np.frombuffer(bytes(bits), dtype=np.uint8).copy()
    out = np.zeros(max(w * h, 1), dtype=np.uint8)
    st = lib.oracle_mask_indices(bits.ctypes.data if bits.size else None, bits.size, w, h, int(fh),
                                 int(fv), out.ctypes.data)
    return st, out[: w * h].reshape(h, w) if st == 0 else None


def quant_tables(q):
    a = np.zeros(64, np.uint8)
    b = np.zeros(64, np.uint8)
    lib.oracle_jpeg_quant_tables(float(q), a.ctypes.data, b.ctypes.data)
    return a, b


def encode_jpeg(argb, w, h, q):
    argb = np.ascontiguousarray(argb, dtype=np.uint32)
    cap = w * h * 8 + 65536
    out = np.zeros(cap, np.uint8)
    n = lib.oracle_encode_jpeg(argb.ctypes.data, w, h, float(q), out.ctypes.data, cap)
    return out[:n].tobytes()


def jpeg_coefficients(argb, w, h, q):
    argb = np.ascontiguousarray(argb, dtype=np.uint32)
    nb = ((w + 15) // 16) * ((h + 15) // 16) * 6
    out = np.zeros((nb, 64), np.int16)
    lib.oracle_jpeg_coefficients(argb.ctypes.data, w, h, float(q), out.ctypes.data, nb)
    return out


def render_tiles_mt(channels, tile_planes, n_tiles, pixel_type, width, height, model="rgb",
                    big_endian=False, flip_h=False, flip_v=False, n_threads=1, keep_output=True,
                    fast=False):
    """Reference-CPU proxy: per-request LUT rebuild + render (+flip) over a thread pool.
    tile_planes: list (per tile) of lists (per channel) of numpy planes.  Returns (seconds, out);
    keep_output=False renders into per-thread scratch (bounded memory for timing samples);
    fast=True runs the ISA-tuned build (timing only)."""
    arr, keep = make_bindings(channels)
    q = make_qdef(model)
    size_c = len(channels)
    flat = []
    for t in range(n_tiles):
        flat.extend(_p(p) for p in tile_planes[t])
    ptrs = (ctypes.c_void_p * max(len(flat), 1))(*flat)
    out = np.zeros((n_tiles, height, width), dtype=np.uint32) if keep_output else None
    L = fast_lib if fast else lib
    secs = L.oracle_render_tiles_mt(ctypes.byref(q), arr, size_c, ptrs, n_tiles, pixel_type,
                                      int(big_endian), width, height, int(flip_h), int(flip_v),
                                      _p(out), n_threads)
    return secs, out
