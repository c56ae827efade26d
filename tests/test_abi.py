"""libomr.so loads (no GPU needed) and exports every symbol include/omr/omr.h declares."""
import ctypes
import os
import re

from omr import _lib

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(REPO, "include", "omr", "omr.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(omr_[a-z0-9_]+)\s*\(", src)))


def test_header_symbols_exported():
    names = declared_symbols()
    assert len(names) >= 30
    missing = [n for n in names if not hasattr(_lib.lib, n)]
    assert not missing, missing


def test_binding_covers_header():
    assert set(declared_symbols()) <= set(_lib._SIGS), set(declared_symbols()) - set(_lib._SIGS)
    assert not _lib.MISSING


def test_abi_version_and_struct_layout():
    assert _lib.lib.omr_abi_version() == 2
    assert ctypes.sizeof(_lib.TileJob) == 88 and _lib.TileJob.has_projection.offset == 68
    assert ctypes.sizeof(_lib.MaskJob) == 40 and _lib.MaskJob.flip_h.offset == 28
    # struct layouts a Panama/JNI binding must reproduce
    assert ctypes.sizeof(_lib.QuantumDef) == 16
    assert ctypes.sizeof(_lib.ChannelBinding) == 72
    assert _lib.ChannelBinding.lut.offset == 64
    assert ctypes.sizeof(_lib.Region) == 16


def test_context_create_without_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        return
    h = ctypes.c_void_p()
    assert _lib.lib.omr_ctx_create(0, ctypes.byref(h)) == _lib.DEVICE


def test_jpeg_tables_host_helper_matches_oracle(oracle):
    for q in (0.05, 0.3, 0.5, 0.75, 0.8, 0.85, 0.9, 0.95, 1.0):
        a = (ctypes.c_uint8 * 64)()
        b = (ctypes.c_uint8 * 64)()
        assert _lib.lib.omr_jpeg_quant_tables(q, a, b) == 0
        ol, oc = oracle.quant_tables(q)
        assert list(a) == list(ol) and list(b) == list(oc)
