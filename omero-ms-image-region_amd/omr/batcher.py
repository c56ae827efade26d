"""Batcher and Pool: concurrent tile requests coalesced into GPU batches.

Batcher (omr_batcher_*): worker threads call submit()/wait(); a dispatcher
thread in libomr.so groups pending jobs by image + settings, renders and encodes each group in
one batch, and renders identical in-flight tiles once (ImageRegionCtx.cacheKey,
ImageRegionCtx.java:165-177).

Pool (omr_pool_*): one batcher per GPU of the node, each job to the least-queued
one -- the reference's N worker-verticle instances over one worker pool
(ImageRegionMicroserviceVerticle.java:84-85, :149-165) spread over the node's GPUs.
"""
import ctypes

import numpy as np

from . import _lib
from ._lib import lib
from .context import make_bindings

FORMATS = {"jpeg": _lib.FORMAT_JPEG, "png": _lib.FORMAT_PNG, "argb": _lib.FORMAT_ARGB,
           "tif": _lib.FORMAT_TIFF}


PROJECTIONS = {"intmax": _lib.PROJECTION_MAX, "intmean": _lib.PROJECTION_MEAN, "intsum": _lib.PROJECTION_SUM}


def _job(pixbuf, qdef, channels, z, t, x, y, width, height, flip_h, flip_v, fmt, quality, bindings,
         projection=None, projection_start=-1, projection_end=-1):
    arr, keep = bindings if bindings is not None else make_bindings(channels)
    alg = PROJECTIONS[projection] if isinstance(projection, str) else projection
    job = _lib.TileJob(pixbuf.h.value if hasattr(pixbuf.h, "value") else pixbuf.h,
                       ctypes.addressof(qdef), ctypes.addressof(arr), len(channels), z, t, x, y, width, height,
                       int(flip_h), int(flip_v), FORMATS.get(fmt, 99), float(quality),
                       int(alg is not None), int(alg or 0), int(projection_start), int(projection_end))
    return job, (arr, keep)


class _Queue:
    _submit = _submit_mask = _wait = _set_semantics = _destroy = None

    def close(self):
        if self.h:
            type(self)._destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def submit(self, pixbuf, qdef, channels, z, t, x, y, width, height, flip_h=False, flip_v=False,
               fmt="jpeg", quality=0.85, bindings=None, projection=None, projection_start=-1,
               projection_end=-1):
        """A render_image_region job.  projection ("intmax" / "intmean" / "intsum" or OMR_PROJECTION_*):
        the full plane projected over [projection_start, projection_end] (negative: 0 / sizeZ-1)
        at t; z, x, y, width, height are then ignored (ImageRegionRequestHandler.java:506-558)."""
        job, keep = _job(pixbuf, qdef, channels, z, t, x, y, width, height, flip_h, flip_v, fmt, quality,
                         bindings, projection, projection_start, projection_end)
        ticket = ctypes.c_uint64()
        _lib.check(type(self)._submit(self.h, ctypes.byref(job), ctypes.byref(ticket)))
        return ticket.value

    def submit_mask(self, bits, width, height, rgba, flip_h=False, flip_v=False):
        """A render_shape_mask job (ShapeMaskRequestHandler.java:165-207); wait() returns the PNG."""
        b = None if bits is None else np.frombuffer(bytes(bits), dtype=np.uint8).copy()
        job = _lib.MaskJob()
        job.bits = b.ctypes.data if b is not None and b.size else (None if b is None else ctypes.addressof(job))
        job.n_bytes = 0 if b is None else b.size
        job.width, job.height = int(width), int(height)
        job.rgba[:] = [int(v) for v in rgba]
        job.flip_h, job.flip_v = int(bool(flip_h)), int(bool(flip_v))
        ticket = ctypes.c_uint64()
        _lib.check(type(self)._submit_mask(self.h, ctypes.byref(job), ctypes.byref(ticket)))
        return ticket.value

    def set_semantics(self, flags):
        """OMR_SEM_* switches for the jobs submitted after this call."""
        _lib.check(type(self)._set_semantics(self.h, int(flags)))

    def wait(self, ticket, cap=1 << 22):
        n = ctypes.c_size_t(0)
        out = np.empty(cap, dtype=np.uint8)
        st = type(self)._wait(self.h, ticket, out.ctypes.data, cap, ctypes.byref(n))
        if st == _lib.BUFFER_TOO_SMALL:
            out = np.empty(n.value, dtype=np.uint8)
            st = type(self)._wait(self.h, ticket, out.ctypes.data, n.value, ctypes.byref(n))
        _lib.check(st)
        return out[:n.value].tobytes()


class Batcher(_Queue):
    _submit = lib.omr_batcher_submit
    _submit_mask = lib.omr_batcher_submit_mask
    _wait = lib.omr_batcher_wait
    _set_semantics = lib.omr_batcher_set_semantics
    _destroy = lib.omr_batcher_destroy

    def __init__(self, device=0, max_batch=64, max_wait_us=500):
        h = ctypes.c_void_p()
        st = lib.omr_batcher_create(device, max_batch, max_wait_us, ctypes.byref(h))
        if st != _lib.OK:
            raise _lib.OmrError(st, "omr_batcher_create failed")
        self.h = h

    def stats(self):
        s = (ctypes.c_uint64 * 4)()
        _lib.check(lib.omr_batcher_stats(self.h, s))
        return {"jobs": s[0], "batches": s[1], "rendered": s[2], "dedup": s[3]}

    def set_stack_cache(self, max_bytes):
        """HBM cache of the projection jobs' Z-stacks (0 disables)."""
        _lib.check(lib.omr_batcher_set_stack_cache(self.h, int(max_bytes)))

    def stack_cache_stats(self):
        s = (ctypes.c_uint64 * 3)()
        _lib.check(lib.omr_batcher_stack_cache_stats(self.h, s))
        return {"hits": s[0], "misses": s[1], "resident_bytes": s[2]}


class Pool(_Queue):
    _submit = lib.omr_pool_submit
    _submit_mask = lib.omr_pool_submit_mask
    _wait = lib.omr_pool_wait
    _set_semantics = lib.omr_pool_set_semantics
    _destroy = lib.omr_pool_destroy

    def __init__(self, devices, max_batch=64, max_wait_us=500):
        devs = (ctypes.c_int32 * len(devices))(*devices)
        h = ctypes.c_void_p()
        st = lib.omr_pool_create(devs, len(devices), max_batch, max_wait_us, ctypes.byref(h))
        if st != _lib.OK:
            raise _lib.OmrError(st, "omr_pool_create failed")
        self.h = h
        self.devices = list(devices)

    def device_index(self, ticket):
        return lib.omr_pool_device_index(self.h, ticket)

    def set_stack_cache(self, max_bytes_per_device):
        _lib.check(lib.omr_pool_set_stack_cache(self.h, int(max_bytes_per_device)))

    def stats(self):
        n = len(self.devices)
        s = (ctypes.c_uint64 * (4 * n))()
        _lib.check(lib.omr_pool_stats(self.h, s, n))
        return [{"jobs": s[4 * i], "batches": s[4 * i + 1], "rendered": s[4 * i + 2], "dedup": s[4 * i + 3]}
                for i in range(n)]
