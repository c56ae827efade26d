"""Context: Python handle on one omr_ctx (device + stream + workspace).

Host arrays are numpy; device buffers are torch tensors on the context's GPU (torch is
only used as the device-memory allocator — all compute runs in libomr.so kernels).
"""
import ctypes
import functools

import numpy as np

from . import _lib
from ._lib import lib, check


def _ptr(a):
    """Address of a numpy array, torch tensor, bytes-like or int."""
    if a is None:
        return None
    if isinstance(a, int):
        return a
    if isinstance(a, np.ndarray):
        return a.ctypes.data
    if hasattr(a, "data_ptr"):
        return a.data_ptr()
    raise TypeError(f"cannot take the address of {type(a)}")


def make_bindings(channels):
    """ChannelBinding[] from a list of dicts / ChannelSettings; keeps LUT buffers alive."""
    n = len(channels)
    arr = (_lib.ChannelBinding * max(n, 1))()
    keep = []
    for i, ch in enumerate(channels):
        d = ch if isinstance(ch, dict) else ch.as_dict()
        b = arr[i]
        b.active = int(bool(d.get("active", True)))
        b.family = int(d.get("family", _lib.FAMILY_LINEAR))
        b.coefficient = float(d.get("coefficient", 1.0))
        b.noise_reduction = int(bool(d.get("noise_reduction", False)))
        b.reverse = int(bool(d.get("reverse", False)))
        b.input_start = float(d["input_start"])
        b.input_end = float(d["input_end"])
        b.global_min = float(d.get("global_min", 0.0))
        b.global_max = float(d.get("global_max", 0.0))
        rgba = d.get("rgba", (255, 0, 0, 255))
        for k in range(4):
            b.rgba[k] = int(rgba[k])
        lut = d.get("lut")
        if lut is not None:
            buf = np.ascontiguousarray(np.asarray(lut, dtype=np.uint8).reshape(768))
            keep.append(buf)
            b.lut = buf.ctypes.data_as(_lib._u8p)
        else:
            b.lut = None
    return arr, keep


def make_qdef(model, cd_start=0, cd_end=255, bit_resolution=255):
    q = _lib.QuantumDef()
    q.cd_start, q.cd_end, q.bit_resolution = cd_start, cd_end, bit_resolution
    q.model = _lib.MODEL_RGB if model in (_lib.MODEL_RGB, "rgb", "c") else _lib.MODEL_GREYSCALE
    return q


class Context:
    """One omr_ctx.  Its launches run on the context's own non-blocking HIP stream.

    torch_order (default True): every *_device call is stream-ordered with torch's current
    stream at the API boundary, without a host sync: the context stream first waits for the
    work torch has queued (the inputs), and torch's stream then waits for the call's kernels
    (the outputs), so a following tensor op (.cpu(), a kernel, a free) sees the result.  Keep
    tensors alive until the call's work is done when torch might reuse their memory (the
    caching allocator reuses on torch's stream, which the second wait orders).  With
    torch_order=False (the bench: explicit synchronize around timed regions) nothing is added
    to a call; order_after_torch() / order_torch_after() do the same by hand."""

    def __init__(self, device=0, torch_order=True):
        h = ctypes.c_void_p()
        st = lib.omr_ctx_create(int(device), ctypes.byref(h))
        if st != _lib.OK:
            raise _lib.OmrError(st, f"omr_ctx_create(device={device}) failed")
        self.h = h
        self.device = device
        self.torch_order = bool(torch_order)
        self._ext = None

    def close(self):
        if self.h:
            lib.omr_ctx_destroy(self.h)
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

    @property
    def stream(self):
        return lib.omr_ctx_get_stream(self.h)

    def set_stream(self, stream_ptr):
        check(lib.omr_ctx_set_stream(self.h, stream_ptr), self.h)

    def synchronize(self):
        check(lib.omr_ctx_synchronize(self.h), self.h)

    def _ext_stream(self):
        import torch
        if self._ext is None or self._ext[0] != self.stream:
            self._ext = (self.stream, torch.cuda.ExternalStream(self.stream, device=torch.device("cuda", self.device)))
        return self._ext[1]

    def order_after_torch(self):
        """The context's stream waits for the work queued so far on torch's current stream."""
        import torch
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(torch.device("cuda", self.device)))
        self._ext_stream().wait_event(ev)

    def order_torch_after(self):
        """torch's current stream waits for the work queued so far on the context's stream."""
        import torch
        ev = torch.cuda.Event()
        ev.record(self._ext_stream())
        torch.cuda.current_stream(torch.device("cuda", self.device)).wait_event(ev)

    def set_semantics(self, flags):
        """OMR_SEM_* switches (omr._lib.SEM_*) for later calls on this context."""
        check(lib.omr_ctx_set_semantics(self.h, int(flags)), self.h)

    @property
    def semantics(self):
        return int(lib.omr_ctx_get_semantics(self.h))

    def enable_kernel_timing(self, enable=True):
        check(lib.omr_ctx_enable_kernel_timing(self.h, int(enable)), self.h)

    def kernel_timings(self, cap=1 << 16):
        """[(ms, kind)] of the timed hot-kernel launches since the last call (kind 2 render,
        3 projection, 4 jpeg); synchronises the stream."""
        ms = np.zeros(cap, np.float32)
        kind = np.zeros(cap, np.int32)
        n = lib.omr_ctx_kernel_timings(self.h, ms.ctypes.data, kind.ctypes.data, cap)
        if n < 0:
            raise _lib.OmrError(_lib.DEVICE, "kernel timing query failed")
        return list(zip(ms[:n].tolist(), kind[:n].tolist()))

    def last_error(self):
        raw = lib.omr_last_error(self.h)
        return raw.decode() if raw else ""

    # ---- render -----------------------------------------------------------------------
    def render_packed_int(self, qdef, channels, planes, pixel_type, width, height,
                          big_endian=False, flip_h=False, flip_v=False, row_stride=0):
        arr, keep = make_bindings(channels)
        ptrs = (ctypes.c_void_p * max(len(planes), 1))(*[_ptr(p) for p in planes])
        out = np.empty((height, width), dtype=np.uint32)
        check(lib.omr_render_packed_int(self.h, ctypes.byref(qdef), arr, len(channels), ptrs,
                                        row_stride, pixel_type, int(big_endian), width, height,
                                        int(flip_h), int(flip_v), out.ctypes.data), self.h)
        return out

    def render_packed_int_device(self, qdef, channels, planes, pixel_type, width, height, out,
                                 big_endian=False, flip_h=False, flip_v=False, row_stride=0):
        arr, keep = make_bindings(channels)
        ptrs = (ctypes.c_void_p * max(len(planes), 1))(*[_ptr(p) for p in planes])
        check(lib.omr_render_packed_int_device(self.h, ctypes.byref(qdef), arr, len(channels),
                                               ptrs, row_stride, pixel_type, int(big_endian),
                                               width, height, int(flip_h), int(flip_v),
                                               _ptr(out)), self.h)
        return out

    def render_batch_device(self, qdef, channels, d_plane_ptrs, n_tiles, pixel_type, width, height,
                            out, status=None, big_endian=False, flip_h=False, flip_v=False,
                            row_stride=0, bindings=None):
        if bindings is None:
            bindings = make_bindings(channels)
        arr, keep = bindings
        check(lib.omr_render_batch_device(self.h, ctypes.byref(qdef), arr, len(channels),
                                          _ptr(d_plane_ptrs), n_tiles, row_stride, pixel_type,
                                          int(big_endian), width, height, int(flip_h),
                                          int(flip_v), _ptr(out), _ptr(status)), self.h)
        return out

    def render_batch_strided_device(self, qdef, channels, d_base, tile_stride, channel_stride, n_tiles,
                                    pixel_type, width, height, out, status=None, big_endian=False,
                                    flip_h=False, flip_v=False, row_stride=0, bindings=None):
        """Batch whose planes sit at d_base + t*tile_stride + c*channel_stride (bytes)."""
        if bindings is None:
            bindings = make_bindings(channels)
        arr, keep = bindings
        check(lib.omr_render_batch_strided_device(self.h, ctypes.byref(qdef), arr, len(channels),
                                                  _ptr(d_base), tile_stride, channel_stride, n_tiles,
                                                  row_stride, pixel_type, int(big_endian), width,
                                                  height, int(flip_h), int(flip_v), _ptr(out),
                                                  _ptr(status)), self.h)
        return out

    def render_pixel_buffer_tiles(self, qdef, channels, pixbuf, requests, width, height, out=None,
                                  flip_h=False, flip_v=False, bindings=None):
        """Pipelined host-fed tiles: requests = [(z, t, x, y)]; out: host numpy [n][h][w] uint32
        (allocated when None) or a device tensor (rendered in place)."""
        if bindings is None:
            bindings = make_bindings(channels)
        arr, keep = bindings
        n = len(requests)
        reqs = (_lib.TileRequest * max(n, 1))(*[_lib.TileRequest(*r) for r in requests])
        on_device = out is not None and hasattr(out, "data_ptr")
        if out is None:
            out = np.empty((n, height, width), dtype=np.uint32)
        check(lib.omr_render_pixel_buffer_tiles(self.h, pixbuf.h, ctypes.byref(qdef), arr, len(channels), reqs, n,
                                                width, height, int(flip_h), int(flip_v), _ptr(out),
                                                int(on_device)), self.h)
        return out

    def flip_argb_device(self, src, dst, width, height, flip_h, flip_v):
        check(lib.omr_flip_argb_device(self.h, _ptr(src), _ptr(dst), width, height, int(flip_h),
                                       int(flip_v)), self.h)

    def flip_mask_device(self, src, dst, width, height, flip_h, flip_v):
        check(lib.omr_flip_mask_device(self.h, _ptr(src), _ptr(dst), width, height, int(flip_h),
                                       int(flip_v)), self.h)

    # ---- projection --------------------------------------------------------------------
    def project_stack(self, stack, pixel_type, size_x, size_y, size_z, algorithm, start, end,
                      stepping=1, big_endian_in=False, big_endian_out=False):
        bpp = _lib.BYTES_PER_PIXEL[pixel_type]
        out = np.empty(size_x * size_y * bpp, dtype=np.uint8)
        check(lib.omr_project_stack(self.h, _ptr(stack), pixel_type, int(big_endian_in), size_x,
                                    size_y, size_z, algorithm, start, end, stepping,
                                    out.ctypes.data, int(big_endian_out)), self.h)
        return out

    def project_stack_device(self, stack, pixel_type, size_x, size_y, size_z, algorithm, start,
                             end, out, stepping=1, big_endian_in=False, big_endian_out=False):
        check(lib.omr_project_stack_device(self.h, _ptr(stack), pixel_type, int(big_endian_in),
                                           size_x, size_y, size_z, algorithm, start, end,
                                           stepping, _ptr(out), int(big_endian_out)), self.h)
        return out

    def project_stacks_device(self, stacks, pixel_type, size_x, size_y, size_z, algorithm, start, end, outs,
                              stepping=1, big_endian_in=False, big_endian_out=False):
        """Several same-geometry stacks projected in one launch (the glue's K3)."""
        n = len(stacks)
        s = (ctypes.c_void_p * max(n, 1))(*[_ptr(x) for x in stacks])
        o = (ctypes.c_void_p * max(n, 1))(*[_ptr(x) for x in outs])
        check(lib.omr_project_stacks_device(self.h, s, n, pixel_type, int(big_endian_in), size_x, size_y, size_z,
                                            algorithm, start, end, stepping, o, int(big_endian_out)), self.h)
        return outs

    def render_projected_device(self, qdef, channels, stacks, pixel_type, size_x, size_y, size_z,
                                algorithm, start, end, out, stepping=1, big_endian=False,
                                flip_h=False, flip_v=False, bindings=None):
        arr, keep = make_bindings(channels) if bindings is None else bindings
        ptrs = (ctypes.c_void_p * max(len(stacks), 1))(*[_ptr(s) for s in stacks])
        check(lib.omr_render_projected_device(self.h, ctypes.byref(qdef), arr, len(channels), ptrs,
                                              pixel_type, int(big_endian), size_x, size_y, size_z,
                                              algorithm, start, end, stepping, int(flip_h),
                                              int(flip_v), _ptr(out)), self.h)
        return out

    # ---- encode ------------------------------------------------------------------------
    def _encode(self, fn, src, *args, cap):
        out = np.empty(cap, dtype=np.uint8)
        n = ctypes.c_size_t(0)
        check(fn(self.h, _ptr(src), *args, out.ctypes.data, cap, ctypes.byref(n)), self.h)
        return out[:n.value].tobytes()

    def encode_jpeg(self, argb, width, height, quality):
        argb = np.ascontiguousarray(argb, dtype=np.uint32)
        return self._encode(lib.omr_encode_jpeg, argb, width, height, float(quality),
                            cap=lib.omr_jpeg_max_bytes(width, height))

    def encode_jpeg_device(self, d_argb, width, height, quality):
        return self._encode(lib.omr_encode_jpeg_device, d_argb, width, height, float(quality),
                            cap=lib.omr_jpeg_max_bytes(width, height))

    def encode_jpeg_batch_device(self, d_argb, n_tiles, width, height, quality, d_out, d_offsets,
                                 d_lengths, d_status=None, tile_stride=0):
        """Async batch encode on the device; files packed in d_out (uint8 tensor)."""
        check(lib.omr_encode_jpeg_batch_device(self.h, _ptr(d_argb), tile_stride, n_tiles, width, height,
                                               float(quality), _ptr(d_out), d_out.numel(), _ptr(d_offsets),
                                               _ptr(d_lengths), _ptr(d_status)), self.h)

    def render_jpeg_batch_strided_device(self, qdef, channels, d_base, tile_stride, channel_stride, n_tiles,
                                         pixel_type, width, height, quality, d_out, d_offsets, d_lengths,
                                         d_status=None, big_endian=False, flip_h=False, flip_v=False, row_stride=0,
                                         bindings=None):
        """Render + JPEG of a strided plane batch in one call (fused F1 kernel where it applies):
        files packed in d_out, as encode_jpeg_batch_device."""
        arr, keep = make_bindings(channels) if bindings is None else bindings
        check(lib.omr_render_jpeg_batch_strided_device(
            self.h, ctypes.byref(qdef), arr, len(channels), _ptr(d_base), tile_stride, channel_stride, n_tiles,
            row_stride, pixel_type, int(big_endian), width, height, int(flip_h), int(flip_v), float(quality),
            _ptr(d_out), d_out.numel(), _ptr(d_offsets), _ptr(d_lengths), _ptr(d_status)), self.h)

    def render_jpeg_device(self, qdef, channels, planes, pixel_type, width, height, quality, big_endian=False,
                           flip_h=False, flip_v=False, row_stride=0, bindings=None):
        """One request in the default format (omr_render_jpeg): device planes (one tensor or
        address per channel, None for an inactive one) -> JPEG bytes."""
        arr, keep = make_bindings(channels) if bindings is None else bindings
        ptrs = (ctypes.c_void_p * max(len(planes), 1))(*[_ptr(p) for p in planes])
        cap = lib.omr_jpeg_max_bytes(width, height)
        out = np.empty(cap, dtype=np.uint8)
        n = ctypes.c_size_t(0)
        check(lib.omr_render_jpeg(self.h, ctypes.byref(qdef), arr, len(channels), ptrs, row_stride, pixel_type,
                                  int(big_endian), width, height, int(flip_h), int(flip_v), float(quality),
                                  out.ctypes.data, cap, ctypes.byref(n)), self.h)
        return out[:n.value].tobytes()

    def render_jpeg_batch_device(self, qdef, channels, d_plane_ptrs, n_tiles, pixel_type, width, height, quality,
                                 d_out, d_offsets, d_lengths, d_status=None, big_endian=False, flip_h=False,
                                 flip_v=False, row_stride=0, bindings=None):
        arr, keep = make_bindings(channels) if bindings is None else bindings
        check(lib.omr_render_jpeg_batch_device(
            self.h, ctypes.byref(qdef), arr, len(channels), _ptr(d_plane_ptrs), n_tiles, row_stride, pixel_type,
            int(big_endian), width, height, int(flip_h), int(flip_v), float(quality), _ptr(d_out), d_out.numel(),
            _ptr(d_offsets), _ptr(d_lengths), _ptr(d_status)), self.h)

    def encode_jpeg_batch(self, d_argb, n_tiles, width, height, quality, cap=None, tile_stride=0):
        """Batch encode device ARGB tiles -> list of JPEG byte strings (one host sync)."""
        if cap is None:
            cap = n_tiles * (width * height + 4096)
        out = np.empty(cap, dtype=np.uint8)
        offs = np.zeros(n_tiles, dtype=np.uint64)
        lens = np.zeros(n_tiles, dtype=np.uint32)
        check(lib.omr_encode_jpeg_batch(self.h, _ptr(d_argb), tile_stride, n_tiles, width, height,
                                        float(quality), out.ctypes.data, cap, offs.ctypes.data,
                                        lens.ctypes.data), self.h)
        return [out[int(o):int(o) + int(n)].tobytes() for o, n in zip(offs, lens)]

    def encode_png(self, argb, width, height):
        argb = np.ascontiguousarray(argb, dtype=np.uint32)
        return self._encode(lib.omr_encode_png, argb, width, height,
                            cap=lib.omr_png_max_bytes(width, height, 3))

    def encode_png_device(self, d_argb, width, height):
        return self._encode(lib.omr_encode_png_device, d_argb, width, height,
                            cap=lib.omr_png_max_bytes(width, height, 3))

    def encode_png_batch_device(self, d_argb, n_tiles, width, height, d_out, d_offsets=None, d_lengths=None,
                                d_status=None, tile_stride=0):
        """Batched PNG of n_tiles device ARGB tiles into d_out (device bytes); asynchronous."""
        check(lib.omr_encode_png_batch_device(self.h, _ptr(d_argb), tile_stride, n_tiles, width, height,
                                              _ptr(d_out), d_out.numel() * d_out.element_size(), _ptr(d_offsets),
                                              _ptr(d_lengths), _ptr(d_status)), self.h)

    def render_shape_mask_png_batch(self, masks, cap=None):
        """masks: [(bits, width, height, rgba, flip_h, flip_v)] -> [(status, png bytes)] (host in/out)."""
        n = len(masks)
        keep = [np.frombuffer(bytes(m[0]), dtype=np.uint8).copy() if m[0] is not None else None for m in masks]
        jobs = (_lib.MaskJob * max(n, 1))()
        for i, (m, b) in enumerate(zip(masks, keep)):
            jobs[i].bits = b.ctypes.data if b is not None and b.size else None
            jobs[i].n_bytes = 0 if b is None else b.size
            jobs[i].width, jobs[i].height = int(m[1]), int(m[2])
            jobs[i].rgba[:] = [int(v) for v in m[3]]
            jobs[i].flip_h, jobs[i].flip_v = int(bool(m[4])), int(bool(m[5]))
        if cap is None:
            cap = sum(lib.omr_png_batch_max_bytes(max(1, int(m[1])), max(1, int(m[2])), 1, 1) for m in masks)
        out = np.empty(max(cap, 1), dtype=np.uint8)
        offs = np.zeros(max(n, 1), np.uint64)
        lens = np.zeros(max(n, 1), np.uint32)
        stat = np.zeros(max(n, 1), np.int32)
        check(lib.omr_render_shape_mask_png_batch(self.h, jobs, n, out.ctypes.data, cap, offs.ctypes.data,
                                                  lens.ctypes.data, stat.ctypes.data), self.h)
        return [(int(stat[i]), out[int(offs[i]):int(offs[i]) + int(lens[i])].tobytes() if stat[i] == 0 else b"")
                for i in range(n)]

    def encode_tiff(self, argb, width, height):
        argb = np.ascontiguousarray(argb, dtype=np.uint32)
        return self._encode(lib.omr_encode_tiff, argb, width, height,
                            cap=lib.omr_tiff_max_bytes(width, height))

    def encode_tiff_device(self, d_argb, width, height):
        return self._encode(lib.omr_encode_tiff_device, d_argb, width, height,
                            cap=lib.omr_tiff_max_bytes(width, height))

    def render_shape_mask_png(self, bits, width, height, rgba, flip_h=False, flip_v=False):
        bits = np.frombuffer(bytes(bits), dtype=np.uint8).copy()
        col = (ctypes.c_uint8 * 4)(*[int(v) for v in rgba])
        cap = lib.omr_png_max_bytes(width, height, 1)
        out = np.empty(cap, dtype=np.uint8)
        n = ctypes.c_size_t(0)
        check(lib.omr_render_shape_mask_png(self.h, bits.ctypes.data if bits.size else None,
                                            bits.size, width, height, col, int(flip_h),
                                            int(flip_v), out.ctypes.data, cap, ctypes.byref(n)),
              self.h)
        return out[:n.value].tobytes()


def _torch_ordered(fn):
    """Wrap a *_device method: inputs after torch's queued work, torch after the outputs."""
    @functools.wraps(fn)
    def call(self, *a, **k):
        if self.torch_order:
            self.order_after_torch()
        try:
            return fn(self, *a, **k)
        finally:
            if self.torch_order and self.h:
                self.order_torch_after()
    return call


for _name in [n for n in vars(Context) if n.endswith("_device") or n == "encode_jpeg_batch"]:
    setattr(Context, _name, _torch_ordered(getattr(Context, _name)))
