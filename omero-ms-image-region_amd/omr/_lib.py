"""ctypes binding of libomr.so (include/omr/omr.h).

This is the ONLY way Python reaches the product path; there is no CPU fallback.
If libomr.so is missing, importing this module raises immediately.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("OMR_LIB") or os.path.join(_HERE, "libomr.so")   # OMR_LIB: a deployed build

if not os.path.exists(LIB_PATH):
    raise ImportError(
        f"libomr.so not found at {LIB_PATH}: build it with `make -C omero-ms-image-region_amd` "
        "(or __graft_entry__.build()); there is no fallback path")

# One HIP runtime per process: torch-ROCm bundles its own libamdhip64.so.7 (same soname as
# /opt/rocm's).  Loading torch first makes libomr.so bind to that already-loaded runtime
# instead of pulling in a second HIP/HSA runtime that would fight over the device.
try:
    import torch  # noqa: F401
except Exception:  # no torch: libomr.so uses /opt/rocm's runtime (the Java/FFI case)
    pass

lib = ctypes.CDLL(LIB_PATH)

# ---- enums (omr.h) ----------------------------------------------------------------------
OK, INVALID_ARGUMENT, NOT_FOUND, QUANTIZATION, DEVICE, OOM, BUFFER_TOO_SMALL, INTERNAL = range(8)
STATUS_NAMES = {0: "OK", 1: "INVALID_ARGUMENT", 2: "NOT_FOUND", 3: "QUANTIZATION", 4: "DEVICE",
                5: "OOM", 6: "BUFFER_TOO_SMALL", 7: "INTERNAL"}
# HTTP status the reference answers with for each outcome
HTTP_STATUS = {OK: 200, INVALID_ARGUMENT: 400, NOT_FOUND: 404, QUANTIZATION: 500, DEVICE: 500,
               OOM: 500, BUFFER_TOO_SMALL: 500, INTERNAL: 500}
MAX_REQUEST_CHANNELS = 64
MAP_NONE, MAP_REVERSE, MAP_NULL, MAP_BAD = range(4)
PIXELS_INT8, PIXELS_UINT8, PIXELS_INT16, PIXELS_UINT16, PIXELS_INT32, PIXELS_UINT32, \
    PIXELS_FLOAT, PIXELS_DOUBLE = range(8)
FAMILY_LINEAR, FAMILY_POLYNOMIAL, FAMILY_LOGARITHMIC, FAMILY_EXPONENTIAL = range(4)
MODEL_GREYSCALE, MODEL_RGB = 0, 1
PROJECTION_MAX, PROJECTION_MEAN, PROJECTION_SUM = 0, 1, 2
# OMR_SEM_* switches of the un-vendored upstream semantics (include/omr/omr.h)
SEM_WINDOW_INT_BOUNDS, SEM_ALPHA_SEPARATE, SEM_GREYSCALE_LUT, SEM_JPEG_CHROMA_DIV2 = 1, 2, 4, 8
SEM_PROJECTION_ALL_ACTIVE = 16
SEM_LOG_UNGUARDED, SEM_NOISE_REDUCTION_OFF, SEM_EXP_NORMALIZED, SEM_MASK_PIXEL_FLIP = 32, 64, 128, 256
SEM_ALL = 0x1FF
SEM_FLAGS = {"WINDOW_INT_BOUNDS": SEM_WINDOW_INT_BOUNDS, "ALPHA_SEPARATE": SEM_ALPHA_SEPARATE,
             "GREYSCALE_LUT": SEM_GREYSCALE_LUT, "JPEG_CHROMA_DIV2": SEM_JPEG_CHROMA_DIV2,
             "PROJECTION_ALL_ACTIVE": SEM_PROJECTION_ALL_ACTIVE, "LOG_UNGUARDED": SEM_LOG_UNGUARDED,
             "NOISE_REDUCTION_OFF": SEM_NOISE_REDUCTION_OFF, "EXP_NORMALIZED": SEM_EXP_NORMALIZED,
             "MASK_PIXEL_FLIP": SEM_MASK_PIXEL_FLIP}

PIXEL_TYPE_NAMES = {"int8": PIXELS_INT8, "uint8": PIXELS_UINT8, "int16": PIXELS_INT16,
                    "uint16": PIXELS_UINT16, "int32": PIXELS_INT32, "uint32": PIXELS_UINT32,
                    "float": PIXELS_FLOAT, "double": PIXELS_DOUBLE}
BYTES_PER_PIXEL = {PIXELS_INT8: 1, PIXELS_UINT8: 1, PIXELS_INT16: 2, PIXELS_UINT16: 2,
                   PIXELS_INT32: 4, PIXELS_UINT32: 4, PIXELS_FLOAT: 4, PIXELS_DOUBLE: 8}


class QuantumDef(ctypes.Structure):
    _fields_ = [("cd_start", ctypes.c_int32), ("cd_end", ctypes.c_int32),
                ("bit_resolution", ctypes.c_int32), ("model", ctypes.c_int32)]


class ChannelBinding(ctypes.Structure):
    _fields_ = [("active", ctypes.c_int32), ("family", ctypes.c_int32),
                ("coefficient", ctypes.c_double), ("noise_reduction", ctypes.c_int32),
                ("reverse", ctypes.c_int32), ("input_start", ctypes.c_double),
                ("input_end", ctypes.c_double), ("global_min", ctypes.c_double),
                ("global_max", ctypes.c_double), ("rgba", ctypes.c_uint8 * 4),
                ("lut", ctypes.POINTER(ctypes.c_uint8))]


class TileRequest(ctypes.Structure):
    _fields_ = [("z", ctypes.c_int32), ("t", ctypes.c_int32), ("x", ctypes.c_int32), ("y", ctypes.c_int32)]


class TileJob(ctypes.Structure):
    _fields_ = [("pb", ctypes.c_void_p), ("qdef", ctypes.c_void_p), ("channels", ctypes.c_void_p),
                ("size_c", ctypes.c_int32), ("z", ctypes.c_int32), ("t", ctypes.c_int32), ("x", ctypes.c_int32),
                ("y", ctypes.c_int32), ("width", ctypes.c_int32), ("height", ctypes.c_int32),
                ("flip_h", ctypes.c_int32), ("flip_v", ctypes.c_int32), ("format", ctypes.c_int32),
                ("quality", ctypes.c_float), ("has_projection", ctypes.c_int32), ("projection", ctypes.c_int32),
                ("projection_start", ctypes.c_int32), ("projection_end", ctypes.c_int32)]


FORMAT_JPEG, FORMAT_PNG, FORMAT_ARGB, FORMAT_TIFF = 0, 1, 2, 3


class MaskJob(ctypes.Structure):
    _fields_ = [("bits", ctypes.c_void_p), ("n_bytes", ctypes.c_size_t), ("width", ctypes.c_int32),
                ("height", ctypes.c_int32), ("rgba", ctypes.c_uint8 * 4), ("flip_h", ctypes.c_int32),
                ("flip_v", ctypes.c_int32)]


class Region(ctypes.Structure):
    _fields_ = [("x", ctypes.c_int32), ("y", ctypes.c_int32),
                ("width", ctypes.c_int32), ("height", ctypes.c_int32)]


_NCH = 64


class ImageRegionCtxStruct(ctypes.Structure):
    _fields_ = [("image_id", ctypes.c_int64), ("z", ctypes.c_int32), ("t", ctypes.c_int32),
                ("has_tile", ctypes.c_int32), ("tile", Region),
                ("has_resolution", ctypes.c_int32), ("resolution", ctypes.c_int32),
                ("has_region", ctypes.c_int32), ("region", Region),
                ("n_channels", ctypes.c_int32), ("channels", ctypes.c_int32 * _NCH),
                ("window_set", ctypes.c_int32 * _NCH), ("windows", (ctypes.c_float * 2) * _NCH),
                ("color_set", ctypes.c_int32 * _NCH), ("colors", (ctypes.c_char * 64) * _NCH),
                ("model", ctypes.c_int32), ("has_quality", ctypes.c_int32),
                ("quality", ctypes.c_float), ("inverted_axis", ctypes.c_int32),
                ("projection", ctypes.c_int32), ("has_projection_start", ctypes.c_int32),
                ("projection_start", ctypes.c_int32), ("has_projection_end", ctypes.c_int32),
                ("projection_end", ctypes.c_int32), ("n_maps", ctypes.c_int32),
                ("map_reverse", ctypes.c_int32 * _NCH), ("flip_h", ctypes.c_int32),
                ("flip_v", ctypes.c_int32), ("format", ctypes.c_char * 16),
                ("cache_key", ctypes.c_char * 17)]


class ShapeMaskCtxStruct(ctypes.Structure):
    _fields_ = [("shape_id", ctypes.c_int64), ("has_color", ctypes.c_int32),
                ("color", ctypes.c_char * 64), ("flip_h", ctypes.c_int32),
                ("flip_v", ctypes.c_int32), ("cache_key", ctypes.c_char * 128)]


_vp = ctypes.c_void_p
_i32 = ctypes.c_int32
_i64 = ctypes.c_int64
_sz = ctypes.c_size_t
_f32 = ctypes.c_float
_u8p = ctypes.POINTER(ctypes.c_uint8)
_QD = ctypes.POINTER(QuantumDef)
_CB = ctypes.POINTER(ChannelBinding)

_SIGS = {
    "omr_abi_version": (_i32, []),
    "omr_ctx_create": (_i32, [_i32, ctypes.POINTER(_vp)]),
    "omr_ctx_destroy": (None, [_vp]),
    "omr_last_error": (ctypes.c_char_p, [_vp]),
    "omr_ctx_synchronize": (_i32, [_vp]),
    "omr_ctx_set_stream": (_i32, [_vp, _vp]),
    "omr_ctx_get_stream": (_vp, [_vp]),
    "omr_ctx_set_semantics": (_i32, [_vp, ctypes.c_uint32]),
    "omr_ctx_get_semantics": (ctypes.c_uint32, [_vp]),
    "omr_ctx_enable_kernel_timing": (_i32, [_vp, _i32]),
    "omr_ctx_kernel_timings": (_i32, [_vp, _vp, _vp, _i32]),
    "omr_pinned_alloc": (_vp, [_vp, _sz]),
    "omr_pinned_free": (None, [_vp, _vp]),
    "omr_pixel_buffer_open": (_i32, [ctypes.c_char_p, _i32, _i32, _i32, _i32, _i32, _i32, ctypes.POINTER(_vp)]),
    "omr_pixel_buffer_close": (None, [_vp]),
    "omr_pixel_buffer_plane_offset": (_i64, [_vp, _i32, _i32, _i32]),
    "omr_pixel_buffer_get_tile": (_i32, [_vp, _i32, _i32, _i32, _i32, _i32, _i32, _i32, _vp, _sz]),
    "omr_ctx_set_pixel_buffer_dma": (_i32, [_vp, _i32]),
    "omr_batcher_create": (_i32, [_i32, _i32, _i32, ctypes.POINTER(_vp)]),
    "omr_batcher_destroy": (None, [_vp]),
    "omr_batcher_submit": (_i32, [_vp, _vp, ctypes.POINTER(ctypes.c_uint64)]),
    "omr_batcher_submit_mask": (_i32, [_vp, _vp, ctypes.POINTER(ctypes.c_uint64)]),
    "omr_batcher_wait": (_i32, [_vp, ctypes.c_uint64, _vp, _sz, ctypes.POINTER(_sz)]),
    "omr_batcher_stats": (_i32, [_vp, _vp]),
    "omr_batcher_set_semantics": (_i32, [_vp, ctypes.c_uint32]),
    "omr_batcher_set_stack_cache": (_i32, [_vp, _i64]),
    "omr_batcher_stack_cache_stats": (_i32, [_vp, _vp]),
    "omr_pool_set_stack_cache": (_i32, [_vp, _i64]),
    "omr_pool_create": (_i32, [_vp, _i32, _i32, _i32, ctypes.POINTER(_vp)]),
    "omr_pool_destroy": (None, [_vp]),
    "omr_pool_size": (_i32, [_vp]),
    "omr_pool_submit": (_i32, [_vp, _vp, ctypes.POINTER(ctypes.c_uint64)]),
    "omr_pool_submit_mask": (_i32, [_vp, _vp, ctypes.POINTER(ctypes.c_uint64)]),
    "omr_pool_wait": (_i32, [_vp, ctypes.c_uint64, _vp, _sz, ctypes.POINTER(_sz)]),
    "omr_pool_device_index": (_i32, [_vp, ctypes.c_uint64]),
    "omr_pool_set_semantics": (_i32, [_vp, ctypes.c_uint32]),
    "omr_pool_stats": (_i32, [_vp, _vp, _i32]),
    "omr_render_pixel_buffer_tiles": (_i32, [_vp, _vp, _QD, _CB, _i32, _vp, _i32, _i32, _i32, _i32, _i32, _vp,
                                             _i32]),
    "omr_render_packed_int": (_i32, [_vp, _QD, _CB, _i32, _vp, _i64, _i32, _i32, _i32, _i32, _i32,
                                     _i32, _vp]),
    "omr_render_packed_int_device": (_i32, [_vp, _QD, _CB, _i32, _vp, _i64, _i32, _i32, _i32, _i32,
                                            _i32, _i32, _vp]),
    "omr_render_batch_device": (_i32, [_vp, _QD, _CB, _i32, _vp, _i32, _i64, _i32, _i32, _i32, _i32,
                                       _i32, _i32, _vp, _vp]),
    "omr_render_batch_strided_device": (_i32, [_vp, _QD, _CB, _i32, _vp, _i64, _i64, _i32, _i64, _i32, _i32,
                                               _i32, _i32, _i32, _i32, _vp, _vp]),
    "omr_flip_argb_device": (_i32, [_vp, _vp, _vp, _i32, _i32, _i32, _i32]),
    "omr_flip_mask_device": (_i32, [_vp, _vp, _vp, _i32, _i32, _i32, _i32]),
    "omr_project_stack": (_i32, [_vp, _vp, _i32, _i32, _i32, _i32, _i32, _i32, _i32, _i32, _i32,
                                 _vp, _i32]),
    "omr_project_stack_device": (_i32, [_vp, _vp, _i32, _i32, _i32, _i32, _i32, _i32, _i32, _i32,
                                        _i32, _vp, _i32]),
    "omr_render_projected_device": (_i32, [_vp, _QD, _CB, _i32, _vp, _i32, _i32, _i32, _i32, _i32,
                                           _i32, _i32, _i32, _i32, _i32, _i32, _vp]),
    "omr_jpeg_max_bytes": (_sz, [_i32, _i32]),
    "omr_png_max_bytes": (_sz, [_i32, _i32, _i32]),
    "omr_encode_jpeg": (_i32, [_vp, _vp, _i32, _i32, _f32, _vp, _sz, ctypes.POINTER(_sz)]),
    "omr_encode_jpeg_device": (_i32, [_vp, _vp, _i32, _i32, _f32, _vp, _sz, ctypes.POINTER(_sz)]),
    "omr_encode_jpeg_batch_device": (_i32, [_vp, _vp, _i64, _i32, _i32, _i32, _f32, _vp, _sz, _vp, _vp, _vp]),
    "omr_encode_jpeg_batch": (_i32, [_vp, _vp, _i64, _i32, _i32, _i32, _f32, _vp, _sz, _vp, _vp]),
    "omr_jpeg_quant_tables": (_i32, [_f32, _vp, _vp]),
    "omr_render_jpeg_batch_strided_device": (_i32, [_vp, _QD, _CB, _i32, _vp, _i64, _i64, _i32, _i64, _i32, _i32,
                                                    _i32, _i32, _i32, _i32, _f32, _vp, _sz, _vp, _vp, _vp]),
    "omr_render_jpeg_batch_device": (_i32, [_vp, _QD, _CB, _i32, _vp, _i32, _i64, _i32, _i32, _i32, _i32, _i32,
                                            _i32, _f32, _vp, _sz, _vp, _vp, _vp]),
    "omr_render_jpeg": (_i32, [_vp, _QD, _CB, _i32, _vp, _i64, _i32, _i32, _i32, _i32, _i32, _i32, _f32, _vp, _sz,
                               ctypes.POINTER(_sz)]),
    "omr_jpeg_quant_tables_sem": (_i32, [_f32, ctypes.c_uint32, _vp, _vp]),
    "omr_tiff_max_bytes": (_sz, [_i32, _i32]),
    "omr_encode_tiff": (_i32, [_vp, _vp, _i32, _i32, _vp, _sz, ctypes.POINTER(_sz)]),
    "omr_encode_tiff_device": (_i32, [_vp, _vp, _i32, _i32, _vp, _sz, ctypes.POINTER(_sz)]),
    "omr_encode_png": (_i32, [_vp, _vp, _i32, _i32, _vp, _sz, ctypes.POINTER(_sz)]),
    "omr_encode_png_device": (_i32, [_vp, _vp, _i32, _i32, _vp, _sz, ctypes.POINTER(_sz)]),
    "omr_render_shape_mask_png": (_i32, [_vp, _vp, _sz, _i32, _i32, _vp, _i32, _i32, _vp, _sz,
                                         ctypes.POINTER(_sz)]),
    "omr_project_stacks_device": (_i32, [_vp, _vp, _i32, _i32, _i32, _i32, _i32, _i32, _i32, _i32, _i32, _i32, _vp,
                                         _i32]),
    "omr_encode_png_batch_device": (_i32, [_vp, _vp, _i64, _i32, _i32, _i32, _vp, _sz, _vp, _vp, _vp]),
    "omr_png_batch_max_bytes": (_sz, [_i32, _i32, _i32, _i32]),
    "omr_render_shape_mask_png_batch": (_i32, [_vp, ctypes.POINTER(MaskJob), _i32, _vp, _sz, _vp, _vp, _vp]),
    "omr_split_html_color": (_i32, [ctypes.c_char_p, ctypes.POINTER(_i32)]),
    "omr_shape_mask_fill_color": (_i32, [_i32, _i32, ctypes.c_char_p, _vp]),
    "omr_get_region_def": (_i32, [_i32, ctypes.POINTER(Region), _i32, ctypes.POINTER(_i32), _i32,
                                  _i32, _i32, _i32, _i32, _i32, ctypes.POINTER(Region)]),
    "omr_resolution_level": (_i32, [_i32, _i32]),
    "omr_check_plane_def": (_i32, [ctypes.POINTER(Region), _i32, _i32]),
    "omr_parse_lut": (_i32, [_vp, _sz, _vp]),
    "omr_image_region_ctx_parse": (_i32, [ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_char_p),
                                          _i32, ctypes.POINTER(ImageRegionCtxStruct), _vp, _sz]),
    "omr_shape_mask_ctx_parse": (_i32, [ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_char_p),
                                        _i32, ctypes.POINTER(ShapeMaskCtxStruct), _vp, _sz]),
    "omr_lut_provider_create": (_i32, [ctypes.c_char_p, ctypes.POINTER(_vp)]),
    "omr_lut_provider_destroy": (None, [_vp]),
    "omr_lut_provider_count": (_i32, [_vp]),
    "omr_lut_provider_add": (_i32, [_vp, ctypes.c_char_p, _vp]),
    "omr_lut_provider_get": (_vp, [_vp, ctypes.c_char_p]),
    "omr_create_rendering_def": (_i32, [_i32, _i32, _QD, _CB]),
    "omr_update_settings": (_i32, [ctypes.POINTER(ImageRegionCtxStruct), _i32, _QD, _CB, _vp, _vp, _sz]),
}

MISSING = []
for _name, (_res, _args) in _SIGS.items():
    try:
        _fn = getattr(lib, _name)
    except AttributeError:
        MISSING.append(_name)
        continue
    _fn.restype = _res
    _fn.argtypes = _args

EXPORTED = [n for n in _SIGS if n not in MISSING]


class OmrError(RuntimeError):
    def __init__(self, status, message=""):
        self.status = status
        super().__init__(f"{STATUS_NAMES.get(status, status)}: {message}")


def check(status, ctx=None):
    if status != OK:
        msg = ""
        if ctx is not None:
            raw = lib.omr_last_error(ctx)
            msg = raw.decode() if raw else ""
        raise OmrError(status, msg)
    return status
