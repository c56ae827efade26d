/*
 * omr.h — C ABI of the MI355X-native image-region rendering path.
 *
 * This is the drop-in boundary between the reference's Java host code
 * (omero-ms-image-region's ImageRegionRequestHandler / ShapeMaskRequestHandler)
 * and hand-written gfx950 HIP kernels.  Every entry point names the reference
 * call site it replaces.  Paths are relative to
 *   src/main/java/com/glencoesoftware/omero/ms/image/region/
 * of the reference.  Plain pointers and sizes only; no torch or HIP types.
 *
 * Status codes map onto the reference's HTTP outcomes
 * (ImageRegionVerticle.java:163-186, ImageRegionMicroserviceVerticle.java:301-304):
 *   OMR_INVALID_ARGUMENT -> 400 (IllegalArgumentException / ValidationException)
 *   OMR_NOT_FOUND        -> 404 (handler returned null, e.g. unknown format)
 *   OMR_QUANTIZATION     -> 500 (QuantizationException, ImageRegionRequestHandler.java:479)
 *   OMR_DEVICE / OMR_OOM -> 500
 *   OMR_INTERNAL         -> 500 (unchecked exceptions the reference would throw: NPE, CCE, ...)
 *
 * Threading: one omr_ctx per worker thread.  Calls on distinct contexts may run
 * concurrently; one context must not be called concurrently.  All buffers are
 * caller-owned.  Unlike the reference (global mutable compression level,
 * ImageRegionRequestHandler.java:457-460 on a Spring singleton), JPEG quality is
 * a per-call argument.
 */
#ifndef OMR_OMR_H
#define OMR_OMR_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OMR_ABI_VERSION 2   /* 2 (round 4): omr_tile_job gained the projection fields */

typedef int32_t omr_status;
enum {
    OMR_OK = 0,
    OMR_INVALID_ARGUMENT = 1,
    OMR_NOT_FOUND = 2,
    OMR_QUANTIZATION = 3,
    OMR_DEVICE = 4,
    OMR_OOM = 5,
    OMR_BUFFER_TOO_SMALL = 6,
    OMR_INTERNAL = 7          /* NPE / ClassCastException / IndexOutOfBounds in the reference -> 500 */
};

/* ome.model.enums.PixelsType values the path supports. */
enum {
    OMR_PIXELS_INT8 = 0,
    OMR_PIXELS_UINT8 = 1,
    OMR_PIXELS_INT16 = 2,
    OMR_PIXELS_UINT16 = 3,
    OMR_PIXELS_INT32 = 4,
    OMR_PIXELS_UINT32 = 5,
    OMR_PIXELS_FLOAT = 6,
    OMR_PIXELS_DOUBLE = 7
};

/* ome.model.enums.Family (ImageRegionVerticle.java:72-76 lists the families). */
enum {
    OMR_FAMILY_LINEAR = 0,
    OMR_FAMILY_POLYNOMIAL = 1,
    OMR_FAMILY_LOGARITHMIC = 2,
    OMR_FAMILY_EXPONENTIAL = 3
};

/* RenderingModel: Renderer.MODEL_GREYSCALE / MODEL_RGB (ImageRegionCtx.java:333-341). */
enum { OMR_MODEL_GREYSCALE = 0, OMR_MODEL_RGB = 1 };

/* IProjection constants used by ProjectionService.java:75-91. */
enum { OMR_PROJECTION_MAX = 0, OMR_PROJECTION_MEAN = 1, OMR_PROJECTION_SUM = 2 };

/* QuantumDef + RenderingDef model (ImageRegionRequestHandler.java:262-277). */
typedef struct omr_quantum_def {
    int32_t cd_start;        /* 0 */
    int32_t cd_end;          /* 255 (QuantumFactory.DEPTH_8BIT) */
    int32_t bit_resolution;  /* 255 */
    int32_t model;           /* OMR_MODEL_* */
} omr_quantum_def;

/*
 * One ChannelBinding as the Renderer sees it after updateSettings
 * (ImageRegionRequestHandler.java:281-298 defaults, :689-741 request settings).
 */
typedef struct omr_channel_binding {
    int32_t active;           /* Renderer.setActive (:696) */
    int32_t family;           /* OMR_FAMILY_*; HTTP path is always linear (:285) */
    double coefficient;       /* curve coefficient k; HTTP path 1.0 (:286) */
    int32_t noise_reduction;  /* HTTP path false (:287) */
    int32_t reverse;          /* ReverseIntensityContext in the codomain chain (:725-726) */
    double input_start;       /* Renderer.setChannelWindow start (:703), float-rounded by ImageRegionCtx.java:313 */
    double input_end;         /* window end */
    double global_min;        /* LUT domain = StatsInfo/type range (StatsFactory.initPixelsRange, :290-291) */
    double global_max;
    uint8_t rgba[4];          /* Renderer.setRGBA (:712) */
    const uint8_t* lut;       /* setChannelLookupTable (:708): 768 bytes R[256] G[256] B[256]; NULL = use rgba */
} omr_channel_binding;

/* RegionDef (omeis.providers.re.data.RegionDef). */
typedef struct omr_region {
    int32_t x, y, width, height;
} omr_region;

typedef struct omr_ctx omr_ctx;

/* ---- context --------------------------------------------------------- */
int32_t     omr_abi_version(void);
omr_status  omr_ctx_create(int32_t device_ordinal, omr_ctx** out);
void        omr_ctx_destroy(omr_ctx* ctx);
const char* omr_last_error(const omr_ctx* ctx);
omr_status  omr_ctx_synchronize(omr_ctx* ctx);
/* Run subsequent device-side calls on a caller-owned hipStream_t (NULL = ctx's own). */
omr_status  omr_ctx_set_stream(omr_ctx* ctx, void* hip_stream);
void*       omr_ctx_get_stream(omr_ctx* ctx);
/*
 * Kernel timing (perf4j StopWatch analogue, ImageRegionRequestHandler.java:502): when enabled,
 * every hot-kernel launch (K2 render, K3 projection, K4 JPEG) is bracketed by HIP events on
 * the stream it is launched on.  omr_ctx_kernel_timings synchronises, writes up to `cap`
 * per-launch durations in ms (launch order) and clears the record; returns the count.
 * kind_out (optional) receives 2 = render, 3 = projection, 4 = jpeg per entry.
 */
omr_status  omr_ctx_enable_kernel_timing(omr_ctx* ctx, int32_t enable);
int32_t     omr_ctx_kernel_timings(omr_ctx* ctx, float* ms_out, int32_t* kind_out, int32_t cap);
/* Pinned host staging (PixelBuffer tile reads land here). */
void*       omr_pinned_alloc(omr_ctx* ctx, size_t bytes);
void        omr_pinned_free(omr_ctx* ctx, void* p);

/*
 * Un-vendored upstream semantics.  The quantization, compositing and
 * JPEG-table arithmetic lives in omero:server 5.4.10 jars that are absent here, so every choice
 * that could not be pinned is a named switch; 0 (all off) is the restatement the repo defaults
 * to (DESIGN.md §2 gives the reasoning per switch).  The CPU restatement (oracle/) implements the
 * same switches, and the GPU tests cover each one against it.
 */
enum {
    /* Quantization_8_16_bit LUT window ends as Java (int) casts of the double window
     * (x < (int)start -> cdStart, x >= (int)end -> cdEnd) instead of double compares
     * (x < start, x >= end).  Integer pixel types (the LUT path) only. */
    OMR_SEM_WINDOW_INT_BOUNDS = 1u << 0,
    /* Channel colour scaling in two truncating steps, colour then alpha,
     * (int)((int)(c/255f * v) * (a/255f)), instead of (int)((c/255f * a/255f) * v).  (The
     * one-step order (int)((c/255f * v) * (a/255f)) needs no switch: it equals the default for
     * every c, a, v in 0..255, tests/test_semantics.py.) */
    OMR_SEM_ALPHA_SEPARATE = 1u << 1,
    /* Greyscale model: a .lut channel renders (R[v],G[v],B[v]) instead of ignoring the LUT. */
    OMR_SEM_GREYSCALE_LUT = 1u << 2,
    /* JPEG chroma base table K2Div2Chrominance (Annex K chroma halved, JPEGQTable) scaled by the
     * quality instead of K2Chrominance. */
    OMR_SEM_JPEG_CHROMA_DIV2 = 1u << 3,
    /* Projection glue: render every active channel.  By default
     * omr_render_projected_device reproduces the reference, whose InMemoryPlanarPixelBuffer is
     * sized sizeC = #active channels (ImageRegionRequestHandler.java:538-555) but read at the
     * original channel index (:525, :549): a rendered channel whose index is >= #active fails its
     * bounds check (DimensionsOutOfBoundsException -> 500, here OMR_INTERNAL). */
    OMR_SEM_PROJECTION_ALL_ACTIVE = 1u << 4,
    /* S2 logarithmic map without the x <= 0 guard: f(x) = Math.log(x) for every x (NaN below 0,
     * -Infinity at 0, propagated through both rounding stages as Java does: Math.round(NaN) = 0).
     * By default f(x) = x > 0 ? log(x) : 0. */
    OMR_SEM_LOG_UNGUARDED = 1u << 5,
    /* S4 noise reduction off: a channel's noiseReduction flag has no effect.  By default the first
     * and last decile of the window clip to cdStart / cdEnd. */
    OMR_SEM_NOISE_REDUCTION_OFF = 1u << 6,
    /* Exponential map on the window-normalised input (Appendix C): f(x) = exp(pow((x - start) /
     * (end - start), k)).  By default f(x) = exp(pow(x, k)), which overflows to +Infinity above
     * x ~ 709 for k = 1 (a 16-bit window then renders cdStart below its end). */
    OMR_SEM_EXP_NORMALIZED = 1u << 7,
    /* Shape mask, width % 8 == 0 with a flip: flip at pixel level (the evident intent).  By default
     * the reference is reproduced: it flips the still bit-packed buffer as if it held one byte per
     * pixel (ShapeMaskRequestHandler.java:175-181, :145-150), which indexes past the array
     * (ArrayIndexOutOfBoundsException -> the future fails -> 404, ShapeMaskVerticle.java:119-128,
     * here OMR_NOT_FOUND) unless the buffer holds >= width*height bytes, when the byte-flipped
     * buffer is rendered as packed bits. */
    OMR_SEM_MASK_PIXEL_FLIP = 1u << 8,
    OMR_SEM_ALL = 0x1FFu
};
/* Semantics of every later call on this context (renders, projections' renders, JPEG). */
omr_status omr_ctx_set_semantics(omr_ctx* ctx, uint32_t flags);
uint32_t   omr_ctx_get_semantics(const omr_ctx* ctx);

/* ---- pixel buffer: ROMIO repository file -> pinned staging -> HBM ---------- */
/*
 * Replaces pixelsService.getPixelBuffer(pixels, false) (ImageRegionRequestHandler.java:302-309)
 * for repository-backed images (upstream ome.io.nio.RomioPixelBuffer):
 * one file of big-endian planes in XYZCT order, plane (z, c, t) at
 * ((t*sizeC + c)*sizeZ + z) * sizeX*sizeY*bytesPerPixel.  Read-only; safe to share between
 * contexts and threads (pread).  open: OMR_NOT_FOUND when the file does not exist,
 * OMR_INVALID_ARGUMENT when it is shorter than the dimensions say.
 */
typedef struct omr_pixel_buffer omr_pixel_buffer;
omr_status omr_pixel_buffer_open(const char* path, int32_t size_x, int32_t size_y, int32_t size_z,
                                 int32_t size_c, int32_t size_t_, int32_t pixel_type,
                                 omr_pixel_buffer** out);
void       omr_pixel_buffer_close(omr_pixel_buffer* pb);
/* RomioPixelBuffer.getPlaneOffset(z, c, t) in bytes; -1 when out of range. */
int64_t    omr_pixel_buffer_plane_offset(const omr_pixel_buffer* pb, int32_t z, int32_t c, int32_t t);
/* PixelBuffer.getTile(z, c, t, x, y, w, h): w*h pixels, rows packed, file (big-endian) byte order.
 * OMR_INVALID_ARGUMENT outside the image (DimensionsOutOfBoundsException). */
omr_status omr_pixel_buffer_get_tile(const omr_pixel_buffer* pb, int32_t z, int32_t c, int32_t t,
                                     int32_t x, int32_t y, int32_t w, int32_t h, void* dst, size_t cap);
typedef struct omr_tile_request { int32_t z, t, x, y; } omr_tile_request;
/*
 * n render_image_region tile requests (ImageRegionRequestHandler.java:430-600: getPixelBuffer ->
 * renderAsPackedInt -> flip) of one image at one rendering setting, all width x height: reader
 * threads pread each group of tiles straight into pinned memory while the previous group is
 * copied to HBM (own copy stream), rendered (K1+K2) and copied back.  argb_out: n*height*width
 * uint32 in host memory (out_on_device 0; pinned memory from omr_pinned_alloc skips a bounce
 * copy) or in device memory (1: e.g. for omr_encode_jpeg_batch_device).  Synchronous.
 */
/* Tile rows DMA'd straight from the registered file mapping (1, default) or copied by reader
 * threads into pinned staging first (0).  The DMA path falls back to staging on its own when the
 * driver refuses to register the mapping. */
omr_status omr_ctx_set_pixel_buffer_dma(omr_ctx* ctx, int32_t enable);
omr_status omr_render_pixel_buffer_tiles(omr_ctx* ctx, const omr_pixel_buffer* pb,
                                         const omr_quantum_def* qdef,
                                         const omr_channel_binding* channels, int32_t size_c,
                                         const omr_tile_request* reqs, int32_t n, int32_t width,
                                         int32_t height, int32_t flip_h, int32_t flip_v,
                                         uint32_t* argb_out, int32_t out_on_device);

/* ---- request batching ------------------------------ */
/*
 * Concurrent render_image_region requests coalesced into GPU batches.  The reference runs each
 * request on its own worker thread (ImageRegionMicroserviceVerticle.java:149-165) with its own
 * Renderer (ImageRegionRequestHandler.java:436-440) and caches finished regions in Redis under
 * ImageRegionCtx.cacheKey (ImageRegionCtx.java:165-177).  A batcher owns one GPU context and a
 * dispatcher thread: submitted jobs are grouped by image + rendering settings + tile size + flip +
 * format, each group is rendered by one omr_render_pixel_buffer_tiles call and encoded by one
 * batched JPEG / PNG launch, and identical tiles in flight together are rendered once.
 * Projection requests (p=intmax|intmean|intsum, :506-558) are jobs with has_projection set: the
 * active channels' Z-stacks at t go to HBM by DMA, K3 + K2 (or K3R) project and render the full
 * plane, and the group's planes are encoded in one batch; jobs with the same image, settings,
 * projection and t are rendered once.  Shape masks (render_shape_mask,
 * ShapeMaskRequestHandler.java:165-207, one per worker at ShapeMaskVerticle.java:121-149) are
 * jobs of their own (omr_batcher_submit_mask): every mask of a dispatch round is encoded by one
 * omr_render_shape_mask_png_batch call.  A failing job (OMR_QUANTIZATION, the quirk-3 OMR_INTERNAL
 * of the projection glue, a mask's 404) fails alone.
 * submit/wait are thread-safe; the pixel buffer must outlive its jobs.
 */
enum { OMR_FORMAT_JPEG = 0, OMR_FORMAT_PNG = 1, OMR_FORMAT_ARGB = 2 /* packed int[] */,
       OMR_FORMAT_TIFF = 3 /* TIFFImageWriter branch, :583-596 */ };
typedef struct omr_tile_job {
    const omr_pixel_buffer* pb;
    const struct omr_quantum_def* qdef;            /* copied at submit */
    const struct omr_channel_binding* channels;    /* size_c entries, copied (LUTs too) */
    int32_t size_c;
    int32_t z, t, x, y, width, height;
    int32_t flip_h, flip_v;
    int32_t format;                                /* OMR_FORMAT_*; others -> OMR_NOT_FOUND (404) */
    float quality;                                 /* JPEG */
    /* p=intmax|intmean|intsum[|start:end] (ImageRegionCtx.projection, ImageRegionRequestHandler.java
     * :506-558): with has_projection != 0 every active channel is projected (OMR_PROJECTION_*) over
     * z in [projection_start, projection_end] at t -- a negative bound takes the reference's default,
     * 0 / sizeZ - 1 (:510-515) -- and the full projected plane is rendered: z, x, y, width and height
     * are ignored, as the glue replaces the plane definition (:550-552).  Zero-initialised: none. */
    int32_t has_projection, projection, projection_start, projection_end;
} omr_tile_job;
struct omr_mask_job;   /* shape-mask job, declared with omr_render_shape_mask_png_batch below */
typedef struct omr_batcher omr_batcher;
omr_status omr_batcher_create(int32_t device_ordinal, int32_t max_batch, int32_t max_wait_us,
                              omr_batcher** out);
void       omr_batcher_destroy(omr_batcher* b);
omr_status omr_batcher_submit(omr_batcher* b, const omr_tile_job* job, uint64_t* ticket);
/* A render_shape_mask job (the mask bytes are copied at submit); its result is the PNG file. */
omr_status omr_batcher_submit_mask(omr_batcher* b, const struct omr_mask_job* job, uint64_t* ticket);
/* Blocks until the job is done; copies its encoded bytes.  OMR_BUFFER_TOO_SMALL sets *len and
 * keeps the result for a retry with a larger buffer. */
omr_status omr_batcher_wait(omr_batcher* b, uint64_t ticket, uint8_t* out, size_t cap, size_t* len);
/* jobs submitted, dispatch rounds, tiles rendered (distinct renders: tiles, projected planes and
 * masks), duplicate jobs served from a sibling job's result */
omr_status omr_batcher_stats(omr_batcher* b, uint64_t stats_out[4]);
/* OMR_SEM_* flags for jobs submitted after this call (each job keeps the flags it was submitted
 * under; jobs with different flags never share a render). */
omr_status omr_batcher_set_semantics(omr_batcher* b, uint32_t flags);
/* HBM stack cache of the projection jobs: the (pixel buffer, c, t) Z-stacks stay resident (least
 * recently used evicted) up to max_bytes (default 4 GiB, env OMR_STACK_CACHE_MB; 0 disables), so
 * repeated p= requests on an image skip the PCIe upload.  stats: hits, misses, resident bytes. */
omr_status omr_batcher_set_stack_cache(omr_batcher* b, int64_t max_bytes);
omr_status omr_batcher_stack_cache_stats(omr_batcher* b, uint64_t stats_out[3]);

/* ---- node-level serving pool: the request batches of all worker threads over the node's GPUs ---- */
/*
 * The reference's only parallelism is N worker-verticle instances over one worker pool
 * (ImageRegionMicroserviceVerticle.java:84-85, :149-165).  A pool holds one batcher per entry of
 * devices[] (its own context, stream, dispatcher thread and plan / LUT replicas in that GPU's
 * HBM; an ordinal may repeat, e.g. two batchers on one card) and sends each submitted job to the
 * batcher with the fewest jobs queued or in flight.  Tiles are independent, so nothing crosses
 * between GPUs: no collective, no peer copies.  submit / wait are thread-safe and keep the
 * batcher's per-tile statuses (OMR_QUANTIZATION fails only its own tile).  At most 256 devices.
 */
typedef struct omr_pool omr_pool;
omr_status omr_pool_create(const int32_t* devices, int32_t n_devices, int32_t max_batch, int32_t max_wait_us,
                           omr_pool** out);
void       omr_pool_destroy(omr_pool* p);
int32_t    omr_pool_size(const omr_pool* p);
omr_status omr_pool_submit(omr_pool* p, const omr_tile_job* job, uint64_t* ticket);
omr_status omr_pool_submit_mask(omr_pool* p, const struct omr_mask_job* job, uint64_t* ticket);
/* omr_batcher_wait of the batcher holding the ticket. */
omr_status omr_pool_wait(omr_pool* p, uint64_t ticket, uint8_t* out, size_t cap, size_t* len);
/* Index into devices[] of the batcher a ticket went to (-1: not a ticket of this pool). */
int32_t    omr_pool_device_index(const omr_pool* p, uint64_t ticket);
omr_status omr_pool_set_semantics(omr_pool* p, uint32_t flags);
omr_status omr_pool_set_stack_cache(omr_pool* p, int64_t max_bytes_per_device);
/* stats_out[4*i .. 4*i+3] = omr_batcher_stats of device i; n_entries >= omr_pool_size. */
omr_status omr_pool_stats(omr_pool* p, uint64_t* stats_out, int32_t n_entries);

/* ---- render (quantize + codomain + composite + flip) ------------------ */
/*
 * Replaces renderer.renderAsPackedInt(planeDef, null)  (ImageRegionRequestHandler.java:559)
 * followed by flip(buf, sizeX, sizeY, flipH, flipV)      (ImageRegionRequestHandler.java:574-575, :616-642).
 * planes[c] points at the region of channel c (size_c pointers; NULL allowed for inactive
 * channels); row_stride is in pixels (0 = width).  big_endian: ROMIO planes are big-endian.
 * Host memory in and out; synchronous.
 */
omr_status omr_render_packed_int(omr_ctx* ctx, const omr_quantum_def* qdef,
                                 const omr_channel_binding* channels, int32_t size_c,
                                 const void* const* planes, int64_t row_stride,
                                 int32_t pixel_type, int32_t big_endian,
                                 int32_t width, int32_t height,
                                 int32_t flip_h, int32_t flip_v,
                                 uint32_t* argb_out);

/* Same, device pointers, asynchronous on the context stream. */
omr_status omr_render_packed_int_device(omr_ctx* ctx, const omr_quantum_def* qdef,
                                        const omr_channel_binding* channels, int32_t size_c,
                                        const void* const* d_planes, int64_t row_stride,
                                        int32_t pixel_type, int32_t big_endian,
                                        int32_t width, int32_t height,
                                        int32_t flip_h, int32_t flip_v,
                                        uint32_t* d_argb_out);

/*
 * Batch of n_tiles same-settings tile requests (one viewer's tiles; the request-level
 * parallelism of ImageRegionMicroserviceVerticle.java:149-165 coalesced into one launch).
 * d_plane_ptrs: DEVICE array of n_tiles*size_c device pointers ([tile][channel]); each plane
 * must start 16-byte aligned when width and row_stride are multiples of 16 bytes' worth of pixels
 * (the vector path: 16-B loads), which the library cannot check on the host.
 * d_argb_out: device [n_tiles][height][width].  d_status (optional, device int32[n_tiles]):
 * per-tile OMR_OK / OMR_QUANTIZATION.  Asynchronous on the context stream.
 */
omr_status omr_render_batch_device(omr_ctx* ctx, const omr_quantum_def* qdef,
                                   const omr_channel_binding* channels, int32_t size_c,
                                   const void* const* d_plane_ptrs, int32_t n_tiles,
                                   int64_t row_stride, int32_t pixel_type, int32_t big_endian,
                                   int32_t width, int32_t height,
                                   int32_t flip_h, int32_t flip_v,
                                   uint32_t* d_argb_out, int32_t* d_status);

/*
 * Same batch with the planes laid out regularly in device memory (e.g. a pyramid level kept
 * resident as [tile][channel][y][x]): plane(t, c) = d_base + t*tile_stride_bytes +
 * c*channel_stride_bytes.  No pointer table; otherwise identical to omr_render_batch_device.
 */
omr_status omr_render_batch_strided_device(omr_ctx* ctx, const omr_quantum_def* qdef,
                                           const omr_channel_binding* channels, int32_t size_c,
                                           const void* d_base, int64_t tile_stride_bytes,
                                           int64_t channel_stride_bytes, int32_t n_tiles,
                                           int64_t row_stride, int32_t pixel_type, int32_t big_endian,
                                           int32_t width, int32_t height,
                                           int32_t flip_h, int32_t flip_v,
                                           uint32_t* d_argb_out, int32_t* d_status);

/*
 * Standalone output flip of an already-rendered ARGB buffer on the device
 * (ImageRegionRequestHandler.flip, :616-642).  src and dest must not alias.
 * Identity (no flip) copies.
 */
omr_status omr_flip_argb_device(omr_ctx* ctx, const uint32_t* d_src, uint32_t* d_dest,
                                int32_t size_x, int32_t size_y, int32_t flip_h, int32_t flip_v);
/* ShapeMaskRequestHandler.flip(byte[]...) (:128-154), byte-per-pixel. */
omr_status omr_flip_mask_device(omr_ctx* ctx, const uint8_t* d_src, uint8_t* d_dest,
                                int32_t size_x, int32_t size_y, int32_t flip_h, int32_t flip_v);

/* ---- Z-projection ------------------------------------------------------ */
/*
 * ProjectionService.projectStack(pixels, buf, alg, t, c, stepping, start, end)
 * (ProjectionService.java:46-120): one channel's stack [size_z][size_y][size_x] -> one plane
 * of the same pixel type.  Max over z in [start,end] inclusive; mean/sum over [start,end)
 * (ProjectionService.java:184 vs :271).  Host memory; synchronous.
 */
omr_status omr_project_stack(omr_ctx* ctx, const void* stack, int32_t pixel_type,
                             int32_t big_endian_in, int32_t size_x, int32_t size_y, int32_t size_z,
                             int32_t algorithm, int32_t start, int32_t end, int32_t stepping,
                             void* plane_out, int32_t big_endian_out);
omr_status omr_project_stack_device(omr_ctx* ctx, const void* d_stack, int32_t pixel_type,
                                    int32_t big_endian_in, int32_t size_x, int32_t size_y,
                                    int32_t size_z, int32_t algorithm, int32_t start, int32_t end,
                                    int32_t stepping, void* d_plane_out, int32_t big_endian_out);
/*
 * n_stacks same-geometry stacks (e.g. every active channel of one p= request, the glue's
 * projectStack loop at ImageRegionRequestHandler.java:516-533) projected in one launch.
 * d_stacks / d_planes_out: HOST arrays of n_stacks device pointers; n_stacks <= 32.
 * Asynchronous on the context stream.
 */
omr_status omr_project_stacks_device(omr_ctx* ctx, const void* const* d_stacks, int32_t n_stacks,
                                     int32_t pixel_type, int32_t big_endian_in, int32_t size_x,
                                     int32_t size_y, int32_t size_z, int32_t algorithm, int32_t start,
                                     int32_t end, int32_t stepping, void* const* d_planes_out,
                                     int32_t big_endian_out);
/*
 * Projection glue + render (ImageRegionRequestHandler.java:506-559): project every active
 * channel's stack (d_stacks[c], NULL for inactive) and render the full projected plane.
 * Projected planes stay in HBM (native byte order); output device [size_y][size_x].
 */
omr_status omr_render_projected_device(omr_ctx* ctx, const omr_quantum_def* qdef,
                                       const omr_channel_binding* channels, int32_t size_c,
                                       const void* const* d_stacks, int32_t pixel_type,
                                       int32_t big_endian, int32_t size_x, int32_t size_y,
                                       int32_t size_z, int32_t algorithm, int32_t start,
                                       int32_t end, int32_t stepping, int32_t flip_h,
                                       int32_t flip_v, uint32_t* d_argb_out);

/* ---- encode --------------------------------------------------------------- */
/* Upper bound of the encoded size (callers size `out` with it). */
size_t omr_jpeg_max_bytes(int32_t width, int32_t height);
size_t omr_png_max_bytes(int32_t width, int32_t height, int32_t channels);
/*
 * JPEG baseline (JFIF, YCbCr 4:2:0, IJG islow FDCT, Java ImageIO quality scaling,
 * standard Huffman tables) of the 24-bit RGB view of ARGB pixels
 * (ImageUtil.createBufferedImage + compressionService.compressToStream,
 *  ImageRegionRequestHandler.java:576-582).  Quality is per call.
 * Host ARGB in, host bytes out.  *out_len always receives the file length; a NULL `out` or
 * cap < length returns OMR_BUFFER_TOO_SMALL (query, then call again).  Tiles up to 4096 px
 * run the batched pipeline below with one tile; larger images the single-tile kernels.
 */
omr_status omr_encode_jpeg(omr_ctx* ctx, const uint32_t* argb, int32_t width, int32_t height,
                           float quality, uint8_t* out, size_t cap, size_t* out_len);
/* Device ARGB in (e.g. straight from omr_render_*_device), host bytes out. */
omr_status omr_encode_jpeg_device(omr_ctx* ctx, const uint32_t* d_argb, int32_t width,
                                  int32_t height, float quality, uint8_t* out, size_t cap,
                                  size_t* out_len);
/*
 * Batched JPEG (same encoder, byte-identical per tile) of n_tiles device ARGB tiles
 * (tile i at d_argb + i*tile_stride_px; 0 = width*height), e.g. the output of
 * omr_render_batch_*_device.  Complete JFIF files are packed back to back in d_out
 * (capacity out_cap bytes): file i at d_out + d_offsets[i], d_lengths[i] bytes (0 and
 * d_status[i] = OMR_BUFFER_TOO_SMALL when it did not fit; d_status optional).
 * Asynchronous on the context stream; width, height <= 4096.  This is the batch form of the
 * per-request compressToStream calls (ImageRegionRequestHandler.java:580-582).
 */
omr_status omr_encode_jpeg_batch_device(omr_ctx* ctx, const uint32_t* d_argb, int64_t tile_stride_px,
                                        int32_t n_tiles, int32_t width, int32_t height, float quality,
                                        uint8_t* d_out, size_t out_cap, uint64_t* d_offsets,
                                        uint32_t* d_lengths, int32_t* d_status);
/*
 * render_image_region's default response for a batch of tiles in one call: render (quantize,
 * codomain, composite, flip: renderAsPackedInt + flip, :559, :574-575) and JPEG-encode
 * (createBufferedImage + compressToStream, :576-582) n_tiles same-settings tiles whose planes
 * are already in HBM.  Output exactly as omr_encode_jpeg_batch_device (byte-identical files);
 * d_status[i] (optional) also reports OMR_QUANTIZATION for a tile with a pixel outside its LUT
 * domain.  8/16-bit integer pixels with 1..4 active channels on tiles whose sides are multiples
 * of 16 render inside the encoder's first kernel (the ARGB tile never reaches HBM); other
 * requests render with K2 first.  Plane rows must start 4-byte aligned (16-bit) / 2-byte
 * aligned (8-bit) for the fused path.  Asynchronous on the context stream.
 */
omr_status omr_render_jpeg_batch_strided_device(omr_ctx* ctx, const omr_quantum_def* qdef,
                                                const omr_channel_binding* channels, int32_t size_c,
                                                const void* d_base, int64_t tile_stride_bytes,
                                                int64_t channel_stride_bytes, int32_t n_tiles, int64_t row_stride,
                                                int32_t pixel_type, int32_t big_endian, int32_t width, int32_t height,
                                                int32_t flip_h, int32_t flip_v, float quality, uint8_t* d_out,
                                                size_t out_cap, uint64_t* d_offsets, uint32_t* d_lengths,
                                                int32_t* d_status);
/*
 * One render_image_region request in its default format (format=jpeg, ImageRegionCtx.java:146):
 * renderAsPackedInt + flip + createBufferedImage + compressToStream
 * (ImageRegionRequestHandler.java:559-582) of one tile whose planes are already in HBM, the JPEG
 * file landing in `out` (host memory).  d_planes is a HOST array of size_c device pointers, one per
 * channel (an inactive channel's may be null).  Same files as omr_render_packed_int_device +
 * omr_encode_jpeg_device, in one call with one stream sync (K2's small-launch render + the one-tile
 * JPEG pipeline: measured faster for a single tile than the fused kernel).  Synchronous; a pixel outside its LUT
 * domain returns OMR_QUANTIZATION (-> 500); *out_len is set whenever the length is known
 * (OMR_BUFFER_TOO_SMALL when cap is short).  Tiles up to 4096 x 4096.
 */
omr_status omr_render_jpeg(omr_ctx* ctx, const omr_quantum_def* qdef, const omr_channel_binding* channels,
                           int32_t size_c, const void* const* d_planes, int64_t row_stride, int32_t pixel_type,
                           int32_t big_endian, int32_t width, int32_t height, int32_t flip_h, int32_t flip_v,
                           float quality, uint8_t* out, size_t cap, size_t* out_len);
/* Same with a device plane-pointer table [tile][channel] (omr_render_batch_device's layout). */
omr_status omr_render_jpeg_batch_device(omr_ctx* ctx, const omr_quantum_def* qdef,
                                        const omr_channel_binding* channels, int32_t size_c,
                                        const void* const* d_plane_ptrs, int32_t n_tiles, int64_t row_stride,
                                        int32_t pixel_type, int32_t big_endian, int32_t width, int32_t height,
                                        int32_t flip_h, int32_t flip_v, float quality, uint8_t* d_out,
                                        size_t out_cap, uint64_t* d_offsets, uint32_t* d_lengths,
                                        int32_t* d_status);
/* Same, host output: files packed in out (cap bytes), offsets/lengths host arrays; synchronous. */
omr_status omr_encode_jpeg_batch(omr_ctx* ctx, const uint32_t* d_argb, int64_t tile_stride_px,
                                 int32_t n_tiles, int32_t width, int32_t height, float quality,
                                 uint8_t* out, size_t cap, uint64_t* offsets, uint32_t* lengths);
/* Java ImageIO quality -> quantisation tables (natural order), JPEGQTable.getScaledInstance. */
omr_status omr_jpeg_quant_tables(float quality, uint8_t luma[64], uint8_t chroma[64]);
/* Same under OMR_SEM_* flags (OMR_SEM_JPEG_CHROMA_DIV2 selects the chroma base table). */
omr_status omr_jpeg_quant_tables_sem(float quality, uint32_t semantics, uint8_t luma[64], uint8_t chroma[64]);

/* PNG RGB8 of ARGB pixels (ImageIO.write(image, "png"), ImageRegionRequestHandler.java:598). */
omr_status omr_encode_png(omr_ctx* ctx, const uint32_t* argb, int32_t width, int32_t height,
                          uint8_t* out, size_t cap, size_t* out_len);
omr_status omr_encode_png_device(omr_ctx* ctx, const uint32_t* d_argb, int32_t width,
                                 int32_t height, uint8_t* out, size_t cap, size_t* out_len);
/*
 * Batched PNG (same encoder family, decoded pixels identical per tile) of n_tiles device ARGB
 * tiles (tile i at d_argb + i*tile_stride_px; 0 = width*height): the batch form of the
 * per-request ImageIO.write(image, "png", ...) calls (ImageRegionRequestHandler.java:597-599).
 * Complete PNG files in d_out (capacity out_cap bytes): file i at d_out + d_offsets[i] (16-byte
 * aligned slots, in tile order), d_lengths[i] bytes; 0 and d_status[i] = OMR_BUFFER_TOO_SMALL when
 * it did not fit (d_offsets / d_lengths / d_status optional).  Every stage is one launch over all
 * tiles; no host sync (asynchronous on the context stream).  width, height <= 4096.
 */
omr_status omr_encode_png_batch_device(omr_ctx* ctx, const uint32_t* d_argb, int64_t tile_stride_px,
                                       int32_t n_tiles, int32_t width, int32_t height, uint8_t* d_out,
                                       size_t out_cap, uint64_t* d_offsets, uint32_t* d_lengths,
                                       int32_t* d_status);
/* Output capacity that always holds n batched PNG files of width x height (channels 3: RGB
 * tiles, 1: masks), 16-byte slots included. */
size_t omr_png_batch_max_bytes(int32_t width, int32_t height, int32_t channels, int32_t n);

/*
 * TIFF of the 24-bit RGB view (TIFFImageWriter branch, ImageRegionRequestHandler.java:584-596):
 * baseline uncompressed big-endian RGB, 8-bit samples, >= 8 KiB strips.  Host writer.
 */
size_t omr_tiff_max_bytes(int32_t width, int32_t height);
omr_status omr_encode_tiff(omr_ctx* ctx, const uint32_t* argb, int32_t width, int32_t height,
                           uint8_t* out, size_t cap, size_t* out_len);
omr_status omr_encode_tiff_device(omr_ctx* ctx, const uint32_t* d_argb, int32_t width,
                                  int32_t height, uint8_t* out, size_t cap, size_t* out_len);

/* ---- shape mask ------------------------------------------------------------- */
/*
 * ShapeMaskRequestHandler.renderShapeMask(Color, byte[], w, h) (:165-207): MSB-first bit mask
 * (no row padding) -> flip -> 2-entry palette PNG (index 0 transparent, index 1 = rgba).
 * width % 8 == 0 with a flip follows the reference's packed-buffer flip unless the context has
 * OMR_SEM_MASK_PIXEL_FLIP (see there).  Every exception the reference raises inside
 * renderShapeMask (a null or short mask, a zero size, the packed-buffer flip's
 * ArrayIndexOutOfBoundsException, width*height past Java int) completes its future exceptionally,
 * which ShapeMaskVerticle.java:119-128 answers with 404: OMR_NOT_FOUND.  A null rgba or out is
 * OMR_INVALID_ARGUMENT.  Host in/out.
 */
omr_status omr_render_shape_mask_png(omr_ctx* ctx, const uint8_t* bits, size_t n_bytes,
                                     int32_t width, int32_t height, const uint8_t rgba[4],
                                     int32_t flip_h, int32_t flip_v,
                                     uint8_t* out, size_t cap, size_t* out_len);
/*
 * N render_shape_mask requests in one call (the per-worker renderShapeMask calls of
 * ShapeMaskVerticle.java:121-149 coalesced): the masks may differ in size, colour and flips, and
 * are encoded by the batched PNG pipeline (one launch per stage for all of them).  Host in/out,
 * synchronous.  File i lands at out + offsets[i] (16-byte aligned slots), lengths[i] bytes;
 * status[i] is OMR_OK, OMR_NOT_FOUND for every case the single call answers with 404 (the same
 * checks and the same packed-buffer flip), or OMR_BUFFER_TOO_SMALL when cap ran out
 * (omr_png_batch_max_bytes(w, h, 1, 1) per mask always suffices).  Returns OMR_OK when the call
 * ran; per-mask outcomes are in status.
 */
typedef struct omr_mask_job {
    const uint8_t* bits;        /* MSB-first mask bits (byte[] of the Mask) */
    size_t n_bytes;
    int32_t width, height;
    uint8_t rgba[4];            /* fill colour (omr_shape_mask_fill_color) */
    int32_t flip_h, flip_v;
} omr_mask_job;
omr_status omr_render_shape_mask_png_batch(omr_ctx* ctx, const omr_mask_job* jobs, int32_t n,
                                           uint8_t* out, size_t cap, uint64_t* offsets,
                                           uint32_t* lengths, int32_t* status);

/* ---- host-side request helpers (no device work) ---------------------------------- */
/* ImageRegionRequestHandler.splitHTMLColor (:865-890), bug-compatible; OMR_INVALID_ARGUMENT = null. */
omr_status omr_split_html_color(const char* color, int32_t rgba_out[4]);
/* ShapeMaskRequestHandler.renderShapeMask(Mask) fill colour (:97-106).  OMR_INVALID_ARGUMENT where the
 * reference throws (NPE on an unparsable colour, Color's IAE); inside renderShapeMask that fails the
 * future, which the verticle answers with 404 (ShapeMaskVerticle.java:119-128). */
omr_status omr_shape_mask_fill_color(int32_t has_mask_fill, int32_t mask_fill_color,
                                     const char* request_color, uint8_t rgba_out[4]);
/*
 * getRegionDef + truncateRegionDef + flipRegionDef (ImageRegionRequestHandler.java:789-832,
 * :751-758, :770-780).  mode: 0 = tile (tile.x/y in tile units, width/height 0 = use
 * tile_size_*), 1 = region (pixels), 2 = neither (full plane).  level_sizes holds
 * n_levels (sizeX,sizeY) pairs; resolution < 0 means "not given" (0).
 */
omr_status omr_get_region_def(int32_t mode, const omr_region* request, int32_t resolution,
                              const int32_t* level_sizes, int32_t n_levels,
                              int32_t tile_size_x, int32_t tile_size_y, int32_t max_tile_length,
                              int32_t flip_h, int32_t flip_v, omr_region* out);
/* setResolutionLevel (:840-853): Renderer level = nLevels - resolution - 1. */
int32_t omr_resolution_level(int32_t n_levels, int32_t resolution);
/* checkPlaneDef (:651-681): truncate region to the level size. */
omr_status omr_check_plane_def(omr_region* region, int32_t size_x, int32_t size_y);
/* LutReader: parse an ImageJ .lut file image (768 B binary, 800 B with header, or text). */
omr_status omr_parse_lut(const uint8_t* data, size_t n, uint8_t lut_out[768]);

/* ---- request decode + renderer settings (omr_request.cpp; host only) -------------------- */
#define OMR_MAX_REQUEST_CHANNELS 64
/* per-channel entry of omr_image_region_ctx.map_reverse (the `maps` JSON list) */
enum { OMR_MAP_NONE = 0, OMR_MAP_REVERSE = 1, OMR_MAP_NULL = 2, OMR_MAP_BAD = 3 };

/*
 * ImageRegionCtx (ImageRegionCtx.java:44-109) after assignParams (:127-153).  has_* / -1 encode
 * Java nulls.  windows are the Float values (:313-314); colors[i] is the raw `$...` string
 * (HTML colour or a *.lut name).
 */
typedef struct omr_image_region_ctx {
    int64_t image_id;
    int32_t z, t;
    int32_t has_tile;          /* tile: x/y in tile units, width/height 0 for the short form */
    omr_region tile;
    int32_t has_resolution, resolution;
    int32_t has_region;
    omr_region region;
    int32_t n_channels;        /* -1: no 'c' parameter (channels == null) */
    int32_t channels[OMR_MAX_REQUEST_CHANNELS];      /* signed 1-based, negative = inactive */
    int32_t window_set[OMR_MAX_REQUEST_CHANNELS];    /* 0: Float[2]{null,null} */
    float windows[OMR_MAX_REQUEST_CHANNELS][2];
    int32_t color_set[OMR_MAX_REQUEST_CHANNELS];     /* 0: colour null */
    char colors[OMR_MAX_REQUEST_CHANNELS][64];
    int32_t model;             /* -1 null, OMR_MODEL_GREYSCALE ("g"), OMR_MODEL_RGB ("c") */
    int32_t has_quality;
    float quality;
    int32_t inverted_axis;     /* -1 null, 0/1 (parsed, unused, :93-97) */
    int32_t projection;        /* -1 null, OMR_PROJECTION_* */
    int32_t has_projection_start, projection_start;
    int32_t has_projection_end, projection_end;
    int32_t n_maps;            /* -1: no `maps` parameter */
    int32_t map_reverse[OMR_MAX_REQUEST_CHANNELS];   /* OMR_MAP_* per list element */
    int32_t flip_h, flip_v;
    char format[16];           /* default "jpeg" */
    char cache_key[17];        /* Guava sipHash24 hex of the sorted parameters (:165-177) */
} omr_image_region_ctx;

/* ShapeMaskCtx (ShapeMaskCtx.java:38-81). */
typedef struct omr_shape_mask_ctx {
    int64_t shape_id;
    int32_t has_color;
    char color[64];
    int32_t flip_h, flip_v;
    char cache_key[128];       /* "ome.model.roi.Mask:<id>:<color>" (:77-81) */
} omr_shape_mask_ctx;

/*
 * new ImageRegionCtx(params, key) (ImageRegionCtx.java:122-153).  names/values: the request's
 * MultiMap entries in insertion order (case-insensitive names, first value wins).
 * OMR_INVALID_ARGUMENT = IllegalArgumentException (400); OMR_INTERNAL = an unchecked exception
 * the reference does not catch (500).  err (optional) receives the message.
 */
omr_status omr_image_region_ctx_parse(const char* const* names, const char* const* values, int32_t n,
                                      omr_image_region_ctx* out, char* err, size_t err_cap);
/* new ShapeMaskCtx(params, key) (ShapeMaskCtx.java:61-72); bad shapeId -> OMR_INTERNAL (500). */
omr_status omr_shape_mask_ctx_parse(const char* const* names, const char* const* values, int32_t n,
                                    omr_shape_mask_ctx* out, char* err, size_t err_cap);

/* LutProviderImpl (LutProviderImpl.java:29-75): *.lut files under root, keyed by basename. */
typedef struct omr_lut_provider omr_lut_provider;
omr_status     omr_lut_provider_create(const char* root, omr_lut_provider** out);
void           omr_lut_provider_destroy(omr_lut_provider* p);
int32_t        omr_lut_provider_count(const omr_lut_provider* p);
omr_status     omr_lut_provider_add(omr_lut_provider* p, const char* name, const uint8_t lut_rgb768[768]);
/* 768-byte R[256] G[256] B[256] table owned by the provider, or NULL (getLutReaders -> null). */
const uint8_t* omr_lut_provider_get(const omr_lut_provider* p, const char* name);

/* createRenderingDef (ImageRegionRequestHandler.java:258-300) for size_c channels. */
omr_status omr_create_rendering_def(int32_t pixel_type, int32_t size_c, omr_quantum_def* qdef,
                                    omr_channel_binding* channels);
/*
 * updateSettings (ImageRegionRequestHandler.java:689-741) applied to a rendering def: active
 * flags, windows, colours or LUTs (luts may be NULL), reverse-intensity maps, model.
 * Reference failures (null channels / window / colour / model, short lists, bad maps entries)
 * return OMR_INTERNAL (500).
 */
omr_status omr_update_settings(const omr_image_region_ctx* ctx, int32_t size_c, omr_quantum_def* qdef,
                               omr_channel_binding* channels, const omr_lut_provider* luts,
                               char* err, size_t err_cap);

#ifdef __cplusplus
}
#endif
#endif /* OMR_OMR_H */
