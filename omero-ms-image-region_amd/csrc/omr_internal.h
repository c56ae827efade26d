// omr_internal.h — shared definitions of the MI355X image-region library (libomr.so).
// Host runtime pieces (context, workspace, staging) and the device-side parameter
// blocks the kernels read.  Reference citations: see include/omr/omr.h.
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <algorithm>
#include <cmath>
#include <cstddef>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "omr/omr.h"

struct omr_ctx;

namespace omr {

constexpr int kMaxActive = 32;        // active channels per render call
constexpr int kBlock = 256;           // threads per workgroup (4 waves)
constexpr uint32_t kErrBit = 0x80000000u;  // contrib-table entry flag: value outside LUT domain

// Per-active-channel quantization mode.
enum ChanMode : int32_t {
    kModeTable8 = 0,   // 8-bit types: quantization+codomain+colour folded into contrib[raw byte]
    kModeLinear16 = 1, // 16-bit linear: exact double evaluation of the LUT entry, contrib[v]
    kModeLut16 = 2,    // 16-bit other families / noise reduction: byte LUT gather, contrib[v]
    kModeEval = 3,     // 32-bit int / float / double: per-pixel q(x) in double, contrib[v]
    kModeThresh = 4    // float / int32 / uint32 with q monotone in x: K1 finds the 255 code
                       // thresholds of q in key space, K2 binary-searches them in LDS
};

// Family map the kernels evaluate (ChanParam::family): the omr.h family with the OMR_SEM_* variant
// of its map folded in by the host (prepare_plan).
enum FamilyCode : int32_t {
    kFamLinear = OMR_FAMILY_LINEAR,
    kFamPoly = OMR_FAMILY_POLYNOMIAL,
    kFamLog = OMR_FAMILY_LOGARITHMIC,       // x > 0 ? log(x) : 0
    kFamExp = OMR_FAMILY_EXPONENTIAL,       // exp(pow(x, k))
    kFamLogRaw = 4,                         // log(x) for every x (OMR_SEM_LOG_UNGUARDED)
    kFamExpNorm = 5                         // exp(pow((x - ws)/(we - ws), k)) (OMR_SEM_EXP_NORMALIZED)
};
// Host and device evaluate the same expressions (-ffp-contract=off): the CPU restatement's S2.
__host__ __device__ inline double family_map_code(int family, double x, double k, double ws, double we) {
    switch (family) {
    case kFamPoly: return pow(x, k);
    case kFamLog: return x > 0 ? log(x) : 0.0;
    case kFamExp: return exp(pow(x, k));
    case kFamLogRaw: return log(x);
    case kFamExpNorm: return exp(pow((x - ws) / (we - ws), k));
    default: return x;
    }
}

// One active channel as the kernels see it (device memory, read uniformly).
struct ChanParam {
    int32_t index;      // channel index into the [tile][size_c] plane table
    int32_t mode;
    int32_t lo, hi;     // integer window thresholds: x < lo -> cdStart, x >= hi -> cdEnd
    int32_t gmin, gmax; // LUT domain (QuantizationException outside)
    int32_t family, nr; // FamilyCode; noise reduction in effect
    int32_t reverse, has_lut;
    int32_t second;     // apply the a1*v + cdStart rounding stage (not identity)
    int32_t pad0;
    double ws, we, k;   // window, coefficient
    double ys, a0, a1;  // f(ws), bitRes/(f(we)-f(ws)), (cdEnd-cdStart)/bitRes
    double dec;         // noise-reduction decile width
    float ratio[3];     // (c/255f)*(alpha/255f)
    float alpha;        // alpha/255f (OMR_SEM_ALPHA_SEPARATE)
    float cratio[3];    // c/255f     (OMR_SEM_ALPHA_SEPARATE)
    float pad1;
    uint64_t lut_addr;  // device address of this channel's quantization byte LUT (kModeLut16;
                        // the context's device LUT cache, Ctx::dev_luts)
    uint8_t qtab[256];  // kModeTable8: q of raw byte t, built on the host (host libm, exact)
    uint8_t lut_rgb[768];  // LutReader colours (valid when has_lut)
};

struct RenderPlan {
    int32_t n_active;
    int32_t cd_start, cd_end;
    int32_t greyscale;
    uint32_t sem;       // OMR_SEM_* flags
    int32_t pad[3];
    ChanParam ch[kMaxActive];
};

struct Ctx {
    int device = 0;
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;
    std::string last_error;
    // device workspace (grow-only bump arena, reset per call)
    void* ws = nullptr;
    size_t ws_cap = 0;
    // device buffer for intermediate results that must outlive the workspace's reuse within one
    // call (the unfused render -> JPEG path's ARGB batch); grow-only
    void* aux = nullptr;
    size_t aux_cap = 0;
    // device-side sticky status word (quantization errors of async calls)
    int32_t* d_flag = nullptr;
    int32_t* h_flag = nullptr;   // fine-grained pinned word: d_flag copied here by a kernel at sync
    // fine-grained pinned landing buffer for single-file results (one-tile JPEG): a kernel writes
    // the file and its length here, so the caller needs one stream sync
    uint8_t* h_out = nullptr;
    size_t h_out_cap = 0;
    // pinned staging for parameter blocks (2-slot ring)
    static constexpr int kPinSlots = 8;   // parameter blocks in flight: the host runs this many ahead
    void* pin[kPinSlots] = {};
    size_t pin_cap = 0;
    hipEvent_t pin_ev[kPinSlots] = {};
    int pin_slot = 0;
    int cu_count = 256;
    bool k2_nt_store = false;   // env OMR_K2_NT_STORE=1: non-temporal ARGB stores (measurement switch)
    uint32_t sem = 0;            // OMR_SEM_* (omr_ctx_set_semantics)
    // projection glue through the fused K3R kernel (env OMR_K3R=1; measured slower than K3 + K2
    // on C3, DESIGN.md §K3R, so off by default)
    bool k3r = false;
    // PNG D3 (Huffman tables) on the device (env OMR_PNG_DEVICE_D3=1): no mid-encode host round
    // trip, but the single-workgroup build measured slower than the host's
    bool png_device_d3 = false;
    bool png_single_batched = true;   // single PNG / mask requests through the batched pipeline (n = 1)
    // x^(8*256*j) mod P (CRC-32) for the batched PNG's segment combine: [0, 4096) j = lo, then
    // [4096, 6144) j = hi * 4096; built on the device on first use (omr_png.hip)
    uint32_t* d_crc_pow = nullptr;
    bool f1_f32 = true;              // F1's Fast16 quantize in f32 when proven exact (OMR_F1_F32=0: f64)
    // JPEG B4a / B6 grids: chunk groups for streams of this many bytes per pixel x 100 (longer
    // streams loop; env OMR_JPEG_EST_CENTIBPP)
    int jpeg_est_centibpp = 100;
    // chunks per lane of K2's float / 32-bit grid-stride modes (env OMR_K2_EVAL_CPT=2|4; 4
    // measured 6% slower on C5, DESIGN.md §K2, so 2 by default)
    int k2_eval_cpt = -2;            // float / 32-bit K2: -1 / -2 pipelined chunks per lane, 2 / 4 plain
    // Device cache of the kModeLut16 byte LUTs (non-linear 16-bit families, noise reduction): a
    // setting's LUT is built on the host once (host_quant_lut) and uploaded once, and every later
    // request with that setting reads it in place (omr_render.hip device_quant_lut).  LRU, at most
    // kDevLutEntries LUTs and kDevLutBytes in all.
    struct DevLut { std::vector<uint8_t> key; uint8_t* d = nullptr; size_t bytes = 0; uint64_t used = 0; };
    static constexpr int kDevLutEntries = 64;
    static constexpr size_t kDevLutBytes = (size_t)256 << 20;
    std::vector<DevLut> dev_luts;
    size_t dev_lut_bytes = 0;
    uint64_t dev_lut_clock = 0;
    // kernel timing (omr_ctx_enable_kernel_timing)
    bool timing = false;
    struct Timed { hipEvent_t start, stop; int kind; };
    std::vector<Timed> timed;
    std::vector<hipEvent_t> event_pool;
    // pixel-buffer pipeline (omr_pixbuf.cpp): reader threads + double-buffered staging
    void* pixbuf_state = nullptr;
    bool pixbuf_direct = true;   // DMA tile rows from a registered file mapping when possible
    void (*pixbuf_state_free)(void*) = nullptr;
};

// Bracket one hot-kernel launch with events when timing is enabled.
struct KernelTimer {
    Ctx* c;
    int kind;
    hipEvent_t start = nullptr, stop = nullptr;
    bool ext = false, used = false;             // ext: the next omr_launch stamps the events itself
    KernelTimer* prev = nullptr;
    // ext = true for a scope holding one kernel launched through omr_launch: the events are then
    // the dispatch's own start / end timestamps (hipExtLaunchKernel), the duration a rocprofv3
    // kernel trace reports, instead of two queue packets around it (which read ~1 us high on a
    // 16 us kernel)
    KernelTimer(Ctx* ctx, int k, bool ext_launch = false);
    ~KernelTimer();
};
extern thread_local KernelTimer* tl_ext_timer;

template <typename F, typename... Args>
inline void omr_launch(F kernel, const dim3& g, const dim3& b, uint32_t lds, hipStream_t s, Args... args) {
    KernelTimer* t = tl_ext_timer;
    if (t && !t->used && t->stop) {
        t->used = true;
        hipExtLaunchKernelGGL(kernel, g, b, lds, s, t->start, t->stop, 0u, args...);
    } else {
        hipLaunchKernelGGL(kernel, g, b, lds, s, args...);
    }
}

omr_status fail(Ctx* c, omr_status s, const std::string& msg);
omr_status hip_fail(Ctx* c, hipError_t e, const char* what);
// Ensure the workspace holds at least `bytes`; invalidates previous contents.
omr_status ensure_workspace(Ctx* c, size_t bytes);
// Ensure ctx->aux holds at least `bytes` (contents not preserved across growth).
omr_status ensure_aux(Ctx* c, size_t bytes);
// Fine-grained pinned landing buffer (ctx->h_out) of at least `bytes` (grow-only).
omr_status ensure_host_out(Ctx* c, size_t bytes);
// Copy `bytes` from host `src` to device `dst` through the pinned ring (async on ctx stream).
// Move the sticky device status word to fine-grained host memory and clear it, on `s`
// (omr_render.hip): omr_ctx_synchronize then needs one stream sync and no copy round trip.
hipError_t launch_flag_out(hipStream_t s, int32_t* d_flag, int32_t* h_flag);
// Copy `bytes` from device-accessible pinned host memory to device memory with a kernel on `s`
// (omr_render.hip).
hipError_t launch_h2d_small(hipStream_t s, void* dst1, const void* pinned_src1, size_t n1,
                            void* dst2 = nullptr, const void* pinned_src2 = nullptr, size_t n2 = 0);
omr_status stage_h2d(Ctx* c, void* dst, const void* src, size_t bytes);
// Two parameter blocks through one ring slot and one copy launch.
omr_status stage_h2d2(Ctx* c, void* dst1, const void* src1, size_t n1, void* dst2, const void* src2, size_t n2);
int bytes_per_pixel(int32_t pixel_type);
// K3 launch over up to 32 stacks (omr_project.hip).
struct FusedRender;
// The fused projection glue (omr_project.hip, K3R): stacks[a] per rendered channel in plan order;
// *done = false when it does not apply (the caller projects with K3 and renders with K2).
omr_status enqueue_project_render(Ctx* ctx, const void* const* stacks, const FusedRender& R, int32_t pixel_type,
                                  int32_t be_in, int32_t size_x, int32_t size_y, int32_t algorithm, int32_t start,
                                  int32_t end, int32_t stepping, int32_t flip_h, int32_t flip_v, uint32_t* d_out,
                                  bool* done);
omr_status validate_projection_args(Ctx* c, int32_t pixel_type, int32_t size_x, int32_t size_y,
                                    int32_t size_z, int32_t algorithm, int32_t start, int32_t end,
                                    int32_t stepping);
omr_status enqueue_projection(Ctx* c, const void* const* d_stacks, void* const* d_outs, int n,
                              int32_t pixel_type, int32_t be_in, int32_t size_x, int32_t size_y,
                              int32_t algorithm, int32_t start, int32_t end, int32_t stepping,
                              int32_t be_out);

// omr_render_pixel_buffer_tiles with optional per-tile statuses (device int32[n], OMR_OK /
// OMR_QUANTIZATION): then a QuantizationException fails only the tiles it hit (omr_pixbuf.cpp).
omr_status render_pixel_buffer_tiles(omr_ctx* ctx, const omr_pixel_buffer* pb, const omr_quantum_def* qdef,
                                     const omr_channel_binding* channels, int32_t size_c,
                                     const omr_tile_request* reqs, int32_t n, int32_t width, int32_t height,
                                     int32_t flip_h, int32_t flip_v, uint32_t* argb_out, int32_t out_on_device,
                                     int32_t* d_status);

// dims = {sizeX, sizeY, sizeZ, sizeC, sizeT, pixelType} of an open pixel buffer (omr_pixbuf.cpp).
void pixel_buffer_dims(const omr_pixel_buffer* pb, int32_t dims[6]);
// Process-unique id of an open pixel buffer (cache keys outlive a buffer's address).
uint64_t pixel_buffer_serial(const omr_pixel_buffer* pb);
// The (c, t) Z-stack of a pixel buffer into device memory on ctx's stream (omr_pixbuf.cpp).
omr_status pixel_buffer_upload_stack(omr_ctx* ctx, const omr_pixel_buffer* pb, int32_t c, int32_t t, void* d_dst);

#define OMR_HIP(ctx, expr)                                          \
    do {                                                            \
        hipError_t _e = (expr);                                     \
        if (_e != hipSuccess) return ::omr::hip_fail((ctx), _e, #expr); \
    } while (0)

inline size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

}  // namespace omr

struct omr_ctx : omr::Ctx {};
