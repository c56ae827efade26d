// omr_k2.h — K2's per-channel quantization as device helpers, shared by the render kernel
// (omr_render.hip) and the fused render -> JPEG kernel (omr_jpeg.hip), plus the host interface
// the fused path uses to prepare a render without launching K2.
#pragma once

#include "omr_device.h"

namespace omr {

// Per-active-channel parameters K2 reads from the kernarg segment (scalar loads, no
// per-pixel memory traffic for settings).
struct K2Chan {
    int32_t index;      // plane-table column (channel index)
    int32_t mode;       // kModeTable8 / kModeLinear16 / kModeLut16 / kModeEval
    int32_t lo, hi;     // window thresholds for integer x: x < lo -> cdStart, x >= hi -> cdEnd
    int32_t gmin, gmax; // LUT domain
    int32_t check;      // pixel values may fall outside [gmin, gmax] (QuantizationException)
    int32_t second;     // the a1*v + cdStart rounding stage is not the identity
    int32_t wsi;        // integral window start (FusedRender::f32: x - wsi in int32)
    double ws, a0, a1;
    uint64_t lut_addr;  // device address of the byte LUT (kModeLut16; the context's LUT cache)
};


__device__ __forceinline__ uint32_t clamp_fields(uint32_t a) {
    const uint32_t r = min(a >> 20, 255u), g = min((a >> 10) & 1023u, 255u), b = min(a & 1023u, 255u);
    return (r << 20) | (g << 10) | b;
}

// Exact LUT entry of a 16-bit pixel for the linear family, branch-free:
// v = round(a0*(x - ws)) (Java Math.round), window ends by integer compare.
__device__ __forceinline__ uint32_t linear16(int x, const K2Chan& p, int cds, int cds8, int cde8) {
    const double d = p.a0 * ((double)x - p.ws);
    int v = __double2int_rz(floor(d + 0.5));          // exact in the window (d in [0, bitRes])
    v = (d == 0x1.fffffffffffffp-2) ? 0 : v;
    if (p.second) v = (int)java_round_d(p.a1 * (double)v + (double)cds);   // uniform branch
    v = x >= p.hi ? cde8 : v;
    v = x < p.lo ? cds8 : v;                          // checked first upstream: wins for ws > we
    return (uint32_t)v & 0xFFu;
}

// Default QuantumDef (cd 0..255, bitRes 255), window start < end, and no window pixel at
// Java's 0.49999999999999994 special case (checked on the host): round(a0*(x - ws)) clamped
// to [0,255] equals the LUT entry for every x (below the window d < 0 -> 0, above it
// d >= 255 -> 255), so the window compares fold into one med3.  Truncation stands in for the
// floor: they differ only for d + 0.5 < 0, where both clamp to 0 (v_cvt_i32_f64 saturates, so
// d + 0.5 >= 2^31 still clamps to 255).
__device__ __forceinline__ uint32_t fast16(int x, const K2Chan& p) {
    const double d = p.a0 * ((double)x - p.ws);
    const int v = __double2int_rz(d + 0.5);
    return (uint32_t)min(max(v, 0), 255);
}

// fast16 for an integral window start: (double)(x - ws) is the same double as (double)x - ws
// (both exact), with the subtraction in int32 instead of f64 (one f64 operation fewer).
__device__ __forceinline__ uint32_t fast16i(int x, const K2Chan& p) {
    const double d = p.a0 * (double)(x - (int)p.ws);
    const int v = __double2int_rz(d + 0.5);
    return (uint32_t)min(max(v, 0), 255);
}

// fast16i in single precision: round(a0*(x - ws)) clamped is a non-decreasing step function of
// x with 255 steps, and so is the f32 form below; the host picks fa so that the two step at the
// same 255 pixel values (fast16_f32_params), i.e. agree on every x of the type, or the launch
// keeps the f64 form.  fb is the magic 1.5 * 2^23: in [2^23, 2^24) an f32 has ulp 1, so the one
// rounding of the fma is round-to-nearest-even of the exact (x - ws) * fa, and the float's bits
// are 0x4B400000 + that integer; an integer med3 on the bits clamps to [0, 255] (beyond
// +-2^22 the exponent moves and the clamp still saturates the right way).  Full-rate f32 and no
// float -> int conversion instead of four f64 operations.
constexpr int32_t kMagicBits = 0x4B400000;            // bits of 12582912.0f = 1.5 * 2^23
__device__ __forceinline__ uint32_t fast16f(int x, int wsi, float fa, float fb) {
    const float y = __builtin_fmaf((float)(x - wsi), fa, fb);
    const int32_t b = __float_as_int(y);
    return (uint32_t)(min(max(b, kMagicBits), kMagicBits + 255) - kMagicBits);
}


__device__ __forceinline__ uint32_t pack_contrib(const ChanParam& p, int v, int cds, int cde, int grey, uint32_t sem) {
    const int vv = p.reverse ? ((cde - v + cds) & 0xFF) : v;
    if (grey && !(p.has_lut && (sem & OMR_SEM_GREYSCALE_LUT)))
        return ((uint32_t)vv << 20) | ((uint32_t)vv << 10) | (uint32_t)vv;
    uint32_t r, g, b;
    if (p.has_lut) {
        r = p.lut_rgb[vv]; g = p.lut_rgb[256 + vv]; b = p.lut_rgb[512 + vv];
    } else if (sem & OMR_SEM_ALPHA_SEPARATE) {
        r = (uint32_t)(int)((float)(int)(p.cratio[0] * (float)vv) * p.alpha);
        g = (uint32_t)(int)((float)(int)(p.cratio[1] * (float)vv) * p.alpha);
        b = (uint32_t)(int)((float)(int)(p.cratio[2] * (float)vv) * p.alpha);
    } else {
        r = (uint32_t)(int)(p.ratio[0] * (float)vv);
        g = (uint32_t)(int)(p.ratio[1] * (float)vv);
        b = (uint32_t)(int)(p.ratio[2] * (float)vv);
    }
    return (r << 20) | (g << 10) | b;
}

// Contribution-table entry t of active channel a (K1, and K2's in-LDS build for small launches).
// Table8 channels are indexed by the raw byte.
__device__ __forceinline__ uint32_t contrib_entry(const RenderPlan* __restrict__ plan, int a, int t, int is_signed8) {
    const ChanParam& p = plan->ch[a];
    const int cds = plan->cd_start, cde = plan->cd_end;
    if (p.mode == kModeTable8) {
        const int value = is_signed8 ? (int)(int8_t)(uint8_t)t : t;
        if (value < p.gmin || value > p.gmax) return kErrBit;
        const int v = p.qtab[t];                      // q(value), from the host (prepare_plan)
        return pack_contrib(p, v, cds, cde, plan->greyscale, plan->sem);
    }
    return pack_contrib(p, t, cds, cde, plan->greyscale, plan->sem);
}

// A render prepared for the fused render -> JPEG path (omr_jpeg.hip): the plan is staged and
// the contribution tables (K1) and byte LUTs built on the context stream; the fused kernel
// quantizes + composites each pixel as K2 does (same helpers, same tables) and encodes it.
constexpr int kFusedMaxActive = 4;
enum FusedMode : int32_t { kFusedTable8 = 0, kFusedLinear16 = 1, kFusedMixed16 = 2, kFusedFast16 = 4,
                           kFusedFast16I = 5 /* launch-only: Fast16 with integral window starts */,
                           kFusedFast16F = 6 /* launch-only: Fast16I in f32 (FusedRender::f32) */,
                           kFusedFast16FS = 7 /* launch-only: kFusedFast16F on int16 pixels (sign bias) */ };
struct FusedRender {
    K2Chan ch[kFusedMaxActive];
    const uint32_t* contrib;     // [n_active][256] (workspace; built by K1 unless the kernel builds it)
    const RenderPlan* plan;      // the staged plan (kernels that build the tables themselves)
    int32_t* flag;               // sticky quantization-error word
    int32_t n_active, mode, cd_start, cds8, cde8, is_signed;
    int32_t any_check;           // some channel's LUT domain is narrower than its pixel type
    int32_t ws_int;              // every window start is an integer (|ws| < 2^30): x - ws in int32
    int32_t f32;                 // Fast16 with every channel's (fa, fb) proven exact: kFusedFast16F
    float fa[kFusedMaxActive], fb[kFusedMaxActive];
    float fc[kFusedMaxActive];   // 2^23 + wsi (exact: |wsi| <= 2^23): F1's packed form of x - wsi
    // 16-bit LUT domains of the checked channels in the kernel's (biased) pixel domain, clamped to
    // [0, 65535] and packed twice (lo | lo << 16) for v_pk_min/max_u16 compares; dnone: some
    // checked channel's domain holds no 16-bit value at all (every pixel fails)
    uint32_t dlo2[kFusedMaxActive], dhi2[kFusedMaxActive];
    int32_t dnone;
    // an all-grey MCU (every pixel r == g == b) is possible: the greyscale model, or every channel's
    // colour grey without a .lut; otherwise F1 skips its grey-MCU test (~15 VALU per MCU)
    int32_t grey_ok;
};

// (fa, fb) for fast16f such that fast16f(x) == fast16i(x) for every x in [0, xmax] (the pixel
// domain, int16 biased to unsigned) given the window start wsi and slope a0; false when no f32
// slope within a few ulps of a0 steps at exactly fast16i's 255 pixel values.
bool fast16_f32_params(double a0, int64_t wsi, int32_t xmax, float* fa, float* fb);

// Host side (omr_render.hip).  render_fused_plan: true when the fused kernel covers these
// settings (8/16-bit integer pixels, 1..4 active channels); *st != OMR_OK is a request error.
// Opaque plan storage: the caller passes a FusedPlanBuf it owns.
struct FusedPlanBuf;
FusedPlanBuf* fused_plan_new();
void fused_plan_free(FusedPlanBuf* fp);
bool render_fused_plan(Ctx* ctx, const omr_quantum_def* q, const omr_channel_binding* ch, int32_t size_c,
                       int32_t pixel_type, FusedPlanBuf* fp, omr_status* st);
size_t render_fused_ws_bytes(const FusedPlanBuf* fp);
// Stage the plan at ctx->ws + ws_off (the workspace must hold render_fused_ws_bytes from there),
// build the tables on the context stream and fill `out`.
// build_contrib false: the fused kernel builds the tables from `plan` (contrib_entry) itself.
// bias_int16: int16 pixel-domain parameters (ws, lo, hi, gmin, gmax) + 32768, for a kernel that
// reads int16 pixels biased to unsigned (the fused JPEG kernel; plans from render_fused_plan).
omr_status render_fused_stage(Ctx* ctx, FusedPlanBuf* fp, size_t ws_off, FusedRender& out, bool build_contrib = true,
                              bool bias_int16 = false);

}  // namespace omr
