// omr_render.hip — K1 (per-request tables) and K2 (quantize + codomain + composite + flip).
//
// Replaces, per tile request:
//   renderer.renderAsPackedInt(planeDef, null)   ImageRegionRequestHandler.java:559
//     (upstream omeis Renderer: QuantumStrategy LUT, CodomainChain, HSB/GreyScale strategy)
//   flip(buf, sizeX, sizeY, flipH, flipV)         ImageRegionRequestHandler.java:574-575, :616-642
// Semantics: SEMANTICS TABLE in oracle/omr_oracle.c (the parity checker).
//
// Design:
//  * K1 folds everything that depends only on the quantized value v — reverse intensity,
//    channel colour or .lut table, greyscale — into a 256-entry table per active channel
//    whose entries pack (r,g,b) contributions as 10-bit fields.  For 8-bit pixel types the
//    quantization LUT is folded in as well (table indexed by the raw byte).
//  * K2 streams the channel planes once (16 B per lane per channel), quantizes each pixel
//    (16-bit linear: exact double evaluation of the LUT entry, no 64 KiB LUT gather;
//    other families: byte LUT gather; float/32-bit: per-pixel double q(x)), sums the
//    channel contributions from LDS with plain integer adds, clamps and packs ARGB, and
//    writes it at the flipped position (the flip costs nothing).  HBM-bound.
#include "omr_device.h"
#include "omr_k2.h"

#include <memory>
#include <mutex>

namespace omr {

// ------------------------------------------------------------------------------- K1
// Parameter blocks (plans, pointer tables, headers: a few KiB) from pinned host memory;
// blockIdx.y selects one of two (dst, src, bytes) segments.
__global__ void __launch_bounds__(256) k_h2d_small(uint8_t* __restrict__ dst1, const uint8_t* __restrict__ src1,
                                                   uint64_t n1, uint8_t* __restrict__ dst2,
                                                   const uint8_t* __restrict__ src2, uint64_t n2) {
    uint8_t* dst = blockIdx.y ? dst2 : dst1;
    const uint8_t* src = blockIdx.y ? src2 : src1;
    const uint64_t bytes = blockIdx.y ? n2 : n1;
    const uint64_t i = ((uint64_t)blockIdx.x * 256 + threadIdx.x) * 16;
    if (i + 16 <= bytes && ((reinterpret_cast<uintptr_t>(dst) | reinterpret_cast<uintptr_t>(src)) & 15) == 0) {
        *reinterpret_cast<uint4*>(dst + i) = *reinterpret_cast<const uint4*>(src + i);
    } else {
        for (uint64_t j = i; j < i + 16 && j < bytes; ++j) dst[j] = src[j];
    }
}

__global__ void k_flag_out(int32_t* __restrict__ d_flag, int32_t* __restrict__ h_flag) {
    const int32_t f = *d_flag;
    *h_flag = f;                    // visible to the host after the stream synchronises
    if (f) *d_flag = 0;
}

hipError_t launch_flag_out(hipStream_t s, int32_t* d_flag, int32_t* h_flag) {
    hipLaunchKernelGGL(k_flag_out, dim3(1), dim3(1), 0, s, d_flag, h_flag);
    return hipGetLastError();
}

hipError_t launch_h2d_small(hipStream_t s, void* dst1, const void* pinned_src1, size_t n1,
                            void* dst2, const void* pinned_src2, size_t n2) {
    const size_t bytes = std::max(n1, n2);
    if (bytes == 0) return hipSuccess;
    const uint64_t blocks = (bytes + 16 * 256 - 1) / (16 * 256);
    hipLaunchKernelGGL(k_h2d_small, dim3((unsigned)blocks, n2 ? 2u : 1u), dim3(256), 0, s, static_cast<uint8_t*>(dst1),
                       static_cast<const uint8_t*>(pinned_src1), (uint64_t)n1, static_cast<uint8_t*>(dst2),
                       static_cast<const uint8_t*>(pinned_src2), (uint64_t)n2);
    return hipGetLastError();
}

// grid: n_active blocks x 256 threads.
__global__ void __launch_bounds__(256) k_build_contrib(const RenderPlan* __restrict__ plan,
                                                       uint32_t* __restrict__ contrib, int is_signed8) {
    contrib[blockIdx.x * 256 + threadIdx.x] = contrib_entry(plan, blockIdx.x, threadIdx.x, is_signed8);
}

// ------------------------------------------------------------------------------- K2
enum K2Mode : int { kK2Table8 = 0, kK2Linear16 = 1, kK2Mixed16 = 2, kK2Eval = 3, kK2Fast16 = 4,
                    kK2Thresh = 5 /* float / 32-bit, every channel kModeThresh: no double math */ };

struct K2Args {
    const RenderPlan* plan;     // full plan in HBM (eval mode reads the family parameters)
    const void* const* planes;  // [n_tiles][size_c] (pointer-table batches)
    const uint8_t* sbase;       // strided batches: plane(t, c) = sbase + t*tile_stride + c*chan_stride
    int64_t tile_stride, chan_stride;
    int32_t strided;
    const uint32_t* contrib;    // [n_active][256]
    const uint32_t* thresh;     // [n_active][256] kModeThresh code thresholds (K1)
    const uint32_t* buckets;    // [n_active][bk_n] kModeThresh key buckets (K1)
    int32_t bk_n;               // buckets per channel: k2_launch_buckets(n_active)
    int32_t use_thresh;         // some channel is kModeThresh: stage thresh + buckets in LDS too
    uint32_t n_work;            // work blocks of 256*CPT chunks (grid-stride in eval mode)
    uint32_t* out;              // [n_tiles][H][W]
    int32_t* status;            // optional per-tile status
    int32_t* flag;              // sticky error word
    int64_t row_stride;         // pixels
    int32_t size_c, n_tiles, width, height;
    int32_t flip_h, flip_v;
    int32_t n_active, cd_start, cd_end, cds8, cde8;
    int32_t tile_uniform;       // every block lies inside one tile (chunks per tile % block chunks == 0)
    int32_t nt_store;           // non-temporal ARGB stores (OMR_K2_NT_STORE=1; measurement switch)
    uint32_t total;             // work items (chunks of VEC pixels)
    FastDiv cpt, cpr;           // chunks per tile, chunks per row
    K2Chan ch[kMaxActive];
};

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

// Raw chunk of VEC pixels of BPP bytes.
template <int BPP, int VEC>
struct Chunk {
    static constexpr int kBytes = BPP * VEC;
    static constexpr int kDw = kBytes >= 4 ? kBytes / 4 : 1;
    uint32_t dw[kDw];
};

// Plane pointers arrive as generic pointers (pointer table / strided base); loading through
// the global address space gives global_load_* instead of flat_load_*, whose shared
// vmcnt/lgkmcnt accounting forced a full wait between the channel loads.
#define OMR_GLOBAL __attribute__((address_space(1)))
template <typename T> __device__ __forceinline__ const OMR_GLOBAL T* gload_ptr(const void* p) { return (const OMR_GLOBAL T*)(p); }
template <typename T> __device__ __forceinline__ OMR_GLOBAL T* gstore_ptr(void* p) { return (OMR_GLOBAL T*)(p); }

// K2 streams every pixel once and writes every output once: 16-byte loads are non-temporal.
// The ARGB stores are plain by default: non-temporal stores cost 10 % extra HBM write traffic
// (PMC WRITE_SIZE 1.103x the algorithmic bytes, profiles/pmc_render_c2.json) for no measured
// gain once the clocks are up (sustained K2 0.549 vs 0.547 ms, profiles/r02/k2_series_*.json);
// OMR_K2_NT_STORE=1 turns them back on for measurement (never for the 1-byte single-channel
// case: a write-only stream drops from 6.7 to 2.4 TB/s with nt stores).
#ifndef OMR_K2_NT
#define OMR_K2_NT 1
#endif

template <int BPP, int VEC>
__device__ __forceinline__ void load_chunk(Chunk<BPP, VEC>& c, const uint8_t* p) {
    constexpr int B = BPP * VEC;
    if constexpr (B == 16) {
        const u32x4 v = OMR_K2_NT ? __builtin_nontemporal_load(gload_ptr<u32x4>(p)) : *gload_ptr<u32x4>(p);
        c.dw[0] = v[0]; c.dw[1] = v[1]; c.dw[2] = v[2]; c.dw[3] = v[3];
    } else if constexpr (B == 8) {
        const u32x2 v = *gload_ptr<u32x2>(p);
        c.dw[0] = v[0]; c.dw[1] = v[1];
    } else if constexpr (B == 4) {
        c.dw[0] = *gload_ptr<uint32_t>(p);
    } else if constexpr (B == 2) {
        c.dw[0] = *gload_ptr<uint16_t>(p);
    } else {
        c.dw[0] = *gload_ptr<uint8_t>(p);
    }
}

// Integer value of pixel j (16-bit types).
template <int VEC, bool BE, bool SIGNED>
__device__ __forceinline__ int pixel16(const Chunk<2, VEC>& c, int j) {
    uint32_t d = c.dw[j >> 1];
    if constexpr (BE) d = bswap16x2(d);
    const uint32_t h = (j & 1) ? (d >> 16) : (d & 0xFFFF);
    return SIGNED ? (int)(int16_t)h : (int)h;
}

// Raw byte of pixel j (8-bit types: the contrib table is indexed by the raw byte; K1
// decodes the signed value of int8 entries).
template <int VEC>
__device__ __forceinline__ uint32_t byte_index(const Chunk<1, VEC>& c, int j) {
    return (c.dw[j >> 2] >> (8 * (j & 3))) & 0xFF;
}

// Double value of pixel j (32/64-bit types).
template <int BPP, int VEC, bool BE, int PT>
__device__ __forceinline__ double pixel_double(const Chunk<BPP, VEC>& c, int j) {
    if constexpr (BPP == 4) {
        uint32_t d = c.dw[j];
        if constexpr (BE) d = bswap32(d);
        if constexpr (PT == OMR_PIXELS_FLOAT) return (double)__uint_as_float(d);
        else if constexpr (PT == OMR_PIXELS_INT32) return (double)(int32_t)d;
        else return (double)d;
    } else {
        uint32_t lo = c.dw[2 * j], hi = c.dw[2 * j + 1];
        if constexpr (BE) { const uint32_t t = bswap32(lo); lo = bswap32(hi); hi = t; }
        return __hiloint2double((int)hi, (int)lo);
    }
}

// General q(x) in double (float / 32-bit types): Java semantics, selects instead of branches.
// Host and device: the host runs it to find the kModeThresh code thresholds (host_thresholds).
__host__ __device__ __forceinline__ uint32_t eval_q(double x, const ChanParam& p, int cds, int cde) {
    const double f = family_map(p, x);
    const double a = p.a0 * (f - p.ys);
    double r = floor(a + 0.5);
    r = (a == 0x1.fffffffffffffp-2 || r != r) ? 0.0 : r;
    r = fmin(fmax(r, -9223372036854775808.0), 9223372036854775808.0);   // (double)(long) round
    uint32_t v = (uint32_t)(java_round_d(p.a1 * r + (double)cds) & 0xFF);
    const bool lo = x < p.ws || (p.nr && x < p.ws + p.dec);
    const bool hi = x >= p.we || (p.nr && x >= p.we - p.dec);
    v = hi && !(x < p.ws) ? (uint32_t)(cde & 0xFF) : v;
    v = lo ? (uint32_t)(cds & 0xFF) : v;
    return v;
}

// ---- kModeThresh: q(x) through its code thresholds in order-preserving key space.
// key(x) is a uint32 whose unsigned order is the numeric order of x (NaN aside), so for a
// q that is monotone non-decreasing in x (checked on the host: window, NR, family and both
// rounding stages are all monotone once f is monotone on [ws, we)):
//   q(x) = min(#{c in 1..255 : T[c] <= key(x)}, q(max key)),  T[c] = min{key : q(key) >= c}.
// T is found on the host with eval_q (host_thresholds), the q K2's kModeEval path evaluates on
// the device; K2 then costs a bucket read and a short search instead of a double log/pow.
__device__ __forceinline__ uint32_t float_key(uint32_t bits) {
    return (bits & 0x80000000u) ? ~bits : (bits | 0x80000000u);
}

template <int PT> __device__ __forceinline__ uint32_t raw_key(uint32_t raw) {
    if constexpr (PT == OMR_PIXELS_FLOAT) return float_key(raw);
    else if constexpr (PT == OMR_PIXELS_INT32) return raw ^ 0x80000000u;
    else return raw;
}


// thr[a][0] = q(max key) | q(NaN) << 8; thr[a][c] = T[c] (0xFFFFFFFF when no key reaches c): built
// on the host (host_thresholds) and staged with the plan.

// Buckets over the key range where a kModeThresh channel's code varies: bucket b covers 2^shift
// keys from origin + b·2^shift; its entry is (#T <= its first key) | (#T in the rest of it) << 8,
// so K2 searches only the few thresholds of its bucket (usually 0-2) instead of all 255.  The
// origin sits one whole bucket below T[1] (round 3), so bucket 0 holds no threshold, and the
// table runs on past T[cmax] to its full extent `hi`: K2 clamps the key into [origin, hi] for the
// bucket index only (one med3), and a key below T[1] (bucket 0) or past T[cmax]'s bucket finds
// len 0 -- no search.  Before, both clamped ends shared a bucket with a threshold, and every
// pixel outside the window (half the plane for a window that starts above the data's median)
// ran one search step.  The (origin, hi, shift) of each channel follow its buckets in the table.
#ifndef OMR_K2_BUCKETS_LOG2
#define OMR_K2_BUCKETS_LOG2 11
#endif
constexpr int kBucketsLog2 = OMR_K2_BUCKETS_LOG2, kBuckets = 1 << kBucketsLog2;
// Buckets per channel: kBuckets u32 entries (8 KiB) for up to 4 threshold channels, half as many
// above, so 8 channels' threshold + bucket tables still fit K2's 48 KiB (the 16-byte bucket maps
// ride on top).
__host__ __device__ constexpr int k2_buckets_log2(int na) { return na <= 4 ? kBucketsLog2 : kBucketsLog2 - 1; }
__host__ __device__ constexpr int k2_buckets(int na) { return 1 << k2_buckets_log2(na); }
// the launch's bucket count: k2_buckets, or for measurement OMR_K2_BUCKETS_LG (10..11: 2^lg) /
// OMR_K2_BUCKETS (a multiple of 256 from 1024 to 2048), read per call (tests A/B them)
static inline int k2_launch_buckets(int na) {
    int env = 0;
    if (const char* ev = std::getenv("OMR_K2_BUCKETS")) {
        const int v = std::atoi(ev);
        if (v >= 1024 && v <= kBuckets && v % 256 == 0) env = v;
    } else if (const char* el = std::getenv("OMR_K2_BUCKETS_LG")) {
        const int v = std::atoi(el);
        if (v >= 10 && v <= kBucketsLog2) env = 1 << v;
    }
    if (env && (size_t)na * (2048 + 4u * env + 16) <= 64 * 1024) return env;
    return k2_buckets(na);
}
constexpr int kMaxThreshActive = (int)((48u * 1024u) / (1024u + 1024u + 4u * (kBuckets / 2)));

// Bucket map of a channel with thresholds T[1] = t1 .. T[cmax] = k1: the smallest shift with
// (k1 - t1) >> shift <= kBuckets - 3, origin = t1 - 2^shift rounded down to a multiple of 2^shift
// (0 when t1 < 2^shift) -- so a key's bucket is (key >> shift) - (origin >> shift) and K2 folds
// the second term into its table address -- and hi = the last key of bucket kBuckets - 1
// (saturated at 2^32 - 1).  T[1] lands in bucket 1 (bucket 0 holds no threshold), T[cmax] at most
// in bucket (span >> shift) + 2.
struct BucketMap { uint32_t org, hi, sh, pad; };
__device__ __forceinline__ BucketMap bucket_map(uint32_t t1, uint32_t k1, uint32_t nbk) {
    const uint32_t span = k1 - t1;
    const uint32_t bits = span ? 32u - (uint32_t)__clz(span) : 0u;
    const uint32_t lg = 31u - (uint32_t)__clz(nbk);
    uint32_t sh = bits > lg ? bits - lg : 0u;
    while ((span >> sh) > nbk - 3u) ++sh;                 // sh <= 23 (span < 2^32, nbk >= 1024)
    BucketMap m;
    m.sh = sh;
    const uint64_t step = 1ull << sh;
    m.org = t1 >= step ? (uint32_t)((t1 - step) & ~(step - 1)) : 0u;
    const uint64_t end = (uint64_t)m.org + ((uint64_t)nbk << sh) - 1u;
    m.hi = end > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)end;
    m.pad = m.org >= 0x80000000u ? 1u : 0u;               // float keys: K2 may clamp the raw bits
    // (org >= key(+0.0) -- every threshold of a float channel sits above +0)
    return m;
}

__device__ __forceinline__ uint32_t med3_u32(uint32_t x, uint32_t lo, uint32_t hi) {
    uint32_t r;
    asm("v_med3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(x), "v"(lo), "v"(hi));
    return r;
}

__device__ __forceinline__ int32_t med3_i32(int32_t x, int32_t lo, int32_t hi) {
    int32_t r;
    asm("v_med3_i32 %0, %1, %2, %3" : "=v"(r) : "v"(x), "v"(lo), "v"(hi));
    return r;
}

// #{c in 1..255 : T[c] <= key} over the sorted thresholds.
__device__ __forceinline__ uint32_t thresh_count(const uint32_t* __restrict__ T, uint32_t key) {
    uint32_t pos = 0;
#pragma unroll
    for (uint32_t st = 128; st >= 1; st >>= 1) pos += (T[pos + st] <= key) ? st : 0u;
    return pos;
}

// grid: (buckets / 256, n_active) x 256 threads; the maps follow the n_active bucket tables.
// Entry of bucket [ks, ke]: lo = #T <= ks in bits 0-7, and in bits 8-31 the offset t - ks of its
// one threshold t when it holds exactly one (1 .. 2^23 - 1: T[c] > ks, sh <= 23), 0xFFFFFF when
// it holds none, 0x800000 | n when it holds n >= 2 (both above every in-bucket offset).  K2 then
// quantizes a key of the bucket as lo + ((key - ks) >= offset) -- one table read, no threshold
// read -- and only keys in a bucket of two or more thresholds search its n thresholds.
__global__ void __launch_bounds__(256) k_build_buckets(const RenderPlan* __restrict__ plan,
                                                       const uint32_t* __restrict__ thr,
                                                       uint32_t* __restrict__ bkt, int nbk) {
    const int a = blockIdx.y;
    if (plan->ch[a].mode != kModeThresh) return;
    const uint32_t* T = thr + a * 256;
    const uint32_t cmax = T[0] & 0xFFu;
    const uint32_t b = blockIdx.x * 256 + threadIdx.x;
    const uint32_t k1 = cmax ? T[cmax] : 0u;
    const BucketMap m = bucket_map(cmax ? T[1] : 0u, k1, (uint32_t)nbk);
    if (b == 0) reinterpret_cast<BucketMap*>(bkt + gridDim.y * nbk)[a] = m;
    uint32_t e = 0xFFFFFF00u;
    if (cmax) {
        const uint64_t ks = (uint64_t)m.org + ((uint64_t)b << m.sh);
        const uint64_t ke = ks + (1ull << m.sh) - 1;
        const uint32_t lo = thresh_count(T, (uint32_t)std::min<uint64_t>(ks, k1));
        const uint32_t hi = thresh_count(T, (uint32_t)std::min<uint64_t>(ke, k1));
        const uint32_t n = hi - lo;
        const uint32_t off = n == 0 ? 0xFFFFFFu : n == 1 ? T[lo + 1] - (uint32_t)ks : 0x800000u | n;
        e = lo | (off << 8);
    }
    bkt[a * nbk + b] = e;
}

#ifndef OMR_K2_CPT
#define OMR_K2_CPT 2
#endif
constexpr int kCPT = OMR_K2_CPT;   // chunks per thread of the fixed-channel-count kernels

// LDS of one K2 block: contrib [na][256] u32, then (kModeThresh) thresholds [na][256] u32 and
// buckets [na][k2_buckets(na)] u32 + their maps.
__host__ __device__ constexpr size_t k2_lds_bytes(int na, bool thresh, int nbk) {
    return (size_t)na * (1024 + (thresh ? 1024 + 4 * nbk + sizeof(BucketMap) : 0));
}

template <int MODE, int BPP>
__device__ __forceinline__ void k2_stage_tables(const K2Args& A, uint32_t* s_contrib, int na) {
    // one 16-byte load per lane for up to 4 channels of contrib; the threshold tables follow
    for (int i = threadIdx.x * 4; i < na * 256; i += blockDim.x * 4)
        *reinterpret_cast<uint4*>(s_contrib + i) = *reinterpret_cast<const uint4*>(A.contrib + i);
    if constexpr ((MODE == kK2Eval || MODE == kK2Thresh) && BPP == 4) {
        if (A.use_thresh) {
            uint32_t* s_thr = s_contrib + na * 256;
            for (int i = threadIdx.x * 4; i < na * 256; i += blockDim.x * 4)
                *reinterpret_cast<uint4*>(s_thr + i) = *reinterpret_cast<const uint4*>(A.thresh + i);
            uint32_t* s_b = s_thr + na * 256;
            const uint32_t* g_b = reinterpret_cast<const uint32_t*>(A.buckets);
            for (int i = threadIdx.x * 4; i < na * (A.bk_n + 4); i += blockDim.x * 4)   // + the maps
                *reinterpret_cast<uint4*>(s_b + i) = *reinterpret_cast<const uint4*>(g_b + i);
        }
    }
}

// One chunk of 8/16 bytes per channel (loaded, or NA == 0: loaded here channel by channel):
// quantize + codomain + composite, then the ARGB store (flips folded into the address).
template <int BPP, int VEC, bool BE, bool SIGNED, int PT, int NA, int MODE>
__device__ __forceinline__ void k2_chunk(const K2Args& A, Chunk<BPP, VEC> (&ckk)[NA > 0 ? NA : 1], uint32_t tile,
                                         uint32_t row, uint32_t cc, const uint32_t* s_contrib) {
    constexpr int NL = NA > 0 ? NA : 1;
    const int na = NA > 0 ? NA : A.n_active;
    const int cds = A.cd_start, cds8 = A.cds8, cde8 = A.cde8;
    const int W = A.width, H = A.height;
    auto plane_base = [&](uint32_t t, int a) -> const uint8_t* {
        if (A.strided) return A.sbase + (int64_t)t * A.tile_stride + (int64_t)A.ch[a].index * A.chan_stride;
        return static_cast<const uint8_t*>(A.planes[(int64_t)t * A.size_c + A.ch[a].index]);
    };
    const uint32_t* const s_thr = s_contrib + na * 256;
    const uint32_t* const s_bkt = s_thr + na * 256;
    const int nbk = A.bk_n;
    const int64_t in_off = ((int64_t)row * A.row_stride + (int64_t)cc * VEC) * BPP;
    uint32_t acc[VEC];
#pragma unroll
    for (int j = 0; j < VEC; ++j) acc[j] = 0;
    uint32_t err_bits = 0;
    bool err = false;
#pragma unroll
    for (int a = 0; a < (NA > 0 ? NA : kMaxActive); ++a) {
        if (NA == 0 && a >= na) break;
        const K2Chan& p = A.ch[a];
        Chunk<BPP, VEC>& c = ckk[NA > 0 ? a : 0];
        if constexpr (NA == 0) {
            load_chunk<BPP, VEC>(c, plane_base(tile, a) + in_off);
        }
        const uint32_t* tab = s_contrib + a * 256;
        if constexpr ((MODE == kK2Eval || MODE == kK2Thresh) && BPP == 4) {
            if (MODE == kK2Thresh || p.mode == kModeThresh) {          // uniform: bucket, then the few thresholds in it
                const uint32_t* T = s_thr + a * 256;
                const uint32_t* Bk = s_bkt + a * nbk;
                const uint32_t cnan = (T[0] >> 8) & 0xFFu;
                const BucketMap& M = reinterpret_cast<const BucketMap*>(s_bkt + na * nbk)[a];
                const uint32_t org = M.org, hi = M.hi, sh = M.sh, inb = (1u << sh) - 1u;
                if constexpr (PT == OMR_PIXELS_FLOAT || PT == OMR_PIXELS_INT32) {
                    if (PT == OMR_PIXELS_INT32 || M.pad) {              // uniform: clamp the raw bits (k_build_buckets)
                        // raw pixel bits as int32: key = raw ^ 2^31 is a monotone bijection for
                        // int32, and for floats on the non-negative half (every negative float
                        // and -0 clamps to org_r >= 0, where the count is 0 like theirs).  The
                        // bucket of raw r is (r >> sh, arithmetic) + 2^(31 - sh) - (org >> sh).
                        const int32_t org_r = (int32_t)(org ^ 0x80000000u), hi_r = (int32_t)(hi ^ 0x80000000u);
                        const uint32_t* const Bkr = Bk - (org >> sh) + (0x80000000u >> sh);
#pragma unroll
                        for (int j = 0; j < VEC; ++j) {
                            uint32_t raw = c.dw[j];
                            if constexpr (BE) raw = bswap32(raw);
                            const int32_t kc = med3_i32((int32_t)raw, org_r, hi_r);
                            const uint32_t e = Bkr[kc >> sh];
                            const uint32_t off = e >> 8;
                            uint32_t base = (e & 0xFFu) + (((uint32_t)kc & inb) >= off ? 1u : 0u);
                            if (off - 0x800000u < 0x7FFFFFu) {          // two or more thresholds here
                                const uint32_t key = (uint32_t)kc ^ 0x80000000u;   // the clamped key: same count
                                uint32_t len = off & 0xFFu;
                                while (len > 0) {
                                    const uint32_t half = len >> 1;
                                    const bool le = T[base + half + 1] <= key;
                                    base = le ? base + half + 1 : base;
                                    len = le ? len - half - 1 : half;
                                }
                            }
                            if constexpr (PT == OMR_PIXELS_FLOAT) base = __builtin_isnan(__uint_as_float(raw)) ? cnan : base;
                            acc[j] += tab[base];
                            if (NA == 0 || NA > 4) acc[j] = clamp_fields(acc[j]);
                        }
                        continue;
                    }
                }
                const uint32_t* const Bk0 = Bk - (org >> sh);           // org is a multiple of 2^sh
#pragma unroll
                for (int j = 0; j < VEC; ++j) {
                    uint32_t raw = c.dw[j];
                    if constexpr (BE) raw = bswap32(raw);
                    uint32_t key;
                    if constexpr (PT == OMR_PIXELS_FLOAT) key = raw ^ ((uint32_t)((int32_t)raw >> 31) | 0x80000000u);
                    else key = raw_key<PT>(raw);
                    const uint32_t kc = med3_u32(key, org, hi);
                    const uint32_t e = Bk0[kc >> sh];
                    const uint32_t off = e >> 8;
                    uint32_t base = (e & 0xFFu) + ((kc & inb) >= off ? 1u : 0u);
                    if (off - 0x800000u < 0x7FFFFFu) {              // two or more thresholds here
                        uint32_t len = off & 0xFFu;
                        while (len > 0) {
                            const uint32_t half = len >> 1;
                            const bool le = T[base + half + 1] <= key;
                            base = le ? base + half + 1 : base;
                            len = le ? len - half - 1 : half;
                        }
                    }
                    if constexpr (PT == OMR_PIXELS_FLOAT) base = __builtin_isnan(__uint_as_float(raw)) ? cnan : base;
                    acc[j] += tab[base];
                    if (NA == 0 || NA > 4) acc[j] = clamp_fields(acc[j]);
                }
                continue;
            }
        }
#pragma unroll
        for (int j = 0; j < VEC; ++j) {
            uint32_t e;
            if constexpr (MODE == kK2Table8) {
                e = tab[byte_index<VEC>(c, j)];
                err_bits |= e;
                e &= ~kErrBit;
            } else if constexpr (MODE == kK2Fast16 || MODE == kK2Linear16 || MODE == kK2Mixed16) {
                const int x = pixel16<VEC, BE, SIGNED>(c, j);
                if (p.check) err |= (x < p.gmin) | (x > p.gmax);
                uint32_t v;
                if constexpr (MODE == kK2Fast16) {
                    v = fast16(x, p);
                } else if (MODE == kK2Linear16 || p.mode == kModeLinear16) {
                    v = linear16(x, p, cds, cds8, cde8);
                } else {
                    const int xi = min(max(x, p.gmin), p.gmax);
                    v = reinterpret_cast<const uint8_t*>(p.lut_addr)[(uint32_t)(xi - p.gmin)];
                }
                e = tab[v];
            } else if constexpr (MODE == kK2Eval) {
                const double x = pixel_double<BPP, VEC, BE, PT>(c, j);
                e = tab[eval_q(x, A.plan->ch[a], A.cd_start, A.cd_end)];
            } else {
                e = 0;   // kK2Thresh: every channel took the threshold path above
            }
            acc[j] += e;
            if (NA == 0 || NA > 4) acc[j] = clamp_fields(acc[j]);
        }
    }
    if ((err_bits & kErrBit) || err) {
        atomicOr(A.flag, 1);
        if (A.status) A.status[tile] = OMR_QUANTIZATION;
    }
    uint32_t px[VEC];
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
        const uint32_t c = clamp_fields(acc[j]);
        px[j] = 0xFF000000u | ((c >> 4) & 0xFF0000u) | ((c >> 2) & 0xFF00u) | (c & 0xFFu);
    }
    const uint32_t orow = A.flip_v ? (uint32_t)H - 1 - row : row;
    const uint32_t ocol = A.flip_h ? (uint32_t)W - (cc + 1) * VEC : cc * VEC;
    OMR_GLOBAL uint32_t* o = gstore_ptr<uint32_t>(A.out + (int64_t)tile * W * H + (int64_t)orow * W + ocol);
    if (A.flip_h) {
#pragma unroll
        for (int j = 0; j < VEC / 2; ++j) { const uint32_t t = px[j]; px[j] = px[VEC - 1 - j]; px[VEC - 1 - j] = t; }
    }
    if constexpr (VEC % 4 == 0) {
#pragma unroll
        for (int j = 0; j < VEC; j += 4)
        {
            const u32x4 v = u32x4{px[j], px[j + 1], px[j + 2], px[j + 3]};
            if (OMR_K2_NT && BPP * NL >= 4 && A.nt_store) __builtin_nontemporal_store(v, (OMR_GLOBAL u32x4*)(o + j));
            else *(OMR_GLOBAL u32x4*)(o + j) = v;
        }
    } else if constexpr (VEC == 2) {
        *(OMR_GLOBAL u32x2*)(o) = u32x2{px[0], px[1]};
    } else {
        o[0] = px[0];
    }
}

// The chunks of work block wb: [wb*256*CPT, (wb+1)*256*CPT), thread t the chunks
// wb*256*CPT + k*256 + t.  Every channel load of every chunk is issued before any compute
// (CPT*NA 16-B loads in flight per lane); plain loads (measured faster than non-temporal here,
// tools/probe_stream.hip).  NA == 0: runtime channel count, one chunk per thread, clamp per add.
// STAGE: load the LDS tables here, after the pixel loads are in flight (one-pass grids).
// The chunks of a work block in flight: positions and (NA > 0) every channel's pixels.
template <int BPP, int VEC, int NA, int CPT>
struct K2Batch {
    uint32_t gk[CPT], tk[CPT], rk[CPT], ck[CPT];
    Chunk<BPP, VEC> c[CPT][NA > 0 ? NA : 1];
};

// Positions of work block wb's chunks for this thread, then (NA > 0) every plane pointer (scalar
// when the block sits in one tile) and every pixel load back to back: no wait between them.
template <int BPP, int VEC, int NA, int CPT>
__device__ __forceinline__ void k2_issue(const K2Args& A, uint32_t wb, K2Batch<BPP, VEC, NA, CPT>& B,
                                         uint32_t tid = threadIdx.x) {
    constexpr int NL = NA > 0 ? NA : 1;
    const uint32_t cpr = A.cpr.d, cptd = A.cpt.d;
    const uint32_t g0 = wb * (kBlock * CPT);
    uint32_t btile = 0;
    if (A.tile_uniform) btile = fdiv(g0, A.cpt);          // whole block inside one tile (scalar)
    auto plane_base = [&](uint32_t t, int a) -> const uint8_t* {
        if (A.strided) return A.sbase + (int64_t)t * A.tile_stride + (int64_t)A.ch[a].index * A.chan_stride;
        return static_cast<const uint8_t*>(A.planes[(int64_t)t * A.size_c + A.ch[a].index]);
    };
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
        B.gk[k] = g0 + k * kBlock + tid;
        const uint32_t g = min(B.gk[k], A.total - 1);   // tail lanes load a valid chunk, store nothing
        const uint32_t t = A.tile_uniform ? btile : fdiv(g, A.cpt);
        const uint32_t rem = g - t * cptd;
        const uint32_t r = fdiv(rem, A.cpr);
        B.tk[k] = t;
        B.rk[k] = r;
        B.ck[k] = rem - r * cpr;
    }
    if constexpr (NA > 0) {
        const uint8_t* ubase[NL];
        if (A.tile_uniform) {
#pragma unroll
            for (int a = 0; a < NL; ++a) ubase[a] = plane_base(btile, a);
        }
        const uint8_t* pb[CPT][NL];
#pragma unroll
        for (int k = 0; k < CPT; ++k)
#pragma unroll
            for (int a = 0; a < NA; ++a) pb[k][a] = A.tile_uniform ? ubase[a] : plane_base(B.tk[k], a);
#pragma unroll
        for (int k = 0; k < CPT; ++k) {
            const int64_t off = ((int64_t)B.rk[k] * A.row_stride + (int64_t)B.ck[k] * VEC) * BPP;
#pragma unroll
            for (int a = 0; a < NA; ++a) load_chunk<BPP, VEC>(B.c[k][a], pb[k][a] + off);
        }
    }
}

template <int BPP, int VEC, bool BE, bool SIGNED, int PT, int NA, int MODE, int CPT>
__device__ __forceinline__ void k2_finish(const K2Args& A, K2Batch<BPP, VEC, NA, CPT>& B, const uint32_t* s_contrib) {
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
        if (B.gk[k] >= A.total) continue;
        k2_chunk<BPP, VEC, BE, SIGNED, PT, NA, MODE>(A, B.c[k], B.tk[k], B.rk[k], B.ck[k], s_contrib);
    }
}

// The chunks of work block wb: [wb*256*CPT, (wb+1)*256*CPT), thread t the chunks
// wb*256*CPT + k*256 + t.  Every channel load of every chunk is issued before any compute
// (CPT*NA 16-B loads in flight per lane); plain loads (measured faster than non-temporal here).
// NA == 0: runtime channel count, one chunk per thread, clamp per add.
// STAGE: load the LDS tables here, after the pixel loads are in flight (one-pass grids).
template <int BPP, int VEC, bool BE, bool SIGNED, int PT, int NA, int MODE, bool STAGE, int CPTT>
__device__ __forceinline__ void k2_work(const K2Args& A, uint32_t wb, uint32_t* s_contrib) {
    constexpr int CPT = NA > 0 ? CPTT : 1;
    const int na = NA > 0 ? NA : A.n_active;
    K2Batch<BPP, VEC, NA, CPT> B;
    k2_issue<BPP, VEC, NA, CPT>(A, wb, B);
    if constexpr (STAGE) {
        // tables -> LDS, issued after the pixel loads so their latencies overlap.  Small launches
        // (CPTT 1, integer modes) build them from the plan here instead: no K1 launch per request.
        if constexpr (CPTT == 1 && kCPT > 1 && BPP <= 2) {
            for (int i = threadIdx.x; i < na * 256; i += kBlock)
                s_contrib[i] = contrib_entry(A.plan, i >> 8, i & 255, PT == OMR_PIXELS_INT8 ? 1 : 0);
        } else {
            k2_stage_tables<MODE, BPP>(A, s_contrib, na);
        }
        __syncthreads();
    }
    k2_finish<BPP, VEC, BE, SIGNED, PT, NA, MODE, CPT>(A, B, s_contrib);
}

// Float / 32-bit modes, software-pipelined grid stride (round 3): the pixel loads of the
// workgroup's next work block are issued before the current block is quantized, so every lane
// keeps NA * CPT 16-byte loads in flight through the compute (the plain grid stride above waits
// out the HBM latency once per block, then computes with nothing in flight).
// SUB: work blocks per workgroup (256 threads each) sharing one copy of the LDS tables, so a
// register-light form (one chunk per lane) can hold more waves per CU than the tables' LDS
// would allow 256-thread workgroups.
template <int BPP, int VEC, bool BE, bool SIGNED, int PT, int NA, int MODE, int CPT, int SUB = 1>
__global__ void __launch_bounds__(kBlock * SUB) k_render_pipe(const K2Args A) {
    extern __shared__ __attribute__((aligned(16))) uint32_t s_contrib[];
    K2Batch<BPP, VEC, NA, CPT> b0, b1;
    const uint32_t tid = SUB == 1 ? threadIdx.x : threadIdx.x % kBlock;
    const uint32_t stride = gridDim.x * SUB;
    uint32_t wb = blockIdx.x * SUB + (SUB == 1 ? 0u : threadIdx.x / kBlock);   // wave-uniform
    if (wb < A.n_work) k2_issue<BPP, VEC, NA, CPT>(A, wb, b0, tid);
    k2_stage_tables<MODE, BPP>(A, s_contrib, NA);                 // behind the first loads
    __syncthreads();
    while (wb < A.n_work) {                                       // wave-uniform; two blocks per trip
        const uint32_t w1 = wb + stride;
        if (w1 < A.n_work) k2_issue<BPP, VEC, NA, CPT>(A, w1, b1, tid);
        k2_finish<BPP, VEC, BE, SIGNED, PT, NA, MODE, CPT>(A, b0, s_contrib);
        if (w1 >= A.n_work) break;
        const uint32_t w2 = w1 + stride;
        if (w2 < A.n_work) k2_issue<BPP, VEC, NA, CPT>(A, w2, b0, tid);
        k2_finish<BPP, VEC, BE, SIGNED, PT, NA, MODE, CPT>(A, b1, s_contrib);
        wb = w2;
    }
}

// Integer / 8-bit modes: one full (non-persistent) grid, one work block per workgroup, tables
// staged behind the pixel loads.  Eval mode (float / 32-bit; threshold + bucket tables up to
// 6 KiB per channel): a grid of a few workgroups per CU that stage the tables once and stride
// over the work blocks.  CPTT: chunks per thread when NA > 0 — kCPT for batches, 1 for launches
// too small to fill the chip at kCPT (a one-tile request, a C3 composite), twice the workgroups.
template <int BPP, int VEC, bool BE, bool SIGNED, int PT, int NA, int MODE, int CPTT = kCPT>
__global__ void __launch_bounds__(kBlock) k_render(const K2Args A) {
    extern __shared__ __attribute__((aligned(16))) uint32_t s_contrib[];
    if constexpr (MODE == kK2Eval || MODE == kK2Thresh) {
        k2_stage_tables<MODE, BPP>(A, s_contrib, NA > 0 ? NA : A.n_active);
        __syncthreads();
        for (uint32_t wb = blockIdx.x; wb < A.n_work; wb += gridDim.x)
            k2_work<BPP, VEC, BE, SIGNED, PT, NA, MODE, false, CPTT>(A, wb, s_contrib);
    } else {
        k2_work<BPP, VEC, BE, SIGNED, PT, NA, MODE, true, CPTT>(A, blockIdx.x, s_contrib);
    }
}

// Small-launch threshold: below this many kCPT work blocks K2 runs one chunk per thread.
static inline bool k2_small_launch(uint64_t total_chunks, int cu_count) {
    return kCPT > 1 && total_chunks < (uint64_t)kBlock * kCPT * (uint64_t)cu_count * 4;
}

// ------------------------------------------------------------------------------- host side
struct PreparedPlan {
    RenderPlan plan;
    size_t plan_bytes = 0;
    int n_lut = 0;                   // kModeLut16 channels (their LUTs: the context's device cache)
};

static double host_family_map(const ChanParam& p, double x) { return family_map_code(p.family, x, p.k, p.ws, p.we); }

static int32_t java_d2i_host(double v) {   // Java (int) of a double: NaN -> 0, saturating
    if (v != v) return 0;
    if (v >= 2147483647.0) return INT32_MAX;
    if (v <= -2147483648.0) return INT32_MIN;
    return (int32_t)v;
}

static int32_t ceil_to_i32(double v) {
    if (v != v) return INT32_MIN;
    const double c = ceil(v);
    if (c <= -2147483647.0) return -2147483647;
    if (c >= 2147483647.0) return 2147483647;
    return (int32_t)c;
}

// kModeThresh precondition: q is monotone non-decreasing in x.  Below ws it is cdStart, at or
// above we cdEnd, and inside [ws, we) it is round(a1*round(a0*(f(x) - f(ws))) + cdStart) with
// a0, a1 >= 0 — monotone once f is increasing and finite on [ws, we]: always for linear; for
// log / poly / exp when ws > 0 and k > 0 (x^k, ln x, e^(x^k) increase on x > 0); for the
// window-normalised exp (OMR_SEM_EXP_NORMALIZED) when k > 0 (its input is in [0, 1)).  Noise
// reduction only widens the two constant ends.  Codes must stay inside one byte without wrap.
static bool monotone_q(const ChanParam& p, const omr_quantum_def& q) {
    if (q.cd_start < 0 || q.cd_end > 255 || q.cd_start > q.cd_end) return false;
    if (!std::isfinite(p.ws) || !std::isfinite(p.we) || !(p.ws < p.we)) return false;
    if (p.nr && !std::isfinite(p.dec)) return false;
    // a0 NaN (e.g. x^0.5 with ws < 0 gives f(ws) = NaN): a0*(f(x) - ys) is NaN for every x, so
    // the window maps to round(a1*0 + cdStart) = cdStart — a step function, monotone.
    if (p.a0 != p.a0) return true;
    if (!std::isfinite(p.ys) || !std::isfinite(p.a0) || !(p.a0 > 0) || !std::isfinite(p.a1) || p.a1 < 0) return false;
    if (p.nr && !std::isfinite(p.dec)) return false;
    if (p.family == kFamLinear) return true;
    const double ye = host_family_map(p, p.we);
    if (!std::isfinite(ye) || !(ye > p.ys)) return false;
    const bool is_log = p.family == kFamLog || p.family == kFamLogRaw;
    if (!is_log && !(p.k > 0 && std::isfinite(p.k))) return false;
    if (p.family == kFamExpNorm) return true;
    return p.ws > 0;
}

static bool thresh_ok(const ChanParam& p, const omr_quantum_def& q, int32_t pixel_type) {
    if (pixel_type != OMR_PIXELS_FLOAT && pixel_type != OMR_PIXELS_INT32 && pixel_type != OMR_PIXELS_UINT32)
        return false;
    return monotone_q(p, q);
}

// ---- kModeThresh code thresholds, on the host (round 5).  T[c] = the smallest key whose q is
// >= c, found with eval_q run on the host: the family map then goes through the host libm (the
// same log / pow / exp the CPU restatement calls), so the thresholds -- and hence every code K2
// produces for a Thresh channel -- are exactly the restatement's, where the device libm left a
// code boundary one ulp off now and then (+-1 code value, two of them on a composite component
// two channels feed).  Per code a galloping search from an estimate (the family map inverted at
// the code's rounding boundary) brackets T[c] within a few keys, then bisection: ~8 q evaluations
// per code instead of 32, and the estimate only steers the search, so the result does not depend
// on it.  Results are cached per (pixel type, codomain, family, window, coefficient, NR).
static double host_key_value(int32_t pt, uint32_t k) {
    if (pt == OMR_PIXELS_FLOAT) {
        const uint32_t b = (k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k;
        float f;
        std::memcpy(&f, &b, 4);
        return (double)f;
    }
    if (pt == OMR_PIXELS_INT32) return (double)(int32_t)(k ^ 0x80000000u);
    return (double)k;
}

// The key of the representable pixel value nearest x (an estimate only; NaN -> 0).
static uint64_t host_key_of(int32_t pt, double x) {
    if (x != x) return 0;
    if (pt == OMR_PIXELS_FLOAT) {
        const float f = (float)x;
        uint32_t b;
        std::memcpy(&b, &f, 4);
        return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
    }
    if (pt == OMR_PIXELS_INT32) {
        const double c = std::min(2147483647.0, std::max(-2147483648.0, std::floor(x)));
        return (uint32_t)(int32_t)c ^ 0x80000000u;
    }
    return (uint32_t)std::min(4294967295.0, std::max(0.0, std::floor(x)));
}

// Inverse of the family map (estimate of the x where f(x) = y).
static double host_family_inverse(const ChanParam& p, double y) {
    switch (p.family) {
    case kFamPoly: return std::pow(y, 1.0 / p.k);
    case kFamLog:
    case kFamLogRaw: return std::exp(y);
    case kFamExp: return std::pow(std::log(y), 1.0 / p.k);
    case kFamExpNorm: return p.ws + (p.we - p.ws) * std::pow(std::log(y), 1.0 / p.k);
    default: return y;
    }
}

// Smallest k in [L, R] with ge(k), given ge(R) and a guess h in [L, R]: gallop away from h until
// the answer is bracketed, then bisect.  Exact for any monotone ge whatever h is.
template <typename Ge>
static uint64_t first_true(uint64_t L, uint64_t R, uint64_t h, Ge ge) {
    if (ge(h)) {
        R = h;
        for (uint64_t step = 1; R - L >= step; step <<= 1) {
            const uint64_t m = R - step;
            if (ge(m)) R = m;
            else { L = m + 1; break; }
        }
    } else {
        L = h + 1;
        for (uint64_t step = 1; L + step - 1 < R; step <<= 1) {
            const uint64_t m = L + step - 1;
            if (ge(m)) { R = m; break; }
            L = m + 1;
        }
    }
    while (L < R) {
        const uint64_t m = L + (R - L) / 2;
        if (ge(m)) R = m;
        else L = m + 1;
    }
    return L;
}

// Estimate of the pixel value where q reaches code c: the first-stage value r the code needs,
// then f(x) = ys + (r - 0.5) / a0 inverted, clamped into the window.
static double code_estimate(const ChanParam& p, uint32_t c, int cds) {
    double r = (double)c;
    if (p.second) r = std::ceil(((double)c - 0.5 - (double)cds) / p.a1);
    double xe = host_family_inverse(p, p.ys + (r - 0.5) / p.a0);
    if (!(xe >= p.ws)) xe = p.ws;                    // NaN included
    if (!(xe <= p.we)) xe = p.we;
    return xe;
}

static void host_thresholds_compute(const ChanParam& p, int32_t pt, int cds, int cde, uint32_t* T) {
    const uint32_t klo = pt == OMR_PIXELS_FLOAT ? 0x007FFFFFu : 0u;
    const uint32_t khi = pt == OMR_PIXELS_FLOAT ? 0xFF800000u : 0xFFFFFFFFu;
    auto q = [&](uint64_t k) { return eval_q(host_key_value(pt, (uint32_t)k), p, cds, cde); };
    const uint32_t cmax = q(khi);
    const uint32_t qnan = pt == OMR_PIXELS_FLOAT ? eval_q(std::nan(""), p, cds, cde) : 0u;
    T[0] = cmax | (qnan << 8);
    uint64_t lower = klo;                            // T[c] >= T[c - 1]: q is monotone
    for (uint32_t c = 1; c < 256; ++c) {
        if (c > cmax) {                              // no key reaches c
            T[c] = 0xFFFFFFFFu;
            continue;
        }
        const uint64_t h = std::min<uint64_t>(std::max<uint64_t>(host_key_of(pt, code_estimate(p, c, cds)), lower), khi);
        lower = first_true(lower, khi, h, [&](uint64_t k) { return q(k) >= c; });
        T[c] = (uint32_t)lower;
    }
}

// The byte LUT of a kModeLut16 channel over its domain [gmin, gmax] (the Quantization_8_16_bit
// LUT), with quantize_eval on the host: for a monotone q through its 255 code thresholds (a few
// thousand evaluations instead of 65,536 for a u16 domain), otherwise entry by entry.  Cached
// (most recent 16 domains up to 2^17 entries).
static void host_quant_lut_compute(const ChanParam& p, int cds, int cde, bool mono, uint8_t* out) {
    const int64_t gmin = p.gmin, gmax = p.gmax, n = gmax - gmin + 1;
    auto q = [&](int64_t x) { return (uint32_t)quantize_eval((double)x, p, cds, cde); };
    if (!mono) {
        for (int64_t i = 0; i < n; ++i) out[i] = (uint8_t)q(gmin + i);
        return;
    }
    const uint32_t cmax = q(gmax);
    int64_t T[256];
    uint64_t lower = 0;                              // offsets from gmin
    for (uint32_t c = 1; c <= cmax; ++c) {
        double xe = std::ceil(code_estimate(p, c, cds));
        if (!(xe >= (double)gmin)) xe = (double)gmin;
        if (!(xe <= (double)gmax)) xe = (double)gmax;
        const uint64_t h = std::max<uint64_t>((uint64_t)((int64_t)xe - gmin), lower);
        lower = first_true(lower, (uint64_t)(n - 1), h, [&](uint64_t k) { return q(gmin + (int64_t)k) >= c; });
        T[c] = (int64_t)lower;
    }
    uint32_t c = 0;
    for (int64_t i = 0; i < n; ++i) {
        while (c < cmax && T[c + 1] <= i) ++c;
        out[i] = (uint8_t)c;
    }
}

// Everything a kModeLut16 byte LUT depends on (host and device LUT caches).
struct QuantLutKey {
    int32_t cds, cde, family, nr, gmin, gmax, lo, hi, second, mono;
    double ws, we, k, ys, a0, a1, dec;
};
static QuantLutKey quant_lut_key(const ChanParam& p, int cds, int cde, bool mono) {
    QuantLutKey key;
    std::memset(&key, 0, sizeof(key));
    key.cds = cds; key.cde = cde; key.family = p.family; key.nr = p.nr; key.gmin = p.gmin; key.gmax = p.gmax;
    key.lo = p.lo; key.hi = p.hi; key.second = p.second; key.mono = mono;
    key.ws = p.ws; key.we = p.we; key.k = p.k; key.ys = p.ys; key.a0 = p.a0; key.a1 = p.a1; key.dec = p.dec;
    return key;
}

static void host_quant_lut(const ChanParam& p, int cds, int cde, bool mono, uint8_t* out) {
    const int64_t n = (int64_t)p.gmax - p.gmin + 1;
    using Key = QuantLutKey;
    const Key key = quant_lut_key(p, cds, cde, mono);
    struct Entry { Key k; std::vector<uint8_t> lut; };
    static std::mutex mu;
    static std::vector<Entry> cache;                 // most recent last
    const bool cacheable = n <= (1 << 17);
    if (cacheable) {
        std::lock_guard<std::mutex> lk(mu);
        for (size_t i = cache.size(); i-- > 0;)
            if (std::memcmp(&cache[i].k, &key, sizeof(Key)) == 0) {
                std::memcpy(out, cache[i].lut.data(), (size_t)n);
                if (i + 1 != cache.size()) std::swap(cache[i], cache.back());
                return;
            }
    }
    host_quant_lut_compute(p, cds, cde, mono, out);
    if (!cacheable) return;
    Entry e{key, std::vector<uint8_t>(out, out + n)};
    std::lock_guard<std::mutex> lk(mu);
    if (cache.size() >= 16) cache.erase(cache.begin());
    cache.push_back(std::move(e));
}

static void host_thresholds(const ChanParam& p, int32_t pt, int cds, int cde, uint32_t* T) {
    struct Key {
        int32_t pt, cds, cde, family, nr, pad;
        double ws, we, k, ys, a0, a1, dec;
        int32_t second, pad2;
    };
    Key key;
    std::memset(&key, 0, sizeof(key));
    key.pt = pt; key.cds = cds; key.cde = cde; key.family = p.family; key.nr = p.nr;
    key.ws = p.ws; key.we = p.we; key.k = p.k; key.ys = p.ys; key.a0 = p.a0; key.a1 = p.a1; key.dec = p.dec;
    key.second = p.second;
    struct Entry { Key k; uint32_t T[256]; };
    static std::mutex mu;
    static std::vector<Entry> cache;                 // most recent last, at most 64 entries
    {
        std::lock_guard<std::mutex> lk(mu);
        for (size_t i = cache.size(); i-- > 0;)
            if (std::memcmp(&cache[i].k, &key, sizeof(Key)) == 0) {
                std::memcpy(T, cache[i].T, sizeof(cache[i].T));
                if (i + 1 != cache.size()) std::swap(cache[i], cache.back());
                return;
            }
    }
    Entry e;
    e.k = key;
    host_thresholds_compute(p, pt, cds, cde, e.T);
    std::memcpy(T, e.T, sizeof(e.T));
    std::lock_guard<std::mutex> lk(mu);
    if (cache.size() >= 64) cache.erase(cache.begin());
    cache.push_back(e);
}

// The device copy of a channel's kModeLut16 byte LUT, from the context's LRU cache (Ctx::dev_luts).
// A miss builds the LUT on the host (host_quant_lut) and uploads it once; a hit costs a key compare:
// no host evaluation, no PCIe traffic and no pinned-slot growth per request.
static omr_status device_quant_lut(Ctx* ctx, const ChanParam& p, int cds, int cde, bool mono, uint64_t* addr) {
    const QuantLutKey key = quant_lut_key(p, cds, cde, mono);
    const uint8_t* kb = reinterpret_cast<const uint8_t*>(&key);
    const size_t n = (size_t)((int64_t)p.gmax - p.gmin + 1);
    for (auto& e : ctx->dev_luts)
        if (e.bytes == n && std::memcmp(e.key.data(), kb, sizeof(key)) == 0) {
            e.used = ++ctx->dev_lut_clock;
            *addr = reinterpret_cast<uint64_t>(e.d);
            return OMR_OK;
        }
    // evict least recently used entries past the count / byte budget; queued kernels of this
    // context's stream may still read them, so the stream drains first (misses only)
    bool drained = false;
    while (!ctx->dev_luts.empty() && ((int)ctx->dev_luts.size() >= Ctx::kDevLutEntries ||
                                      ctx->dev_lut_bytes + n > Ctx::kDevLutBytes)) {
        if (!drained) { OMR_HIP(ctx, hipStreamSynchronize(ctx->stream)); drained = true; }
        auto lru = std::min_element(ctx->dev_luts.begin(), ctx->dev_luts.end(),
                                    [](const Ctx::DevLut& a, const Ctx::DevLut& b) { return a.used < b.used; });
        OMR_HIP(ctx, hipFree(lru->d));
        ctx->dev_lut_bytes -= lru->bytes;
        ctx->dev_luts.erase(lru);
    }
    std::vector<uint8_t> host(n);
    host_quant_lut(p, cds, cde, mono, host.data());
    Ctx::DevLut e;
    e.key.assign(kb, kb + sizeof(key));
    e.bytes = n;
    void* d = nullptr;
    if (hipMalloc(&d, n) != hipSuccess) return fail(ctx, OMR_OOM, "device LUT allocation failed");
    e.d = static_cast<uint8_t*>(d);
    hipError_t er = hipMemcpyAsync(e.d, host.data(), n, hipMemcpyHostToDevice, ctx->stream);
    if (er == hipSuccess) er = hipStreamSynchronize(ctx->stream);     // `host` is freed on return
    if (er != hipSuccess) {
        (void)hipFree(e.d);
        return hip_fail(ctx, er, "device LUT upload");
    }
    e.used = ++ctx->dev_lut_clock;
    ctx->dev_lut_bytes += n;
    ctx->dev_luts.push_back(std::move(e));
    *addr = reinterpret_cast<uint64_t>(ctx->dev_luts.back().d);
    return OMR_OK;
}

static omr_status prepare_plan(Ctx* ctx, const omr_quantum_def* q, const omr_channel_binding* ch,
                               int32_t size_c, int32_t pixel_type, PreparedPlan& pp) {
    if (!q) return fail(ctx, OMR_INVALID_ARGUMENT, "null quantum def");
    if (size_c < 0 || (size_c > 0 && !ch)) return fail(ctx, OMR_INVALID_ARGUMENT, "bad channel bindings");
    if (q->bit_resolution <= 0) return fail(ctx, OMR_INVALID_ARGUMENT, "bit resolution must be > 0");
    if (q->model != OMR_MODEL_GREYSCALE && q->model != OMR_MODEL_RGB)
        return fail(ctx, OMR_INVALID_ARGUMENT, "unknown rendering model");
    const int bpp = bytes_per_pixel(pixel_type);
    if (!bpp) return fail(ctx, OMR_INVALID_ARGUMENT, "unsupported pixel type");
    RenderPlan& P = pp.plan;
    // header only: a channel's slot is cleared when it is filled (the plan is ~29 KiB at 32
    // channels, and only its first n_active slots are staged or read)
    std::memset(&P, 0, offsetof(RenderPlan, ch));
    P.cd_start = q->cd_start;
    P.cd_end = q->cd_end;
    P.greyscale = q->model == OMR_MODEL_GREYSCALE;
    P.sem = ctx->sem;
    int na = 0;
    pp.n_lut = 0;
    for (int c = 0; c < size_c; ++c) {
        if (!ch[c].active) continue;
        if (P.greyscale && na == 1) break;   // GreyScaleStrategy renders the first active channel (S8)
        if (na == kMaxActive) return fail(ctx, OMR_INVALID_ARGUMENT, "more than 32 active channels");
        const omr_channel_binding& b = ch[c];
        if (b.family < OMR_FAMILY_LINEAR || b.family > OMR_FAMILY_EXPONENTIAL)
            return fail(ctx, OMR_INVALID_ARGUMENT, "unknown family");
        ChanParam& p = P.ch[na];
        std::memset(&p, 0, offsetof(ChanParam, lut_rgb));   // the 768-byte LUT copy only when used
        p.index = c;
        p.family = b.family;
        if (b.family == OMR_FAMILY_LOGARITHMIC && (P.sem & OMR_SEM_LOG_UNGUARDED)) p.family = kFamLogRaw;
        if (b.family == OMR_FAMILY_EXPONENTIAL && (P.sem & OMR_SEM_EXP_NORMALIZED)) p.family = kFamExpNorm;
        p.nr = b.noise_reduction != 0 && !(P.sem & OMR_SEM_NOISE_REDUCTION_OFF);
        p.reverse = b.reverse != 0;
        p.has_lut = b.lut != nullptr;
        if (b.lut) std::memcpy(p.lut_rgb, b.lut, 768);
        p.ws = b.input_start;
        p.we = b.input_end;
        p.k = b.coefficient;
        p.ys = host_family_map(p, p.ws);
        const double ye = host_family_map(p, p.we);
        p.a0 = (double)q->bit_resolution / (ye - p.ys);
        p.a1 = (double)(q->cd_end - q->cd_start) / (double)q->bit_resolution;
        p.dec = (p.we - p.ws) / 10.0;
        p.second = !(p.a1 == 1.0 && q->cd_start == 0);
        if (P.sem & OMR_SEM_WINDOW_INT_BOUNDS) {   // x < (int)ws, x >= (int)we (Java d2i)
            p.lo = java_d2i_host(p.ws);
            p.hi = java_d2i_host(p.we);
        } else {                                   // x < ws <=> x < ceil(ws) for integer x
            p.lo = ceil_to_i32(p.ws);
            p.hi = ceil_to_i32(p.we);
            if (p.we != p.we) p.hi = INT32_MAX;
        }
        const float alpha = (float)b.rgba[3] / 255.0f;
        p.alpha = alpha;
        for (int k = 0; k < 3; ++k) {
            p.cratio[k] = (float)b.rgba[k] / 255.0f;
            p.ratio[k] = p.cratio[k] * alpha;
        }
        if (bpp <= 2) {
            const double gmin = std::trunc(b.global_min), gmax = std::trunc(b.global_max);
            if (!(gmin == gmin) || !(gmax == gmax) || gmax < gmin || gmin < -2147483648.0 || gmax > 2147483647.0)
                return fail(ctx, OMR_INVALID_ARGUMENT, "bad LUT domain (global min/max)");
            p.gmin = (int32_t)gmin;
            p.gmax = (int32_t)gmax;
            if (bpp == 1) {
                p.mode = kModeTable8;
                for (int t = 0; t < 256; ++t) {            // q of every raw byte in the domain
                    const int value = pixel_type == OMR_PIXELS_INT8 ? (int)(int8_t)(uint8_t)t : t;
                    p.qtab[t] = value < p.gmin || value > p.gmax
                                    ? 0
                                    : (uint8_t)quantize_eval((double)value, p, q->cd_start, q->cd_end);
                }
            } else {
                const bool fast = b.family == OMR_FAMILY_LINEAR && !p.nr && std::isfinite(p.ws) &&
                                  std::isfinite(p.a0) && std::fabs(p.a0) < 1e300 && !p.second &&
                                  q->bit_resolution <= 65535;
                const bool fast2 = b.family == OMR_FAMILY_LINEAR && !p.nr && std::isfinite(p.ws) &&
                                   std::isfinite(p.a0) && std::fabs(p.a0) < 1e300 && std::isfinite(p.a1) &&
                                   q->bit_resolution <= 65535;
                p.mode = (fast || fast2) ? kModeLinear16 : kModeLut16;
                if (p.mode == kModeLut16) {
                    const int64_t n = (int64_t)p.gmax - p.gmin + 1;
                    if (n > (1 << 24)) return fail(ctx, OMR_INVALID_ARGUMENT, "LUT domain too large");
                    pp.n_lut++;
                }
            }
        } else {
            p.mode = thresh_ok(p, *q, pixel_type) ? kModeThresh : kModeEval;
            p.gmin = INT32_MIN;
            p.gmax = INT32_MAX;
        }
        ++na;
    }
    P.n_active = na;
    if (na > kMaxThreshActive)   // threshold + bucket tables (6 KiB of LDS per channel): K2 within 48 KiB
        for (int i = 0; i < na; ++i)
            if (P.ch[i].mode == kModeThresh) P.ch[i].mode = kModeEval;
    pp.plan_bytes = offsetof(RenderPlan, ch) + sizeof(ChanParam) * (size_t)(na > 0 ? na : 1);
    if (pp.n_lut > 0) {
        const bool int_bounds = (P.sem & OMR_SEM_WINDOW_INT_BOUNDS) != 0;   // x in [(int)ws, ws): may wrap
        OMR_HIP(ctx, hipSetDevice(ctx->device));
        for (int i = 0; i < na; ++i)
            if (P.ch[i].mode == kModeLut16) {
                const omr_status st = device_quant_lut(ctx, P.ch[i], q->cd_start, q->cd_end,
                                                       !int_bounds && monotone_q(P.ch[i], *q), &P.ch[i].lut_addr);
                if (st) return st;
            }
    }
    return OMR_OK;
}

// Workspace layout for one render launch: [plan][contrib][thresholds][buckets][extra...] (the
// byte LUTs live in the context's device LUT cache)
struct RenderLayout {
    size_t plan_off = 0, contrib_off = 0, thresh_off = 0, bucket_off = 0, extra_off = 0, total = 0;
};

static RenderLayout layout_for(const PreparedPlan&, size_t extra) {
    RenderLayout L;
    L.plan_off = 0;
    L.contrib_off = align_up(sizeof(RenderPlan), 256);
    L.thresh_off = L.contrib_off + align_up((size_t)kMaxActive * 256 * 4, 256);
    L.bucket_off = L.thresh_off + align_up((size_t)kMaxActive * 256 * 4, 256);
    L.extra_off = L.bucket_off + align_up((size_t)kMaxActive * (kBuckets * 4 + sizeof(BucketMap)), 256);
    L.total = L.extra_off + extra;
    return L;
}

// The pipelined float kernel holds two work blocks in registers (87 VGPRs at three channels: 5
// waves per SIMD), so its grid-stride grid is sized by the kernel's own occupancy, queried once
// per instantiation: a grid sized for 8 resident blocks per CU left 3 of every 8 waiting for a
// second round.
static thread_local int tl_cu_count = 0;
template <auto KERN, int SUB = 1>
static int pipe_grid(const K2Args& a, int grid, size_t lds) {
    // occupancy per (device, LDS bytes) of this instantiation: the LDS footprint differs between
    // launches (threshold tables or not), and a pool's batchers launch it on several devices
    struct Entry { int dev; size_t lds; int occ; };
    static std::mutex mu;
    static Entry cache[16];
    static int n_cache = 0;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || tl_cu_count <= 0) return grid;
    int occ = -1;
    {
        std::lock_guard<std::mutex> lk(mu);
        for (int i = 0; i < n_cache; ++i)
            if (cache[i].dev == dev && cache[i].lds == lds) { occ = cache[i].occ; break; }
        if (occ < 0) {
            int o = 0;
            occ = hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, KERN, kBlock * SUB, lds) == hipSuccess ? o : 0;
            if (n_cache < 16) cache[n_cache++] = {dev, lds, occ};
        }
    }
    if (occ <= 0) return grid;
    return (int)std::min<uint64_t>((a.n_work + SUB - 1) / SUB, (uint64_t)tl_cu_count * (uint64_t)occ);
}

template <int BPP, int VEC, bool BE, bool SIGNED, int PT, int MODE>
static hipError_t launch_render_na(const K2Args& a, int na, int grid, bool small, hipStream_t s, int cpt = kCPT) {
    const size_t lds = k2_lds_bytes(na > 0 ? na : 1, a.use_thresh != 0, a.bk_n);
    if constexpr (BPP == 4 && VEC > 1 && (MODE == kK2Thresh || MODE == kK2Eval)) {
        // software-pipelined grid stride (k_render_pipe; cpt -1: one chunk per lane and block,
        // -2: two), the default for 1..4 channels
        if (cpt < 0) {
#define OMR_PIPE(NAV, CPTV)                                                                       \
    {                                                                                             \
        constexpr auto kern = &k_render_pipe<BPP, VEC, BE, SIGNED, PT, NAV, MODE, CPTV>;         \
        omr_launch(kern, dim3(pipe_grid<kern>(a, grid, lds)), dim3(kBlock), lds, s, a);   \
        return hipGetLastError();                                                                 \
    }
            if (cpt == -3 && na == 3) {   // measurement: one chunk per lane, two work blocks per workgroup
                constexpr auto kern = &k_render_pipe<BPP, VEC, BE, SIGNED, PT, 3, MODE, 1, 2>;
                omr_launch(kern, dim3(pipe_grid<kern, 2>(a, grid, lds)), dim3(kBlock * 2), lds, s, a);
                return hipGetLastError();
            }
            switch (na * 2 + (cpt == -2 ? 1 : 0)) {
            case 2: OMR_PIPE(1, 1)
            case 3: OMR_PIPE(1, 2)
            case 4: OMR_PIPE(2, 1)
            case 5: OMR_PIPE(2, 2)
            case 6: OMR_PIPE(3, 1)
            case 7: OMR_PIPE(3, 2)
            case 8: OMR_PIPE(4, 1)
            case 9: OMR_PIPE(4, 2)
            default: break;
            }
#undef OMR_PIPE
        }
        // grid-stride float / 32-bit modes, OMR_K2_EVAL_CPT=4: 4 chunks per lane (12 loads in
        // flight at 3 channels; measured slower than kCPT on C5)
        if (cpt == 4) {
            switch (na) {
            case 1: omr_launch((k_render<BPP, VEC, BE, SIGNED, PT, 1, MODE, 4>), dim3(grid), dim3(kBlock), lds, s, a); return hipGetLastError();
            case 2: omr_launch((k_render<BPP, VEC, BE, SIGNED, PT, 2, MODE, 4>), dim3(grid), dim3(kBlock), lds, s, a); return hipGetLastError();
            case 3: omr_launch((k_render<BPP, VEC, BE, SIGNED, PT, 3, MODE, 4>), dim3(grid), dim3(kBlock), lds, s, a); return hipGetLastError();
            case 4: omr_launch((k_render<BPP, VEC, BE, SIGNED, PT, 4, MODE, 4>), dim3(grid), dim3(kBlock), lds, s, a); return hipGetLastError();
            default: break;
            }
        }
    }
    if constexpr (BPP <= 2 && kCPT > 1) {   // grid-stride eval modes size their own grid
        if (small) {
            switch (na) {
            case 1: omr_launch((k_render<BPP, VEC, BE, SIGNED, PT, 1, MODE, 1>), dim3(grid), dim3(kBlock), lds, s, a); return hipGetLastError();
            case 2: omr_launch((k_render<BPP, VEC, BE, SIGNED, PT, 2, MODE, 1>), dim3(grid), dim3(kBlock), lds, s, a); return hipGetLastError();
            case 3: omr_launch((k_render<BPP, VEC, BE, SIGNED, PT, 3, MODE, 1>), dim3(grid), dim3(kBlock), lds, s, a); return hipGetLastError();
            case 4: omr_launch((k_render<BPP, VEC, BE, SIGNED, PT, 4, MODE, 1>), dim3(grid), dim3(kBlock), lds, s, a); return hipGetLastError();
            default: break;
            }
        }
    }
    switch (na) {
    case 1: omr_launch((k_render<BPP, VEC, BE, SIGNED, PT, 1, MODE>), dim3(grid), dim3(kBlock), lds, s, a); break;
    case 2: omr_launch((k_render<BPP, VEC, BE, SIGNED, PT, 2, MODE>), dim3(grid), dim3(kBlock), lds, s, a); break;
    case 3: omr_launch((k_render<BPP, VEC, BE, SIGNED, PT, 3, MODE>), dim3(grid), dim3(kBlock), lds, s, a); break;
    case 4: omr_launch((k_render<BPP, VEC, BE, SIGNED, PT, 4, MODE>), dim3(grid), dim3(kBlock), lds, s, a); break;
    default: omr_launch((k_render<BPP, VEC, BE, SIGNED, PT, 0, MODE>), dim3(grid), dim3(kBlock), lds, s, a); break;
    }
    return hipGetLastError();
}

template <int BPP, int VEC, bool BE>
static hipError_t launch_render_pt(const K2Args& a, int pt, int na, int mode16, int grid, bool small, hipStream_t s,
                                   int cpt) {
    if constexpr (BPP == 1) {
        return pt == OMR_PIXELS_INT8 ? launch_render_na<1, VEC, BE, true, OMR_PIXELS_INT8, kK2Table8>(a, na, grid, small, s)
                                     : launch_render_na<1, VEC, BE, false, OMR_PIXELS_UINT8, kK2Table8>(a, na, grid, small, s);
    } else if constexpr (BPP == 2) {
        if (pt == OMR_PIXELS_INT16) {
            if (mode16 == kK2Fast16) return launch_render_na<2, VEC, BE, true, OMR_PIXELS_INT16, kK2Fast16>(a, na, grid, small, s);
            return mode16 == kK2Linear16 ? launch_render_na<2, VEC, BE, true, OMR_PIXELS_INT16, kK2Linear16>(a, na, grid, small, s)
                                         : launch_render_na<2, VEC, BE, true, OMR_PIXELS_INT16, kK2Mixed16>(a, na, grid, small, s);
        }
        if (mode16 == kK2Fast16) return launch_render_na<2, VEC, BE, false, OMR_PIXELS_UINT16, kK2Fast16>(a, na, grid, small, s);
        return mode16 == kK2Linear16 ? launch_render_na<2, VEC, BE, false, OMR_PIXELS_UINT16, kK2Linear16>(a, na, grid, small, s)
                                     : launch_render_na<2, VEC, BE, false, OMR_PIXELS_UINT16, kK2Mixed16>(a, na, grid, small, s);
    } else if constexpr (BPP == 4) {
        if (mode16 == kK2Thresh) {
            if (pt == OMR_PIXELS_FLOAT) return launch_render_na<4, VEC, BE, false, OMR_PIXELS_FLOAT, kK2Thresh>(a, na, grid, small, s, cpt);
            if (pt == OMR_PIXELS_INT32) return launch_render_na<4, VEC, BE, true, OMR_PIXELS_INT32, kK2Thresh>(a, na, grid, small, s, cpt);
            return launch_render_na<4, VEC, BE, false, OMR_PIXELS_UINT32, kK2Thresh>(a, na, grid, small, s, cpt);
        }
        if (pt == OMR_PIXELS_FLOAT) return launch_render_na<4, VEC, BE, false, OMR_PIXELS_FLOAT, kK2Eval>(a, na, grid, small, s, cpt);
        if (pt == OMR_PIXELS_INT32) return launch_render_na<4, VEC, BE, true, OMR_PIXELS_INT32, kK2Eval>(a, na, grid, small, s, cpt);
        return launch_render_na<4, VEC, BE, false, OMR_PIXELS_UINT32, kK2Eval>(a, na, grid, small, s, cpt);
    } else {
        return launch_render_na<8, VEC, BE, false, OMR_PIXELS_DOUBLE, kK2Eval>(a, na, grid, small, s);
    }
}

template <int BPP, int VEC>
static hipError_t launch_render_be(const K2Args& a, int pt, bool be, int na, int mode16, int grid, bool small,
                                   hipStream_t s, int cpt) {
    return be ? launch_render_pt<BPP, VEC, true>(a, pt, na, mode16, grid, small, s, cpt)
              : launch_render_pt<BPP, VEC, false>(a, pt, na, mode16, grid, small, s, cpt);
}

// kK2Fast16 preconditions (see fast16): default codomain, increasing window, finite slope,
// and no integer x in the window with a0*(x - ws) == 0.49999999999999994 (Java's
// Math.round special case, where floor(d + 0.5) would differ).
static bool fast_linear_ok(const ChanParam& c, const RenderPlan& P) {
    if (P.sem & OMR_SEM_WINDOW_INT_BOUNDS) return false;   // the window may start below ws: d < 0 wraps
    if (P.cd_start != 0 || P.cd_end != 255 || c.second || !(c.we > c.ws) || !(c.a0 > 0) || !std::isfinite(c.a0))
        return false;
    const double x0 = std::floor(c.ws + 0.5 / c.a0);
    for (double x = x0 - 3; x <= x0 + 3; x += 1.0) {
        if (x < c.lo || x >= c.hi) continue;
        const double d = c.a0 * (x - c.ws);
        if (d == 0x1.fffffffffffffp-2) return false;
    }
    return true;
}

// fast16i on the host, operation for operation (the library builds with -ffp-contract=off)
static int host_fast16i(int64_t t, double a0) {
    const double e = a0 * (double)t + 0.5;
    if (!(e < 256.0)) return 255;                      // also covers e beyond the int range
    return e < 1.0 ? 0 : (int)e;                       // trunc, clamped below at 0
}

static int host_fast16f(int64_t t, float fa, float fb) {
    const float y = std::fmaf((float)t, fa, fb);       // correctly rounded, as v_fma_f32
    int32_t b;
    std::memcpy(&b, &y, 4);
    return std::min(std::max(b, kMagicBits), kMagicBits + 255) - kMagicBits;
}

bool fast16_f32_params(double a0, int64_t wsi, int32_t xmax, float* fa, float* fb) {
    if (!(a0 > 0) || !(a0 < 1e6) || wsi < -(1 << 23) || wsi > (1 << 23)) return false;
    // fast16i steps from k-1 to k at x = wsi + bp[k]: t = x - wsi over [tlo, thi]
    const int64_t tlo = -wsi, thi = (int64_t)xmax - wsi;
    int64_t bp[256];
    for (int k = 1; k <= 255; ++k) {
        // clamp in double before the conversion: a tiny a0 (a very wide window) puts the quotient
        // past 2^63, where the int64 conversion is undefined
        const double q = std::ceil((k - 0.5) / a0);
        int64_t t = (int64_t)std::max<double>((double)tlo, std::min<double>((double)(thi + 1), q));
        while (t > tlo && host_fast16i(t - 1, a0) >= k) --t;
        while (t <= thi && host_fast16i(t, a0) < k) ++t;
        bp[k] = t;                                     // thi + 1: level k is never reached
    }
    // both functions are non-decreasing in t, so agreeing on both sides of every step means
    // agreeing everywhere
    const float B = 12582912.0f;                       // kMagicBits
    auto exact = [&](float A) {
        for (int k = 1; k <= 255; ++k) {
            const int64_t b = bp[k];
            if (b <= thi && host_fast16f(b, A, B) < k) return false;
            if (b > tlo && host_fast16f(b - 1, A, B) >= k) return false;
        }
        return true;
    };
    const float A0 = (float)a0;
    for (int da = 0; da < 17; ++da) {                  // A0, +1, -1, ..., +8, -8 ulps
        float A = A0;
        for (int i = 0; i < (da + 1) / 2; ++i) A = std::nextafterf(A, (da & 1) ? INFINITY : 0.0f);
        if (A > 0 && exact(A)) { *fa = A; *fb = B; return true; }
    }
    return false;
}

static void type_bounds(int32_t t, double& lo, double& hi) {
    switch (t) {
    case OMR_PIXELS_INT8: lo = -128; hi = 127; break;
    case OMR_PIXELS_UINT8: lo = 0; hi = 255; break;
    case OMR_PIXELS_INT16: lo = -32768; hi = 32767; break;
    case OMR_PIXELS_UINT16: lo = 0; hi = 65535; break;
    default: lo = 0; hi = 0; break;
    }
}

// Enqueue K1 + K2 for a batch whose plane pointer table is already on the device.
struct Strided {
    const void* base;
    int64_t tile_stride, chan_stride;   // bytes
};

static omr_status enqueue_render(Ctx* ctx, PreparedPlan& pp, int32_t pixel_type, int32_t big_endian,
                                 const void* const* d_plane_ptrs, int32_t size_c, int32_t n_tiles,
                                 int64_t row_stride, int32_t width, int32_t height, int32_t flip_h,
                                 int32_t flip_v, uint32_t* d_out, int32_t* d_status, bool aligned,
                                 const RenderLayout& L, const Strided* strided = nullptr,
                                 const void* ptr_src = nullptr, size_t ptr_bytes = 0) {
    // ptr_bytes > 0: the host plane-pointer table ptr_src goes to d_plane_ptrs in the same
    // staging launch as the plan
    uint8_t* ws = static_cast<uint8_t*>(ctx->ws);
    RenderPlan* d_plan = reinterpret_cast<RenderPlan*>(ws + L.plan_off);
    uint32_t* d_contrib = reinterpret_cast<uint32_t*>(ws + L.contrib_off);
    const int na = pp.plan.n_active;
    bool use_thresh = false;
    for (int i = 0; i < na; ++i) use_thresh |= pp.plan.ch[i].mode == kModeThresh;
    uint32_t* d_thresh = reinterpret_cast<uint32_t*>(ws + L.thresh_off);
    uint32_t* d_buckets = reinterpret_cast<uint32_t*>(ws + L.bucket_off);
    std::vector<uint32_t> thr;
    if (use_thresh) {                               // the code thresholds, on the host (exact)
        thr.assign((size_t)na * 256, 0u);
        for (int i = 0; i < na; ++i)
            if (pp.plan.ch[i].mode == kModeThresh)
                host_thresholds(pp.plan.ch[i], pixel_type, pp.plan.cd_start, pp.plan.cd_end, thr.data() + 256 * i);
    }
    const bool thr_with_plan = use_thresh && !(ptr_src && ptr_bytes);   // one staging launch for both
    omr_status st = thr_with_plan
                        ? stage_h2d2(ctx, d_plan, &pp.plan, pp.plan_bytes, d_thresh, thr.data(), thr.size() * 4)
                        : stage_h2d2(ctx, d_plan, &pp.plan, pp.plan_bytes, const_cast<const void**>(d_plane_ptrs),
                                     ptr_src, ptr_src ? ptr_bytes : 0);
    if (st != OMR_OK) return st;
    if (use_thresh && !thr_with_plan && (st = stage_h2d(ctx, d_thresh, thr.data(), thr.size() * 4))) return st;
    const int bpp = bytes_per_pixel(pixel_type);
    const int vec = aligned ? (bpp <= 2 ? 8 : 16 / bpp) : 1;
    const uint64_t cpr = (uint64_t)width / vec;
    const uint64_t cpt = cpr * (uint64_t)height;
    const uint64_t total = cpt * (uint64_t)n_tiles;
    // one chunk per thread for launches too small to fill the chip (launch_render_na); those
    // K2 instantiations (1..4 active channels) build the contribution tables in LDS themselves
    const bool small = bpp <= 2 && k2_small_launch(total, ctx->cu_count);
    const bool k2_builds_contrib = small && na >= 1 && na <= 4;
    if (na > 0) {
        if (!k2_builds_contrib) {
            hipLaunchKernelGGL(k_build_contrib, dim3(na), dim3(256), 0, ctx->stream, d_plan, d_contrib,
                               pixel_type == OMR_PIXELS_INT8 ? 1 : 0);
            OMR_HIP(ctx, hipGetLastError());
        }
    }
    if (use_thresh) {
        hipLaunchKernelGGL(k_build_buckets, dim3(k2_launch_buckets(na) / 256, na), dim3(256), 0,
                           ctx->stream, d_plan, d_thresh, d_buckets, k2_launch_buckets(na));
        OMR_HIP(ctx, hipGetLastError());
    }
    if (total == 0) return OMR_OK;
    if (total >= (1ull << 31)) return fail(ctx, OMR_INVALID_ARGUMENT, "batch too large for one launch");
    K2Args a;
    std::memset(&a, 0, sizeof(a));
    a.plan = d_plan;
    a.planes = d_plane_ptrs;
    if (strided) {
        a.strided = 1;
        a.sbase = static_cast<const uint8_t*>(strided->base);
        a.tile_stride = strided->tile_stride;
        a.chan_stride = strided->chan_stride;
    }
    a.contrib = d_contrib;
    a.thresh = d_thresh;
    a.buckets = d_buckets;
    a.bk_n = k2_launch_buckets(na);
    a.use_thresh = use_thresh ? 1 : 0;
    a.out = d_out;
    a.status = d_status;
    a.flag = ctx->d_flag;
    a.row_stride = row_stride;
    a.size_c = size_c;
    a.n_tiles = n_tiles;
    a.width = width;
    a.height = height;
    a.flip_h = flip_h ? 1 : 0;
    a.flip_v = flip_v ? 1 : 0;
    a.n_active = na;
    a.cd_start = pp.plan.cd_start;
    a.cd_end = pp.plan.cd_end;
    a.cds8 = pp.plan.cd_start & 0xFF;
    a.cde8 = pp.plan.cd_end & 0xFF;
    // chunks per lane: kCPT (the float / 32-bit vector path: the context's k2_eval_cpt), 1 for
    // small launches and the runtime-channel-count kernels
    // (negative: the software-pipelined float kernel, k_render_pipe, at |cpt| chunks)
    const int cpt_sel = (na >= 1 && na <= 4 && !small) ? (bpp == 4 && aligned ? ctx->k2_eval_cpt : kCPT) : 1;
    const int cpt_thread = cpt_sel == -3 ? 1 : cpt_sel < 0 ? -cpt_sel : cpt_sel;   // -3: one chunk, two blocks per WG
    a.tile_uniform = (cpt % ((uint64_t)kBlock * cpt_thread)) == 0 ? 1 : 0;
    a.nt_store = ctx->k2_nt_store ? 1 : 0;
    a.total = (uint32_t)total;
    a.cpt = make_fastdiv((uint32_t)cpt);
    a.cpr = make_fastdiv((uint32_t)cpr);
    bool all_linear = true, all_fast = true;
    double tlo, thi;
    type_bounds(pixel_type, tlo, thi);
    for (int i = 0; i < na; ++i) {
        const ChanParam& c = pp.plan.ch[i];
        K2Chan& k = a.ch[i];
        k.index = c.index;
        k.mode = c.mode;
        k.lo = c.lo;
        k.hi = c.hi;
        k.gmin = c.gmin;
        k.gmax = c.gmax;
        k.check = (bpp <= 2 && (c.gmin > tlo || c.gmax < thi)) ? 1 : 0;
        k.second = c.second;
        k.ws = c.ws;
        k.a0 = c.a0;
        k.a1 = c.a1;
        k.lut_addr = c.lut_addr;
        if (c.mode != kModeLinear16) all_linear = false;
        if (!(c.mode == kModeLinear16 && fast_linear_ok(c, pp.plan))) all_fast = false;
    }
    bool all_thresh = na > 0;
    for (int i = 0; i < na; ++i) all_thresh &= pp.plan.ch[i].mode == kModeThresh;
    const int mode16 = bpp == 4 ? (all_thresh ? kK2Thresh : kK2Eval)
                                : all_fast ? kK2Fast16 : all_linear ? kK2Linear16 : kK2Mixed16;
    const uint64_t per_block = (uint64_t)kBlock * cpt_thread;
    a.n_work = (uint32_t)((total + per_block - 1) / per_block);
    const bool eval_mode = bpp >= 4;     // kK2Eval: grid-stride over the work blocks
    // resident blocks per CU: 8 (2 per SIMD), fewer when the LDS tables (160 KiB per CU) allow fewer
    const uint64_t k2_res = std::min<uint64_t>(8, (160u * 1024u) / k2_lds_bytes(na > 0 ? na : 1, a.use_thresh != 0, a.bk_n));
    const int grid = eval_mode ? (int)std::min<uint64_t>(a.n_work, (uint64_t)ctx->cu_count * k2_res) : (int)a.n_work;
    hipError_t e;
    const bool be = big_endian != 0;
    KernelTimer timer(ctx, 2, true);      // K2's one launch stamps its own events (hipExtLaunchKernel)
    tl_cu_count = ctx->cu_count;
    if (aligned) {
        switch (bpp) {
        case 1: e = launch_render_be<1, 8>(a, pixel_type, be, na, mode16, grid, small, ctx->stream, cpt_thread); break;
        case 2: e = launch_render_be<2, 8>(a, pixel_type, be, na, mode16, grid, small, ctx->stream, cpt_thread); break;
        case 4: e = launch_render_be<4, 4>(a, pixel_type, be, na, mode16, grid, small, ctx->stream, cpt_sel); break;
        default: e = launch_render_be<8, 2>(a, pixel_type, be, na, mode16, grid, small, ctx->stream, cpt_thread); break;
        }
    } else {
        switch (bpp) {
        case 1: e = launch_render_be<1, 1>(a, pixel_type, be, na, mode16, grid, small, ctx->stream, cpt_thread); break;
        case 2: e = launch_render_be<2, 1>(a, pixel_type, be, na, mode16, grid, small, ctx->stream, cpt_thread); break;
        case 4: e = launch_render_be<4, 1>(a, pixel_type, be, na, mode16, grid, small, ctx->stream, cpt_thread); break;
        default: e = launch_render_be<8, 1>(a, pixel_type, be, na, mode16, grid, small, ctx->stream, cpt_thread); break;
        }
    }
    OMR_HIP(ctx, e);
    return OMR_OK;
}

// ---- fused render -> JPEG (omr_k2.h): the plan and K1 of a render, K2 left to the caller
struct FusedPlanBuf {
    PreparedPlan pp;
    RenderLayout L;
    int32_t pixel_type = 0;
    int32_t mode = 0;
};

FusedPlanBuf* fused_plan_new() { return new FusedPlanBuf(); }
void fused_plan_free(FusedPlanBuf* fp) { delete fp; }
size_t render_fused_ws_bytes(const FusedPlanBuf* fp) { return fp->L.total; }

static bool fused_from_prepared(FusedPlanBuf* fp, int32_t pixel_type) {
    const int bpp = bytes_per_pixel(pixel_type);
    const int na = fp->pp.plan.n_active;
    if (bpp > 2 || na < 1 || na > kFusedMaxActive) return false;
    fp->pixel_type = pixel_type;
    fp->L = layout_for(fp->pp, 0);
    bool all_linear = true, all_fast = true;
    for (int i = 0; i < na; ++i) {
        const ChanParam& c = fp->pp.plan.ch[i];
        if (c.mode != kModeLinear16) all_linear = false;
        if (!(c.mode == kModeLinear16 && fast_linear_ok(c, fp->pp.plan))) all_fast = false;
    }
    fp->mode = bpp == 1 ? kFusedTable8 : all_fast ? kFusedFast16 : all_linear ? kFusedLinear16 : kFusedMixed16;
    return true;
}

bool render_fused_plan(Ctx* ctx, const omr_quantum_def* q, const omr_channel_binding* ch, int32_t size_c,
                       int32_t pixel_type, FusedPlanBuf* fp, omr_status* st) {
    *st = prepare_plan(ctx, q, ch, size_c, pixel_type, fp->pp);
    if (*st) return false;
    // int16: the fused JPEG kernel reads pixels biased to unsigned (x + 32768) and takes
    // ws + 32768, which must be exact so that (x + 32768) - (ws + 32768) rounds like x - ws
    for (int i = 0; i < fp->pp.plan.n_active; ++i) {
        const double ws = fp->pp.plan.ch[i].ws;
        if (pixel_type == OMR_PIXELS_INT16 && (ws + 32768.0) - 32768.0 != ws) return false;
    }
    return fused_from_prepared(fp, pixel_type);
}

omr_status render_fused_stage(Ctx* ctx, FusedPlanBuf* fp, size_t ws_off, FusedRender& F, bool build_contrib,
                              bool bias_int16) {
    PreparedPlan& pp = fp->pp;
    const RenderLayout& L = fp->L;
    uint8_t* ws = static_cast<uint8_t*>(ctx->ws) + ws_off;
    RenderPlan* d_plan = reinterpret_cast<RenderPlan*>(ws + L.plan_off);
    uint32_t* d_contrib = reinterpret_cast<uint32_t*>(ws + L.contrib_off);
    const int na = pp.plan.n_active;
    omr_status st = stage_h2d(ctx, d_plan, &pp.plan, pp.plan_bytes);
    if (st) return st;
    if (build_contrib) {
        hipLaunchKernelGGL(k_build_contrib, dim3(na), dim3(256), 0, ctx->stream, d_plan, d_contrib,
                           fp->pixel_type == OMR_PIXELS_INT8 ? 1 : 0);
        OMR_HIP(ctx, hipGetLastError());
    }
    std::memset(&F, 0, sizeof(F));
    double tlo, thi;
    type_bounds(fp->pixel_type, tlo, thi);
    // int16 with bias_int16 (the fused JPEG kernel): pixels are read biased to unsigned, so every
    // pixel-domain parameter moves by 32768 with them (x - ws, x - gmin and the compares are
    // unchanged; render_fused_plan checked that ws + 32768 is exact)
    const int bias = bias_int16 && fp->pixel_type == OMR_PIXELS_INT16 ? 32768 : 0;
    for (int i = 0; i < na; ++i) {
        const ChanParam& c = pp.plan.ch[i];
        K2Chan& k = F.ch[i];
        k.index = c.index;
        k.mode = c.mode;
        // saturating: a window end at +-inf / NaN / beyond 2^31 is already clamped to INT32_MAX / MIN
        auto sat = [](int64_t v) { return (int32_t)std::min<int64_t>(std::max<int64_t>(v, INT32_MIN), INT32_MAX); };
        k.lo = sat((int64_t)c.lo + bias);
        k.hi = sat((int64_t)c.hi + bias);
        // the biased LUT domain is compared with u16 pixels: clamp it to one step beyond the
        // int16 range first, so that + 32768 cannot overflow and the compares are unchanged
        k.gmin = bias ? (int32_t)std::min<int64_t>(std::max<int64_t>(c.gmin, -32768), 32768) + bias : c.gmin;
        k.gmax = bias ? (int32_t)std::min<int64_t>(std::max<int64_t>(c.gmax, -32769), 32767) + bias : c.gmax;
        k.check = (c.gmin > tlo || c.gmax < thi) ? 1 : 0;
        F.any_check |= k.check;
        {
            const int64_t dl = std::max<int64_t>(k.gmin, 0), dh = std::min<int64_t>(k.gmax, 65535);
            if (k.check && dl > dh) F.dnone = 1;
            const uint32_t l = (uint32_t)std::min<int64_t>(dl, 65535), h = (uint32_t)std::max<int64_t>(dh, 0);
            F.dlo2[i] = l | (l << 16);
            F.dhi2[i] = h | (h << 16);
        }
        const bool wint = c.ws == std::floor(c.ws) && std::fabs(c.ws) < 1073741824.0;
        F.ws_int = (i == 0 ? 1 : F.ws_int) & (wint ? 1 : 0);
        k.second = c.second;
        k.ws = c.ws + (double)bias;
        k.wsi = wint ? (int32_t)k.ws : 0;
        k.a0 = c.a0;
        k.a1 = c.a1;
        k.lut_addr = c.lut_addr;
    }
    // The fused JPEG kernel (bias_int16), Fast16 with integral window starts: the f32 form where
    // it is proven exact for every pixel value (16-bit pixels: x in [0, 65535] after the bias)
    if (bias_int16 && fp->mode == kFusedFast16 && F.ws_int && ctx->f1_f32) {
        F.f32 = 1;
        for (int i = 0; i < na && F.f32; ++i)
            F.f32 = fast16_f32_params(F.ch[i].a0, F.ch[i].wsi, 65535, &F.fa[i], &F.fb[i]) ? 1 : 0;
        for (int i = 0; i < na && F.f32; ++i) F.fc[i] = (float)((int64_t)(1 << 23) + F.ch[i].wsi);
    }
    F.contrib = d_contrib;
    F.plan = d_plan;
    F.flag = ctx->d_flag;
    F.n_active = na;
    F.mode = fp->mode;
    F.cd_start = pp.plan.cd_start;
    F.cds8 = pp.plan.cd_start & 0xFF;
    F.cde8 = pp.plan.cd_end & 0xFF;
    F.is_signed = fp->pixel_type == OMR_PIXELS_INT8 || fp->pixel_type == OMR_PIXELS_INT16;
    // grey MCUs: the greyscale model renders (v, v, v) unless a .lut colours it (OMR_SEM_GREYSCALE_LUT);
    // the rgb model only when every channel's colour has r == g == b and no .lut
    F.grey_ok = 1;
    for (int i = 0; i < na; ++i) {
        const ChanParam& c = pp.plan.ch[i];
        const bool lut = c.has_lut && (!pp.plan.greyscale || (pp.plan.sem & OMR_SEM_GREYSCALE_LUT));
        const bool grey_colour = pp.plan.greyscale || (c.ratio[0] == c.ratio[1] && c.ratio[1] == c.ratio[2] &&
                                                       c.cratio[0] == c.cratio[1] && c.cratio[1] == c.cratio[2]);
        if (lut || !grey_colour) F.grey_ok = 0;
    }
    return OMR_OK;
}

static bool vec_aligned(int bpp, int32_t width, int64_t row_stride) {
    const int vec = bpp <= 2 ? 8 : 16 / bpp;
    return width % vec == 0 && row_stride % vec == 0;
}

static omr_status check_dims(Ctx* ctx, int32_t width, int32_t height, int32_t flip_h, int32_t flip_v,
                             int64_t& row_stride) {
    if (width < 0 || height < 0) return fail(ctx, OMR_INVALID_ARGUMENT, "negative region size");
    if ((flip_h || flip_v) && (width == 0 || height == 0))
        return fail(ctx, OMR_INVALID_ARGUMENT, "Attempted to flip image with 0 size");
    if (row_stride == 0) row_stride = width;
    if (row_stride < width) return fail(ctx, OMR_INVALID_ARGUMENT, "row stride smaller than width");
    return OMR_OK;
}

}  // namespace omr

using namespace omr;

extern "C" {

omr_status omr_render_batch_device(omr_ctx* ctx, const omr_quantum_def* qdef,
                                   const omr_channel_binding* channels, int32_t size_c,
                                   const void* const* d_plane_ptrs, int32_t n_tiles,
                                   int64_t row_stride, int32_t pixel_type, int32_t big_endian,
                                   int32_t width, int32_t height, int32_t flip_h, int32_t flip_v,
                                   uint32_t* d_argb_out, int32_t* d_status) {
    if (!ctx) return OMR_INVALID_ARGUMENT;
    if (n_tiles < 0) return fail(ctx, OMR_INVALID_ARGUMENT, "negative tile count");
    omr_status st = check_dims(ctx, width, height, flip_h, flip_v, row_stride);
    if (st) return st;
    PreparedPlan pp;
    st = prepare_plan(ctx, qdef, channels, size_c, pixel_type, pp);
    if (st) return st;
    if (n_tiles == 0 || width == 0 || height == 0) return OMR_OK;
    if (pp.plan.n_active > 0 && !d_plane_ptrs) return fail(ctx, OMR_INVALID_ARGUMENT, "null plane table");
    if (!d_argb_out) return fail(ctx, OMR_INVALID_ARGUMENT, "null output");
    OMR_HIP(ctx, hipSetDevice(ctx->device));
    const RenderLayout L = layout_for(pp, 0);
    st = ensure_workspace(ctx, L.total);
    if (st) return st;
    if (d_status) OMR_HIP(ctx, hipMemsetAsync(d_status, 0, sizeof(int32_t) * (size_t)n_tiles, ctx->stream));
    const int bpp = bytes_per_pixel(pixel_type);
    // the plane pointers live on the device: 16-B alignment is the caller's contract (omr.h); the
    // output is checked here (its 16-B vector stores fall back to scalar ones when misaligned)
    const bool aligned = vec_aligned(bpp, width, row_stride) && reinterpret_cast<uintptr_t>(d_argb_out) % 16 == 0;
    return enqueue_render(ctx, pp, pixel_type, big_endian, d_plane_ptrs, size_c, n_tiles, row_stride,
                          width, height, flip_h, flip_v, d_argb_out, d_status, aligned, L);
}

omr_status omr_render_batch_strided_device(omr_ctx* ctx, const omr_quantum_def* qdef,
                                           const omr_channel_binding* channels, int32_t size_c,
                                           const void* d_base, int64_t tile_stride_bytes,
                                           int64_t channel_stride_bytes, int32_t n_tiles,
                                           int64_t row_stride, int32_t pixel_type, int32_t big_endian,
                                           int32_t width, int32_t height, int32_t flip_h, int32_t flip_v,
                                           uint32_t* d_argb_out, int32_t* d_status) {
    if (!ctx) return OMR_INVALID_ARGUMENT;
    if (n_tiles < 0) return fail(ctx, OMR_INVALID_ARGUMENT, "negative tile count");
    omr_status st = check_dims(ctx, width, height, flip_h, flip_v, row_stride);
    if (st) return st;
    PreparedPlan pp;
    st = prepare_plan(ctx, qdef, channels, size_c, pixel_type, pp);
    if (st) return st;
    if (n_tiles == 0 || width == 0 || height == 0) return OMR_OK;
    if (pp.plan.n_active > 0 && !d_base) return fail(ctx, OMR_INVALID_ARGUMENT, "null batch base");
    if (!d_argb_out) return fail(ctx, OMR_INVALID_ARGUMENT, "null output");
    OMR_HIP(ctx, hipSetDevice(ctx->device));
    const RenderLayout L = layout_for(pp, 0);
    st = ensure_workspace(ctx, L.total);
    if (st) return st;
    if (d_status) OMR_HIP(ctx, hipMemsetAsync(d_status, 0, sizeof(int32_t) * (size_t)n_tiles, ctx->stream));
    const int bpp = bytes_per_pixel(pixel_type);
    const bool aligned = vec_aligned(bpp, width, row_stride) && reinterpret_cast<uintptr_t>(d_base) % 16 == 0 &&
                         tile_stride_bytes % 16 == 0 && channel_stride_bytes % 16 == 0 &&
                         reinterpret_cast<uintptr_t>(d_argb_out) % 16 == 0;
    const Strided sd{d_base, tile_stride_bytes, channel_stride_bytes};
    return enqueue_render(ctx, pp, pixel_type, big_endian, nullptr, size_c, n_tiles, row_stride, width, height,
                          flip_h, flip_v, d_argb_out, d_status, aligned, L, &sd);
}

omr_status omr_render_packed_int_device(omr_ctx* ctx, const omr_quantum_def* qdef,
                                        const omr_channel_binding* channels, int32_t size_c,
                                        const void* const* d_planes, int64_t row_stride,
                                        int32_t pixel_type, int32_t big_endian, int32_t width,
                                        int32_t height, int32_t flip_h, int32_t flip_v,
                                        uint32_t* d_argb_out) {
    if (!ctx) return OMR_INVALID_ARGUMENT;
    omr_status st = check_dims(ctx, width, height, flip_h, flip_v, row_stride);
    if (st) return st;
    PreparedPlan pp;
    st = prepare_plan(ctx, qdef, channels, size_c, pixel_type, pp);
    if (st) return st;
    if (width == 0 || height == 0) return OMR_OK;
    for (int a = 0; a < pp.plan.n_active; ++a)
        if (!d_planes || !d_planes[pp.plan.ch[a].index]) return fail(ctx, OMR_INVALID_ARGUMENT, "null plane for active channel");
    if (!d_argb_out) return fail(ctx, OMR_INVALID_ARGUMENT, "null output");
    OMR_HIP(ctx, hipSetDevice(ctx->device));
    const size_t ptr_bytes = sizeof(void*) * (size_t)(size_c > 0 ? size_c : 1);
    const RenderLayout L = layout_for(pp, align_up(ptr_bytes, 256));
    st = ensure_workspace(ctx, L.total);
    if (st) return st;
    const void** d_ptrs = reinterpret_cast<const void**>(static_cast<uint8_t*>(ctx->ws) + L.extra_off);
    std::vector<const void*> ptrs(size_c > 0 ? size_c : 1, nullptr);
    for (int c = 0; c < size_c; ++c) ptrs[c] = d_planes ? d_planes[c] : nullptr;
    const int bpp = bytes_per_pixel(pixel_type);
    bool aligned = vec_aligned(bpp, width, row_stride);
    for (int c = 0; c < size_c && aligned; ++c)
        if (ptrs[c] && (reinterpret_cast<uintptr_t>(ptrs[c]) % 16)) aligned = false;
    if (reinterpret_cast<uintptr_t>(d_argb_out) % 16) aligned = false;
    return enqueue_render(ctx, pp, pixel_type, big_endian, d_ptrs, size_c, 1, row_stride, width, height,
                          flip_h, flip_v, d_argb_out, nullptr, aligned, L, nullptr, ptrs.data(),
                          sizeof(void*) * ptrs.size());
}

omr_status omr_render_packed_int(omr_ctx* ctx, const omr_quantum_def* qdef,
                                 const omr_channel_binding* channels, int32_t size_c,
                                 const void* const* planes, int64_t row_stride, int32_t pixel_type,
                                 int32_t big_endian, int32_t width, int32_t height, int32_t flip_h,
                                 int32_t flip_v, uint32_t* argb_out) {
    if (!ctx) return OMR_INVALID_ARGUMENT;
    omr_status st = check_dims(ctx, width, height, flip_h, flip_v, row_stride);
    if (st) return st;
    PreparedPlan pp;
    st = prepare_plan(ctx, qdef, channels, size_c, pixel_type, pp);
    if (st) return st;
    if (width == 0 || height == 0) return OMR_OK;
    for (int a = 0; a < pp.plan.n_active; ++a)
        if (!planes || !planes[pp.plan.ch[a].index]) return fail(ctx, OMR_INVALID_ARGUMENT, "null plane for active channel");
    if (!argb_out) return fail(ctx, OMR_INVALID_ARGUMENT, "null output");
    OMR_HIP(ctx, hipSetDevice(ctx->device));
    const int bpp = bytes_per_pixel(pixel_type);
    const size_t plane_bytes = align_up((size_t)width * height * bpp, 256);
    const size_t out_bytes = align_up((size_t)width * height * 4, 256);
    const size_t ptr_bytes = align_up(sizeof(void*) * (size_t)(size_c > 0 ? size_c : 1), 256);
    const int na = pp.plan.n_active;
    const RenderLayout L = layout_for(pp, ptr_bytes + plane_bytes * (size_t)na + out_bytes);
    st = ensure_workspace(ctx, L.total);
    if (st) return st;
    uint8_t* ws = static_cast<uint8_t*>(ctx->ws);
    const void** d_ptrs = reinterpret_cast<const void**>(ws + L.extra_off);
    uint8_t* d_planes = ws + L.extra_off + ptr_bytes;
    uint32_t* d_out = reinterpret_cast<uint32_t*>(d_planes + plane_bytes * (size_t)na);
    std::vector<const void*> ptrs(size_c > 0 ? size_c : 1, nullptr);
    for (int a = 0; a < na; ++a) {
        const int c = pp.plan.ch[a].index;
        uint8_t* dst = d_planes + plane_bytes * (size_t)a;
        ptrs[c] = dst;
        OMR_HIP(ctx, hipMemcpy2DAsync(dst, (size_t)width * bpp, planes[c], (size_t)row_stride * bpp,
                                      (size_t)width * bpp, height, hipMemcpyHostToDevice, ctx->stream));
    }
    st = enqueue_render(ctx, pp, pixel_type, big_endian, d_ptrs, size_c, 1, width, width, height, flip_h,
                        flip_v, d_out, nullptr, vec_aligned(bpp, width, width), L, nullptr, ptrs.data(),
                        sizeof(void*) * ptrs.size());
    if (st) return st;
    OMR_HIP(ctx, hipMemcpyAsync(argb_out, d_out, (size_t)width * height * 4, hipMemcpyDeviceToHost, ctx->stream));
    return omr_ctx_synchronize(ctx);
}

}  // extern "C"

extern "C" omr_status omr_render_projected_device(
    omr_ctx* ctx, const omr_quantum_def* qdef, const omr_channel_binding* channels, int32_t size_c,
    const void* const* d_stacks, int32_t pixel_type, int32_t big_endian, int32_t size_x, int32_t size_y,
    int32_t size_z, int32_t algorithm, int32_t start, int32_t end, int32_t stepping, int32_t flip_h,
    int32_t flip_v, uint32_t* d_argb_out) {
    // ImageRegionRequestHandler.java:506-559: project every active channel (full plane, the
    // tile/region is dropped, :556-557), then render the projected planes at z=0,t=0.
    if (!ctx) return OMR_INVALID_ARGUMENT;
    omr_status st = validate_projection_args(ctx, pixel_type, size_x, size_y, size_z, algorithm, start, end, stepping);
    if (st) return st;
    int64_t row_stride = size_x;
    st = check_dims(ctx, size_x, size_y, flip_h, flip_v, row_stride);
    if (st) return st;
    PreparedPlan pp;
    st = prepare_plan(ctx, qdef, channels, size_c, pixel_type, pp);
    if (st) return st;
    if (size_x == 0 || size_y == 0) return OMR_OK;
    const int na = pp.plan.n_active;
    for (int a = 0; a < na; ++a)
        if (!d_stacks || !d_stacks[pp.plan.ch[a].index]) return fail(ctx, OMR_INVALID_ARGUMENT, "null stack for active channel");
    if (!(ctx->sem & OMR_SEM_PROJECTION_ALL_ACTIVE)) {
        // :507-555: the projected buffer holds sizeC = #active channels but is read at each rendered
        // channel's original index (Appendix B quirk 3) -> the buffer's bounds check fails
        int projected_size_c = 0;
        for (int c = 0; c < size_c; ++c) projected_size_c += channels[c].active ? 1 : 0;
        for (int a = 0; a < na; ++a)
            if (pp.plan.ch[a].index >= projected_size_c)
                return fail(ctx, OMR_INTERNAL, "DimensionsOutOfBoundsException: C '" +
                                                   std::to_string(pp.plan.ch[a].index) + "' greater than sizeC '" +
                                                   std::to_string(projected_size_c) + "'");
    }
    if (!d_argb_out) return fail(ctx, OMR_INVALID_ARGUMENT, "null output");
    OMR_HIP(ctx, hipSetDevice(ctx->device));
    const int bpp = bytes_per_pixel(pixel_type);
    if (ctx->k3r && na >= 1 && na <= kFusedMaxActive && bpp <= 2 && (size_x * (int64_t)size_y * bpp) % 16 == 0 &&
        reinterpret_cast<uintptr_t>(d_argb_out) % 4 == 0) {
        // K3R: project + render in one kernel (the projected planes never reach HBM); the
        // contribution tables are built by K3R itself from the staged plan (no K1 launch)
        FusedPlanBuf fp;
        fp.pp = pp;
        if (fused_from_prepared(&fp, pixel_type)) {
            const void* st_ptrs[kFusedMaxActive] = {};
            bool aligned = true;
            for (int a = 0; a < na; ++a) {
                st_ptrs[a] = d_stacks[fp.pp.plan.ch[a].index];
                aligned &= reinterpret_cast<uintptr_t>(st_ptrs[a]) % 16 == 0;
            }
            if (aligned && (bpp == 2 || algorithm == OMR_PROJECTION_MAX)) {
                st = ensure_workspace(ctx, render_fused_ws_bytes(&fp));
                if (st) return st;
                FusedRender R;
                st = render_fused_stage(ctx, &fp, 0, R, /*build_contrib=*/false);
                if (st) return st;
                bool done = false;
                st = enqueue_project_render(ctx, st_ptrs, R, pixel_type, big_endian, size_x, size_y, algorithm, start,
                                            end, stepping, flip_h, flip_v, d_argb_out, &done);
                if (st || done) return st;    // else (too many planes summed): K3 + K2 below
            }
        }
    }
    const size_t plane_bytes = align_up((size_t)size_x * size_y * bpp, 256);
    const size_t ptr_bytes = align_up(sizeof(void*) * (size_t)(size_c > 0 ? size_c : 1), 256);
    const RenderLayout L = layout_for(pp, ptr_bytes + plane_bytes * (size_t)na);
    st = ensure_workspace(ctx, L.total);
    if (st) return st;
    uint8_t* ws = static_cast<uint8_t*>(ctx->ws);
    const void** d_ptrs = reinterpret_cast<const void**>(ws + L.extra_off);
    uint8_t* d_planes = ws + L.extra_off + ptr_bytes;
    std::vector<const void*> ptrs(size_c > 0 ? size_c : 1, nullptr);
    std::vector<const void*> srcs;
    std::vector<void*> dsts;
    for (int a = 0; a < na; ++a) {
        const int c = pp.plan.ch[a].index;
        uint8_t* dst = d_planes + plane_bytes * (size_t)a;
        ptrs[c] = dst;
        srcs.push_back(d_stacks[c]);
        dsts.push_back(dst);
    }
    for (size_t i = 0; i < srcs.size(); i += 32) {
        const int n = (int)std::min<size_t>(32, srcs.size() - i);
        st = enqueue_projection(ctx, srcs.data() + i, dsts.data() + i, n, pixel_type, big_endian, size_x,
                                size_y, algorithm, start, end, stepping, 0);
        if (st) return st;
    }
    const bool aligned = vec_aligned(bpp, size_x, size_x) && (reinterpret_cast<uintptr_t>(d_argb_out) % 16 == 0);
    return enqueue_render(ctx, pp, pixel_type, 0, d_ptrs, size_c, 1, size_x, size_x, size_y, flip_h, flip_v,
                          d_argb_out, nullptr, aligned, L, nullptr, ptrs.data(), sizeof(void*) * ptrs.size());
}

// Test hook (not part of omr.h): the F1 f32 quantize parameters, for the host-side exhaustive
// check in tests/test_f32_quantize.py.
extern "C" int32_t omr_debug_fast16_f32_params(double a0, int64_t wsi, int32_t xmax, float* fa, float* fb) {
    return omr::fast16_f32_params(a0, wsi, xmax, fa, fb) ? 1 : 0;
}
