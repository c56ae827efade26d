// omr_project.hip — K3 Z-projection and the standalone flip kernels.
//
// K3 replaces ProjectionService.projectStack (ProjectionService.java:46-120) with
// projectStackMax (:176-199) and projectStackMeanOrSum (:259-291).  Each lane owns a
// 16-byte column chunk of the XY plane and walks z with several loads in flight, so the
// Z-stack streams through HBM exactly once (coalesced rows; no transposition).
// The flips replace ImageRegionRequestHandler.flip (:616-642) and
// ShapeMaskRequestHandler.flip (:128-154) for callers holding an already-rendered buffer.
#include "omr_device.h"
#include "omr_k2.h"

namespace omr {

constexpr int kMaxStacks = 32;

struct K3Args {
    const uint8_t* stacks[kMaxStacks];
    uint8_t* outs[kMaxStacks];
    int32_t n_stacks;
    int32_t start, end, stepping;
    int64_t plane;        // pixels per plane
    uint32_t chunks;      // chunks per plane
    // exact unsigned division by the mean's plane count (Granlund-Montgomery, any 32-bit
    // numerator): q = (t + ((n - t) >> s1)) >> s2, t = umulhi(m, n)
    uint32_t div_m, div_s1, div_s2;
};

// Granlund-Montgomery constants of unsigned division by d (1 <= d < 2^31).
static inline void set_udiv(K3Args& a, uint32_t d) {
    uint32_t l = 0;
    while (l < 32 && (1ull << l) < d) ++l;
    a.div_m = (uint32_t)((((1ull << 32) * ((1ull << l) - d)) / d) + 1);
    a.div_s1 = l ? 1u : 0u;
    a.div_s2 = l ? l - 1 : 0u;
}

__device__ __forceinline__ uint32_t udiv_inv(uint32_t n, const K3Args& a) {
    const uint32_t t = __umulhi(a.div_m, n);
    return (t + ((n - t) >> a.div_s1)) >> a.div_s2;
}

template <typename T> struct Raw;
template <> struct Raw<int8_t> { using U = uint8_t; };
template <> struct Raw<uint8_t> { using U = uint8_t; };
template <> struct Raw<int16_t> { using U = uint16_t; };
template <> struct Raw<uint16_t> { using U = uint16_t; };
template <> struct Raw<int32_t> { using U = uint32_t; };
template <> struct Raw<uint32_t> { using U = uint32_t; };
template <> struct Raw<float> { using U = uint32_t; };
template <> struct Raw<double> { using U = uint64_t; };

template <typename U>
__device__ __forceinline__ U bswap_any(U v) {
    if constexpr (sizeof(U) == 1) return v;
    else if constexpr (sizeof(U) == 2) return (U)(((v & 0xFF) << 8) | (v >> 8));
    else if constexpr (sizeof(U) == 4) return bswap32(v);
    else return ((uint64_t)bswap32((uint32_t)v) << 32) | bswap32((uint32_t)(v >> 32));
}

template <typename T, bool BE>
__device__ __forceinline__ T load_px(const uint8_t* p) {
    using U = typename Raw<T>::U;
    U u = *reinterpret_cast<const U*>(p);
    if constexpr (BE) u = bswap_any<U>(u);
    T t;
    __builtin_memcpy(&t, &u, sizeof(T));
    return t;
}

template <typename T, bool BE>
__device__ __forceinline__ void store_px(uint8_t* p, T t) {
    using U = typename Raw<T>::U;
    U u;
    __builtin_memcpy(&u, &t, sizeof(T));
    if constexpr (BE) u = bswap_any<U>(u);
    *reinterpret_cast<U*>(p) = u;
}

template <typename T> __device__ __forceinline__ double type_max() {
    if constexpr (std::is_same<T, int8_t>::value) return 127.0;
    else if constexpr (std::is_same<T, uint8_t>::value) return 255.0;
    else if constexpr (std::is_same<T, int16_t>::value) return 32767.0;
    else if constexpr (std::is_same<T, uint16_t>::value) return 65535.0;
    else if constexpr (std::is_same<T, int32_t>::value) return 2147483647.0;
    else if constexpr (std::is_same<T, uint32_t>::value) return 4294967295.0;
    else if constexpr (std::is_same<T, float>::value) return 3.4028234663852886e38;
    else return 1.7976931348623157e308;
}

__device__ __forceinline__ int32_t java_d2i(double d) {
    if (d != d) return 0;
    if (d >= 2147483647.0) return INT32_MAX;
    if (d <= -2147483648.0) return INT32_MIN;
    return (int32_t)d;
}
__device__ __forceinline__ int64_t java_d2l(double d) {
    if (d != d) return 0;
    if (d >= 9223372036854775807.0) return INT64_MAX;
    if (d <= -9223372036854775808.0) return INT64_MIN;
    return (int64_t)d;
}

// PixelData.setPixelValue narrowing (S9 in oracle/omr_oracle.c).
template <typename T> __device__ __forceinline__ T narrow(double v) {
    if constexpr (std::is_same<T, float>::value) return (float)v;
    else if constexpr (std::is_same<T, double>::value) return v;
    else if constexpr (std::is_same<T, uint32_t>::value) return (uint32_t)java_d2l(v);
    else return (T)java_d2i(v);
}

// Accumulator: exact integer sum for integer types (== Java's double sum, every partial
// sum < 2^53), double for float types (same order as the reference loop).
template <typename T> struct Acc { using type = double; };
template <> struct Acc<int8_t> { using type = int64_t; };
template <> struct Acc<uint8_t> { using type = int64_t; };
template <> struct Acc<int16_t> { using type = int64_t; };
template <> struct Acc<uint16_t> { using type = int64_t; };
template <> struct Acc<int32_t> { using type = int64_t; };
template <> struct Acc<uint32_t> { using type = int64_t; };

template <typename T, bool BEI, bool BEO, int ALG>
__global__ void __launch_bounds__(kBlock) k_project(K3Args A) {
    constexpr int V = sizeof(T) >= 8 ? 2 : 16 / (int)sizeof(T);   // pixels per lane (16 B)
    const int s = blockIdx.y;
    const uint8_t* __restrict__ stack = A.stacks[s];
    uint8_t* __restrict__ out = A.outs[s];
    const int64_t plane_bytes = A.plane * (int64_t)sizeof(T);
    for (uint32_t c = blockIdx.x * kBlock + threadIdx.x; c < A.chunks; c += gridDim.x * kBlock) {
        const int64_t px0 = (int64_t)c * V;
        const int nv = (int)min<int64_t>(V, A.plane - px0);
        if (ALG == OMR_PROJECTION_MAX) {
            T best[V];
#pragma unroll
            for (int j = 0; j < V; ++j) best[j] = (T)0;
            const uint8_t* p = stack + (int64_t)A.start * plane_bytes + px0 * (int64_t)sizeof(T);
            const int64_t step = plane_bytes * A.stepping;
            if (nv == V) {
                int z = A.start;
#pragma unroll 4
                for (; z <= A.end; z += A.stepping, p += step) {
#pragma unroll
                    for (int j = 0; j < V; ++j) {
                        const T v = load_px<T, BEI>(p + j * sizeof(T));
                        if (v > best[j]) best[j] = v;   // stackValue > projectedValue (:187)
                    }
                }
            } else {
                for (int z = A.start; z <= A.end; z += A.stepping, p += step)
                    for (int j = 0; j < nv; ++j) {
                        const T v = load_px<T, BEI>(p + j * sizeof(T));
                        if (v > best[j]) best[j] = v;
                    }
            }
            for (int j = 0; j < nv; ++j) store_px<T, BEO>(out + (px0 + j) * sizeof(T), best[j]);
        } else {
            using AT = typename Acc<T>::type;
            AT sum[V];
#pragma unroll
            for (int j = 0; j < V; ++j) sum[j] = 0;
            int count = 0;
            const uint8_t* p = stack + (int64_t)A.start * plane_bytes + px0 * (int64_t)sizeof(T);
            const int64_t step = plane_bytes * A.stepping;
            if (nv == V) {
#pragma unroll 4
                for (int z = A.start; z < A.end; z += A.stepping, p += step) {
#pragma unroll
                    for (int j = 0; j < V; ++j) sum[j] += (AT)load_px<T, BEI>(p + j * sizeof(T));
                    ++count;
                }
            } else {
                for (int z = A.start; z < A.end; z += A.stepping, p += step) {
                    for (int j = 0; j < nv; ++j) sum[j] += (AT)load_px<T, BEI>(p + j * sizeof(T));
                    ++count;
                }
            }
            const double pmax = type_max<T>();
            for (int j = 0; j < nv; ++j) {
                double v = (double)sum[j];
                if (ALG == OMR_PROJECTION_MEAN) v = v / (double)count;
                if (v > pmax) v = pmax;
                store_px<T, BEO>(out + (px0 + j) * sizeof(T), narrow<T>(v));
            }
        }
    }
}

// K3v: 16-byte vector loads (one per lane per plane) when the stack is 16-B aligned and a plane
// is a whole number of 16-B chunks.  SPLIT: the 4 waves of a block take consecutive quarters of
// the z range for the same 64 chunks and combine through LDS in z order — legal where the
// combine is exact: max (order-free, NaN skipped, +0 start) and integer sums (int64, exact).
// Float / double mean and sum keep one lane per chunk walking every z in the reference order.
#define OMR_GLOBAL __attribute__((address_space(1)))
typedef uint32_t p32x4 __attribute__((ext_vector_type(4)));
template <typename T> struct VecPx {
    using U = typename Raw<T>::U;
    static constexpr int V = 16 / (int)sizeof(T);
    static __device__ __forceinline__ void split(const p32x4& q, U (&u)[V]) {
        __builtin_memcpy(&u[0], &q, 16);
    }
};

template <typename T, bool BE>
__device__ __forceinline__ T px_of(typename Raw<T>::U u) {
    if constexpr (BE) u = bswap_any<typename Raw<T>::U>(u);
    T t;
    __builtin_memcpy(&t, &u, sizeof(T));
    return t;
}

// 32-bit sums for 8/16-bit types when at most 65535 planes are summed: exact (65535 x 65535 <
// 2^32, 65535 x 32768 < 2^31), and one add per pixel instead of a 64-bit add pair.
template <typename T> struct Acc32 { using type = typename Acc<T>::type; };
template <> struct Acc32<int8_t> { using type = int32_t; };
template <> struct Acc32<uint8_t> { using type = uint32_t; };
template <> struct Acc32<int16_t> { using type = int32_t; };
template <> struct Acc32<uint16_t> { using type = uint32_t; };
constexpr uint32_t kAcc32MaxPlanes = 65535;

template <typename T, bool BEI, bool BEO, int ALG, bool SPLIT, bool NARROW = false>
__global__ void __launch_bounds__(kBlock) k_project_v(K3Args A, uint32_t n_iter) {
    using U = typename Raw<T>::U;
    using AT = typename std::conditional<NARROW, typename Acc32<T>::type, typename Acc<T>::type>::type;
    constexpr int V = VecPx<T>::V;
    constexpr bool MAX = ALG == OMR_PROJECTION_MAX;
    using Part = typename std::conditional<MAX, T, AT>::type;
    __shared__ Part s_part[SPLIT ? 3 * 64 * V : 1];
    const int s = blockIdx.y;
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63u;
    const uint32_t c = SPLIT ? blockIdx.x * 64 + lane : blockIdx.x * kBlock + threadIdx.x;
    const bool live = c < A.chunks;
    const uint32_t cc = live ? c : A.chunks - 1;
    const OMR_GLOBAL p32x4* base = (const OMR_GLOBAL p32x4*)(const void*)(A.stacks[s]) + cc;
    const uint64_t pchunks = (uint64_t)A.chunks * (uint64_t)A.stepping;   // uint4s between used planes
    const uint32_t i0 = SPLIT ? (uint32_t)((uint64_t)n_iter * wave / 4) : 0u;
    const uint32_t i1 = SPLIT ? (uint32_t)((uint64_t)n_iter * (wave + 1) / 4) : n_iter;
    Part acc[V];
#pragma unroll
    for (int j = 0; j < V; ++j) acc[j] = (Part)0;
    const OMR_GLOBAL p32x4* p = base + ((uint64_t)A.start + 0) * A.chunks + (uint64_t)i0 * pchunks;
    uint32_t i = i0;
    auto fold = [&](const p32x4 q) {
        U u[V];
        VecPx<T>::split(q, u);
#pragma unroll
        for (int j = 0; j < V; ++j) {
            const T v = px_of<T, BEI>(u[j]);
            if constexpr (MAX) { if (v > acc[j]) acc[j] = v; }   // stackValue > projectedValue (:187)
            else acc[j] += (Part)v;
        }
    };
    // 8 independent 16-B loads in flight (16 measured slower on C3: 124 VGPRs, 4 waves per SIMD)
    for (; i + 8 <= i1; i += 8, p += 8 * pchunks) {
        p32x4 q[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) q[u] = __builtin_nontemporal_load(p + u * pchunks);   // read once
#pragma unroll
        for (int u = 0; u < 8; ++u) fold(q[u]);
    }
    if (i < i1) {
        // the remainder (< 8 planes) as one batch of loads too: planes past i1 re-read the last
        // one (a cache hit) and are not folded.  One load at a time here made the z split's
        // wave with the remainder (the mean's 63 planes: 15 / 16 / 16 / 16) hold its workgroup
        const uint32_t rem = i1 - i;
        p32x4 q[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) q[u] = __builtin_nontemporal_load(p + (uint64_t)min((uint32_t)u, rem - 1) * pchunks);
#pragma unroll
        for (int u = 0; u < 8; ++u)
            if ((uint32_t)u < rem) fold(q[u]);
    }
    if constexpr (SPLIT) {
        if (wave > 0) {
#pragma unroll
            for (int j = 0; j < V; ++j) s_part[((wave - 1) * 64 + lane) * V + j] = acc[j];
        }
        __syncthreads();
        if (wave > 0) return;
#pragma unroll
        for (int w = 0; w < 3; ++w)
#pragma unroll
            for (int j = 0; j < V; ++j) {
                const Part v = s_part[(w * 64 + lane) * V + j];
                if constexpr (MAX) { if (v > acc[j]) acc[j] = v; }
                else acc[j] += v;
            }
    }
    if (!live) return;
    U o[V];
#pragma unroll
    for (int j = 0; j < V; ++j) {
        T t;
        if constexpr (MAX) {
            t = acc[j];
        } else if constexpr (NARROW && ALG == OMR_PROJECTION_MEAN) {
            // (int)(sum / (double)n) == the integer quotient toward zero: |sum| < 2^32, n < 2^16,
            // so the double quotient's error (< 2^-21) never crosses an integer the true
            // quotient is >= 1/n away from; the mean of in-range values is in range
            const int64_t sv = (int64_t)acc[j];
            const uint32_t q = udiv_inv((uint32_t)(sv < 0 ? -sv : sv), A);
            t = (T)(sv < 0 ? -(int64_t)q : (int64_t)q);
        } else {
            double v = (double)acc[j];
            if (ALG == OMR_PROJECTION_MEAN) v = v / (double)n_iter;
            if (v > type_max<T>()) v = type_max<T>();
            t = narrow<T>(v);
        }
        U u;
        __builtin_memcpy(&u, &t, sizeof(T));
        if constexpr (BEO) u = bswap_any<U>(u);
        o[j] = u;
    }
    p32x4 q;
    __builtin_memcpy(&q, o, 16);
    ((OMR_GLOBAL p32x4*)(void*)(A.outs[s]))[c] = q;
}

// K3R: the projection glue (ImageRegionRequestHandler.java:506-559) in one kernel — every active
// channel's stack projected and the projected pixel rendered (quantize, codomain, colour,
// composite, flip) without the projected planes going through HBM.  A workgroup owns 64 16-byte
// chunks (512 pixels at 16 bits) of the plane for every channel; its 4 waves take consecutive
// quarters of the z range (exact: max is order-free, integer sums are exact), combine through
// LDS, and each thread then narrows (PixelData.setPixelValue, as K3 stores), quantizes (K2's
// helpers and contribution tables) and composites 2 pixels.
struct K3RArgs {
    const uint8_t* stacks[kFusedMaxActive];   // per active channel (plan order)
    uint32_t* out;
    FusedRender R;
    int32_t start, stepping, width, height, flip_h, flip_v, mean;
    uint32_t chunks, n_iter;
    FastDiv ndiv;         // n_iter (mean: exact integer quotient, see below)
};

constexpr int kK3RChunks = 32;   // 16-B chunks per workgroup (256 pixels at 16 bits)
constexpr int kK3RParts = 8;     // z parts per workgroup: 4 waves x 2 half-waves

template <typename T, bool BEI, bool MAX, bool FAST>
__global__ void __launch_bounds__(kBlock) k_project_render(K3RArgs A) {
    using U = typename Raw<T>::U;
    constexpr int V = VecPx<T>::V;                      // 8 (16-bit) or 16 (8-bit) pixels per chunk
    constexpr int NPX = kK3RChunks * V;                 // pixels per workgroup
    using Part = typename std::conditional<MAX, T, typename Acc32<T>::type>::type;
    __shared__ Part s_part[kK3RParts][kFusedMaxActive][NPX];
    __shared__ uint32_t s_contrib[kFusedMaxActive * 256];
    const int na = A.R.n_active;
    for (int i = threadIdx.x; i < na * 256; i += kBlock)     // K1's tables, built here (no K1 launch)
        s_contrib[i] = contrib_entry(A.R.plan, i >> 8, i & 255, std::is_same<T, int8_t>::value ? 1 : 0);
    // lane l of wave w: chunk (l & 31) of the workgroup's 32, z part 2w + (l >> 5) of 8
    const uint32_t lane = threadIdx.x & 63u, part = (threadIdx.x >> 6) * 2 + (lane >> 5), ch = lane & 31u;
    const uint32_t c = blockIdx.x * kK3RChunks + ch;
    const uint32_t cc = min(c, A.chunks - 1);
    const uint64_t pchunks = (uint64_t)A.chunks * (uint64_t)A.stepping;
    const uint32_t i0 = (uint32_t)((uint64_t)A.n_iter * part / kK3RParts);
    const uint32_t i1 = (uint32_t)((uint64_t)A.n_iter * (part + 1) / kK3RParts);
#pragma unroll
    for (int a = 0; a < kFusedMaxActive; ++a) {
        if (a >= na) break;                                         // uniform
        Part acc[V];
#pragma unroll
        for (int j = 0; j < V; ++j) acc[j] = (Part)0;
        const OMR_GLOBAL p32x4* p = (const OMR_GLOBAL p32x4*)(const void*)(A.stacks[a]) + cc +
                                    (uint64_t)A.start * A.chunks + (uint64_t)i0 * pchunks;
        auto fold = [&](const p32x4 q) {
            U u[V];
            VecPx<T>::split(q, u);
#pragma unroll
            for (int j = 0; j < V; ++j) {
                const T v = px_of<T, BEI>(u[j]);
                if constexpr (MAX) { if (v > acc[j]) acc[j] = v; }   // stackValue > projectedValue (:187)
                else acc[j] += (Part)v;
            }
        };
        uint32_t i = i0;
        for (; i + 8 <= i1; i += 8, p += 8 * pchunks) {
            p32x4 q[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) q[k] = __builtin_nontemporal_load(p + k * pchunks);
#pragma unroll
            for (int k = 0; k < 8; ++k) fold(q[k]);
        }
        if (i < i1) {                   // the remainder (< 8 planes) as one batch, as K3 does
            const uint32_t rem = i1 - i;
            p32x4 q[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) q[k] = __builtin_nontemporal_load(p + (uint64_t)min((uint32_t)k, rem - 1) * pchunks);
#pragma unroll
            for (int k = 0; k < 8; ++k)
                if ((uint32_t)k < rem) fold(q[k]);
        }
#pragma unroll
        for (int j = 0; j < V; ++j) s_part[part][a][ch * V + j] = acc[j];
    }
    __syncthreads();
    // thread t renders pixel t (16-bit: 256 per workgroup; 8-bit: 512, two per thread)
    const uint64_t plane = (uint64_t)A.chunks * V;
#pragma unroll
    for (int rep = 0; rep < NPX / kBlock; ++rep) {
        const uint32_t lp = rep * kBlock + threadIdx.x;
        const uint64_t px = (uint64_t)blockIdx.x * NPX + lp;
        if (px >= plane) break;
        uint32_t accp = 0;
        bool err = false;
#pragma unroll
        for (int a = 0; a < kFusedMaxActive; ++a) {
            if (a >= na) break;
            const K2Chan& k = A.R.ch[a];
            T t;
            if constexpr (MAX) {
                Part m = s_part[0][a][lp];
#pragma unroll
                for (int w = 1; w < kK3RParts; ++w) { const Part v = s_part[w][a][lp]; if (v > m) m = v; }
                t = m;
            } else {
                // sum as double, mean = sum / count, clamp at the type max, (int) narrowing
                // (ProjectionService.java:268-288): with |sum| < 2^31 and count <= 32767 the
                // double quotient never rounds up across an integer (the gap to the next one is
                // >= 1/count >> its ulp), so the truncated quotient is the integer quotient
                // toward zero; sums below the 16-bit minimum wrap in the short cast as in Java.
                Part sum = s_part[0][a][lp];
#pragma unroll
                for (int w = 1; w < kK3RParts; ++w) sum += s_part[w][a][lp];
                int32_t v = (int32_t)sum;
                if (A.mean) {
                    const uint32_t m = (uint32_t)(v < 0 ? -v : v);
                    const int32_t q = (int32_t)fdiv(m, A.ndiv);
                    v = v < 0 ? -q : q;
                }
                v = min(v, (int32_t)type_max<T>());
                t = (T)v;                                            // setPixelValue (Java narrowing)
            }
            uint32_t e;
            const uint32_t* tab = s_contrib + a * 256;
            if constexpr (sizeof(T) == 1) {                         // Table8: indexed by the raw byte
                e = tab[(uint8_t)t];
                err |= (e & kErrBit) != 0;
                e &= ~kErrBit;
            } else {
                const int x = (int)t;
                if (k.check) err |= (x < k.gmin) | (x > k.gmax);
                uint32_t v;
                if constexpr (FAST) {
                    v = fast16(x, k);
                } else if (k.mode == kModeLinear16) {
                    v = linear16(x, k, A.R.cd_start, A.R.cds8, A.R.cde8);
                } else {
                    const int xi = min(max(x, k.gmin), k.gmax);
                    v = reinterpret_cast<const uint8_t*>(k.lut_addr)[(uint32_t)(xi - k.gmin)];
                }
                e = tab[v];
            }
            accp += e;
        }
        if (__ballot(err)) {
            if (err) atomicOr(A.R.flag, 1);
        }
        const uint32_t f = clamp_fields(accp);
        const uint32_t o = 0xFF000000u | ((f >> 4) & 0xFF0000u) | ((f >> 2) & 0xFF00u) | (f & 0xFFu);
        const uint32_t row = (uint32_t)(px / (uint64_t)A.width), col = (uint32_t)(px - (uint64_t)row * A.width);
        const uint32_t orow = A.flip_v ? (uint32_t)A.height - 1 - row : row;
        const uint32_t ocol = A.flip_h ? (uint32_t)A.width - 1 - col : col;
        A.out[(uint64_t)orow * A.width + ocol] = o;
    }
}

template <typename T, bool BEI>
static hipError_t launch_project_render_t(const K3RArgs& a, bool max, bool fast, dim3 g, hipStream_t s) {
    if constexpr (sizeof(T) == 1) {          // 8-bit: max only (their 32-bit partial sums exceed LDS)
        hipLaunchKernelGGL((k_project_render<T, BEI, true, false>), g, dim3(kBlock), 0, s, a);
        return hipGetLastError();
    }
    if (max) {
        if (fast) hipLaunchKernelGGL((k_project_render<T, BEI, true, true>), g, dim3(kBlock), 0, s, a);
        else hipLaunchKernelGGL((k_project_render<T, BEI, true, false>), g, dim3(kBlock), 0, s, a);
    } else {
        if (fast) hipLaunchKernelGGL((k_project_render<T, BEI, false, true>), g, dim3(kBlock), 0, s, a);
        else hipLaunchKernelGGL((k_project_render<T, BEI, false, false>), g, dim3(kBlock), 0, s, a);
    }
    return hipGetLastError();
}

// The fused glue when it applies (8/16-bit integer stacks, 1..4 rendered channels, 16-B aligned
// stacks holding whole 16-B chunks per plane, even width, 8-B aligned output): *done = true.
omr_status enqueue_project_render(Ctx* ctx, const void* const* stacks, const FusedRender& R, int32_t pixel_type,
                                  int32_t be_in, int32_t size_x, int32_t size_y, int32_t algorithm, int32_t start,
                                  int32_t end, int32_t stepping, int32_t flip_h, int32_t flip_v, uint32_t* d_out,
                                  bool* done) {
    *done = false;
    const int bpp = bytes_per_pixel(pixel_type);
    const int64_t plane = (int64_t)size_x * size_y;
    if (bpp > 2 || R.n_active < 1 || R.n_active > kFusedMaxActive || plane == 0) return OMR_OK;
    if (bpp == 1 && algorithm != OMR_PROJECTION_MAX) return OMR_OK;
    if ((plane * bpp) % 16 || reinterpret_cast<uintptr_t>(d_out) % 4) return OMR_OK;
    for (int a = 0; a < R.n_active; ++a)
        if (!stacks[a] || reinterpret_cast<uintptr_t>(stacks[a]) % 16) return OMR_OK;
    uint32_t n_iter;
    if (algorithm == OMR_PROJECTION_MAX) n_iter = end >= start ? (uint32_t)((end - start) / stepping + 1) : 0u;
    else n_iter = end > start ? (uint32_t)((end - start + stepping - 1) / stepping) : 0u;
    if (n_iter > 32767 || (algorithm != OMR_PROJECTION_MAX && n_iter == 0)) return OMR_OK;   // |sum| < 2^31
    K3RArgs a;
    std::memset(&a, 0, sizeof(a));
    for (int i = 0; i < R.n_active; ++i) a.stacks[i] = static_cast<const uint8_t*>(stacks[i]);
    a.out = d_out;
    a.R = R;
    a.start = start;
    a.stepping = stepping;
    a.width = size_x;
    a.height = size_y;
    a.flip_h = flip_h ? 1 : 0;
    a.flip_v = flip_v ? 1 : 0;
    a.mean = algorithm == OMR_PROJECTION_MEAN ? 1 : 0;
    a.chunks = (uint32_t)(plane * bpp / 16);
    a.n_iter = n_iter;
    a.ndiv = make_fastdiv(n_iter ? n_iter : 1);
    const dim3 g((a.chunks + kK3RChunks - 1) / kK3RChunks);
    const bool mx = algorithm == OMR_PROJECTION_MAX, fast = R.mode == kFusedFast16, be = be_in != 0;
    hipError_t e;
    KernelTimer timer(ctx, 3);
    switch (pixel_type) {
    case OMR_PIXELS_INT8: e = launch_project_render_t<int8_t, false>(a, mx, false, g, ctx->stream); break;
    case OMR_PIXELS_UINT8: e = launch_project_render_t<uint8_t, false>(a, mx, false, g, ctx->stream); break;
    case OMR_PIXELS_INT16:
        e = be ? launch_project_render_t<int16_t, true>(a, mx, fast, g, ctx->stream)
               : launch_project_render_t<int16_t, false>(a, mx, fast, g, ctx->stream);
        break;
    default:
        e = be ? launch_project_render_t<uint16_t, true>(a, mx, fast, g, ctx->stream)
               : launch_project_render_t<uint16_t, false>(a, mx, fast, g, ctx->stream);
        break;
    }
    OMR_HIP(ctx, e);
    *done = true;
    return OMR_OK;
}

template <typename T>
static bool narrow_ok(uint32_t n_iter) {
    return sizeof(T) <= 2 && !std::is_floating_point<T>::value && n_iter <= kAcc32MaxPlanes;
}

template <typename T, bool BEI, bool BEO>
static hipError_t launch_project_v(const K3Args& a, int alg, uint32_t n_iter, bool split, uint32_t chunks16,
                                   int n, hipStream_t s) {
    const dim3 gs((chunks16 + 63) / 64, n), g1((chunks16 + kBlock - 1) / kBlock, n);
    switch (alg) {
    case OMR_PROJECTION_MAX:
        omr_launch((k_project_v<T, BEI, BEO, OMR_PROJECTION_MAX, true>), gs, dim3(kBlock), 0, s, a, n_iter);
        break;
    case OMR_PROJECTION_MEAN:
        if (split && narrow_ok<T>(n_iter)) omr_launch((k_project_v<T, BEI, BEO, OMR_PROJECTION_MEAN, true, true>), gs, dim3(kBlock), 0, s, a, n_iter);
        else if (split) omr_launch((k_project_v<T, BEI, BEO, OMR_PROJECTION_MEAN, true>), gs, dim3(kBlock), 0, s, a, n_iter);
        else omr_launch((k_project_v<T, BEI, BEO, OMR_PROJECTION_MEAN, false>), g1, dim3(kBlock), 0, s, a, n_iter);
        break;
    default:
        if (split && narrow_ok<T>(n_iter)) omr_launch((k_project_v<T, BEI, BEO, OMR_PROJECTION_SUM, true, true>), gs, dim3(kBlock), 0, s, a, n_iter);
        else if (split) omr_launch((k_project_v<T, BEI, BEO, OMR_PROJECTION_SUM, true>), gs, dim3(kBlock), 0, s, a, n_iter);
        else omr_launch((k_project_v<T, BEI, BEO, OMR_PROJECTION_SUM, false>), g1, dim3(kBlock), 0, s, a, n_iter);
        break;
    }
    return hipGetLastError();
}

template <typename T>
static hipError_t launch_project_vt(const K3Args& a, int alg, bool bei, bool beo, uint32_t n_iter, uint32_t chunks16,
                                    int n, hipStream_t s) {
    const bool split = alg == OMR_PROJECTION_MAX || !std::is_floating_point<T>::value;
    if (bei) return beo ? launch_project_v<T, true, true>(a, alg, n_iter, split, chunks16, n, s)
                        : launch_project_v<T, true, false>(a, alg, n_iter, split, chunks16, n, s);
    return beo ? launch_project_v<T, false, true>(a, alg, n_iter, split, chunks16, n, s)
               : launch_project_v<T, false, false>(a, alg, n_iter, split, chunks16, n, s);
}

template <typename T, bool BEI, bool BEO>
static hipError_t launch_project_alg(const K3Args& a, int alg, dim3 grid, hipStream_t s) {
    switch (alg) {
    case OMR_PROJECTION_MAX: hipLaunchKernelGGL((k_project<T, BEI, BEO, OMR_PROJECTION_MAX>), grid, dim3(kBlock), 0, s, a); break;
    case OMR_PROJECTION_MEAN: hipLaunchKernelGGL((k_project<T, BEI, BEO, OMR_PROJECTION_MEAN>), grid, dim3(kBlock), 0, s, a); break;
    default: hipLaunchKernelGGL((k_project<T, BEI, BEO, OMR_PROJECTION_SUM>), grid, dim3(kBlock), 0, s, a); break;
    }
    return hipGetLastError();
}

template <typename T>
static hipError_t launch_project_t(const K3Args& a, int alg, bool bei, bool beo, dim3 grid, hipStream_t s) {
    if (bei) return beo ? launch_project_alg<T, true, true>(a, alg, grid, s) : launch_project_alg<T, true, false>(a, alg, grid, s);
    return beo ? launch_project_alg<T, false, true>(a, alg, grid, s) : launch_project_alg<T, false, false>(a, alg, grid, s);
}

// Validation exactly as ProjectionService.java:53-64 / :154-161 / :140-144 / :88-90.
static omr_status validate_projection(Ctx* ctx, int32_t pixel_type, int32_t size_x, int32_t size_y,
                                      int32_t size_z, int32_t algorithm, int32_t start, int32_t end,
                                      int32_t stepping) {
    if (!bytes_per_pixel(pixel_type)) return fail(ctx, OMR_INVALID_ARGUMENT, "unsupported pixel type");
    if (size_x < 0 || size_y < 0 || size_z <= 0) return fail(ctx, OMR_INVALID_ARGUMENT, "bad stack dimensions");
    if (start < 0 || end < 0) return fail(ctx, OMR_INVALID_ARGUMENT, "Z interval value cannot be negative.");
    if (start >= size_z || end >= size_z)
        return fail(ctx, OMR_INVALID_ARGUMENT, "Z interval value cannot be >= " + std::to_string(size_z));
    if (stepping <= 0) return fail(ctx, OMR_INVALID_ARGUMENT, "stepping: " + std::to_string(stepping) + " <= 0");
    if (algorithm < OMR_PROJECTION_MAX || algorithm > OMR_PROJECTION_SUM)
        return fail(ctx, OMR_INVALID_ARGUMENT, "Unknown algorithm: " + std::to_string(algorithm));
    return OMR_OK;
}

omr_status enqueue_projection(Ctx* ctx, const void* const* d_stacks, void* const* d_outs, int n,
                              int32_t pixel_type, int32_t be_in, int32_t size_x, int32_t size_y,
                              int32_t algorithm, int32_t start, int32_t end, int32_t stepping,
                              int32_t be_out) {
    if (n <= 0) return OMR_OK;
    if (n > kMaxStacks) return fail(ctx, OMR_INVALID_ARGUMENT, "more than 32 stacks per launch");
    K3Args a;
    std::memset(&a, 0, sizeof(a));
    for (int i = 0; i < n; ++i) {
        a.stacks[i] = static_cast<const uint8_t*>(d_stacks[i]);
        a.outs[i] = static_cast<uint8_t*>(d_outs[i]);
    }
    a.n_stacks = n;
    a.start = start;
    a.end = end;
    a.stepping = stepping;
    a.plane = (int64_t)size_x * size_y;
    if (a.plane == 0) return OMR_OK;
    const int bpp = bytes_per_pixel(pixel_type);
    const int v = bpp >= 8 ? 2 : 16 / bpp;
    const int64_t chunks = (a.plane + v - 1) / v;
    if (chunks >= (1ll << 31)) return fail(ctx, OMR_INVALID_ARGUMENT, "plane too large");
    a.chunks = (uint32_t)chunks;
    const int64_t bx = std::min<int64_t>((chunks + kBlock - 1) / kBlock, (int64_t)ctx->cu_count * 8);
    const dim3 grid((unsigned)bx, (unsigned)n);
    const bool bi = be_in != 0, bo = be_out != 0;
    hipError_t e;
    KernelTimer timer(ctx, 3, true);       // the vector path's one launch stamps its own events
    // Vector path: every stack and output 16-B aligned, planes a whole number of 16-B chunks.
    bool vec = (a.plane * bpp) % 16 == 0;
    for (int i = 0; i < n && vec; ++i)
        vec = reinterpret_cast<uintptr_t>(a.stacks[i]) % 16 == 0 && reinterpret_cast<uintptr_t>(a.outs[i]) % 16 == 0;
    if (vec) {
        const uint32_t c16 = (uint32_t)(a.plane * bpp / 16);
        K3Args b = a;
        b.chunks = c16;
        // iterations: max over z in [start, end], mean/sum over z in [start, end) (ProjectionService.java:184, :271)
        uint32_t n_iter = 0;
        if (algorithm == OMR_PROJECTION_MAX) n_iter = end >= start ? (uint32_t)((end - start) / stepping + 1) : 0u;
        else n_iter = end > start ? (uint32_t)((end - start + stepping - 1) / stepping) : 0u;
        set_udiv(b, n_iter ? n_iter : 1u);
        switch (pixel_type) {
        case OMR_PIXELS_INT8: e = launch_project_vt<int8_t>(b, algorithm, bi, bo, n_iter, c16, n, ctx->stream); break;
        case OMR_PIXELS_UINT8: e = launch_project_vt<uint8_t>(b, algorithm, bi, bo, n_iter, c16, n, ctx->stream); break;
        case OMR_PIXELS_INT16: e = launch_project_vt<int16_t>(b, algorithm, bi, bo, n_iter, c16, n, ctx->stream); break;
        case OMR_PIXELS_UINT16: e = launch_project_vt<uint16_t>(b, algorithm, bi, bo, n_iter, c16, n, ctx->stream); break;
        case OMR_PIXELS_INT32: e = launch_project_vt<int32_t>(b, algorithm, bi, bo, n_iter, c16, n, ctx->stream); break;
        case OMR_PIXELS_UINT32: e = launch_project_vt<uint32_t>(b, algorithm, bi, bo, n_iter, c16, n, ctx->stream); break;
        case OMR_PIXELS_FLOAT: e = launch_project_vt<float>(b, algorithm, bi, bo, n_iter, c16, n, ctx->stream); break;
        default: e = launch_project_vt<double>(b, algorithm, bi, bo, n_iter, c16, n, ctx->stream); break;
        }
        OMR_HIP(ctx, e);
        return OMR_OK;
    }
    switch (pixel_type) {
    case OMR_PIXELS_INT8: e = launch_project_t<int8_t>(a, algorithm, bi, bo, grid, ctx->stream); break;
    case OMR_PIXELS_UINT8: e = launch_project_t<uint8_t>(a, algorithm, bi, bo, grid, ctx->stream); break;
    case OMR_PIXELS_INT16: e = launch_project_t<int16_t>(a, algorithm, bi, bo, grid, ctx->stream); break;
    case OMR_PIXELS_UINT16: e = launch_project_t<uint16_t>(a, algorithm, bi, bo, grid, ctx->stream); break;
    case OMR_PIXELS_INT32: e = launch_project_t<int32_t>(a, algorithm, bi, bo, grid, ctx->stream); break;
    case OMR_PIXELS_UINT32: e = launch_project_t<uint32_t>(a, algorithm, bi, bo, grid, ctx->stream); break;
    case OMR_PIXELS_FLOAT: e = launch_project_t<float>(a, algorithm, bi, bo, grid, ctx->stream); break;
    default: e = launch_project_t<double>(a, algorithm, bi, bo, grid, ctx->stream); break;
    }
    OMR_HIP(ctx, e);
    return OMR_OK;
}

omr_status validate_projection_args(Ctx* ctx, int32_t pixel_type, int32_t size_x, int32_t size_y,
                                    int32_t size_z, int32_t algorithm, int32_t start, int32_t end,
                                    int32_t stepping) {
    return validate_projection(ctx, pixel_type, size_x, size_y, size_z, algorithm, start, end, stepping);
}

// ------------------------------------------------------------------------------- flips
template <typename T>
__global__ void __launch_bounds__(kBlock) k_flip(const T* __restrict__ src, T* __restrict__ dst, int W,
                                                 int H, int fh, int fv, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock) {
        const int y = (int)(i / W), x = (int)(i - (int64_t)y * W);
        const int oy = fv ? H - 1 - y : y, ox = fh ? W - 1 - x : x;
        dst[(int64_t)oy * W + ox] = src[i];
    }
}

template <typename T>
static omr_status flip_device(Ctx* ctx, const T* src, T* dst, int32_t W, int32_t H, int32_t fh, int32_t fv) {
    if (!fh && !fv) {
        if (W > 0 && H > 0 && src && dst && src != dst)
            OMR_HIP(ctx, hipMemcpyAsync(dst, src, sizeof(T) * (size_t)W * H, hipMemcpyDeviceToDevice, ctx->stream));
        return OMR_OK;
    }
    if (!src) return fail(ctx, OMR_INVALID_ARGUMENT, "Attempted to flip null image");
    if (W == 0 || H == 0) return fail(ctx, OMR_INVALID_ARGUMENT, "Attempted to flip image with 0 size");
    if (W < 0 || H < 0 || !dst || src == dst) return fail(ctx, OMR_INVALID_ARGUMENT, "bad flip arguments");
    const int64_t n = (int64_t)W * H;
    const int grid = (int)std::min<int64_t>((n + kBlock - 1) / kBlock, (int64_t)ctx->cu_count * 8);
    hipLaunchKernelGGL(k_flip<T>, dim3(grid), dim3(kBlock), 0, ctx->stream, src, dst, W, H, fh ? 1 : 0, fv ? 1 : 0, n);
    OMR_HIP(ctx, hipGetLastError());
    return OMR_OK;
}

}  // namespace omr

using namespace omr;

extern "C" {

omr_status omr_flip_argb_device(omr_ctx* ctx, const uint32_t* d_src, uint32_t* d_dest, int32_t size_x,
                                int32_t size_y, int32_t flip_h, int32_t flip_v) {
    if (!ctx) return OMR_INVALID_ARGUMENT;
    return flip_device<uint32_t>(ctx, d_src, d_dest, size_x, size_y, flip_h, flip_v);
}

omr_status omr_flip_mask_device(omr_ctx* ctx, const uint8_t* d_src, uint8_t* d_dest, int32_t size_x,
                                int32_t size_y, int32_t flip_h, int32_t flip_v) {
    if (!ctx) return OMR_INVALID_ARGUMENT;
    return flip_device<uint8_t>(ctx, d_src, d_dest, size_x, size_y, flip_h, flip_v);
}

omr_status omr_project_stack_device(omr_ctx* ctx, const void* d_stack, int32_t pixel_type,
                                    int32_t big_endian_in, int32_t size_x, int32_t size_y,
                                    int32_t size_z, int32_t algorithm, int32_t start, int32_t end,
                                    int32_t stepping, void* d_plane_out, int32_t big_endian_out) {
    if (!ctx) return OMR_INVALID_ARGUMENT;
    omr_status st = validate_projection(ctx, pixel_type, size_x, size_y, size_z, algorithm, start, end, stepping);
    if (st) return st;
    if (!d_stack || !d_plane_out) return fail(ctx, OMR_INVALID_ARGUMENT, "null stack or output");
    OMR_HIP(ctx, hipSetDevice(ctx->device));
    const void* s[1] = {d_stack};
    void* o[1] = {d_plane_out};
    return enqueue_projection(ctx, s, o, 1, pixel_type, big_endian_in, size_x, size_y, algorithm, start,
                              end, stepping, big_endian_out);
}

omr_status omr_project_stacks_device(omr_ctx* ctx, const void* const* d_stacks, int32_t n_stacks, int32_t pixel_type,
                                     int32_t big_endian_in, int32_t size_x, int32_t size_y, int32_t size_z,
                                     int32_t algorithm, int32_t start, int32_t end, int32_t stepping,
                                     void* const* d_planes_out, int32_t big_endian_out) {
    if (!ctx) return OMR_INVALID_ARGUMENT;
    omr_status st = validate_projection(ctx, pixel_type, size_x, size_y, size_z, algorithm, start, end, stepping);
    if (st) return st;
    if (n_stacks < 0 || n_stacks > kMaxStacks) return fail(ctx, OMR_INVALID_ARGUMENT, "0..32 stacks per call");
    if (n_stacks && (!d_stacks || !d_planes_out)) return fail(ctx, OMR_INVALID_ARGUMENT, "null stack list");
    for (int i = 0; i < n_stacks; ++i)
        if (!d_stacks[i] || !d_planes_out[i]) return fail(ctx, OMR_INVALID_ARGUMENT, "null stack or output");
    OMR_HIP(ctx, hipSetDevice(ctx->device));
    return enqueue_projection(ctx, d_stacks, d_planes_out, n_stacks, pixel_type, big_endian_in, size_x, size_y,
                              algorithm, start, end, stepping, big_endian_out);
}

omr_status omr_project_stack(omr_ctx* ctx, const void* stack, int32_t pixel_type, int32_t big_endian_in,
                             int32_t size_x, int32_t size_y, int32_t size_z, int32_t algorithm,
                             int32_t start, int32_t end, int32_t stepping, void* plane_out,
                             int32_t big_endian_out) {
    if (!ctx) return OMR_INVALID_ARGUMENT;
    omr_status st = validate_projection(ctx, pixel_type, size_x, size_y, size_z, algorithm, start, end, stepping);
    if (st) return st;
    if (!stack || !plane_out) return fail(ctx, OMR_INVALID_ARGUMENT, "null stack or output");
    OMR_HIP(ctx, hipSetDevice(ctx->device));
    const int bpp = bytes_per_pixel(pixel_type);
    const size_t plane = (size_t)size_x * size_y * bpp;
    const size_t in_bytes = plane * size_z;
    st = ensure_workspace(ctx, align_up(in_bytes, 256) + align_up(plane, 256));
    if (st) return st;
    uint8_t* d_in = static_cast<uint8_t*>(ctx->ws);
    uint8_t* d_out = d_in + align_up(in_bytes, 256);
    OMR_HIP(ctx, hipMemcpyAsync(d_in, stack, in_bytes, hipMemcpyHostToDevice, ctx->stream));
    const void* s[1] = {d_in};
    void* o[1] = {d_out};
    st = enqueue_projection(ctx, s, o, 1, pixel_type, big_endian_in, size_x, size_y, algorithm, start, end,
                            stepping, big_endian_out);
    if (st) return st;
    OMR_HIP(ctx, hipMemcpyAsync(plane_out, d_out, plane, hipMemcpyDeviceToHost, ctx->stream));
    OMR_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return OMR_OK;
}

}  // extern "C"
