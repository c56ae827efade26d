// omr_device.h — device helpers shared by the kernels: Java numeric semantics,
// family maps, pixel decoding.  Compiled with -ffp-contract=off so every double
// expression rounds exactly like the CPU restatement (oracle/omr_oracle.c).
#pragma once

#include "omr_internal.h"

namespace omr {

// Java Math.round(double) (JDK 8): floor(a + 0.5) with the 0.49999999999999994 case,
// then (long) conversion (NaN -> 0, saturating).
__host__ __device__ __forceinline__ int64_t java_round_d(double a) {
    if (a == 0x1.fffffffffffffp-2) return 0;
    const double f = floor(a + 0.5);
    if (f != f) return 0;
    if (f >= 9223372036854775807.0) return INT64_MAX;
    if (f <= -9223372036854775808.0) return INT64_MIN;
    return (int64_t)f;
}

// Family maps (SEMANTICS TABLE S2 in oracle/omr_oracle.c) of a channel.
__host__ __device__ __forceinline__ double family_map(const ChanParam& p, double x) {
    return family_map_code(p.family, x, p.k, p.ws, p.we);
}

// q(x) of an integer pixel (the LUT types): window, noise reduction, family map, two rounding
// stages (S3/S4).  The window ends are the integer thresholds p.lo / p.hi the host derived from
// the double window under the OMR_SEM_WINDOW_INT_BOUNDS choice (x < ws <=> x < ceil(ws) for
// integer x by default; x < (int)ws with the switch).
__host__ __device__ __forceinline__ int quantize_eval(double x, const ChanParam& p, int cds, int cde) {
    if (x < (double)p.lo) return cds & 0xFF;
    if (x >= (double)p.hi) return cde & 0xFF;
    if (p.nr) {
        if (x < p.ws + p.dec) return cds & 0xFF;
        if (x >= p.we - p.dec) return cde & 0xFF;
    }
    const double v = (double)java_round_d(p.a0 * (family_map(p, x) - p.ys));
    return (int)(java_round_d(p.a1 * v + (double)cds) & 0xFF);
}

// Swap bytes inside each 16-bit half (big-endian u16 pair -> native).
__device__ __forceinline__ uint32_t bswap16x2(uint32_t d) { return __builtin_amdgcn_perm(d, d, 0x02030001u); }
__device__ __forceinline__ uint32_t bswap32(uint32_t d) { return __builtin_amdgcn_perm(d, d, 0x00010203u); }

// Packed 2 x u16 minimum / maximum (v_pk_min_u16 / v_pk_max_u16).
typedef uint16_t omr_u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pk_min_u16(uint32_t a, uint32_t b) {
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_min(__builtin_bit_cast(omr_u16x2, a), __builtin_bit_cast(omr_u16x2, b)));
}
__device__ __forceinline__ uint32_t pk_max_u16(uint32_t a, uint32_t b) {
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(omr_u16x2, a), __builtin_bit_cast(omr_u16x2, b)));
}

// Load through an explicit global (addrspace 1) pointer.  A pointer the compiler cannot prove
// global (read from a device table, or selected between such a pointer and a kernarg one)
// otherwise becomes a flat load, which also counts against lgkmcnt: every later LDS wait
// (s_waitcnt lgkmcnt(0)) then waits for that HBM load too, serialising a prefetch.
template <typename T>
__device__ __forceinline__ T ld_global(const void* p) {
    return *(const __attribute__((address_space(1))) T*)p;
}

// 32-bit magic-number division (n < 2^31, d >= 1).
struct FastDiv {
    uint32_t d, mul, shift;
};
inline FastDiv make_fastdiv(uint32_t d) {
    FastDiv f;
    f.d = d;
    uint32_t s = 0;
    while ((1ull << s) < d) ++s;
    f.shift = s;
    f.mul = (uint32_t)(((1ull << 32) * ((1ull << s) - d)) / d + 1);
    return f;
}
__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv& f) {
    if (f.d == 1) return n;
    const uint32_t t = __umulhi(n, f.mul);
    return (t + ((n - t) >> 1)) >> (f.shift - 1);
}

}  // namespace omr
