// omr_jpeg.hip — K4 baseline JPEG encoder, bit-exact with IJG 6b / libjpeg-turbo.
//
// Replaces ImageUtil.createBufferedImage + compressionService.compressToStream
// (ImageRegionRequestHandler.java:576-582): the JDK ImageIO JPEG writer (IJG libjpeg 6b)
// with JFIF YCbCr 4:2:0, islow FDCT, Java-scaled standard tables, standard Huffman tables,
// no restart markers.  The entropy-coded segment is produced byte-identically to a serial
// encoder without restart intervals:
//   J1  one wave per 16x16 MCU: RGB->YCbCr (jccolor fixed point), h2v2 downsample with the
//       1,2 bias, IJG edge replication, level shift, islow FDCT, quantisation, dummy blocks
//   J2  one lane per 8x8 block: Huffman bit length (DC prediction from the previous block
//       of the same component in scan order)
//   J3  exclusive scan of bit lengths -> bit offsets
//   J4  one lane per block: re-encode and OR the bits into a big-endian word stream
//   J5  count 0xFF per 16-byte chunk -> scan -> J6 scatter with 0x00 stuffing + 1-bit pad
#include "omr_device.h"
#include "omr_k2.h"

#include <memory>
#include <type_traits>

namespace omr {

// ------------------------------------------------------------------ tables
static constexpr uint8_t kBitsDcL[17] = {0, 0, 1, 5, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0, 0, 0};
static constexpr uint8_t kBitsDcC[17] = {0, 0, 3, 1, 1, 1, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0};
static constexpr uint8_t kValDc[12] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11};
static constexpr uint8_t kBitsAcL[17] = {0, 0, 2, 1, 3, 3, 2, 4, 3, 5, 5, 4, 4, 0, 0, 1, 0x7d};
static constexpr uint8_t kValAcL[162] = {
    0x01, 0x02, 0x03, 0x00, 0x04, 0x11, 0x05, 0x12, 0x21, 0x31, 0x41, 0x06, 0x13, 0x51, 0x61, 0x07,
    0x22, 0x71, 0x14, 0x32, 0x81, 0x91, 0xa1, 0x08, 0x23, 0x42, 0xb1, 0xc1, 0x15, 0x52, 0xd1, 0xf0,
    0x24, 0x33, 0x62, 0x72, 0x82, 0x09, 0x0a, 0x16, 0x17, 0x18, 0x19, 0x1a, 0x25, 0x26, 0x27, 0x28,
    0x29, 0x2a, 0x34, 0x35, 0x36, 0x37, 0x38, 0x39, 0x3a, 0x43, 0x44, 0x45, 0x46, 0x47, 0x48, 0x49,
    0x4a, 0x53, 0x54, 0x55, 0x56, 0x57, 0x58, 0x59, 0x5a, 0x63, 0x64, 0x65, 0x66, 0x67, 0x68, 0x69,
    0x6a, 0x73, 0x74, 0x75, 0x76, 0x77, 0x78, 0x79, 0x7a, 0x83, 0x84, 0x85, 0x86, 0x87, 0x88, 0x89,
    0x8a, 0x92, 0x93, 0x94, 0x95, 0x96, 0x97, 0x98, 0x99, 0x9a, 0xa2, 0xa3, 0xa4, 0xa5, 0xa6, 0xa7,
    0xa8, 0xa9, 0xaa, 0xb2, 0xb3, 0xb4, 0xb5, 0xb6, 0xb7, 0xb8, 0xb9, 0xba, 0xc2, 0xc3, 0xc4, 0xc5,
    0xc6, 0xc7, 0xc8, 0xc9, 0xca, 0xd2, 0xd3, 0xd4, 0xd5, 0xd6, 0xd7, 0xd8, 0xd9, 0xda, 0xe1, 0xe2,
    0xe3, 0xe4, 0xe5, 0xe6, 0xe7, 0xe8, 0xe9, 0xea, 0xf1, 0xf2, 0xf3, 0xf4, 0xf5, 0xf6, 0xf7, 0xf8,
    0xf9, 0xfa};
static constexpr uint8_t kBitsAcC[17] = {0, 0, 2, 1, 2, 4, 4, 3, 4, 7, 5, 4, 4, 0, 1, 2, 0x77};
static constexpr uint8_t kValAcC[162] = {
    0x00, 0x01, 0x02, 0x03, 0x11, 0x04, 0x05, 0x21, 0x31, 0x06, 0x12, 0x41, 0x51, 0x07, 0x61, 0x71,
    0x13, 0x22, 0x32, 0x81, 0x08, 0x14, 0x42, 0x91, 0xa1, 0xb1, 0xc1, 0x09, 0x23, 0x33, 0x52, 0xf0,
    0x15, 0x62, 0x72, 0xd1, 0x0a, 0x16, 0x24, 0x34, 0xe1, 0x25, 0xf1, 0x17, 0x18, 0x19, 0x1a, 0x26,
    0x27, 0x28, 0x29, 0x2a, 0x35, 0x36, 0x37, 0x38, 0x39, 0x3a, 0x43, 0x44, 0x45, 0x46, 0x47, 0x48,
    0x49, 0x4a, 0x53, 0x54, 0x55, 0x56, 0x57, 0x58, 0x59, 0x5a, 0x63, 0x64, 0x65, 0x66, 0x67, 0x68,
    0x69, 0x6a, 0x73, 0x74, 0x75, 0x76, 0x77, 0x78, 0x79, 0x7a, 0x82, 0x83, 0x84, 0x85, 0x86, 0x87,
    0x88, 0x89, 0x8a, 0x92, 0x93, 0x94, 0x95, 0x96, 0x97, 0x98, 0x99, 0x9a, 0xa2, 0xa3, 0xa4, 0xa5,
    0xa6, 0xa7, 0xa8, 0xa9, 0xaa, 0xb2, 0xb3, 0xb4, 0xb5, 0xb6, 0xb7, 0xb8, 0xb9, 0xba, 0xc2, 0xc3,
    0xc4, 0xc5, 0xc6, 0xc7, 0xc8, 0xc9, 0xca, 0xd2, 0xd3, 0xd4, 0xd5, 0xd6, 0xd7, 0xd8, 0xd9, 0xda,
    0xe2, 0xe3, 0xe4, 0xe5, 0xe6, 0xe7, 0xe8, 0xe9, 0xea, 0xf2, 0xf3, 0xf4, 0xf5, 0xf6, 0xf7, 0xf8,
    0xf9, 0xfa};
static constexpr int kStdLuma[64] = {
    16, 11, 10, 16, 24, 40, 51, 61, 12, 12, 14, 19, 26, 58, 60, 55,
    14, 13, 16, 24, 40, 57, 69, 56, 14, 17, 22, 29, 51, 87, 80, 62,
    18, 22, 37, 56, 68, 109, 103, 77, 24, 35, 55, 64, 81, 104, 113, 92,
    49, 64, 78, 87, 103, 121, 120, 101, 72, 92, 95, 98, 112, 100, 103, 99};
static constexpr int kStdChroma[64] = {
    17, 18, 24, 47, 99, 99, 99, 99, 18, 21, 26, 66, 99, 99, 99, 99,
    24, 26, 56, 99, 99, 99, 99, 99, 47, 66, 99, 99, 99, 99, 99, 99,
    99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99,
    99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99};
static constexpr int kZigzag[64] = {   // zigzag index -> natural position
    0, 1, 8, 16, 9, 2, 3, 10, 17, 24, 32, 25, 18, 11, 4, 5,
    12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6, 7, 14, 21, 28,
    35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
    58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

struct HuffTab {
    uint16_t code[256];
    uint8_t size[256];
};

constexpr HuffTab make_huff(const uint8_t (&bits)[17], const uint8_t* vals) {
    HuffTab t{};
    int k = 0;
    unsigned code = 0;
    for (int l = 1; l <= 16; ++l) {
        for (int i = 0; i < bits[l]; ++i) {
            t.code[vals[k]] = (uint16_t)code;
            t.size[vals[k]] = (uint8_t)l;
            ++k;
            ++code;
        }
        code <<= 1;
    }
    return t;
}

struct ZzInv {
    uint8_t v[64];
};
constexpr ZzInv make_zzinv() {
    ZzInv z{};
    for (int i = 0; i < 64; ++i) z.v[kZigzag[i]] = (uint8_t)i;
    return z;
}

__constant__ HuffTab c_huff[4] = {make_huff(kBitsDcL, kValDc), make_huff(kBitsAcL, kValAcL),
                                  make_huff(kBitsDcC, kValDc), make_huff(kBitsAcC, kValAcC)};
__constant__ ZzInv c_zzinv = make_zzinv();

// B2a's AC length table, built at compile time: code length of (zero run r < 64, magnitude
// category nb) with the r >> 4 ZRL codes folded in, at r * 16 + nb; 0 for nb == 0 (a zero
// coefficient adds nothing).  Entries with ZRL codes also carry 0x800: a block's sum is then its
// bit count (< 2^11) plus 0x800 per ZRL-prefixed coefficient, so B2a flags B3's ZRL path for free.
// [0] luma, [1] chroma; 2 KiB each, copied to LDS with 16-B loads.
constexpr uint32_t kZrlFlag = 0x800;
// B2a's per-block record also carries the block's int16 flag (B3 then knows which form to load
// before loading anything): bit 15, above the bit count and at most three ZRL flags (< 0x2000).
constexpr uint32_t kWideFlag = 0x8000;
struct AcLen {
    uint16_t v[2][1024];
};
constexpr AcLen make_aclen() {
    AcLen a{};
    const HuffTab t[2] = {make_huff(kBitsAcL, kValAcL), make_huff(kBitsAcC, kValAcC)};
    for (int c = 0; c < 2; ++c)
        for (int i = 0; i < 1024; ++i) {
            const int r = i >> 4, nb = i & 15;
            a.v[c][i] = nb ? (uint16_t)((r >> 4) * t[c].size[0xF0] + t[c].size[((r & 15) << 4) | nb] +
                                        (r >= 16 ? kZrlFlag : 0u)) : 0;
        }
    return a;
}
__constant__ AcLen c_aclen = make_aclen();

// B3's tables, built at compile time and copied to LDS with 16-byte loads: the AC codes packed as
// size << 16 | code with the size-0 entries (run, 0) — EOB and ZRL come from c_huff — zeroed, so
// a zero coefficient codes as zero bits with no select; the DC codes and sizes (12 categories).
struct B3Tabs {
    uint32_t ac[2][256];
    uint32_t dc[2][16];    // size << 16 | code
};
constexpr B3Tabs make_b3tabs() {
    B3Tabs b{};
    const HuffTab ac[2] = {make_huff(kBitsAcL, kValAcL), make_huff(kBitsAcC, kValAcC)};
    const HuffTab dc[2] = {make_huff(kBitsDcL, kValDc), make_huff(kBitsDcC, kValDc)};
    for (int t = 0; t < 2; ++t) {
        for (int i = 0; i < 256; ++i)
            b.ac[t][i] = (i & 15) == 0 ? 0u : ((uint32_t)ac[t].size[i] << 16) | ac[t].code[i];
        for (int i = 0; i < 16; ++i) b.dc[t][i] = ((uint32_t)dc[t].size[i] << 16) | dc[t].code[i];
    }
    return b;
}
__constant__ B3Tabs c_b3tabs = make_b3tabs();

struct QTabs {
    uint16_t q[2][64];  // natural order
    uint32_t m[2][64];  // ceil(2^32 / (8 q)): B1's reciprocal quantiser (set_recips)
};

static void set_recips(QTabs& t) {
    for (int c = 0; c < 2; ++c)
        for (int i = 0; i < 64; ++i) {
            const uint64_t d = (uint64_t)t.q[c][i] << 3;
            t.m[c][i] = (uint32_t)((0x100000000ull + d - 1) / d);
        }
}

// JPEGQTable.getScaledInstance(scale, forceBaseline=true): (int)(q*scale + 0.5f) in [1, 255].
static int scale_entry(int q, float scale) {
    volatile float a = (float)q * scale;      // one float multiply, then the add (no contraction)
    const int sv = (int)(a + 0.5f);
    return sv < 1 ? 1 : sv > 255 ? 255 : sv;
}

// javax.imageio JPEG.convertToLinearQuality + JPEGQTable.getScaledInstance(scale, true) of the
// Annex K luminance table and, by OMR_SEM_JPEG_CHROMA_DIV2, of K2Chrominance (default) or
// K2Div2Chrominance (= K2Chrominance.getScaledInstance(0.5f, true)).
static void quant_tables(float quality, uint32_t sem, uint8_t luma[64], uint8_t chroma[64]) {
    float qf = quality;
    if (qf <= 0.0f) qf = 0.01f;
    if (qf > 1.00f) qf = 1.00f;
    if (qf < 0.5f) qf = 0.5f / qf;
    else qf = 2.0f - (qf * 2.0f);
    for (int i = 0; i < 64; ++i) {
        luma[i] = (uint8_t)scale_entry(kStdLuma[i], qf);
        const int cbase = (sem & OMR_SEM_JPEG_CHROMA_DIV2) ? scale_entry(kStdChroma[i], 0.5f) : kStdChroma[i];
        chroma[i] = (uint8_t)scale_entry(cbase, qf);
    }
}

// ------------------------------------------------------------------ J1: colour + DCT + quant
__device__ __forceinline__ void ycc(uint32_t p, int& y, int& cb, int& cr) {
    const int r = (p >> 16) & 0xFF, g = (p >> 8) & 0xFF, b = p & 0xFF;
    // jccolor.c rgb_ycc_convert, SCALEBITS 16: FIX(x) = (int)(x*65536+0.5)
    y = (19595 * r + 38470 * g + 7471 * b + 32768) >> 16;
    cb = (-11059 * r - 21709 * g + 32768 * b + (128 << 16) + 32767) >> 16;
    cr = (32768 * r - 27439 * g - 5329 * b + (128 << 16) + 32767) >> 16;
}

// The same on separate components (B1/F1 pixel sources hand over r, g, b).
struct Rgb {
    int r, g, b;
};
__device__ __forceinline__ void ycc(const Rgb& p, int& y, int& cb, int& cr) {
    y = (19595 * p.r + 38470 * p.g + 7471 * p.b + 32768) >> 16;
    cb = (-11059 * p.r - 21709 * p.g + 32768 * p.b + (128 << 16) + 32767) >> 16;
    cr = (32768 * p.r - 27439 * p.g - 5329 * p.b + (128 << 16) + 32767) >> 16;
}
__device__ __forceinline__ Rgb rgb_of(uint32_t p) {
    return Rgb{(int)((p >> 16) & 0xFF), (int)((p >> 8) & 0xFF), (int)(p & 0xFF)};
}

// One pixel as two packed 16-bit pairs, r | g << 16 and b | g << 16: the operands of the
// v_dot2 colour transform below (B1/F1 pixel sources hand these over).
struct Px2 {
    uint32_t rg, bg;
};
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
typedef short i16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ Px2 px2_of(uint32_t argb) {   // v_perm: bytes (r, 0, g, 0) and (b, 0, g, 0)
    return Px2{__builtin_amdgcn_perm(0u, argb, 0x0c010c02u), __builtin_amdgcn_perm(0u, argb, 0x0c010c00u)};
}
__device__ __forceinline__ uint32_t udot2(uint32_t a, u16x2 k, uint32_t c) {
    return __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, a), k, c, false);
}
__device__ __forceinline__ int sdot2(uint32_t a, i16x2 k, int c) {
    return __builtin_amdgcn_sdot2(__builtin_bit_cast(i16x2, a), k, c, false);
}
// jccolor.c rgb_ycc_convert as above, each component two v_dot2 (exact: every product and partial
// sum fits 32 bits; 32768 is applied through the unsigned form, the negative weights through the
// signed one).
__device__ __forceinline__ void ycc(const Px2& p, int& y, int& cb, int& cr) {
    y = (int)(udot2(p.rg, u16x2{19595, 38470}, udot2(p.bg, u16x2{7471, 0}, 32768u)) >> 16);
    cb = sdot2(p.rg, i16x2{-11059, -21709}, (int)udot2(p.bg, u16x2{32768, 0}, (128u << 16) + 32767u)) >> 16;
    cr = sdot2(p.bg, i16x2{-5329, -27439}, (int)udot2(p.rg, u16x2{32768, 0}, (128u << 16) + 32767u)) >> 16;
}
__device__ __forceinline__ bool is_grey(const Px2& p) {   // r == g == b
    return (((p.rg ^ (p.rg >> 16)) | (p.bg ^ (p.bg >> 16))) & 0xFFFFu) == 0;
}

#define DESCALE(x, n) (((x) + (1 << ((n)-1))) >> (n))
#define M24(a, c) __mul24((a), (c))

// jfdctint.c one 8-point pass on p[0], p[s], ..., p[7s] (pass 0 rows, pass 1 columns).
template <int PASS>
__device__ __forceinline__ void fdct8(int* p, int s) {
    constexpr int CB = 13, P1 = 2;
    constexpr int sh = PASS ? CB + P1 : CB - P1;
    int tmp0 = p[0] + p[7 * s], tmp7 = p[0] - p[7 * s];
    int tmp1 = p[s] + p[6 * s], tmp6 = p[s] - p[6 * s];
    int tmp2 = p[2 * s] + p[5 * s], tmp5 = p[2 * s] - p[5 * s];
    int tmp3 = p[3 * s] + p[4 * s], tmp4 = p[3 * s] - p[4 * s];
    const int tmp10 = tmp0 + tmp3, tmp13 = tmp0 - tmp3;
    const int tmp11 = tmp1 + tmp2, tmp12 = tmp1 - tmp2;
    if (PASS) {
        p[0] = DESCALE(tmp10 + tmp11, P1);
        p[4 * s] = DESCALE(tmp10 - tmp11, P1);
    } else {
        p[0] = (tmp10 + tmp11) * (1 << P1);
        p[4 * s] = (tmp10 - tmp11) * (1 << P1);
    }
    // Every operand is below 2^17 in magnitude and every product below 2^31 (the jfdctint.c
    // INT32 range for 8-bit samples), so v_mul_i32_i24 (full rate) is exact; a plain `*` lowers
    // to quarter-rate v_mul_lo_u32 / v_mad_u64_u32.
    int z1 = M24(tmp12 + tmp13, 4433);
    p[2 * s] = DESCALE(z1 + M24(tmp13, 6270), sh);
    p[6 * s] = DESCALE(z1 + M24(tmp12, -15137), sh);
    z1 = tmp4 + tmp7;
    int z2 = tmp5 + tmp6, z3 = tmp4 + tmp6, z4 = tmp5 + tmp7;
    const int z5 = M24(z3 + z4, 9633);
    tmp4 = M24(tmp4, 2446); tmp5 = M24(tmp5, 16819); tmp6 = M24(tmp6, 25172); tmp7 = M24(tmp7, 12299);
    z1 = M24(z1, -7373); z2 = M24(z2, -20995); z3 = M24(z3, -16069); z4 = M24(z4, -3196);
    z3 += z5; z4 += z5;
    p[7 * s] = DESCALE(tmp4 + z1 + z3, sh);
    p[5 * s] = DESCALE(tmp5 + z2 + z4, sh);
    p[3 * s] = DESCALE(tmp6 + z2 + z3, sh);
    p[s] = DESCALE(tmp7 + z1 + z4, sh);
}

__device__ __forceinline__ int16_t quant(int t, int q) {   // jcdctmgr.c forward_DCT
    const int div = q << 3;
    if (t < 0) { t = -t; t += div >> 1; t = t >= div ? t / div : 0; return (int16_t)-t; }
    t += div >> 1;
    return (int16_t)(t >= div ? t / div : 0);
}

struct J1Args {
    const uint32_t* argb;
    int16_t* coefs;     // [n_mcu*6][64] zigzag order
    int32_t W, H, mcux, n_mcu;
    QTabs qt;
};

__global__ void __launch_bounds__(256) k_jpeg_fdct(J1Args A) {
    __shared__ int s[4][6 * 64 + 8];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int m = blockIdx.x * 4 + wv;
    const bool valid = m < A.n_mcu;
    int* S = s[wv];
    const int W = A.W, H = A.H;
    const int mx = valid ? m % A.mcux : 0, my = valid ? m / A.mcux : 0;
    const int cx = lane & 7, cy = lane >> 3;
    if (valid) {
        const int x0 = mx * 16 + 2 * cx, y0 = my * 16 + 2 * cy;
        const int xa = min(x0, W - 1), xb = min(x0 + 1, W - 1);
        const int ya = min(y0, H - 1), yb = min(y0 + 1, H - 1);
        const uint32_t* img = A.argb;
        uint32_t p00 = img[(int64_t)ya * W + xa], p01 = img[(int64_t)ya * W + xb];
        uint32_t p10 = img[(int64_t)yb * W + xa], p11 = img[(int64_t)yb * W + xb];
        int y, cb0, cr0, cb1, cr1, cb2, cr2, cb3, cr3;
        const int blk = (cy >> 2) * 2 + (cx >> 2);
        const int o = ((2 * cy) & 7) * 8 + ((2 * cx) & 7);
        ycc(p00, y, cb0, cr0); S[blk * 64 + o] = y - 128;
        ycc(p01, y, cb1, cr1); S[blk * 64 + o + 1] = y - 128;
        ycc(p10, y, cb2, cr2); S[blk * 64 + o + 8] = y - 128;
        ycc(p11, y, cb3, cr3); S[blk * 64 + o + 9] = y - 128;
        const int chv = (H + 1) / 2;            // chroma rows fed by real (even-padded) rows
        const int cyg = my * 8 + cy;
        if (cyg >= chv) {                       // jcprepct bottom padding of the downsampled rows
            const int r0 = min(2 * (chv - 1), H - 1), r1 = min(2 * (chv - 1) + 1, H - 1);
            p00 = img[(int64_t)r0 * W + xa]; p01 = img[(int64_t)r0 * W + xb];
            p10 = img[(int64_t)r1 * W + xa]; p11 = img[(int64_t)r1 * W + xb];
            ycc(p00, y, cb0, cr0); ycc(p01, y, cb1, cr1); ycc(p10, y, cb2, cr2); ycc(p11, y, cb3, cr3);
        }
        const int bias = (cx & 1) ? 2 : 1;     // jcsample.c h2v2_downsample
        S[4 * 64 + cy * 8 + cx] = ((cb0 + cb1 + cb2 + cb3 + bias) >> 2) - 128;
        S[5 * 64 + cy * 8 + cx] = ((cr0 + cr1 + cr2 + cr3 + bias) >> 2) - 128;
    }
    __syncthreads();
    if (valid && lane < 48) fdct8<0>(S + (lane >> 3) * 64 + (lane & 7) * 8, 1);
    __syncthreads();
    if (valid && lane < 48) fdct8<1>(S + (lane >> 3) * 64 + (lane & 7), 8);
    __syncthreads();
    if (!valid) return;
    const int ywib = (W + 7) / 8, yhib = (H + 7) / 8;
    const int zz = c_zzinv.v[lane];
    int16_t* out = A.coefs + (int64_t)m * 6 * 64;
    int16_t dc[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        int16_t q = quant(S[k * 64 + lane], A.qt.q[k < 4 ? 0 : 1][lane]);
        if (k < 4) {
            const int bx = mx * 2 + (k & 1), by = my * 2 + (k >> 1);
            if ((bx >= ywib || by >= yhib) && lane != 0) q = 0;   // dummy block: AC zero
        }
        dc[k] = q;
        if (lane != 0) out[k * 64 + zz] = q;
    }
    if (lane == 0) {   // jccoefct.c dummy-block DC propagation
        const bool c1 = mx * 2 + 1 >= ywib, row1 = my * 2 + 1 >= yhib;
        if (c1) dc[1] = dc[0];
        if (row1) { dc[2] = dc[1]; dc[3] = dc[1]; }
        else if (c1) dc[3] = dc[2];
#pragma unroll
        for (int k = 0; k < 6; ++k) out[k * 64] = dc[k];
    }
}

// ------------------------------------------------------------------ J2/J4: Huffman
struct BitSink {
    uint32_t* words;
    uint64_t acc;
    int nacc;
    uint32_t wi;
    __device__ void put(uint32_t v, int n) {
        acc = (acc << n) | (v & ((1u << n) - 1));
        nacc += n;
        if (nacc >= 32) {
            atomicOr(&words[wi++], (uint32_t)(acc >> (nacc - 32)));
            nacc -= 32;
            acc &= (1ull << nacc) - 1;
        }
    }
    __device__ void flush() {
        if (nacc > 0) atomicOr(&words[wi], (uint32_t)(acc << (32 - nacc)));
    }
};

struct BitCount {
    uint32_t bits = 0;
    __device__ void put(uint32_t, int n) { bits += n; }
    __device__ void flush() {}
};

template <typename Sink>
__device__ __forceinline__ void encode_block(Sink& o, const int16_t* blk, int last_dc, const HuffTab& dct,
                                             const HuffTab& act) {
    int temp = blk[0] - last_dc, temp2 = temp;
    if (temp < 0) { temp = -temp; temp2--; }
    int nbits = temp ? 32 - __clz(temp) : 0;
    o.put(dct.code[nbits], dct.size[nbits]);
    if (nbits) o.put((uint32_t)temp2, nbits);
    int r = 0;
    for (int k = 1; k < 64; ++k) {
        temp = blk[k];
        if (temp == 0) { r++; continue; }
        while (r > 15) { o.put(act.code[0xF0], act.size[0xF0]); r -= 16; }
        temp2 = temp;
        if (temp < 0) { temp = -temp; temp2--; }
        nbits = 32 - __clz(temp);
        const int i = (r << 4) + nbits;
        o.put(act.code[i], act.size[i]);
        o.put((uint32_t)temp2, nbits);
        r = 0;
    }
    if (r > 0) o.put(act.code[0], act.size[0]);
}

__device__ __forceinline__ int prev_block(int b) {
    const int m = b / 6, k = b - m * 6;
    if (k == 1 || k == 2 || k == 3) return b - 1;
    if (m == 0) return -1;
    return k == 0 ? (m - 1) * 6 + 3 : (m - 1) * 6 + k;
}

__global__ void __launch_bounds__(256) k_jpeg_bitlen(const int16_t* __restrict__ coefs, int n_blocks,
                                                     uint32_t* __restrict__ lens) {
    const int b = blockIdx.x * 256 + threadIdx.x;
    if (b >= n_blocks) return;
    const int k = b % 6, pb = prev_block(b);
    const int last = pb >= 0 ? coefs[(int64_t)pb * 64] : 0;
    BitCount c;
    const int t = k < 4 ? 0 : 2;
    encode_block(c, coefs + (int64_t)b * 64, last, c_huff[t], c_huff[t + 1]);
    lens[b] = c.bits;
}

__global__ void __launch_bounds__(256) k_jpeg_write(const int16_t* __restrict__ coefs, int n_blocks,
                                                    const uint32_t* __restrict__ offs, uint32_t* __restrict__ words) {
    const int b = blockIdx.x * 256 + threadIdx.x;
    if (b >= n_blocks) return;
    const int k = b % 6, pb = prev_block(b);
    const int last = pb >= 0 ? coefs[(int64_t)pb * 64] : 0;
    const uint32_t off = offs[b];
    BitSink s{words, 0, (int)(off & 31), off >> 5};
    const int t = k < 4 ? 0 : 2;
    encode_block(s, coefs + (int64_t)b * 64, last, c_huff[t], c_huff[t + 1]);
    s.flush();
}

// ------------------------------------------------------------------ scan (shared with PNG)
__device__ __forceinline__ uint32_t block_exclusive_scan(uint32_t v, uint32_t* s_wave, uint32_t& total) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) s_wave[wid] = x;
    __syncthreads();
    if (wid == 0) {
        uint32_t w = lane < nw ? s_wave[lane] : 0;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(w, o, 64);
            if (lane >= o) w += y;
        }
        if (lane < nw) s_wave[lane] = w;
    }
    __syncthreads();
    const uint32_t off = wid ? s_wave[wid - 1] : 0;
    total = s_wave[nw - 1];
    __syncthreads();
    return off + x - v;
}

constexpr int kScanThreads = 1024, kScanPer = 4, kScanTile = kScanThreads * kScanPer;

__global__ void __launch_bounds__(kScanThreads) k_scan_tiles(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                            int64_t n, uint32_t* __restrict__ tile_sums) {
    __shared__ uint32_t sw[16];
    const int64_t base = (int64_t)blockIdx.x * kScanTile + (int64_t)threadIdx.x * kScanPer;
    uint32_t v[kScanPer], sum = 0;
#pragma unroll
    for (int i = 0; i < kScanPer; ++i) { v[i] = base + i < n ? in[base + i] : 0; sum += v[i]; }
    uint32_t total;
    uint32_t run = block_exclusive_scan(sum, sw, total);
#pragma unroll
    for (int i = 0; i < kScanPer; ++i) {
        if (base + i < n) out[base + i] = run;
        run += v[i];
    }
    if (threadIdx.x == 0) tile_sums[blockIdx.x] = total;
}

__global__ void __launch_bounds__(kScanThreads) k_scan_sums(uint32_t* __restrict__ sums, int n, uint32_t* __restrict__ total_out) {
    __shared__ uint32_t sw[16];
    __shared__ uint32_t carry;
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    for (int base = 0; base < n; base += kScanThreads) {
        const int i = base + threadIdx.x;
        const uint32_t v = i < n ? sums[i] : 0;
        uint32_t total;
        const uint32_t ex = block_exclusive_scan(v, sw, total);
        const uint32_t c = carry;
        if (i < n) sums[i] = ex + c;
        __syncthreads();
        if (threadIdx.x == 0) carry = c + total;
        __syncthreads();
    }
    if (threadIdx.x == 0) *total_out = carry;
}

__global__ void __launch_bounds__(kScanThreads) k_scan_add(uint32_t* __restrict__ out, int64_t n, const uint32_t* __restrict__ tile_sums) {
    const int64_t base = (int64_t)blockIdx.x * kScanTile + (int64_t)threadIdx.x * kScanPer;
    const uint32_t add = tile_sums[blockIdx.x];
#pragma unroll
    for (int i = 0; i < kScanPer; ++i)
        if (base + i < n) out[base + i] += add;
}

size_t scan_scratch_bytes(int64_t n) { return align_up((size_t)((n + kScanTile - 1) / kScanTile + 1) * 4, 256); }

// Exclusive scan of n uint32 (device); *d_total receives the sum.  scratch: scan_scratch_bytes(n).
omr_status device_exclusive_scan(Ctx* ctx, const uint32_t* in, uint32_t* out, int64_t n, uint32_t* d_total,
                                 uint32_t* scratch) {
    const int64_t tiles = (n + kScanTile - 1) / kScanTile;
    if (tiles == 0) {
        OMR_HIP(ctx, hipMemsetAsync(d_total, 0, 4, ctx->stream));
        return OMR_OK;
    }
    hipLaunchKernelGGL(k_scan_tiles, dim3((unsigned)tiles), dim3(kScanThreads), 0, ctx->stream, in, out, n, scratch);
    hipLaunchKernelGGL(k_scan_sums, dim3(1), dim3(kScanThreads), 0, ctx->stream, scratch, (int)tiles, d_total);
    hipLaunchKernelGGL(k_scan_add, dim3((unsigned)tiles), dim3(kScanThreads), 0, ctx->stream, out, n, scratch);
    OMR_HIP(ctx, hipGetLastError());
    return OMR_OK;
}

// ------------------------------------------------------------------ J5/J6: stuffing
constexpr int kStuffChunk = 16;

__device__ __forceinline__ uint32_t stream_byte(const uint32_t* words, uint32_t i, uint32_t nbytes, uint32_t total_bits) {
    uint32_t b = (words[i >> 2] >> (24 - 8 * (i & 3))) & 0xFF;
    if (i == nbytes - 1 && (total_bits & 7)) b |= 0xFFu >> (total_bits & 7);   // jchuff flush: pad with 1s
    return b;
}

__global__ void __launch_bounds__(256) k_stuff_count(const uint32_t* __restrict__ words, const uint32_t* __restrict__ d_total_bits,
                                                     uint32_t max_chunks, uint32_t* __restrict__ counts) {
    const uint32_t c = blockIdx.x * 256 + threadIdx.x;
    if (c >= max_chunks) return;
    const uint32_t tb = *d_total_bits, nbytes = (tb + 7) / 8;
    uint32_t n = 0;
    for (uint32_t i = c * kStuffChunk; i < min(nbytes, (c + 1) * kStuffChunk); ++i)
        n += stream_byte(words, i, nbytes, tb) == 0xFF;
    counts[c] = n;
}

__global__ void __launch_bounds__(256) k_stuff_write(const uint32_t* __restrict__ words, const uint32_t* __restrict__ d_total_bits,
                                                     uint32_t max_chunks, const uint32_t* __restrict__ offs,
                                                     uint8_t* __restrict__ out) {
    const uint32_t c = blockIdx.x * 256 + threadIdx.x;
    if (c >= max_chunks) return;
    const uint32_t tb = *d_total_bits, nbytes = (tb + 7) / 8;
    uint32_t o = c * kStuffChunk + offs[c];
    for (uint32_t i = c * kStuffChunk; i < min(nbytes, (c + 1) * kStuffChunk); ++i) {
        const uint32_t b = stream_byte(words, i, nbytes, tb);
        out[o++] = (uint8_t)b;
        if (b == 0xFF) out[o++] = 0;
    }
}

// ------------------------------------------------------------------ host side
static void jpeg_header(std::vector<uint8_t>& h, int W, int H, const uint8_t* ql, const uint8_t* qc) {
    const uint8_t app0[] = {0xFF, 0xD8, 0xFF, 0xE0, 0x00, 0x10, 'J', 'F', 'I', 'F', 0x00,
                            0x01, 0x01, 0x00, 0x00, 0x01, 0x00, 0x01, 0x00, 0x00};
    h.insert(h.end(), app0, app0 + sizeof(app0));
    for (int t = 0; t < 2; ++t) {
        const uint8_t d[] = {0xFF, 0xDB, 0, 67, (uint8_t)t};
        h.insert(h.end(), d, d + 5);
        for (int i = 0; i < 64; ++i) h.push_back((t ? qc : ql)[kZigzag[i]]);
    }
    const uint8_t sof[] = {0xFF, 0xC0, 0, 17, 8, (uint8_t)(H >> 8), (uint8_t)H, (uint8_t)(W >> 8), (uint8_t)W,
                           3, 1, 0x22, 0, 2, 0x11, 1, 3, 0x11, 1};
    h.insert(h.end(), sof, sof + sizeof(sof));
    auto dht = [&](int id, const uint8_t* bits, const uint8_t* vals) {
        int n = 0;
        for (int i = 1; i <= 16; ++i) n += bits[i];
        const uint8_t m[] = {0xFF, 0xC4, (uint8_t)((19 + n) >> 8), (uint8_t)(19 + n), (uint8_t)id};
        h.insert(h.end(), m, m + 5);
        h.insert(h.end(), bits + 1, bits + 17);
        h.insert(h.end(), vals, vals + n);
    };
    dht(0x00, kBitsDcL, kValDc);
    dht(0x10, kBitsAcL, kValAcL);
    dht(0x01, kBitsDcC, kValDc);
    dht(0x11, kBitsAcC, kValAcC);
    const uint8_t sos[] = {0xFF, 0xDA, 0, 12, 3, 1, 0x00, 2, 0x11, 3, 0x11, 0, 63, 0};
    h.insert(h.end(), sos, sos + sizeof(sos));
}

struct JpegLayout {
    int64_t n_mcu, n_blocks, max_bits, max_words, max_bytes, chunks;
    size_t coef_off, lens_off, offs_off, words_off, cnt_off, cofs_off, out_off, tot_off, scan_off, total;
};

static JpegLayout jpeg_layout(int W, int H, size_t base) {
    JpegLayout L{};
    L.n_mcu = (int64_t)((W + 15) / 16) * ((H + 15) / 16);
    L.n_blocks = L.n_mcu * 6;
    L.max_bits = L.n_blocks * 1700;   // DC <= 27 bits, 63 AC symbols <= 26 bits each
    L.max_words = (L.max_bits + 31) / 32 + 1;
    L.max_bytes = L.max_words * 4;
    L.chunks = (L.max_bytes + kStuffChunk - 1) / kStuffChunk;
    size_t o = align_up(base, 256);
    L.coef_off = o; o = align_up(o + (size_t)L.n_blocks * 128, 256);
    L.lens_off = o; o = align_up(o + (size_t)L.n_blocks * 4, 256);
    L.offs_off = o; o = align_up(o + (size_t)L.n_blocks * 4, 256);
    L.words_off = o; o = align_up(o + (size_t)L.max_words * 4, 256);
    L.cnt_off = o; o = align_up(o + (size_t)L.chunks * 4, 256);
    L.cofs_off = o; o = align_up(o + (size_t)L.chunks * 4, 256);
    L.out_off = o; o = align_up(o + (size_t)L.max_bytes * 2, 256);
    L.tot_off = o; o = align_up(o + 16, 256);
    L.scan_off = o; o += scan_scratch_bytes(std::max(L.n_blocks, L.chunks));
    L.total = o;
    return L;
}

// Encode device ARGB (already in place) into host `out`.  Workspace must hold L.total bytes.
static omr_status encode_jpeg_ws(Ctx* ctx, const uint32_t* d_argb, int W, int H, float quality, uint8_t* out,
                                 size_t cap, size_t* out_len, const JpegLayout& L) {
    uint8_t ql[64], qc[64];
    quant_tables(quality, ctx->sem, ql, qc);
    std::vector<uint8_t> hdr;
    jpeg_header(hdr, W, H, ql, qc);
    uint8_t* ws = static_cast<uint8_t*>(ctx->ws);
    int16_t* coefs = reinterpret_cast<int16_t*>(ws + L.coef_off);
    uint32_t* lens = reinterpret_cast<uint32_t*>(ws + L.lens_off);
    uint32_t* offs = reinterpret_cast<uint32_t*>(ws + L.offs_off);
    uint32_t* words = reinterpret_cast<uint32_t*>(ws + L.words_off);
    uint32_t* cnt = reinterpret_cast<uint32_t*>(ws + L.cnt_off);
    uint32_t* cofs = reinterpret_cast<uint32_t*>(ws + L.cofs_off);
    uint8_t* dout = ws + L.out_off;
    uint32_t* tot = reinterpret_cast<uint32_t*>(ws + L.tot_off);
    uint32_t* scratch = reinterpret_cast<uint32_t*>(ws + L.scan_off);
    J1Args a;
    a.argb = d_argb;
    a.coefs = coefs;
    a.W = W;
    a.H = H;
    a.mcux = (W + 15) / 16;
    a.n_mcu = (int32_t)L.n_mcu;
    for (int i = 0; i < 64; ++i) { a.qt.q[0][i] = ql[i]; a.qt.q[1][i] = qc[i]; }
    {
        KernelTimer timer(ctx, 4);
        OMR_HIP(ctx, hipMemsetAsync(words, 0, (size_t)L.max_words * 4, ctx->stream));
        hipLaunchKernelGGL(k_jpeg_fdct, dim3((unsigned)((L.n_mcu + 3) / 4)), dim3(256), 0, ctx->stream, a);
        const unsigned gb = (unsigned)((L.n_blocks + 255) / 256);
        hipLaunchKernelGGL(k_jpeg_bitlen, dim3(gb), dim3(256), 0, ctx->stream, coefs, (int)L.n_blocks, lens);
        OMR_HIP(ctx, hipGetLastError());
        omr_status st = device_exclusive_scan(ctx, lens, offs, L.n_blocks, tot, scratch);
        if (st) return st;
        hipLaunchKernelGGL(k_jpeg_write, dim3(gb), dim3(256), 0, ctx->stream, coefs, (int)L.n_blocks, offs, words);
        const unsigned gc = (unsigned)((L.chunks + 255) / 256);
        hipLaunchKernelGGL(k_stuff_count, dim3(gc), dim3(256), 0, ctx->stream, words, tot, (uint32_t)L.chunks, cnt);
        OMR_HIP(ctx, hipGetLastError());
        st = device_exclusive_scan(ctx, cnt, cofs, L.chunks, tot + 1, scratch);
        if (st) return st;
        hipLaunchKernelGGL(k_stuff_write, dim3(gc), dim3(256), 0, ctx->stream, words, tot, (uint32_t)L.chunks, cofs, dout);
        OMR_HIP(ctx, hipGetLastError());
    }
    uint32_t h_tot[2] = {0, 0};
    OMR_HIP(ctx, hipMemcpyAsync(h_tot, tot, 8, hipMemcpyDeviceToHost, ctx->stream));
    OMR_HIP(ctx, hipStreamSynchronize(ctx->stream));
    const size_t scan_bytes = (size_t)(h_tot[0] + 7) / 8 + h_tot[1];
    const size_t total = hdr.size() + scan_bytes + 2;
    if (out_len) *out_len = total;
    if (!out || cap < total) return fail(ctx, OMR_BUFFER_TOO_SMALL, "JPEG output buffer too small");
    std::memcpy(out, hdr.data(), hdr.size());
    if (scan_bytes)
        OMR_HIP(ctx, hipMemcpyAsync(out + hdr.size(), dout, scan_bytes, hipMemcpyDeviceToHost, ctx->stream));
    OMR_HIP(ctx, hipStreamSynchronize(ctx->stream));
    out[total - 2] = 0xFF;
    out[total - 1] = 0xD9;
    return OMR_OK;
}

// One tile through the batched pipeline (defined below): B1..B6 with n = 1, then the file is
// copied to `out` (two host syncs, like the legacy J1-J6 path, at a fraction of its kernel time).
static omr_status encode_jpeg_single_batched(Ctx* ctx, const uint32_t* d_argb, int W, int H, float quality,
                                             uint8_t* out, size_t cap, size_t* out_len, size_t base);
static size_t single_batched_bytes(int W, int H, size_t base);
constexpr int kJpegBatchMaxDim = 4096;

static omr_status check_jpeg_dims(Ctx* ctx, int W, int H) {
    if (W <= 0 || H <= 0 || W > 65535 || H > 65535)
        return fail(ctx, OMR_INVALID_ARGUMENT, "JPEG dimensions must be 1..65535");
    return OMR_OK;
}

}  // namespace omr

using namespace omr;

extern "C" {

size_t omr_jpeg_max_bytes(int32_t width, int32_t height) {
    if (width <= 0 || height <= 0) return 1024;
    const size_t mcus = (size_t)((width + 15) / 16) * ((height + 15) / 16);
    return 1024 + mcus * 6 * 1700 / 8 * 2 + 16;
}

omr_status omr_jpeg_quant_tables(float quality, uint8_t luma[64], uint8_t chroma[64]) {
    return omr_jpeg_quant_tables_sem(quality, 0, luma, chroma);
}

omr_status omr_jpeg_quant_tables_sem(float quality, uint32_t semantics, uint8_t luma[64], uint8_t chroma[64]) {
    if (!luma || !chroma) return OMR_INVALID_ARGUMENT;
    quant_tables(quality, semantics, luma, chroma);
    return OMR_OK;
}

omr_status omr_encode_jpeg_device(omr_ctx* ctx, const uint32_t* d_argb, int32_t width, int32_t height,
                                  float quality, uint8_t* out, size_t cap, size_t* out_len) {
    if (!ctx) return OMR_INVALID_ARGUMENT;
    omr_status st = check_jpeg_dims(ctx, width, height);
    if (st) return st;
    if (!d_argb) return fail(ctx, OMR_INVALID_ARGUMENT, "null ARGB buffer");
    OMR_HIP(ctx, hipSetDevice(ctx->device));
    if (width <= kJpegBatchMaxDim && height <= kJpegBatchMaxDim)
        return encode_jpeg_single_batched(ctx, d_argb, width, height, quality, out, cap, out_len, 0);
    const JpegLayout L = jpeg_layout(width, height, 0);
    st = ensure_workspace(ctx, L.total);
    if (st) return st;
    return encode_jpeg_ws(ctx, d_argb, width, height, quality, out, cap, out_len, L);
}

omr_status omr_encode_jpeg(omr_ctx* ctx, const uint32_t* argb, int32_t width, int32_t height, float quality,
                           uint8_t* out, size_t cap, size_t* out_len) {
    if (!ctx) return OMR_INVALID_ARGUMENT;
    omr_status st = check_jpeg_dims(ctx, width, height);
    if (st) return st;
    if (!argb) return fail(ctx, OMR_INVALID_ARGUMENT, "null ARGB buffer");
    OMR_HIP(ctx, hipSetDevice(ctx->device));
    const size_t img = align_up((size_t)width * height * 4, 256);
    if (width <= kJpegBatchMaxDim && height <= kJpegBatchMaxDim) {
        // the image goes to the workspace's first `img` bytes; the batch layout starts after it
        omr_status gs = ensure_workspace(ctx, single_batched_bytes(width, height, img));   // no regrow below
        if (gs) return gs;
        OMR_HIP(ctx, hipMemcpyAsync(ctx->ws, argb, (size_t)width * height * 4, hipMemcpyHostToDevice, ctx->stream));
        return encode_jpeg_single_batched(ctx, nullptr, width, height, quality, out, cap, out_len, img);
    }
    const JpegLayout L = jpeg_layout(width, height, img);
    st = ensure_workspace(ctx, L.total);
    if (st) return st;
    uint32_t* d_argb = static_cast<uint32_t*>(ctx->ws);
    OMR_HIP(ctx, hipMemcpyAsync(d_argb, argb, (size_t)width * height * 4, hipMemcpyHostToDevice, ctx->stream));
    return encode_jpeg_ws(ctx, d_argb, width, height, quality, out, cap, out_len, L);
}

}  // extern "C"

// =====================================================================================
// Batched JPEG: N same-size tiles per call, lane-per-block Huffman, one host sync at most.
//
// The reference encodes every tile on its own worker thread (compressToStream per request,
// ImageRegionRequestHandler.java:580-582).  Here a whole batch of rendered tiles (e.g. the
// output of omr_render_batch_*_device) is encoded by eight launches whose grids span all tiles:
//   B1  k_jpeg_fdct_batch   one wave per MCU: colour, downsample, FDCT, quantise (zig-zag lane
//                           order), the blocks' DCs after dummy-block propagation
//   B2a k_jpeg_block_bits   one lane per block: total bit length (DC needs the previous block's
//                           DC; AC by a walk over the 63 coefficients), sums per 256-block group
//   B2b k_jpeg_group_scan   one workgroup per tile: group bit offsets, tile bit length, zero
//                           the tile's bit-stream words
//   B3  k_jpeg_huff_thread  one lane per block: in-group scan -> bit offset, Huffman-code the 64
//                           register-resident coefficients, whole words stored, shared words ORed
//   B4a k_jpeg_stuff_count  0xFF count per 16-byte chunk of the stream, sums per 256 chunks
//   B4b k_jpeg_group_scan   one workgroup per tile: chunk-group offsets, stuffed length
//   B5  k_jpeg_tile_scan    one workgroup: tile output offsets (header + scan + EOI), status
//   B6  k_jpeg_stuff_batch  per chunk group: in-group scan, stuffed bytes staged in LDS and
//                           copied out coalesced; JFIF header
// Output: complete JFIF files packed back to back in the caller's device buffer.
// =====================================================================================

namespace omr {

struct HuffLds {
    uint16_t code[4][256];
    uint8_t size[4][256];
};

__device__ __forceinline__ void load_huff_lds(HuffLds& h) {
    for (int i = threadIdx.x; i < 1024; i += blockDim.x) {
        h.code[i >> 8][i & 255] = c_huff[i >> 8].code[i & 255];
        h.size[i >> 8][i & 255] = c_huff[i >> 8].size[i & 255];
    }
}

// Inclusive wave64 prefix sum on DPP (row_shr 1/2/4/8 inside each 16-lane row, then
// row_bcast:15 / row_bcast:31 across rows): no LDS traffic, unlike __shfl_up (ds_bpermute).
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, true);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, true);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, true);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, true);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false);
    return v;
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_scan(v), 63);
}

__device__ __forceinline__ uint32_t wave_exclusive(uint32_t v, uint32_t& total) {
    const uint32_t x = wave_incl_scan(v);
    total = (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
    return x - v;
}

// Exact t / d for 0 <= t < 2^16, 1 <= d <= 2040 by one high multiply with m = ceil(2^32 / d):
// n*m/2^32 exceeds n/d by < 2^-16 < 1/d, so the floor never crosses an integer.
__device__ __forceinline__ int quant_recip(int t, int half, uint32_t m) {
    const int sg = t >> 31;                                   // 0 or -1
    const int u = (int)__umulhi((uint32_t)((t ^ sg) - sg + half), m);
    return (u ^ sg) - sg;                                     // sign restored, no branch
}

// v_writelane_b32: the uniform value v into lane `lane` of old (LLVM's intrinsic; the compiler
// routes an SGPR lane select through M0 itself).
__device__ int lane_write(int v, int lane, int old) __asm("llvm.amdgcn.writelane.i32");

__constant__ uint8_t c_zigzag[64] = {
    0, 1, 8, 16, 9, 2, 3, 10, 17, 24, 32, 25, 18, 11, 4, 5,
    12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6, 7, 14, 21, 28,
    35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
    58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

// Measurement-only ablations of B1 / F1 (`tools/ab_build.sh abl<m> -DOMR_ABL=<m>` builds a libomr
// variant; its outputs are wrong).  0 in every real build.
#ifndef OMR_ABL
#define OMR_ABL 0
#endif
enum : int { kAblColour = 2, kAblFdct = 4, kAblLane0 = 8, kAblCoefStore = 16, kAblRender = 32,
             kAblQuant = 64 };

struct B1Args {
    const uint32_t* argb;
    int64_t tile_stride;  // pixels between tiles
    int16_t* coefs;       // [tile][nb][64] zig-zag order, int16: blocks with an AC outside int8
    int8_t* coef8;        // [tile][nb][64] zig-zag order, int8: the other blocks (DC in the record)
    uint32_t* blk;        // [tile][nb] DC after dummy-block propagation << 16 | 1 for an int16 block
    int32_t W, H, mcux, n_mcu, nb;
    int32_t mpw;          // MCUs per wave (prefetch depth vs. waves in flight)
    QTabs qt;
};

constexpr int kB1McuPerWave = 8;   // big batches; a few tiles use 1 so the grid still fills the chip
static_assert(6 * kB1McuPerWave <= 64, "one per-block record per lane");

// Pixels (x, y) and (x+1, y) of one row (clamped to the image), as one 8-byte load when both
// are inside the row.
__device__ __forceinline__ void load_pair(const uint32_t* img, int W, int x, int y, uint32_t& a, uint32_t& b) {
    const uint32_t* r = img + (int64_t)y * W;
    if (x + 1 < W) {
        const uint2 v = *reinterpret_cast<const uint2*>(r + x);   // x even, W*y even when W even
        a = v.x; b = v.y;
    } else {
        a = r[min(x, W - 1)]; b = a;
    }
}

// Per-wave LDS MCU buffer: block b, row r, column c at b*kBS + r*kRS + c.  ds_read_b32 /
// ds_write_b32 bank = word mod 32 per 32-lane half (MI355X_MICROARCH.md §LDS): a row stride of 9
// and a block stride of 72 (8 mod 32) put the 32 rows (pass 0) and the 32 columns (pass 1) of
// four blocks on 32 distinct banks.  The round-2 layout (rows of 8, blocks of 73) was laid out
// for 64 banks: every pass-0 access was 2-way (rows r and r+4), 41 % of B1's LDS-active cycles
// were conflicts (profiles/r02/jpeg_pmc_c2_r02h.txt).
constexpr int kBS = 72, kRS = 9;

// B1's pixel source: rendered ARGB tiles in HBM.  issue<S>() loads the four pixels this lane
// needs for an MCU into prefetch slot S (two slots: the MCUs two ahead are in flight while the
// current one is transformed); take<S>() hands them over at the start of that MCU.
struct ArgbSource {
    static constexpr bool kEdgeRows = true;   // odd heights: the bottom chroma row replicates
    static constexpr int kDepth = 2;          // MCUs of pixels in flight per wave
    const uint32_t* img;
    int W, H;
    bool even_w;
    uint2 na[2] = {make_uint2(0, 0), make_uint2(0, 0)}, nb[2] = {make_uint2(0, 0), make_uint2(0, 0)};
    bool nclamp[2] = {false, false};
    __device__ ArgbSource(const B1Args& A, int tile)
        : img(A.argb + (int64_t)tile * A.tile_stride), W(A.W), H(A.H),
          // 8-byte pixel-pair loads need every row start 8-byte aligned
          even_w((A.W & 1) == 0 && (A.tile_stride & 1) == 0 && ((uintptr_t)A.argb & 7) == 0) {}
    // Even widths: two unconditional 8-byte loads per lane at clamped addresses; the edge
    // replication select happens when the pixels are used, so nothing waits on the prefetch.
    template <int S>
    __device__ __forceinline__ void issue(int x0, int y0) {
        const int ya = min(y0, H - 1), yb = min(y0 + 1, H - 1);
        // 32-bit byte offsets from the uniform tile base (a tile is at most 4096^2 pixels): loads
        // with an SGPR base and a VGPR offset, no 64-bit address arithmetic per load
        if (even_w) {
            const int xl = min(x0, W - 2);                        // even, W >= 2
            na[S] = *px_at<uint2>((uint32_t)(ya * W + xl));
            nb[S] = *px_at<uint2>((uint32_t)(yb * W + xl));
            nclamp[S] = x0 > W - 1;                                // both columns clamp to W-1
        } else {
            const int xa = min(x0, W - 1), xb = min(x0 + 1, W - 1);
            na[S] = make_uint2(*px_at<uint32_t>((uint32_t)(ya * W + xa)), *px_at<uint32_t>((uint32_t)(ya * W + xb)));
            nb[S] = make_uint2(*px_at<uint32_t>((uint32_t)(yb * W + xa)), *px_at<uint32_t>((uint32_t)(yb * W + xb)));
            nclamp[S] = false;
        }
    }
    template <int S>
    __device__ __forceinline__ void take(Px2 (&px)[4]) {
        px[0] = px2_of(nclamp[S] ? na[S].y : na[S].x); px[1] = px2_of(na[S].y);
        px[2] = px2_of(nclamp[S] ? nb[S].y : nb[S].x); px[3] = px2_of(nb[S].y);
    }
    __device__ __forceinline__ uint32_t at(int x, int y) const { return *px_at<uint32_t>((uint32_t)(y * W + x)); }
    __device__ __forceinline__ bool grey_possible() const { return true; }
    template <typename T>
    __device__ __forceinline__ const T* px_at(uint32_t i) const {
        return reinterpret_cast<const T*>(reinterpret_cast<const uint8_t*>(img) + i * 4u);
    }
};

// Fused render -> JPEG: B1 reads the raw channel planes and renders its pixels as K2 does
// (same quantization helpers, contribution tables in LDS), so the ARGB tile never goes through
// HBM (the unfused path writes 4 B and reads 4 B per pixel between K2 and B1).  Tiles whose
// sides are multiples of 16 only (no edge replication); flips map output to source pixels.
struct FusedArgs {
    FusedRender R;
    const uint8_t* sbase;        // strided batches: plane(t, c) = sbase + t*tile_stride + c*chan_stride
    const void* const* planes;   // pointer-table batches: planes[t*size_c + c]
    int64_t tile_stride, chan_stride, row_stride;   // bytes, bytes, pixels
    int32_t strided, size_c, flip_h, flip_v;
    int32_t* rstat;              // [tile] OMR_QUANTIZATION when a pixel left its LUT domain
};

template <int BPP, bool BE, int MODE, int NA>
struct PlaneSource {
    static constexpr bool kEdgeRows = false;  // fused tiles have W % 16 == H % 16 == 0: no edge
                                              // replication and no dummy blocks
    const FusedArgs& F;
    const uint32_t* s_contrib;   // LDS [n_active][256]
    const uint8_t* base[kFusedMaxActive];
    // Pixel prefetch depth (MCUs in flight per wave).  One MCU of cover is ~5 us per wave, far
    // above the load latency; the second slot only costs VGPRs.  Two where that keeps the kernel
    // at <= 64 VGPRs anyway (8 waves per SIMD either way: C1 1-ch u8 -1 % at depth 1), one where
    // the second slot crosses 64: the four-channel table / linear / mixed / fast16-f32 forms
    // (65-72 VGPRs at depth 2, 57-64 at depth 1; C2 fused 229.9k -> 234.2k tiles/s,
    // profiles/r04/ab_jpeg_f1_prefetch_depth.txt).
#ifndef OMR_F1_DEPTH
#define OMR_F1_DEPTH (NA == kFusedMaxActive && MODE != kFusedFast16 && MODE != kFusedFast16I ? 1 : 2)
#endif
    static constexpr int kDepth = OMR_F1_DEPTH;
    uint32_t raw[kDepth][kFusedMaxActive][2];  // [prefetch slot][channel][row]
    int W, H;
    bool err = false;
    __device__ PlaneSource(const FusedArgs& f, const uint32_t* sc, int tile, int w, int h)
        : F(f), s_contrib(sc), W(w), H(h) {
#pragma unroll
        for (int a = 0; a < kFusedMaxActive; ++a) {
            const int c = F.R.ch[a].index;
            base[a] = F.strided ? F.sbase + (int64_t)tile * F.tile_stride + (int64_t)c * F.chan_stride
                                : static_cast<const uint8_t*>(F.planes[(int64_t)tile * F.size_c + c]);
        }
    }
    // Output pixels (x0, x0+1) x (y0, y0+1), x0 even, come from the source pair starting at sx
    // (reversed under flip_h) on rows sy0, sy1.
    template <int S>
    __device__ __forceinline__ void issue(int x0, int y0) {
        const int sx = F.flip_h ? W - 2 - x0 : x0;
        // 32-bit byte offsets from the uniform plane base (the host keeps the plane below 4 GiB):
        // global_load with an SGPR base and a VGPR offset, no 64-bit address arithmetic per load
        const uint32_t rs = (uint32_t)F.row_stride;
        const uint32_t r0 = ((uint32_t)(F.flip_v ? H - 1 - y0 : y0) * rs + (uint32_t)sx) * BPP;
        const uint32_t r1 = ((uint32_t)(F.flip_v ? H - 2 - y0 : y0 + 1) * rs + (uint32_t)sx) * BPP;
#pragma unroll
        for (int a = 0; a < NA; ++a) {
            if constexpr (BPP == 2) {   // global, not flat, loads: see ld_global
                raw[S][a][0] = ld_global<uint32_t>(base[a] + r0);
                raw[S][a][1] = ld_global<uint32_t>(base[a] + r1);
            } else {
                raw[S][a][0] = ld_global<uint16_t>(base[a] + r0);
                raw[S][a][1] = ld_global<uint16_t>(base[a] + r1);
            }
        }
    }
    // 16-bit LUT-domain check (QuantizationException): per channel with a domain narrower than
    // its type, the two rows' packed 2 x 16-bit extremes (v_pk_max/min_u16) are compared with the
    // domain ends packed the same way (FusedRender::dlo2 / dhi2): six VALU per channel and MCU and
    // no registers kept across MCUs (round 2 kept per-lane min/max: 2 x NA VGPRs, 73 instead of
    // 66 for four channels, 6 instead of 7 waves per SIMD).
    // contribution-table entry of pixel j (0: lower address, 1: upper) of raw word w, channel a
    // (16-bit types: w already in native byte order)
    __device__ __forceinline__ uint32_t entry(int a, uint32_t w, int j) {
        const uint32_t* tab = s_contrib + a * 256;
        if constexpr (BPP == 1) {
            const uint32_t e = tab[(w >> (8 * j)) & 0xFF];
            err |= (e & kErrBit) != 0;
            return e & ~kErrBit;
        } else {
            const int x = (int)(j ? (w >> 16) : (w & 0xFFFF));   // int16: biased to unsigned (take())
            const K2Chan& p = F.R.ch[a];
            uint32_t v;
            if constexpr (MODE == kFusedFast16) {
                v = fast16(x, p);
            } else if constexpr (MODE == kFusedFast16I) {
                v = fast16i(x, p);
            } else if constexpr (MODE == kFusedFast16F || MODE == kFusedFast16FS) {
                v = fast16f(x, p.wsi, F.R.fa[a], F.R.fb[a]);
            } else if (MODE == kFusedLinear16 || p.mode == kModeLinear16) {   // uniform
                v = linear16(x, p, F.R.cd_start, F.R.cds8, F.R.cde8);
            } else {
                const int xi = min(max(x, p.gmin), p.gmax);
                v = reinterpret_cast<const uint8_t*>(p.lut_addr)[(uint32_t)(xi - p.gmin)];
            }
            return tab[v];
        }
    }
#ifndef OMR_F1_PK
#define OMR_F1_PK 1
#endif
    // fast16f on a pixel pair in packed f32: each 16-bit half becomes the float 2^23 + x by one
    // v_perm (exponent byte 0x4B over the half's two bytes, big-endian swap included), one
    // v_pk_add_f32 subtracts 2^23 + wsi (exact: integers below 2^24) and one v_pk_fma_f32 applies
    // fa, fb -- the same floats and the same single rounding as fast16f's cvt + fma per pixel.
    __device__ __forceinline__ void entry_pair_f32(int a, uint32_t w, uint32_t& lo, uint32_t& hi) {
        typedef float f2 __attribute__((ext_vector_type(2)));
        const uint32_t* tab = s_contrib + a * 256;
        // w in file order: a big-endian half's first byte is its high byte
        constexpr uint32_t kSelLo = BE ? 0x070C0001u : 0x070C0100u, kSelHi = BE ? 0x070C0203u : 0x070C0302u;
        const f2 X = {__int_as_float((int)__builtin_amdgcn_perm(0x4B000000u, w, kSelLo)),
                      __int_as_float((int)__builtin_amdgcn_perm(0x4B000000u, w, kSelHi))};
        const float c = F.R.fc[a], fa = F.R.fa[a], fb = F.R.fb[a];
        const f2 d = X - (f2){c, c};
        const f2 y = __builtin_elementwise_fma(d, (f2){fa, fa}, (f2){fb, fb});
        const int32_t b0 = __float_as_int(y.x), b1 = __float_as_int(y.y);
        lo += tab[min(max(b0, kMagicBits), kMagicBits + 255) - kMagicBits];
        hi += tab[min(max(b1, kMagicBits), kMagicBits + 255) - kMagicBits];
    }
    template <int S>
    __device__ __forceinline__ void take(Px2 (&px)[4]) {
        uint32_t acc[4] = {0, 0, 0, 0};         // source order: (lo, hi) of row 0, then row 1
#pragma unroll
        for (int a = 0; a < NA; ++a) {
            uint32_t w0 = raw[S][a][0], w1 = raw[S][a][1];
            if constexpr (BPP == 2 && (MODE == kFusedFast16F || MODE == kFusedFast16FS) && OMR_F1_PK &&
                          (OMR_ABL & kAblRender) == 0) {
                // packed form: the byte swap of big-endian pixels is folded into the v_perm that
                // builds 2^23 + x, so the raw word stays in file order (the sign bias moves to
                // each half's first byte; int16 pixels only: a compile-time mode)
                if constexpr (MODE == kFusedFast16FS) {
                    constexpr uint32_t sg = BE ? 0x00800080u : 0x80008000u;
                    w0 ^= sg;
                    w1 ^= sg;
                }
                if (F.R.any_check && F.R.ch[a].check) {      // wave-uniform
                    const uint32_t n0 = BE ? bswap16x2(w0) : w0, n1 = BE ? bswap16x2(w1) : w1;
                    const uint32_t hi2 = F.R.dhi2[a], lo2 = F.R.dlo2[a];
                    err |= ((pk_max_u16(pk_max_u16(n0, n1), hi2) ^ hi2) | (pk_min_u16(pk_min_u16(n0, n1), lo2) ^ lo2)) != 0;
                }
                entry_pair_f32(a, w0, acc[0], acc[1]);
                entry_pair_f32(a, w1, acc[2], acc[3]);
                continue;
            }
            if constexpr (BPP == 2) {
                if constexpr (BE) { w0 = bswap16x2(w0); w1 = bswap16x2(w1); }
                // int16 pixels biased to unsigned (x + 32768, one XOR per pixel pair); the host
                // moved the channel's window, LUT domain and thresholds by the same amount
                const uint32_t sg = F.R.is_signed ? 0x80008000u : 0u;
                w0 ^= sg;
                w1 ^= sg;
                if (F.R.any_check && F.R.ch[a].check) {      // wave-uniform
                    const uint32_t hi2 = F.R.dhi2[a], lo2 = F.R.dlo2[a];
                    err |= ((pk_max_u16(pk_max_u16(w0, w1), hi2) ^ hi2) | (pk_min_u16(pk_min_u16(w0, w1), lo2) ^ lo2)) != 0;
                }
            }
            if constexpr ((OMR_ABL & kAblRender) != 0) {   // raw words instead of quantize + table
                acc[0] += w0 & 0x3FF; acc[1] += w0 >> 22; acc[2] += w1 & 0x3FF; acc[3] += w1 >> 22;
                continue;
            }
            acc[0] += entry(a, w0, 0);
            acc[1] += entry(a, w0, 1);
            acc[2] += entry(a, w1, 0);
            acc[3] += entry(a, w1, 1);
        }
        if (F.flip_h) {                         // the upper half of each pair is the left output pixel
            const uint32_t t0 = acc[0], t2 = acc[2];
            acc[0] = acc[1]; acc[1] = t0; acc[2] = acc[3]; acc[3] = t2;
        }
        // the packed pairs straight from the 10-bit sums (r << 20 | g << 10 | b), each component
        // clamped to 255 by one v_pk_min_u16 per pair (no ARGB pack for the colour transform)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t g = (acc[j] << 6) & 0x03FF0000u;
            px[j] = Px2{pk_min_u16((acc[j] >> 20) | g, 0x00FF00FFu), pk_min_u16((acc[j] & 0x3FFu) | g, 0x00FF00FFu)};
        }
    }
    __device__ __forceinline__ uint32_t at(int, int) const { return 0; }   // never: H % 16 == 0
    __device__ __forceinline__ bool grey_possible() const { return F.R.grey_ok != 0; }
    // after the last MCU: a channel whose domain holds no 16-bit value fails every pixel
    __device__ __forceinline__ void finish() {
        if constexpr (BPP == 2) err |= F.R.dnone != 0;
    }
};

// The B1 body for one pixel source (see k_jpeg_fdct_batch below).
template <class Src>
__device__ __forceinline__ void b1_body(const B1Args& A, Src& src, int* S) {
    const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int tile = blockIdx.y;
    const int W = A.W, H = A.H;
    const int cx = lane & 7, cy = lane >> 3;
    const int ywib = (W + 7) / 8, yhib = (H + 7) / 8;
    const int nat = c_zigzag[lane];                 // this lane owns zig-zag position `lane`
    const int qy = A.qt.q[0][nat], qc = A.qt.q[1][nat];
    const uint32_t my_ = A.qt.m[0][nat], mc_ = A.qt.m[1][nat];   // host-computed (no 64-bit divide)
    // s_waitcnt vmcnt(0) once, here: the quantiser's per-lane table loads are then known complete,
    // so the loop's first use of them does not wait for the pixel prefetches and coefficient
    // stores issued since (vmcnt counts every load and store in issue order)
    __builtin_amdgcn_s_waitcnt(0x0F70);
    const int hy = qy << 2, hc = qc << 2;
    // The workgroup's 4 * mpw MCUs are dealt round robin: at step j its four waves transform four
    // horizontally adjacent MCUs (m = base + 4j + wave), so each row's 4 x 32 bytes of 16-bit
    // planes (or 4 x 64 bytes of ARGB) are one 128-byte line read by the four waves together.
    const int mbase = blockIdx.x * 4 * A.mpw;
    const int cnt = max(0, min(A.mpw, (A.n_mcu - mbase - wv + 3) / 4));   // steps with m < n_mcu
    const int nat_off = (nat >> 3) * kRS + (nat & 7);   // zig-zag position `lane` in the block
    // MCU coordinates advance incrementally (no per-MCU division by the MCU row length)
    int mx = (mbase + wv) % A.mcux, my = (mbase + wv) / A.mcux;
    int nx = mx, ny = my;                          // the next MCU to prefetch
    auto step = [&](int& x, int& y) {              // m += 4
        x += 4;
        while (x >= A.mcux) { x -= A.mcux; ++y; }
    };
    // Every step issues its prefetch -- past the wave's last MCU it reloads the current one -- so
    // the load / store stream is the same on every trip and the compiler's wait counts stay exact
    // (a conditional prefetch made it wait for every outstanding load, the prefetch included).
    auto fetch = [&](auto slot, bool valid) {
        src.template issue<decltype(slot)::value>((valid ? nx : mx) * 16 + 2 * cx, (valid ? ny : my) * 16 + 2 * cy);
        step(nx, ny);
    };
    int abl_sink = 0;                             // ablation builds only: keeps dropped results live
    int rec = 0;                                  // per-block records of this wave's MCUs (lane 6j + k)
    // Grey MCU (every pixel r == g == b, e.g. the greyscale model's output): IJG's Y is then
    // (65536 v + 32768) >> 16 = v exactly and Cb = Cr = 128, so both chroma blocks are zero —
    // the colour transform, their FDCT and their quantisation are skipped.  Wave-uniform; the
    // bottom-edge chroma rows (odd heights) take the general path.
    // Two prefetch slots: step j's pixels arrive in slot j & 1, loaded two steps ahead.
    auto mcu = [&](auto slot, int j) {
        constexpr int SL = decltype(slot)::value;
        const int m = mbase + 4 * j + wv;
        bool grey;
        {
            const int x0 = mx * 16 + 2 * cx;
            Px2 px[4];                                  // (x0, y0) (x0+1, y0) (x0, y0+1) (x0+1, y0+1)
            src.template take<SL>(px);
            fetch(slot, j + Src::kDepth < cnt);
            const int chv = (H + 1) / 2;
            const int cyg = my * 8 + cy;
            const bool edge = Src::kEdgeRows && cyg >= chv;
            // (wave-uniform: only where the source can be grey at all; the general path gives the
            // same coefficients for a grey MCU, so the test is purely a shortcut)
            grey = src.grey_possible() &&
                   __ballot(!(is_grey(px[0]) && is_grey(px[1]) && is_grey(px[2]) && is_grey(px[3])) || edge) == 0;
            int y, cb0, cr0, cb1, cr1, cb2, cr2, cb3, cr3;
            const int blk = (cy >> 2) * 2 + (cx >> 2);
            const int o = blk * kBS + ((2 * cy) & 7) * kRS + ((2 * cx) & 7);
            if (grey) {
                S[o] = (int)(px[0].bg & 0xFFFFu) - 128;
                S[o + 1] = (int)(px[1].bg & 0xFFFFu) - 128;
                S[o + kRS] = (int)(px[2].bg & 0xFFFFu) - 128;
                S[o + kRS + 1] = (int)(px[3].bg & 0xFFFFu) - 128;
            } else if constexpr ((OMR_ABL & kAblColour) != 0) {
                S[o] = px[0].rg & 0xFF; S[o + 1] = px[1].bg >> 16; S[o + kRS] = px[2].bg & 0xFF; S[o + kRS + 1] = px[3].rg & 0xFF;
                S[4 * kBS + cy * kRS + cx] = px[0].rg >> 16;
                S[5 * kBS + cy * kRS + cx] = px[1].bg & 0xFF;
            } else {
            ycc(px[0], y, cb0, cr0); S[o] = y - 128;
            ycc(px[1], y, cb1, cr1); S[o + 1] = y - 128;
            ycc(px[2], y, cb2, cr2); S[o + kRS] = y - 128;
            ycc(px[3], y, cb3, cr3); S[o + kRS + 1] = y - 128;
            if (edge) {
                const int xa = min(x0, W - 1), xb = min(x0 + 1, W - 1);
                const int r0 = min(2 * (chv - 1), H - 1), r1 = min(2 * (chv - 1) + 1, H - 1);
                ycc(px2_of(src.at(xa, r0)), y, cb0, cr0); ycc(px2_of(src.at(xb, r0)), y, cb1, cr1);
                ycc(px2_of(src.at(xa, r1)), y, cb2, cr2); ycc(px2_of(src.at(xb, r1)), y, cb3, cr3);
            }
            const int bias = (cx & 1) ? 2 : 1;
            S[4 * kBS + cy * kRS + cx] = ((cb0 + cb1 + cb2 + cb3 + bias) >> 2) - 128;
            S[5 * kBS + cy * kRS + cx] = ((cr0 + cr1 + cr2 + cr3 + bias) >> 2) - 128;
            }
        }
        const int nfd = grey ? 32 : 48;   // lanes with a block row / column to transform
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        if ((OMR_ABL & kAblFdct) == 0 && lane < nfd) fdct8<0>(S + (lane >> 3) * kBS + (lane & 7) * kRS, 1);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        if ((OMR_ABL & kAblFdct) == 0 && lane < nfd) fdct8<1>(S + (lane >> 3) * kBS + (lane & 7), kRS);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        const int64_t b0 = (int64_t)tile * A.nb + (int64_t)m * 6;
        int16_t* out = A.coefs + b0 * 64;
        int8_t* out8 = A.coef8 + b0 * 64;
        int qv[6];
        int coef[6];                              // all six blocks' coefficients read back to back
#pragma unroll
        for (int k = 0; k < 6; ++k) coef[k] = (k >= 4 && grey) ? 0 : S[k * kBS + nat_off];
#pragma unroll
        for (int k = 0; k < 6; ++k) {
            int q = (k >= 4 && grey) ? 0                       // zero chroma block
                  : (OMR_ABL & kAblQuant) ? coef[k] : k < 4 ? quant_recip(coef[k], hy, my_) : quant_recip(coef[k], hc, mc_);
            if (Src::kEdgeRows && k < 4) {
                const int bx = mx * 2 + (k & 1), by = my * 2 + (k >> 1);
                if ((bx >= ywib || by >= yhib) && lane != 0) q = 0;   // dummy block: AC zero
            }
            qv[k] = q;
        }
        // jccoefct.c dummy-block DC propagation on the wave-uniform DCs (lane 0's coefficient),
        // then each block's 64 coefficients in one store.  A block whose 63 ACs all fit int8 --
        // nearly every block at any quality -- goes out as 64 bytes, so B2a and B3 read half the
        // bytes; one with a larger AC as 128 (int16, lane 0 storing the propagated DC), flagged in
        // bit 0 of its record.  The blocks' Huffman lengths are B2a's (one lane per block walks
        // the stored coefficients: half the instructions of a ballot-per-coefficient length here).
        int dc[6];
#pragma unroll
        for (int k = 0; k < 6; ++k) dc[k] = __builtin_amdgcn_readfirstlane(qv[k]);
        if constexpr (Src::kEdgeRows) {
            const bool c1 = mx * 2 + 1 >= ywib, row1 = my * 2 + 1 >= yhib;
            if (c1) dc[1] = dc[0];
            if (row1) { dc[2] = dc[1]; dc[3] = dc[1]; }
            else if (c1) dc[3] = dc[2];
        }
        // one choice for the MCU's six blocks: an AC outside int8 in any of them (OR of the
        // biased values: a bit above bit 7 in any) makes all six int16
        uint64_t big = 0;                         // lanes holding an AC outside int8 (lane 0: the DC)
#pragma unroll
        for (int k = 0; k < 6; ++k) big |= __ballot((uint32_t)(qv[k] + 128) > 255u);
        const uint32_t wide = (big & ~1ull) != 0 ? 0x3Fu : 0u;   // bit k: block k int16 (all or none)
        // the int16 form is one rarely taken, wave-uniform branch; the int8 stores are
        // unconditional (an int16 MCU's bytes are never read)
        if ((OMR_ABL & kAblCoefStore) == 0 && wide) {
#pragma unroll
            for (int k = 0; k < 6; ++k) {
                const int v = lane == 0 ? dc[k] : qv[k];
                *reinterpret_cast<int16_t*>(reinterpret_cast<uint8_t*>(out) + (uint32_t)(k * 128 + lane * 2)) = (int16_t)v;
            }
        }
#pragma unroll
        for (int k = 0; k < 6; ++k) {
            if constexpr ((OMR_ABL & kAblCoefStore) != 0) abl_sink ^= qv[k];
            else *reinterpret_cast<int8_t*>(reinterpret_cast<uint8_t*>(out8) + (uint32_t)(k * 64 + lane)) = (int8_t)qv[k];
        }
        // the six per-block DC records go to lanes 6j .. 6j+5 of `rec` (j: this MCU's index in
        // the wave's run); one store per wave after the loop instead of six one-lane stores per MCU
        if constexpr ((OMR_ABL & kAblLane0) != 0) {
            abl_sink ^= dc[0] + dc[5];
        } else {
#pragma unroll
            for (int k = 0; k < 6; ++k) rec = lane_write((int)(((uint32_t)dc[k] << 16) | ((wide >> k) & 1u)), 6 * j + k, rec);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");   // S is rewritten by the next MCU
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        step(mx, my);
    };
    using S0 = std::integral_constant<int, 0>;
    using S1 = std::integral_constant<int, 1>;
    if constexpr (Src::kDepth == 1) {
        if (cnt > 0) fetch(S0{}, true);
        for (int j = 0; j < cnt; ++j) mcu(S0{}, j);
    } else {
        if (cnt > 0) {
            fetch(S0{}, true);
            fetch(S1{}, cnt > 1);
        }
        for (int j = 0; j < cnt; j += 2) {   // wave-uniform loop, two steps per trip (static slots)
            mcu(S0{}, j);
            if (j + 1 < cnt) mcu(S1{}, j + 1);
        }
    }
    if ((OMR_ABL & kAblLane0) == 0 && lane < 6 * cnt)
        A.blk[(int64_t)tile * A.nb + (int64_t)(mbase + 4 * (lane / 6) + wv) * 6 + lane % 6] = (uint32_t)rec;
    if constexpr (OMR_ABL != 0)
        if (abl_sink == 0x7FFF1234) A.blk[lane] = (uint32_t)abl_sink;
}

__global__ void __launch_bounds__(256) k_jpeg_fdct_batch(B1Args A) {
    __shared__ int s[4][6 * kBS + 8];
    ArgbSource src(A, blockIdx.y);
    b1_body(A, src, s[__builtin_amdgcn_readfirstlane(threadIdx.x >> 6)]);
}

// F1: fused render + B1 (see PlaneSource).  The contribution tables are staged once per
// workgroup; a pixel outside its channel's LUT domain flags the tile (QuantizationException).
template <int BPP, bool BE, int MODE, int NA>
__global__ void __launch_bounds__(256) k_jpeg_render_fdct(B1Args A, FusedArgs F) {
    __shared__ int s[4][6 * kBS + 8];
    __shared__ uint32_t s_contrib[kFusedMaxActive * 256];
    for (int i = threadIdx.x; i < NA * 256; i += 256) s_contrib[i] = F.R.contrib[i];
    __syncthreads();
    PlaneSource<BPP, BE, MODE, NA> src(F, s_contrib, blockIdx.y, A.W, A.H);
    b1_body(A, src, s[__builtin_amdgcn_readfirstlane(threadIdx.x >> 6)]);
    src.finish();
    if (__ballot(src.err)) {
        if ((threadIdx.x & 63) == 0) {
            atomicOr(F.R.flag, 1);
            if (F.rstat) F.rstat[blockIdx.y] = OMR_QUANTIZATION;
        }
    }
}

__device__ __forceinline__ int prev_block_in_tile(int b) {
    const int m = b / 6, k = b - m * 6;
    if (k == 1 || k == 2 || k == 3) return b - 1;
    if (m == 0) return -1;
    return k == 0 ? (m - 1) * 6 + 3 : (m - 1) * 6 + k;
}

constexpr int kTileThreads = 1024;
constexpr int kB3LdsWords = 4096;   // B3: a group's stream staged in LDS up to 512 bits per block
constexpr int kGrp = 256;   // blocks per B3 workgroup = chunks per B4a/B6 group

__device__ __forceinline__ uint32_t block_reduce_sum(uint32_t v, uint32_t* s_wave) {
    uint32_t total;
    block_exclusive_scan(v, s_wave, total);
    return total;
}

// B2a: one lane per 8x8 block: its bit length, and per-256-block group sums.  The DC part needs
// the previous block's DC in scan order (B1's records); the AC part walks the block's 63
// zig-zag coefficients (eight 16-byte loads into registers, the walk unrolled): run length,
// magnitude category by frexp, code length from an LDS table, ZRLs and EOB, branch-free.
struct B2aArgs {
    const int16_t* coefs;  // [tile][nb][64] zig-zag order (int16 blocks)
    const int8_t* coef8;   // [tile][nb][64] zig-zag order (int8 blocks)
    const uint32_t* blk;   // B1's per-block records (DC << 16 | int16 flag)
    uint16_t* bits;        // [tile][nb]
    uint32_t* gsum;        // [tile][ngb]
    int32_t nb, ngb;
};

// Block b of a 256-block group whose first block is g0: its 64 coefficients from the group's
// uniform base plus a 32-bit byte offset (an SGPR-base load, no 64-bit address VALU).
__device__ __forceinline__ const uint4* group_block_coefs(const int16_t* coefs, int64_t g0, int i) {
    return reinterpret_cast<const uint4*>(reinterpret_cast<const uint8_t*>(coefs + g0 * 64) + (uint32_t)i * 128u);
}
__device__ __forceinline__ const uint4* group_block_coefs8(const int8_t* coef8, int64_t g0, int i) {
    return reinterpret_cast<const uint4*>(reinterpret_cast<const uint8_t*>(coef8 + g0 * 64) + (uint32_t)i * 64u);
}

__device__ __forceinline__ uint32_t u4_at(const uint4& v, int c) {   // c static after unrolling
    return c == 0 ? v.x : c == 1 ? v.y : c == 2 ? v.z : v.w;
}
// Zig-zag coefficient k of a block held in registers: int8 blocks in q[0..3] (byte k), int16
// blocks in q[0..7] (half k).
template <bool NARROW>
__device__ __forceinline__ int block_coef(const uint4 (&q)[8], int k) {
    if constexpr (NARROW) {
        const uint32_t w = u4_at(q[k >> 4], (k >> 2) & 3);
        return (int)(int8_t)(w >> (8 * (k & 3)));
    } else {
        const uint32_t w = u4_at(q[k >> 3], (k >> 1) & 3);
        return (k & 1) ? (int)(int16_t)(w >> 16) : (int)(int16_t)(w & 0xFFFF);
    }
}
// An int8 block in q[0..3] widened in place to the int16 form in q[0..7] (the lanes of a wave
// that also holds an int16 block: the wave then walks every block in the int16 form).
__device__ __forceinline__ void widen_block(uint4 (&q)[8]) {
    auto pair = [](uint32_t w, int h) {
        return ((uint32_t)(int)(int8_t)(w >> (16 * h)) & 0xFFFFu) | ((uint32_t)(int)(int8_t)(w >> (16 * h + 8)) << 16);
    };
#pragma unroll
    for (int i = 7; i >= 0; --i) {   // q[i] from q[i >> 1], which a later (lower) i still reads
        const uint32_t w0 = u4_at(q[i >> 1], (i & 1) * 2), w1 = u4_at(q[i >> 1], (i & 1) * 2 + 1);
        q[i] = make_uint4(pair(w0, 0), pair(w0, 1), pair(w1, 0), pair(w1, 1));
    }
}

// Magnitude category (bit length of |c|, 0 for 0) of a coefficient: frexp's exponent of the exact
// float, sign-independent (two instructions instead of abs + clz + a zero select).
__device__ __forceinline__ int mag_bits(int c) { return __builtin_amdgcn_frexp_expf((float)c); }

// (Staging the workgroup's 32 KiB of coefficients through LDS with coalesced loads, rows of
// 9 x 16 B, measured 2.4x slower than each lane loading its own 128 B: 121 vs 48 us per 64 C2
// tiles, profiles/r03/ab_jpeg_b2a_variants.txt.)
__global__ void __launch_bounds__(kGrp) k_jpeg_block_bits(B2aArgs A) {
    __shared__ uint8_t s_dc[2][16];
    // code length of (run r < 64, category nb) with the r >> 4 ZRL codes folded in, indexed by
    // r * 16 + nb; 0 for nb == 0 (a zero coefficient adds nothing)
    __shared__ __attribute__((aligned(16))) uint16_t s_len[2][1024];
    __shared__ uint32_t sw[16];
    const int tile = blockIdx.y, b0 = blockIdx.x * kGrp, b = b0 + threadIdx.x;
    if (threadIdx.x < 32) s_dc[threadIdx.x >> 4][threadIdx.x & 15] = c_huff[2 * (threadIdx.x >> 4)].size[threadIdx.x & 15];
    reinterpret_cast<uint4*>(&s_len[0][0])[threadIdx.x] = reinterpret_cast<const uint4*>(&c_aclen.v[0][0])[threadIdx.x];
    __syncthreads();
    uint32_t bits = 0;
    if (b < A.nb) {
        const int64_t gb = (int64_t)tile * A.nb + b;
        const uint32_t* blk = A.blk + (int64_t)tile * A.nb;
        // the int8 form is loaded before the record says which form the block has, so the two
        // loads overlap (an int16 block -- rare -- then reads its own form below)
        uint4 q[8];
#pragma unroll
        for (int i = 0; i < 4; ++i) q[i] = group_block_coefs8(A.coef8, (int64_t)tile * A.nb + b0, threadIdx.x)[i];
        const uint32_t rb = blk[b];
        const bool wide = (rb & 1u) != 0;
        const int pb = prev_block_in_tile(b);
        const int d = (int)(int16_t)(rb >> 16) - (pb >= 0 ? (int)(int16_t)(blk[pb] >> 16) : 0);
        const int nbd = mag_bits(d);
        const int t = (b % 6) < 4 ? 0 : 1;
        bits = s_dc[t][nbd] + nbd;
        const uint16_t* len = s_len[t];
        uint32_t r16 = 0;                                  // zero run before coefficient k, times 16
        // eight coefficients at a time: their table indices first (the run chain is VALU only),
        // then the eight LDS reads in flight together
        if (!wide) {
            // an int8 block: its 64 bytes in registers, the walk unrolled
#pragma unroll
            for (int k0 = 0; k0 < 64; k0 += 8) {
                uint32_t idx[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const int k = k0 + j;
                    if (k == 0) { idx[j] = 0; continue; }
                    const int nb = mag_bits(block_coef<true>(q, k));
                    idx[j] = r16 | nb;
                    bits += nb;
                    r16 = nb ? 0u : r16 + 16;
                }
#pragma unroll
                for (int j = 0; j < 8; ++j) bits += (k0 + j) ? len[idx[j]] : 0u;   // zero coefficient: entry 0
            }
        } else {
            // an int16 block (an AC outside int8: rare): eight coefficients per 16-byte load, the
            // next load in flight while these are walked
            const uint4* cp = group_block_coefs(A.coefs, (int64_t)tile * A.nb + b0, threadIdx.x);
            uint4 v = cp[0];
#pragma unroll 1
            for (int i = 0; i < 8; ++i) {
                const uint4 nv = i < 7 ? cp[i + 1] : v;
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    if (i == 0 && j == 0) continue;
                    const uint32_t w = u4_at(v, j >> 1);
                    const int nb = mag_bits((j & 1) ? (int)(int16_t)(w >> 16) : (int)(int16_t)(w & 0xFFFF));
                    bits += nb + len[r16 | nb];
                    r16 = nb ? 0u : r16 + 16;
                }
                v = nv;
            }
        }
        if (r16) bits += c_huff[1 + 2 * t].size[0x00];     // EOB after the last non-zero
        A.bits[gb] = (uint16_t)(bits | (wide ? kWideFlag : 0u));   // bit count | 0x800 x ZRL-prefixed coefficients
        bits &= kZrlFlag - 1;
    }
    const uint32_t total = block_reduce_sum(bits, sw);
    if (threadIdx.x == 0) A.gsum[(int64_t)tile * A.ngb + blockIdx.x] = total;
}

// B2b / B4b: one workgroup per tile: exclusive scan of its group sums (in place), the tile
// total, and (B2b) zeroing of the words the tile's bit stream will occupy.
struct GroupScanArgs {
    uint32_t* gsum;              // [tile][stride] -> exclusive offsets
    const uint32_t* n_groups;    // [tile] (nullptr: fixed_groups)
    uint32_t* total;             // [tile]
    uint32_t* zero_words;        // B2b: [tile][slot_words] words B3 ORs into, zeroed (or nullptr)
    const uint32_t* base_add;    // B4b: total += base_add-derived byte count (or nullptr)
    int64_t stride, slot_words;
    int32_t fixed_groups;
};

__global__ void __launch_bounds__(kTileThreads) k_jpeg_group_scan(GroupScanArgs A) {
    __shared__ uint32_t sw[16];
    __shared__ uint32_t carry;
    __shared__ int s_unstaged;
    const int tile = blockIdx.x;
    uint32_t* g = A.gsum + (int64_t)tile * A.stride;
    const uint32_t ng = A.n_groups ? A.n_groups[tile] : (uint32_t)A.fixed_groups;
    uint32_t* zw = A.zero_words ? A.zero_words + (int64_t)tile * A.slot_words : nullptr;
    if (threadIdx.x == 0) { carry = 0; s_unstaged = 0; }
    __syncthreads();
    for (uint32_t base = 0; base < ng; base += kTileThreads) {
        const uint32_t i = base + threadIdx.x;
        const uint32_t v = i < ng ? g[i] : 0;
        uint32_t tot;
        const uint32_t ex = block_exclusive_scan(v, sw, tot);
        const uint32_t c = carry;
        if (i < ng) g[i] = c + ex;
        // B2b: B3 builds a group's words in LDS and ORs only its first and last word into HBM
        // (shared with the neighbouring groups), so only those need zeroing; a group too long
        // for B3's LDS (ORs at every block boundary) makes the whole tile zeroed below
        if (zw && i < ng && v) {
            const uint32_t w0 = (c + ex) >> 5, w1 = (c + ex + v - 1) >> 5;
            if (w1 - w0 + 1 <= (uint32_t)kB3LdsWords) { zw[w0] = 0; zw[w1] = 0; }
            else s_unstaged = 1;
        }
        __syncthreads();
        if (threadIdx.x == 0) carry = c + tot;
        __syncthreads();
    }
    uint32_t total = carry;
    if (A.base_add) total += (A.base_add[tile] + 7) / 8;   // B4b: stuffed bytes = bytes + 0xFF count
    if (threadIdx.x == 0) A.total[tile] = total;
    if (zw && s_unstaged) {                                // every word of the tile's bit stream
        const uint32_t nw = (total + 31) / 32 + 1;
        uint4* w4 = reinterpret_cast<uint4*>(zw);
        for (uint32_t i = threadIdx.x; i < (nw + 3) / 4; i += kTileThreads) w4[i] = make_uint4(0, 0, 0, 0);
    }
}

struct B3Args {
    const int16_t* coefs;    // int16 blocks
    const int8_t* coef8;     // int8 blocks
    const uint32_t* blk;     // B1's per-block records (DC << 16 | int16 flag)
    const uint16_t* bits;    // [tile][nb]
    const uint32_t* goff;    // [tile][ngb] exclusive bit offset of each 256-block group
    uint32_t* words;
    int32_t nb, ngb;
    int64_t slot_words;
};

// B3: one lane per 8x8 block; the workgroup's 256 consecutive blocks find their bit offsets
// by a block scan on top of the group offset.  The block's 64 zig-zag coefficients arrive as
// eight 16-byte loads into registers (the loop over them is unrolled, so every coefficient is
// a static register), the codes come from the LDS Huffman tables and accumulate in a 64-bit
// register; whole 32-bit words are stored directly, the two words a block may share with its
// neighbours are ORed in.

__global__ void __launch_bounds__(kGrp) k_jpeg_huff_thread(B3Args A) {
    // AC tables packed as size << 16 | code (size-0 entries zeroed: a zero coefficient codes as
    // zero bits with no select in the coefficient loop), then the DC tables
    __shared__ __attribute__((aligned(16))) B3Tabs s_t;
    __shared__ uint32_t s_words[kB3LdsWords];
    __shared__ uint32_t sw[16];
    if (threadIdx.x < (int)(sizeof(B3Tabs) / 16))
        reinterpret_cast<uint4*>(&s_t)[threadIdx.x] = reinterpret_cast<const uint4*>(&c_b3tabs)[threadIdx.x];
    const int tile = blockIdx.y;
    const int b = blockIdx.x * kGrp + threadIdx.x;
    const int64_t gb = (int64_t)tile * A.nb + b;
    const bool live = b < A.nb;
    const uint32_t brec = live ? A.bits[gb] : 0u;
    const uint32_t mybits = brec & (kZrlFlag - 1);
    // no block of the wave has a zero run of 16+ before a non-zero (B2a's kZrlFlag multiples): the
    // walk below drops its per-coefficient ZRL vote
    const bool any_zrl = __ballot((brec & ~kWideFlag) >= kZrlFlag) != 0;
    // B2a's copy of the block's int16 flag: which form to load is known before any coefficient
    // load, so the loads need not wait for the block record
    const bool wide = (brec & kWideFlag) != 0;
    const bool any_wide = __ballot(wide) != 0;
    uint32_t gtot;
    const uint32_t gbit0 = A.goff[(int64_t)tile * A.ngb + blockIdx.x];
    const uint32_t boff = gbit0 + block_exclusive_scan(mybits, sw, gtot);
    // The group's 256 blocks form one contiguous run of the stream: when it fits, it is built in
    // LDS (ds_or) and copied out coalesced, so HBM sees whole lines instead of one 4-byte store
    // per lane per word; the group's first and last words are shared with neighbouring groups.
    const uint32_t gw0 = gbit0 >> 5;
    const uint32_t nw = (uint32_t)__builtin_amdgcn_readfirstlane((int)(gtot ? ((gbit0 + gtot - 1) >> 5) - gw0 + 1 : 0));
    const bool staged = nw <= (uint32_t)kB3LdsWords;
    uint32_t* words = A.words + (int64_t)tile * A.slot_words;
    if (staged) {
        for (uint32_t i = threadIdx.x; i < nw; i += kGrp) s_words[i] = 0;
        __syncthreads();
    }
    // The coder, instantiated for the LDS-staged group (the common case: a flush is one ds_or at
    // a running LDS pointer) and for a group too long for the staging buffer (word stores, the
    // block's shared first word ORed into HBM).
    // NARROW: every block of the wave is int8 (and no ZRL, staged): the walk reads bytes.
    // Otherwise int8 blocks are widened in registers and the wave walks the int16 form.
    auto code_block = [&](auto staged_c, auto narrow_c) {
        constexpr bool STAGED = decltype(staged_c)::value;
        constexpr bool NARROW = decltype(narrow_c)::value;
        const int64_t g0 = (int64_t)tile * A.nb + (int64_t)blockIdx.x * kGrp;
        const uint32_t myrec = A.blk[gb];
        uint4 q[8];
        if (NARROW || !wide) {
#pragma unroll
            for (int i = 0; i < 4; ++i) q[i] = group_block_coefs8(A.coef8, g0, threadIdx.x)[i];
            if constexpr (!NARROW) widen_block(q);
        } else {
#pragma unroll
            for (int i = 0; i < 8; ++i) q[i] = group_block_coefs(A.coefs, g0, threadIdx.x)[i];
        }
        const int pb = prev_block_in_tile(b);
        const int pred = pb >= 0 ? (int)(int16_t)(A.blk[(int64_t)tile * A.nb + pb] >> 16) : 0;
        uint64_t acc = 0;
        int nacc = (int)(boff & 31);
        uint32_t wpos = boff >> 5;
        const uint32_t w0 = wpos;
        uint32_t* sp = &s_words[wpos - gw0];          // STAGED: the LDS word the next flush ORs into
        auto flush = [&](uint32_t w) {
            if constexpr (STAGED) { atomicOr(sp, w); ++sp; }
            else {
                if (wpos == w0) atomicOr(&words[wpos], w);   // shares bits with the previous block
                else words[wpos] = w;
                ++wpos;
            }
        };
        auto put = [&](uint32_t v, int n) {          // n <= 26, v < 2^n
            acc = (acc << n) | v;
            nacc += n;
            if (nacc >= 32) {
                // bits [nacc - 32, nacc) of acc: one v_alignbit_b32 of its halves
                flush(__builtin_amdgcn_alignbit((uint32_t)(acc >> 32), (uint32_t)acc, (uint32_t)(nacc - 32)));
                nacc -= 32;
            }
        };
        auto coef = [&](int k) -> int { return block_coef<NARROW>(q, k); };
        const int kk = b % 6;
        const int ta = kk < 4 ? 0 : 1;
        {
            int d = (int)(int16_t)(myrec >> 16) - pred, d2 = d;
            if (d < 0) { d = -d; d2--; }
            const int nbits = d ? 32 - __clz(d) : 0;
            const uint32_t dcc = s_t.dc[ta][nbits];
            put(((dcc & 0xFFFF) << nbits) | ((uint32_t)d2 & ((1u << nbits) - 1)), (int)(dcc >> 16) + nbits);
        }
        const uint32_t zrl = ((uint32_t)c_huff[1 + 2 * ta].size[0xF0] << 16) | c_huff[1 + 2 * ta].code[0xF0];
        const uint32_t eob = ((uint32_t)c_huff[1 + 2 * ta].size[0x00] << 16) | c_huff[1 + 2 * ta].code[0x00];
        int r16 = 0;                                  // zero run before coefficient k, times 16
        // Branch-free per coefficient: a zero contributes a zero-length code; runs of 16+ zeros
        // before a non-zero (ZRL) take a wave-uniform, rarely entered branch, checked only in
        // waves where B2a saw one.
        auto walk = [&](auto with_zrl) {
#pragma unroll
            for (int k = 1; k < 64; ++k) {
                const int c = coef(k);
                const int nbits = mag_bits(c);                         // 0 for c == 0
                const bool nzk = nbits != 0;                           // one compare on the category
                if constexpr (decltype(with_zrl)::value) {
                    if (k > 16 && __ballot(nzk && r16 > 15 * 16)) {        // r <= k - 1: no ZRL before k 17
                        if (nzk) while (r16 > 15 * 16) { put(zrl & 0xFFFF, (int)(zrl >> 16)); r16 -= 16 * 16; }
                    }
                }
                // (r & 15) << 4 is r16 & 0xF0: one v_and_or builds the table index
                const uint32_t cs = s_t.ac[ta][(r16 & 0xF0) | nbits];
                const uint32_t v = ((cs & 0xFFFF) << nbits) | ((uint32_t)(c < 0 ? c - 1 : c) & ((1u << nbits) - 1));
                put(v, (int)(cs >> 16) + nbits);                        // c == 0: cs == 0, nbits == 0
                r16 = nzk ? 0 : r16 + 16;
            }
        };
        if constexpr (NARROW) walk(std::false_type{});
        else if (any_zrl) walk(std::true_type{});
        else walk(std::false_type{});
        if (r16 > 0) put(eob & 0xFFFF, (int)(eob >> 16));                 // EOB
        if (nacc > 0) {                                                   // shared with the next block
            const uint32_t w = (uint32_t)(acc << (32 - nacc));
            if constexpr (STAGED) atomicOr(sp, w);
            else atomicOr(&words[wpos], w);
        }
    };
    if (live) {
        if (staged && !any_zrl && !any_wide) code_block(std::true_type{}, std::true_type{});
        else if (staged) code_block(std::true_type{}, std::false_type{});
        else code_block(std::false_type{}, std::false_type{});
    }
    if (staged) {
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < nw; i += kGrp) {
            const uint32_t w = s_words[i];
            if (i == 0 || i == nw - 1) atomicOr(&words[gw0 + i], w);
            else words[gw0 + i] = w;
        }
    }
}

constexpr int kStuffBytes = 16;   // bytes per chunk in B4a/B6

// 0x80 in every byte of w that is 0xFF, 0 elsewhere (exact: no borrow between bytes).
__device__ __forceinline__ uint32_t ff_bytes(uint32_t w) {
    const uint32_t t = ~w;
    return ~(((t & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | t | 0x7F7F7F7Fu);
}
// 0x80 in each of the first k (big-endian) bytes of a stream word, k in [0, 4].
__device__ __forceinline__ uint32_t first_bytes_mask(int k) {
    return k >= 4 ? 0x80808080u : k <= 0 ? 0u : 0x80808080u & ~(0xFFFFFFFFu >> (8 * k));
}

__device__ __forceinline__ uint32_t seg_byte(const uint32_t* words, uint32_t i, uint32_t nbytes, uint32_t tb) {
    uint32_t b = (words[i >> 2] >> (24 - 8 * (i & 3))) & 0xFF;
    if (i == nbytes - 1 && (tb & 7)) b |= 0xFFu >> (tb & 7);   // jchuff flush: pad with 1s
    return b;
}

// The 16 bytes of chunk c (big-endian bytes of 4 words), pad bits of the final byte set.
__device__ __forceinline__ void chunk_bytes(const uint32_t* words, uint32_t c, uint32_t nbytes, uint32_t tb,
                                            uint32_t (&w)[4]) {
    const uint4 q = reinterpret_cast<const uint4*>(words)[c];
    w[0] = q.x; w[1] = q.y; w[2] = q.z; w[3] = q.w;
    const uint32_t last = nbytes - 1;
    if ((tb & 7) && last >= c * kStuffBytes && last < (c + 1) * kStuffBytes) {
        const uint32_t i = last - c * kStuffBytes;
        w[i >> 2] |= (0xFFu >> (tb & 7)) << (24 - 8 * (i & 3));
    }
}

// B4a: 0xFF count of every 16-byte chunk of the entropy-coded segment (u8) and per-256-chunk
// group sums; a grid-stride loop over the tile's groups (the grid is sized for typical streams).
struct B4aArgs {
    const uint32_t* words;
    const uint32_t* tile_bits;
    uint8_t* cnt;          // [tile][slot_chunks]
    uint32_t* csum;        // [tile][slot_groups]
    uint32_t* n_groups;    // [tile]
    int64_t slot_words, slot_chunks, slot_groups;
};

__global__ void __launch_bounds__(kGrp) k_jpeg_stuff_count(B4aArgs A) {
    // One wave per 256-chunk group, chunks lane, lane + 64, lane + 128, lane + 192 (each load
    // instruction reads 1 KiB of contiguous stream; the four are issued before any is used), the
    // group sum a wave reduction: no workgroup barrier (the workgroup's four waves take four groups).
    const int tile = blockIdx.y;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t tb = A.tile_bits[tile], nbytes = (tb + 7) / 8;
    const uint32_t nch = (nbytes + kStuffBytes - 1) / kStuffBytes;
    const uint32_t ng = (nch + kGrp - 1) / kGrp;
    if (blockIdx.x == 0 && threadIdx.x == 0) A.n_groups[tile] = ng;
    const uint4* words4 = reinterpret_cast<const uint4*>(A.words + (int64_t)tile * A.slot_words);
    uint8_t* cnt = A.cnt + (int64_t)tile * A.slot_chunks;
    for (uint32_t g = blockIdx.x * 4 + wv; g < ng; g += gridDim.x * 4) {
        uint4 q[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) q[k] = words4[min(g * kGrp + k * 64 + lane, nch - 1)];
        uint32_t tot = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t c = g * kGrp + k * 64 + lane;
            uint32_t w[4] = {q[k].x, q[k].y, q[k].z, q[k].w};
            const uint32_t last = nbytes - 1;
            if ((tb & 7) && last >= c * kStuffBytes && last < (c + 1) * kStuffBytes) {   // jchuff pad bits
                const uint32_t i = last - c * kStuffBytes;
                w[i >> 2] |= (0xFFu >> (tb & 7)) << (24 - 8 * (i & 3));
            }
            const uint32_t e = c < nch ? min(nbytes - c * kStuffBytes, (uint32_t)kStuffBytes) : 0u;
            // four bytes at a time: exact 0xFF-byte detection, popcount of the valid ones
            uint32_t n = 0;
#pragma unroll
            for (int j = 0; j < 4; ++j) n += __popc(ff_bytes(w[j]) & first_bytes_mask((int)e - 4 * j));
            if (c < nch) cnt[c] = (uint8_t)n;
            tot += n;
        }
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) tot += __shfl_xor(tot, o, 64);
        if (lane == 0) A.csum[(int64_t)tile * A.slot_groups + g] = tot;
    }
}

__device__ __forceinline__ uint64_t block_exclusive_scan64(uint64_t v, uint64_t* s_wave, uint64_t& total) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
    uint64_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint64_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) s_wave[wid] = x;
    __syncthreads();
    if (wid == 0) {
        uint64_t w = lane < nw ? s_wave[lane] : 0;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint64_t y = __shfl_up(w, o, 64);
            if (lane >= o) w += y;
        }
        if (lane < nw) s_wave[lane] = w;
    }
    __syncthreads();
    const uint64_t off = wid ? s_wave[wid - 1] : 0;
    total = s_wave[nw - 1];
    __syncthreads();
    return off + x - v;
}

struct B5Args {
    const uint32_t* stuffed;
    uint64_t* offsets;     // [tile] byte offset of the tile's file in out
    uint32_t* lengths;     // [tile] file length (0 when it did not fit)
    int32_t* status;       // [tile] OMR_OK / OMR_BUFFER_TOO_SMALL (optional)
    uint8_t* out;
    uint64_t cap;
    int32_t n_tiles, hdr_len;
    const int32_t* rstat;  // [tile] render status of the fused path (optional; wins over OMR_OK)
};

__global__ void __launch_bounds__(kTileThreads) k_jpeg_tile_scan(B5Args A) {
    __shared__ uint64_t sw[16];
    __shared__ uint64_t carry;
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    for (int base = 0; base < A.n_tiles; base += kTileThreads) {
        const int t = base + threadIdx.x;
        const uint64_t len = t < A.n_tiles ? (uint64_t)A.hdr_len + A.stuffed[t] + 2 : 0;
        uint64_t total;
        const uint64_t ex = block_exclusive_scan64(len, sw, total);
        const uint64_t cr = carry;
        if (t < A.n_tiles) {
            const uint64_t off = cr + ex;
            const bool fits = off + len <= A.cap;
            A.offsets[t] = off;
            A.lengths[t] = fits ? (uint32_t)len : 0;
            if (A.status) A.status[t] = (A.rstat && A.rstat[t]) ? A.rstat[t] : fits ? OMR_OK : OMR_BUFFER_TOO_SMALL;
            if (fits) {                            // EOI
                A.out[off + len - 2] = 0xFF;
                A.out[off + len - 1] = 0xD9;
            }
        }
        __syncthreads();
        if (threadIdx.x == 0) carry = cr + total;
        __syncthreads();
    }
}

constexpr int kJpegHdrMax = 704;   // SOI + APP0 + 2 DQT + SOF0 + 4 DHT + SOS is 607 bytes

struct B6Args {
    const uint32_t* words;
    const uint32_t* tile_bits;
    const uint8_t* cnt;
    const uint32_t* coff;    // [tile][slot_groups] exclusive 0xFF count before each group
    const uint64_t* offsets;
    const uint32_t* lengths;
    uint8_t* out;
    int64_t slot_words, slot_chunks, slot_groups;
    int32_t hdr_len;
    uint8_t hdr[kJpegHdrMax];   // JFIF header by value in the kernarg segment (no staging launch)
};

// B6: per group of 256 chunks: in-group scan of the 0xFF counts, stuffed bytes staged in LDS,
// copied out coalesced.  Block 0 of each tile also writes the JFIF header.  A chunk without 0xFF
// (nearly all of them) lands as five ORed LDS words, funnel-shifted to its byte offset; a chunk
// with 0xFF bytes ORs its expanded bytes one by one.  (Per-byte stores from every lane at a
// 16-byte lane stride had 40 % LDS bank-conflict cycles.)
__global__ void __launch_bounds__(kGrp) __attribute__((amdgpu_waves_per_eu(8))) k_jpeg_stuff_batch(B6Args A) {
    constexpr int kSW = kGrp * kStuffBytes * 2 / 4;
    __shared__ uint32_t swords[kSW + 4];
    __shared__ uint32_t sw[16];
    const int tile = blockIdx.y;
    if (A.lengths[tile] == 0) return;          // did not fit: status says so
    uint8_t* out = A.out + A.offsets[tile];
    if (blockIdx.x == 0)
        for (int i = threadIdx.x; i < A.hdr_len; i += kGrp) out[i] = A.hdr[i];
    out += A.hdr_len;
    const uint32_t tb = A.tile_bits[tile], nbytes = (tb + 7) / 8;
    const uint32_t nch = (nbytes + kStuffBytes - 1) / kStuffBytes;
    const uint32_t ng = (nch + kGrp - 1) / kGrp;
    const uint32_t* words = A.words + (int64_t)tile * A.slot_words;
    for (uint32_t g = blockIdx.x; g < ng; g += gridDim.x) {
        const uint32_t c = g * kGrp + threadIdx.x;
        const uint32_t n = c < nch ? A.cnt[(int64_t)tile * A.slot_chunks + c] : 0u;
        for (int i = threadIdx.x; i < kSW + 4; i += kGrp) swords[i] = 0;   // ordered by the scan's barrier
        uint32_t gtot;
        const uint32_t ex = block_exclusive_scan(n, sw, gtot);
        uint32_t o = threadIdx.x * kStuffBytes + ex;
        if (c < nch) {
            uint32_t w[4];
            chunk_bytes(words, c, nbytes, tb, w);
            const uint32_t e = min(nbytes - c * kStuffBytes, (uint32_t)kStuffBytes);
            if (n == 0 && e == kStuffBytes) {
                // stream byte k -> LDS byte o + k: little-endian words, shifted by o & 3 bytes
                const uint32_t sh = 8 * (o & 3), wi = o >> 2;
                const uint32_t l0 = __builtin_bswap32(w[0]), l1 = __builtin_bswap32(w[1]);
                const uint32_t l2 = __builtin_bswap32(w[2]), l3 = __builtin_bswap32(w[3]);
                atomicOr(&swords[wi], l0 << sh);
                atomicOr(&swords[wi + 1], (uint32_t)((((uint64_t)l1 << 32) | l0) >> (32 - sh)));
                atomicOr(&swords[wi + 2], (uint32_t)((((uint64_t)l2 << 32) | l1) >> (32 - sh)));
                atomicOr(&swords[wi + 3], (uint32_t)((((uint64_t)l3 << 32) | l2) >> (32 - sh)));
                if (sh) atomicOr(&swords[wi + 4], l3 >> (32 - sh));
            } else {
                // byte by byte (a word-wise split — a full word without 0xFF as one shifted pair of
                // ORs — measured 4 % slower: the words with a 0xFF still diverge the wave)
                for (uint32_t i = 0; i < e; ++i) {
                    const uint32_t bv = (w[i >> 2] >> (24 - 8 * (i & 3))) & 0xFF;
                    atomicOr(&swords[o >> 2], bv << (8 * (o & 3)));
                    ++o;
                    if (bv == 0xFF) ++o;                                  // stuffed 0x00 (already zero)
                }
            }
        }
        __syncthreads();
        const uint32_t gbytes = min(nbytes - g * kGrp * kStuffBytes, (uint32_t)(kGrp * kStuffBytes)) + gtot;
        const uint64_t base = (uint64_t)g * kGrp * kStuffBytes + A.coff[(int64_t)tile * A.slot_groups + g];
        // copy out: 16-byte stores from the first 16-byte aligned output byte on (the group's
        // bytes start anywhere), each assembled from five LDS words by a funnel shift; the
        // unaligned head and the tail go byte by byte
        const uint8_t* sbytes = reinterpret_cast<const uint8_t*>(swords);
        uint8_t* dst = out + base;
        const uint32_t head = min((16u - (uint32_t)((uintptr_t)dst & 15u)) & 15u, gbytes);
        const uint32_t nv = (gbytes - head) / 16, tail0 = head + nv * 16;
        if (threadIdx.x < head) dst[threadIdx.x] = sbytes[threadIdx.x];
        const uint32_t sh = 8 * (head & 3u);
        for (uint32_t j = threadIdx.x; j < nv; j += kGrp) {
            const uint32_t* sw4 = swords + (head >> 2) + 4 * j;
            uint32_t v[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) v[k] = sh ? (sw4[k] >> sh) | (sw4[k + 1] << (32 - sh)) : sw4[k];
            *reinterpret_cast<uint4*>(dst + head + 16 * j) = make_uint4(v[0], v[1], v[2], v[3]);
        }
        for (uint32_t i = tail0 + threadIdx.x; i < gbytes; i += kGrp) dst[i] = sbytes[i];
        __syncthreads();
    }
}

// Batch workspace layout.
struct JpegBatchLayout {
    int64_t n_mcu, nb, ngb, slot_words, slot_chunks, slot_groups;
    size_t coef, coef8, blk, bits, gsum, tbits, words, cnt, csum, ngroups, stuffed, hdr, total;
};

static JpegBatchLayout jpeg_batch_layout(int W, int H, int n, size_t base) {
    JpegBatchLayout L{};
    L.n_mcu = (int64_t)((W + 15) / 16) * ((H + 15) / 16);
    L.nb = L.n_mcu * 6;
    L.ngb = (L.nb + kGrp - 1) / kGrp;
    L.slot_words = ((L.nb * 1700 + 31) / 32 + 2 + 3) / 4 * 4;      // 16-B aligned tile slots
    L.slot_chunks = L.slot_words * 4 / kStuffBytes;
    L.slot_groups = (L.slot_chunks + kGrp - 1) / kGrp;
    size_t o = align_up(base, 256);
    auto take = [&](size_t bytes) { const size_t r = o; o = align_up(o + bytes, 256); return r; };
    L.coef = take((size_t)n * L.nb * 128);
    L.coef8 = take((size_t)n * L.nb * 64);
    L.blk = take((size_t)n * L.nb * 4);
    L.bits = take((size_t)n * L.nb * 2);
    L.gsum = take((size_t)n * L.ngb * 4);
    L.tbits = take((size_t)n * 4);
    L.words = take((size_t)n * L.slot_words * 4);
    L.cnt = take((size_t)n * L.slot_chunks);
    L.csum = take((size_t)n * L.slot_groups * 4);
    L.ngroups = take((size_t)n * 4);
    L.stuffed = take((size_t)n * 4);
    L.hdr = take(1024);
    L.total = o;
    return L;
}

template <int BPP, bool BE, int MODE>
static void launch_render_fdct_na(dim3 g, hipStream_t st, const B1Args& a1, const FusedArgs& f) {
    switch (f.R.n_active) {
    case 1: hipLaunchKernelGGL((k_jpeg_render_fdct<BPP, BE, MODE, 1>), g, dim3(256), 0, st, a1, f); break;
    case 2: hipLaunchKernelGGL((k_jpeg_render_fdct<BPP, BE, MODE, 2>), g, dim3(256), 0, st, a1, f); break;
    case 3: hipLaunchKernelGGL((k_jpeg_render_fdct<BPP, BE, MODE, 3>), g, dim3(256), 0, st, a1, f); break;
    default: hipLaunchKernelGGL((k_jpeg_render_fdct<BPP, BE, MODE, 4>), g, dim3(256), 0, st, a1, f); break;
    }
}

template <bool BE>
static void launch_render_fdct_mode(dim3 g, hipStream_t st, const B1Args& a1, const FusedArgs& f) {
    switch (f.R.mode) {
    case kFusedFast16:
        if (f.R.f32 && f.R.is_signed) launch_render_fdct_na<2, BE, kFusedFast16FS>(g, st, a1, f);
        else if (f.R.f32) launch_render_fdct_na<2, BE, kFusedFast16F>(g, st, a1, f);
        else if (f.R.ws_int) launch_render_fdct_na<2, BE, kFusedFast16I>(g, st, a1, f);
        else launch_render_fdct_na<2, BE, kFusedFast16>(g, st, a1, f);
        break;
    case kFusedLinear16: launch_render_fdct_na<2, BE, kFusedLinear16>(g, st, a1, f); break;
    default: launch_render_fdct_na<2, BE, kFusedMixed16>(g, st, a1, f); break;
    }
}

static void launch_render_fdct(dim3 g, hipStream_t st, const B1Args& a1, const FusedArgs& f, int bpp, bool be) {
    if (bpp == 1) launch_render_fdct_na<1, false, kFusedTable8>(g, st, a1, f);
    else if (be) launch_render_fdct_mode<true>(g, st, a1, f);
    else launch_render_fdct_mode<false>(g, st, a1, f);
}

// Fused render -> JPEG: F1 instead of B1 (fused != nullptr; d_argb unused).
struct FusedLaunch {
    FusedArgs args;
    int bpp;
    bool be;
};

static omr_status encode_jpeg_batch_ws(Ctx* ctx, const uint32_t* d_argb, int64_t tile_stride, int n, int W,
                                       int H, float quality, uint8_t* d_out, uint64_t cap, uint64_t* d_offsets,
                                       uint32_t* d_lengths, int32_t* d_status, const JpegBatchLayout& L,
                                       const FusedLaunch* fused = nullptr, const int32_t* rstat = nullptr) {
    uint8_t ql[64], qc[64];
    quant_tables(quality, ctx->sem, ql, qc);
    std::vector<uint8_t> hdr;
    jpeg_header(hdr, W, H, ql, qc);
    uint8_t* ws = static_cast<uint8_t*>(ctx->ws);
    if (hdr.size() > (size_t)kJpegHdrMax) return fail(ctx, OMR_INTERNAL, "JPEG header larger than its kernarg slot");
    auto u32 = [&](size_t off) { return reinterpret_cast<uint32_t*>(ws + off); };
    B1Args a1;
    a1.argb = d_argb;
    a1.tile_stride = tile_stride;
    a1.coefs = reinterpret_cast<int16_t*>(ws + L.coef);
    a1.coef8 = reinterpret_cast<int8_t*>(ws + L.coef8);
    a1.blk = reinterpret_cast<uint32_t*>(ws + L.blk);
    a1.W = W;
    a1.H = H;
    a1.mcux = (W + 15) / 16;
    a1.n_mcu = (int32_t)L.n_mcu;
    a1.nb = (int32_t)L.nb;
    // 4 MCUs per wave once that still gives >= 4 waves per SIMD (16 per CU)
    a1.mpw = (int64_t)n * L.n_mcu >= (int64_t)kB1McuPerWave * 16 * ctx->cu_count ? kB1McuPerWave : 1;
    for (int i = 0; i < 64; ++i) { a1.qt.q[0][i] = ql[i]; a1.qt.q[1][i] = qc[i]; }
    set_recips(a1.qt);
    uint16_t* d_bits = reinterpret_cast<uint16_t*>(ws + L.bits);
    B2aArgs a2{a1.coefs, a1.coef8, a1.blk, d_bits, u32(L.gsum), (int32_t)L.nb, (int32_t)L.ngb};
    GroupScanArgs a2b{u32(L.gsum), nullptr, u32(L.tbits), u32(L.words), nullptr, L.ngb, L.slot_words, (int32_t)L.ngb};
    B3Args a3{a1.coefs, a1.coef8, a1.blk, d_bits, u32(L.gsum), u32(L.words), (int32_t)L.nb, (int32_t)L.ngb, L.slot_words};
    B4aArgs a4{u32(L.words), u32(L.tbits), ws + L.cnt, u32(L.csum), u32(L.ngroups), L.slot_words, L.slot_chunks,
               L.slot_groups};
    GroupScanArgs a4b{u32(L.csum), u32(L.ngroups), u32(L.stuffed), nullptr, u32(L.tbits), L.slot_groups, 0, 0};
    B5Args a5{u32(L.stuffed), d_offsets, d_lengths, d_status, d_out, cap, n, (int32_t)hdr.size(),
              fused ? fused->args.rstat : rstat};
    B6Args a6{u32(L.words), u32(L.tbits), ws + L.cnt, u32(L.csum), d_offsets, d_lengths, d_out,
              L.slot_words, L.slot_chunks, L.slot_groups, (int32_t)hdr.size(), {}};
    std::memcpy(a6.hdr, hdr.data(), hdr.size());
    // chunk groups of a typical stream (<= ~1 B per pixel; q 0.9 C2 tiles are 0.37, uniform noise
    // 0.8); longer streams loop in B4a/B6.  Workgroups past the stream end only exit, but at
    // 2 B per pixel they were 4/5 of both grids.
    const int64_t est_groups = std::max<int64_t>(1, std::min<int64_t>(L.slot_groups,
                                   ((int64_t)W * H * ctx->jpeg_est_centibpp / 100 / kStuffBytes + kGrp - 1) / kGrp));
    KernelTimer whole(ctx, 4);
    {
        KernelTimer t(ctx, 5);
        const dim3 g1((unsigned)((L.n_mcu + 4 * a1.mpw - 1) / (4 * a1.mpw)), (unsigned)n);
        if (!fused) {
            hipLaunchKernelGGL(k_jpeg_fdct_batch, g1, dim3(256), 0, ctx->stream, a1);
        } else {
            launch_render_fdct(g1, ctx->stream, a1, fused->args, fused->bpp, fused->be);
        }
    }
    if constexpr (OMR_ABL != 0) {   // ablation builds time B1 / F1 only: their outputs are not a stream
        OMR_HIP(ctx, hipGetLastError());
        return OMR_OK;
    }
    hipLaunchKernelGGL(k_jpeg_block_bits, dim3((unsigned)L.ngb, (unsigned)n), dim3(kGrp), 0, ctx->stream, a2);
    hipLaunchKernelGGL(k_jpeg_group_scan, dim3((unsigned)n), dim3(kTileThreads), 0, ctx->stream, a2b);
    {
        KernelTimer t(ctx, 6);
        hipLaunchKernelGGL(k_jpeg_huff_thread, dim3((unsigned)L.ngb, (unsigned)n), dim3(kGrp), 0, ctx->stream, a3);
    }
    hipLaunchKernelGGL(k_jpeg_stuff_count, dim3((unsigned)((est_groups + 3) / 4), (unsigned)n), dim3(kGrp), 0, ctx->stream, a4);
    hipLaunchKernelGGL(k_jpeg_group_scan, dim3((unsigned)n), dim3(kTileThreads), 0, ctx->stream, a4b);
    hipLaunchKernelGGL(k_jpeg_tile_scan, dim3(1), dim3(kTileThreads), 0, ctx->stream, a5);
    hipLaunchKernelGGL(k_jpeg_stuff_batch, dim3((unsigned)est_groups, (unsigned)n), dim3(kGrp), 0, ctx->stream, a6);
    OMR_HIP(ctx, hipGetLastError());
    return OMR_OK;
}

// The unfused render -> JPEG path: B1 on rendered ARGB, B5 merging the render's per-tile status.
static omr_status encode_jpeg_batch_ws_rstat(Ctx* ctx, const uint32_t* d_argb, int64_t tile_stride, int n, int W,
                                             int H, float quality, uint8_t* d_out, uint64_t cap, uint64_t* d_offsets,
                                             uint32_t* d_lengths, int32_t* d_status, const JpegBatchLayout& L,
                                             const int32_t* rstat) {
    return encode_jpeg_batch_ws(ctx, d_argb, tile_stride, n, W, H, quality, d_out, cap, d_offsets, d_lengths,
                                d_status, L, nullptr, rstat);
}

static omr_status check_jpeg_batch(Ctx* ctx, const void* d_argb, int n, int W, int H, int64_t stride) {
    if (!d_argb) return fail(ctx, OMR_INVALID_ARGUMENT, "null ARGB batch");
    if (n <= 0 || n > (1 << 20)) return fail(ctx, OMR_INVALID_ARGUMENT, "JPEG batch: n_tiles out of range");
    if (W <= 0 || H <= 0 || W > 4096 || H > 4096)
        return fail(ctx, OMR_INVALID_ARGUMENT, "JPEG batch: tile dimensions must be 1..4096");
    if (stride < (int64_t)W * H) return fail(ctx, OMR_INVALID_ARGUMENT, "JPEG batch: tile stride < width*height");
    return OMR_OK;
}

// The single tile's file and length into fine-grained pinned host memory (host_len first, then
// the bytes at host + 16), 16 B per lane; lanes past the file exit.
__global__ void __launch_bounds__(256) k_file_to_host(const uint8_t* __restrict__ src, const uint32_t* __restrict__ d_len,
                                                      uint8_t* __restrict__ host) {
    const uint32_t len = *d_len;
    const uint64_t i = ((uint64_t)blockIdx.x * 256 + threadIdx.x) * 16;
    if (i == 0) *reinterpret_cast<uint32_t*>(host) = len;
    if (i >= len) return;
    uint8_t* dst = host + 16;
    if (i + 16 <= len) {
        *reinterpret_cast<uint4*>(dst + i) = *reinterpret_cast<const uint4*>(src + i);
    } else {
        for (uint64_t j = i; j < len; ++j) dst[j] = src[j];
    }
}

static size_t single_batched_bytes(int W, int H, size_t base) {
    const JpegBatchLayout L = jpeg_batch_layout(W, H, 1, base);
    return align_up(L.total, 256) + 512 + omr_jpeg_max_bytes(W, H);
}

static omr_status encode_jpeg_single_batched(Ctx* ctx, const uint32_t* d_argb, int W, int H, float quality,
                                             uint8_t* out, size_t cap, size_t* out_len, size_t base) {
    const JpegBatchLayout L = jpeg_batch_layout(W, H, 1, base);
    const size_t o_offs = align_up(L.total, 256), o_lens = o_offs + 256, o_out = o_lens + 256;
    const size_t jcap = omr_jpeg_max_bytes(W, H);
    // (a regrow reallocates without copying: the host-input caller sized the workspace first)
    omr_status st = ensure_workspace(ctx, single_batched_bytes(W, H, base));
    if (st) return st;
    uint8_t* ws = static_cast<uint8_t*>(ctx->ws);
    if (!d_argb) d_argb = reinterpret_cast<const uint32_t*>(ws);   // host-input variant staged at offset 0
    uint64_t* d_offs = reinterpret_cast<uint64_t*>(ws + o_offs);
    uint32_t* d_lens = reinterpret_cast<uint32_t*>(ws + o_lens);
    st = encode_jpeg_batch_ws(ctx, d_argb, (int64_t)W * H, 1, W, H, quality, ws + o_out, jcap, d_offs, d_lens,
                              nullptr, L);
    if (st) return st;
    // the file lands in the context's pinned buffer straight from the device (one sync, no
    // length round trip before the copy)
    st = ensure_host_out(ctx, jcap + 16);
    if (st) return st;
    hipLaunchKernelGGL(k_file_to_host, dim3((unsigned)((jcap + 16 * 256 - 1) / (16 * 256))), dim3(256), 0,
                       ctx->stream, ws + o_out, d_lens, ctx->h_out);
    OMR_HIP(ctx, hipGetLastError());
    OMR_HIP(ctx, hipStreamSynchronize(ctx->stream));
    const uint32_t len = *reinterpret_cast<volatile uint32_t*>(ctx->h_out);
    if (len == 0) return fail(ctx, OMR_DEVICE, "JPEG: stream exceeded the worst-case bound");
    if (out_len) *out_len = len;
    if (!out || cap < len) return fail(ctx, OMR_BUFFER_TOO_SMALL, "JPEG output buffer too small");
    std::memcpy(out, ctx->h_out + 16, len);
    return OMR_OK;
}

}  // namespace omr

extern "C" {

}  // extern "C"

namespace omr {

// Render + JPEG of a batch (omr_render_jpeg_batch_*_device).  The fused path (F1 = render + B1 in
// one kernel) covers 8/16-bit integer pixels with 1..4 active channels on tiles whose sides are
// multiples of 16; anything else renders with K2 into a context buffer and encodes that.
static omr_status render_jpeg_batch(Ctx* ctx, const omr_quantum_def* qdef, const omr_channel_binding* channels,
                                    int32_t size_c, const void* d_base, int64_t tile_stride, int64_t chan_stride,
                                    const void* const* d_ptrs, int32_t n, int64_t row_stride, int32_t pt,
                                    int32_t be, int32_t W, int32_t H, int32_t fh, int32_t fv, float quality,
                                    uint8_t* d_out, size_t cap, uint64_t* d_offsets, uint32_t* d_lengths,
                                    int32_t* d_status) {
    if (!ctx) return OMR_INVALID_ARGUMENT;
    if (n <= 0 || n > (1 << 20)) return fail(ctx, OMR_INVALID_ARGUMENT, "JPEG batch: n_tiles out of range");
    if (W <= 0 || H <= 0 || W > kJpegBatchMaxDim || H > kJpegBatchMaxDim)
        return fail(ctx, OMR_INVALID_ARGUMENT, "JPEG batch: tile dimensions must be 1..4096");
    if (!d_out || !d_offsets || !d_lengths) return fail(ctx, OMR_INVALID_ARGUMENT, "null batch output");
    if (!d_base && !d_ptrs) return fail(ctx, OMR_INVALID_ARGUMENT, "null plane batch");
    if (row_stride == 0) row_stride = W;
    if (row_stride < W) return fail(ctx, OMR_INVALID_ARGUMENT, "row stride smaller than width");
    OMR_HIP(ctx, hipSetDevice(ctx->device));
    std::unique_ptr<FusedPlanBuf, void (*)(FusedPlanBuf*)> fp(fused_plan_new(), fused_plan_free);
    omr_status st = OMR_OK;
    const bool plan_ok = render_fused_plan(ctx, qdef, channels, size_c, pt, fp.get(), &st);
    if (st) return st;
    const int bpp = bytes_per_pixel(pt);
    const int64_t al = bpp == 2 ? 4 : 2;     // the fused loads read pixel pairs
    const bool aligned = (row_stride * bpp) % al == 0 &&
                         (!d_base || ((uintptr_t)d_base % al == 0 && tile_stride % al == 0 && chan_stride % al == 0));
    // F1 addresses a plane's pixels by 32-bit byte offsets from the plane's (uniform) base
    const bool offs32 = (row_stride * (int64_t)(H - 1) + W) * bpp < ((int64_t)1 << 32);
    const bool fused = plan_ok && W % 16 == 0 && H % 16 == 0 && aligned && offs32;
    const size_t rstat_bytes = align_up((size_t)n * 4, 256);
    if (fused) {
        const size_t r_bytes = align_up(render_fused_ws_bytes(fp.get()), 256);
        const JpegBatchLayout L = jpeg_batch_layout(W, H, n, r_bytes + rstat_bytes);
        st = ensure_workspace(ctx, L.total);
        if (st) return st;
        FusedLaunch fl;
        std::memset(&fl, 0, sizeof(fl));
        st = render_fused_stage(ctx, fp.get(), 0, fl.args.R, /*build_contrib=*/true, /*bias_int16=*/true);
        if (st) return st;
        fl.args.sbase = static_cast<const uint8_t*>(d_base);
        fl.args.planes = d_ptrs;
        fl.args.strided = d_base ? 1 : 0;
        fl.args.tile_stride = tile_stride;
        fl.args.chan_stride = chan_stride;
        fl.args.row_stride = row_stride;
        fl.args.size_c = size_c;
        fl.args.flip_h = fh ? 1 : 0;
        fl.args.flip_v = fv ? 1 : 0;
        fl.args.rstat = reinterpret_cast<int32_t*>(static_cast<uint8_t*>(ctx->ws) + r_bytes);
        fl.bpp = bpp;
        fl.be = be != 0;
        OMR_HIP(ctx, hipMemsetAsync(fl.args.rstat, 0, (size_t)n * 4, ctx->stream));
        return encode_jpeg_batch_ws(ctx, nullptr, 0, n, W, H, quality, d_out, cap, d_offsets, d_lengths, d_status,
                                    L, &fl);
    }
    // unfused: K1 + K2 into the context's ARGB buffer, then the batched encoder
    const size_t argb_bytes = align_up((size_t)n * W * H * 4, 256);
    st = ensure_aux(ctx, argb_bytes + rstat_bytes);
    if (st) return st;
    uint32_t* argb = static_cast<uint32_t*>(ctx->aux);
    int32_t* rstat = reinterpret_cast<int32_t*>(static_cast<uint8_t*>(ctx->aux) + argb_bytes);
    omr_ctx* cx = static_cast<omr_ctx*>(ctx);
    st = d_base ? omr_render_batch_strided_device(cx, qdef, channels, size_c, d_base, tile_stride, chan_stride, n,
                                                  row_stride, pt, be, W, H, fh, fv, argb, rstat)
                : omr_render_batch_device(cx, qdef, channels, size_c, d_ptrs, n, row_stride, pt, be, W, H, fh, fv,
                                          argb, rstat);
    if (st) return st;
    const JpegBatchLayout L = jpeg_batch_layout(W, H, n, 0);
    st = ensure_workspace(ctx, L.total);
    if (st) return st;
    return encode_jpeg_batch_ws_rstat(ctx, argb, (int64_t)W * H, n, W, H, quality, d_out, cap, d_offsets, d_lengths,
                                      d_status, L, rstat);
}

// One render_image_region request in its default format: the small-launch render (K2 builds its
// tables in LDS: no K1) into the context's aux ARGB tile, the context's sticky quantization flag
// moved to pinned host memory behind it, then the one-tile JPEG pipeline landing the file in
// pinned memory — one stream sync.  (The fused kernel, and the batch entry at n = 1, measured
// slower for a single tile: tools/omr_latency.cpp.)
static omr_status render_jpeg_one(Ctx* ctx, const omr_quantum_def* qdef, const omr_channel_binding* channels,
                                  int32_t size_c, const void* const* d_planes, int64_t row_stride, int32_t pt,
                                  int32_t be, int32_t W, int32_t H, int32_t fh, int32_t fv, float quality,
                                  uint8_t* out, size_t cap, size_t* out_len) {
    if (!ctx) return OMR_INVALID_ARGUMENT;
    if (!d_planes || size_c <= 0) return fail(ctx, OMR_INVALID_ARGUMENT, "bad plane list");
    omr_status st = check_jpeg_dims(ctx, W, H);
    if (st) return st;
    OMR_HIP(ctx, hipSetDevice(ctx->device));
    st = ensure_aux(ctx, (size_t)W * H * 4);
    if (st) return st;
    uint32_t* argb = static_cast<uint32_t*>(ctx->aux);
    omr_ctx* cx = static_cast<omr_ctx*>(ctx);
    st = omr_render_packed_int_device(cx, qdef, channels, size_c, d_planes, row_stride, pt, be, W, H, fh, fv, argb);
    if (st) return st;
    OMR_HIP(ctx, launch_flag_out(ctx->stream, ctx->d_flag, ctx->h_flag));   // read after the JPEG's sync
    // regions past 4096 a side (region mode is unbounded, ImageRegionRequestHandler.java:817-827):
    // the whole-image J1-J6 encoder, as omr_encode_jpeg_device does
    const omr_status jst = W <= kJpegBatchMaxDim && H <= kJpegBatchMaxDim
                               ? encode_jpeg_single_batched(ctx, argb, W, H, quality, out, cap, out_len, 0)
                               : omr_encode_jpeg_device(cx, argb, W, H, quality, out, cap, out_len);
    OMR_HIP(ctx, hipStreamSynchronize(ctx->stream));     // (already idle unless the encode failed early)
    if (*static_cast<volatile int32_t*>(ctx->h_flag))
        return fail(ctx, OMR_QUANTIZATION, "pixel value outside the quantization LUT domain");
    return jst;
}

}  // namespace omr

extern "C" {

omr_status omr_render_jpeg_batch_strided_device(omr_ctx* ctx, const omr_quantum_def* qdef,
                                                const omr_channel_binding* channels, int32_t size_c,
                                                const void* d_base, int64_t tile_stride_bytes,
                                                int64_t channel_stride_bytes, int32_t n_tiles, int64_t row_stride,
                                                int32_t pixel_type, int32_t big_endian, int32_t width, int32_t height,
                                                int32_t flip_h, int32_t flip_v, float quality, uint8_t* d_out,
                                                size_t out_cap, uint64_t* d_offsets, uint32_t* d_lengths,
                                                int32_t* d_status) {
    if (!d_base) return ctx ? omr::fail(ctx, OMR_INVALID_ARGUMENT, "null batch base") : OMR_INVALID_ARGUMENT;
    return omr::render_jpeg_batch(ctx, qdef, channels, size_c, d_base, tile_stride_bytes, channel_stride_bytes,
                                  nullptr, n_tiles, row_stride, pixel_type, big_endian, width, height, flip_h, flip_v,
                                  quality, d_out, out_cap, d_offsets, d_lengths, d_status);
}

omr_status omr_render_jpeg(omr_ctx* ctx, const omr_quantum_def* qdef, const omr_channel_binding* channels,
                           int32_t size_c, const void* const* d_planes, int64_t row_stride, int32_t pixel_type,
                           int32_t big_endian, int32_t width, int32_t height, int32_t flip_h, int32_t flip_v,
                           float quality, uint8_t* out, size_t cap, size_t* out_len) {
    return omr::render_jpeg_one(ctx, qdef, channels, size_c, d_planes, row_stride, pixel_type, big_endian, width,
                                height, flip_h, flip_v, quality, out, cap, out_len);
}

omr_status omr_render_jpeg_batch_device(omr_ctx* ctx, const omr_quantum_def* qdef,
                                        const omr_channel_binding* channels, int32_t size_c,
                                        const void* const* d_plane_ptrs, int32_t n_tiles, int64_t row_stride,
                                        int32_t pixel_type, int32_t big_endian, int32_t width, int32_t height,
                                        int32_t flip_h, int32_t flip_v, float quality, uint8_t* d_out,
                                        size_t out_cap, uint64_t* d_offsets, uint32_t* d_lengths,
                                        int32_t* d_status) {
    if (!d_plane_ptrs) return ctx ? omr::fail(ctx, OMR_INVALID_ARGUMENT, "null plane table") : OMR_INVALID_ARGUMENT;
    return omr::render_jpeg_batch(ctx, qdef, channels, size_c, nullptr, 0, 0, d_plane_ptrs, n_tiles, row_stride,
                                  pixel_type, big_endian, width, height, flip_h, flip_v, quality, d_out, out_cap,
                                  d_offsets, d_lengths, d_status);
}

omr_status omr_encode_jpeg_batch_device(omr_ctx* ctx, const uint32_t* d_argb, int64_t tile_stride_px,
                                        int32_t n_tiles, int32_t width, int32_t height, float quality,
                                        uint8_t* d_out, size_t out_cap, uint64_t* d_offsets,
                                        uint32_t* d_lengths, int32_t* d_status) {
    using namespace omr;
    if (!ctx) return OMR_INVALID_ARGUMENT;
    if (tile_stride_px == 0) tile_stride_px = (int64_t)width * height;
    omr_status st = check_jpeg_batch(ctx, d_argb, n_tiles, width, height, tile_stride_px);
    if (st) return st;
    if (!d_out || !d_offsets || !d_lengths) return fail(ctx, OMR_INVALID_ARGUMENT, "null batch output");
    OMR_HIP(ctx, hipSetDevice(ctx->device));
    const JpegBatchLayout L = jpeg_batch_layout(width, height, n_tiles, 0);
    st = ensure_workspace(ctx, L.total);
    if (st) return st;
    return encode_jpeg_batch_ws(ctx, d_argb, tile_stride_px, n_tiles, width, height, quality, d_out, out_cap,
                                d_offsets, d_lengths, d_status, L);
}

}  // extern "C"

extern "C" omr_status omr_encode_jpeg_batch(omr_ctx* ctx, const uint32_t* d_argb, int64_t tile_stride_px,
                                            int32_t n_tiles, int32_t width, int32_t height, float quality,
                                            uint8_t* out, size_t cap, uint64_t* offsets, uint32_t* lengths) {
    using namespace omr;
    if (!ctx) return OMR_INVALID_ARGUMENT;
    if (tile_stride_px == 0) tile_stride_px = (int64_t)width * height;
    omr_status st = check_jpeg_batch(ctx, d_argb, n_tiles, width, height, tile_stride_px);
    if (st) return st;
    if (!out || !offsets || !lengths) return fail(ctx, OMR_INVALID_ARGUMENT, "null batch output");
    OMR_HIP(ctx, hipSetDevice(ctx->device));
    JpegBatchLayout L = jpeg_batch_layout(width, height, n_tiles, 0);
    const size_t o_offs = align_up(L.total, 256);
    const size_t o_lens = align_up(o_offs + (size_t)n_tiles * 8, 256);
    const size_t o_out = align_up(o_lens + (size_t)n_tiles * 4, 256);
    st = ensure_workspace(ctx, o_out + cap);
    if (st) return st;
    uint8_t* ws = static_cast<uint8_t*>(ctx->ws);
    uint64_t* d_offs = reinterpret_cast<uint64_t*>(ws + o_offs);
    uint32_t* d_lens = reinterpret_cast<uint32_t*>(ws + o_lens);
    st = encode_jpeg_batch_ws(ctx, d_argb, tile_stride_px, n_tiles, width, height, quality, ws + o_out, cap,
                              d_offs, d_lens, nullptr, L);
    if (st) return st;
    OMR_HIP(ctx, hipMemcpyAsync(offsets, d_offs, (size_t)n_tiles * 8, hipMemcpyDeviceToHost, ctx->stream));
    OMR_HIP(ctx, hipMemcpyAsync(lengths, d_lens, (size_t)n_tiles * 4, hipMemcpyDeviceToHost, ctx->stream));
    OMR_HIP(ctx, hipStreamSynchronize(ctx->stream));
    uint64_t used = 0;
    bool short_buf = false;
    for (int i = 0; i < n_tiles; ++i) {
        if (lengths[i] == 0) short_buf = true;
        else used = std::max<uint64_t>(used, offsets[i] + lengths[i]);
    }
    if (used) OMR_HIP(ctx, hipMemcpyAsync(out, ws + o_out, used, hipMemcpyDeviceToHost, ctx->stream));
    OMR_HIP(ctx, hipStreamSynchronize(ctx->stream));
    if (short_buf) return fail(ctx, OMR_BUFFER_TOO_SMALL, "JPEG batch output buffer too small (lengths 0)");
    return OMR_OK;
}
