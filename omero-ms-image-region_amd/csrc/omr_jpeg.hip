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

struct QTabs {
    uint16_t q[2][64];  // natural order
};

// javax.imageio JPEG.convertToLinearQuality + JPEGQTable.getScaledInstance(scale, true).
static void quant_tables(float quality, uint8_t luma[64], uint8_t chroma[64]) {
    float qf = quality;
    if (qf <= 0.0f) qf = 0.01f;
    if (qf > 1.00f) qf = 1.00f;
    if (qf < 0.5f) qf = 0.5f / qf;
    else qf = 2.0f - (qf * 2.0f);
    for (int i = 0; i < 64; ++i) {
        volatile float a = (float)kStdLuma[i] * qf;
        int sv = (int)(a + 0.5f);
        luma[i] = (uint8_t)(sv < 1 ? 1 : sv > 255 ? 255 : sv);
        volatile float b = (float)kStdChroma[i] * qf;
        sv = (int)(b + 0.5f);
        chroma[i] = (uint8_t)(sv < 1 ? 1 : sv > 255 ? 255 : sv);
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

#define DESCALE(x, n) (((x) + (1 << ((n)-1))) >> (n))

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
    int z1 = (tmp12 + tmp13) * 4433;
    p[2 * s] = DESCALE(z1 + tmp13 * 6270, sh);
    p[6 * s] = DESCALE(z1 + tmp12 * (-15137), sh);
    z1 = tmp4 + tmp7;
    int z2 = tmp5 + tmp6, z3 = tmp4 + tmp6, z4 = tmp5 + tmp7;
    const int z5 = (z3 + z4) * 9633;
    tmp4 *= 2446; tmp5 *= 16819; tmp6 *= 25172; tmp7 *= 12299;
    z1 *= -7373; z2 *= -20995; z3 *= -16069; z4 *= -3196;
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
    quant_tables(quality, ql, qc);
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
    if (!luma || !chroma) return OMR_INVALID_ARGUMENT;
    quant_tables(quality, luma, chroma);
    return OMR_OK;
}

omr_status omr_encode_jpeg_device(omr_ctx* ctx, const uint32_t* d_argb, int32_t width, int32_t height,
                                  float quality, uint8_t* out, size_t cap, size_t* out_len) {
    if (!ctx) return OMR_INVALID_ARGUMENT;
    omr_status st = check_jpeg_dims(ctx, width, height);
    if (st) return st;
    if (!d_argb) return fail(ctx, OMR_INVALID_ARGUMENT, "null ARGB buffer");
    OMR_HIP(ctx, hipSetDevice(ctx->device));
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
    const JpegLayout L = jpeg_layout(width, height, img);
    st = ensure_workspace(ctx, L.total);
    if (st) return st;
    uint32_t* d_argb = static_cast<uint32_t*>(ctx->ws);
    OMR_HIP(ctx, hipMemcpyAsync(d_argb, argb, (size_t)width * height * 4, hipMemcpyHostToDevice, ctx->stream));
    return encode_jpeg_ws(ctx, d_argb, width, height, quality, out, cap, out_len, L);
}

}  // extern "C"
