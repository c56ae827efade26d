// omr_png.hip — K5 PNG encode and K6 shape-mask raster.
//
// K5 replaces ImageIO.write(image, "png", output) for rendered regions
// (ImageRegionRequestHandler.java:583-600): 24-bit RGB (the DirectColorModel view drops
// alpha, :576-578).  K6 replaces ShapeMaskRequestHandler.renderShapeMask(Color, byte[], w, h)
// (:165-221): MSB-first bit mask -> (flip) -> 2-entry palette PNG (index 0 transparent,
// index 1 = fill colour; 1-bit rows when width % 8 == 0, else 8-bit, :174-198).
//
// PNG is compared decoded (pixels), so the filter choice and the deflate parse are ours: the
// zlib stream is one dynamic-Huffman block built on the device (D1-D6 below), or stored blocks
// when that is shorter (noise; every output byte then a pure function of its index).  Adler-32
// is a parallel 64-bit reduction; CRC-32 is per-segment CRCs combined with x^(8n) mod P
// multiplications (XOR-reduction).  The whole IDAT chunk is built on the device, stored vs
// dynamic is decided there, and the chunk lands in pinned host memory: one stream sync per
// encode.
#include "omr_device.h"

namespace omr {

// omr_jpeg.hip
size_t scan_scratch_bytes(int64_t n);
omr_status device_exclusive_scan(Ctx* ctx, const uint32_t* in, uint32_t* out, int64_t n, uint32_t* d_total,
                                 uint32_t* scratch);

constexpr uint32_t kCrcPoly = 0xEDB88320u;
constexpr int kStored = 65535;      // bytes per stored deflate block

struct CrcTab {
    uint32_t t[256];
    uint32_t x2n[32];
};

constexpr uint32_t multmodp_c(uint32_t a, uint32_t b) {
    uint32_t m = 1u << 31, p = 0;
    for (;;) {
        if (a & m) {
            p ^= b;
            if ((a & (m - 1)) == 0) break;
        }
        m >>= 1;
        b = (b & 1) ? (b >> 1) ^ kCrcPoly : b >> 1;
    }
    return p;
}

constexpr CrcTab make_crc() {
    CrcTab c{};
    for (uint32_t n = 0; n < 256; ++n) {
        uint32_t r = n;
        for (int k = 0; k < 8; ++k) r = (r & 1) ? kCrcPoly ^ (r >> 1) : r >> 1;
        c.t[n] = r;
    }
    uint32_t p = 1u << 30;   // x^1
    c.x2n[0] = p;
    for (int n = 1; n < 32; ++n) c.x2n[n] = p = multmodp_c(p, p);
    return c;
}

__constant__ CrcTab c_crc = make_crc();
static constexpr CrcTab h_crc = make_crc();

__device__ uint32_t multmodp(uint32_t a, uint32_t b) {
    uint32_t m = 1u << 31, p = 0;
    for (;;) {
        if (a & m) {
            p ^= b;
            if ((a & (m - 1)) == 0) break;
        }
        m >>= 1;
        b = (b & 1) ? (b >> 1) ^ kCrcPoly : b >> 1;
    }
    return p;
}

__device__ uint32_t x2nmodp(uint64_t n, unsigned k) {   // x^(n * 2^k) mod P
    uint32_t p = 1u << 31;
    while (n) {
        if (n & 1) p = multmodp(c_crc.x2n[k & 31], p);
        n >>= 1;
        ++k;
    }
    return p;
}

static uint32_t host_crc(const uint8_t* d, size_t n, uint32_t crc = 0) {
    uint32_t r = ~crc;
    for (size_t i = 0; i < n; ++i) r = h_crc.t[(r ^ d[i]) & 0xFF] ^ (r >> 8);
    return ~r;
}

// Raw (filtered) scanline byte i of the image: filter 0 per row, then row bytes.
enum PngKind : int32_t { kRgb = 0, kIdx1 = 1, kIdx8 = 2 };

struct PngArgs {
    const uint32_t* argb;    // kRgb
    const uint8_t* bits;     // kIdx*: MSB-first mask bits (unflipped)
    uint8_t* chunk;          // IDAT chunk: [len 4][IDAT 4][zlib ...][adler 4][crc 4]
    unsigned long long* sums;  // adler partial sums (2)
    uint32_t* crc_out;
    int32_t kind, W, H, flip_h, flip_v;
    int64_t rowlen;          // 1 + row bytes
    int64_t raw;             // rowlen * H
    int64_t nblk;            // stored blocks
    int64_t zlen;            // zlib stream length of the stored encoding (2 + 5*nblk + raw + 4)
    // [0] zlib stream length chosen on the device (stored or dynamic), [1] 1 = stored blocks,
    // [2] IDAT chunk bytes (8 + zlen + 4); written by k_png_select
    int64_t* meta;
};

__device__ __forceinline__ int64_t png_zlen(const PngArgs& A) { return A.meta[0]; }

__device__ __forceinline__ uint32_t mask_bit(const PngArgs& A, int x, int y) {
    const int sx = A.flip_h ? A.W - 1 - x : x, sy = A.flip_v ? A.H - 1 - y : y;
    const int64_t i = (int64_t)sy * A.W + sx;
    return (A.bits[i >> 3] >> (7 - (i & 7))) & 1;
}


// One lane per zlib-stream byte of the stored encoding: header, stored-block headers, and the
// filtered stream flt as payload (any filter is valid PNG; storing the same filtered rows the
// dynamic stream codes keeps one Adler-32 -- from D1's row partials -- for both encodings, and
// makes the single-tile and the batched encoder's files identical).
__global__ void __launch_bounds__(256) k_png_layout(PngArgs A, const uint8_t* __restrict__ flt) {
    if (A.meta[1] == 0) return;                     // the dynamic stream was chosen
    uint8_t* z = A.chunk + 8;
    for (int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x; j < A.zlen - 4; j += (int64_t)gridDim.x * 256) {
        uint32_t v;
        if (j < 2) {
            v = j == 0 ? 0x78 : 0x01;                  // CMF/FLG: deflate, 32K window, check bits
        } else {
            const int64_t k = j - 2, b = k / (kStored + 5), o = k - b * (kStored + 5);
            if (o < 5) {
                const int64_t len = min((int64_t)kStored, A.raw - b * kStored);
                const uint32_t l16 = (uint32_t)len;
                switch (o) {
                case 0: v = b == A.nblk - 1 ? 1 : 0; break;   // BFINAL, BTYPE=00
                case 1: v = l16 & 0xFF; break;
                case 2: v = (l16 >> 8) & 0xFF; break;
                case 3: v = (~l16) & 0xFF; break;
                default: v = ((~l16) >> 8) & 0xFF; break;
                }
            } else {
                v = flt[b * kStored + (o - 5)];
            }
        }
        z[j] = (uint8_t)v;
    }
}

__global__ void k_png_adler(PngArgs A) {
    const uint64_t a = (1 + A.sums[0]) % 65521, b = ((uint64_t)A.raw % 65521 + A.sums[1] % 65521) % 65521;
    const uint32_t adler = (uint32_t)((b << 16) | a);
    const int64_t zlen = png_zlen(A);
    uint8_t* t = A.chunk + 8 + zlen - 4;
    t[0] = adler >> 24; t[1] = adler >> 16; t[2] = adler >> 8; t[3] = adler;
    // chunk length and type now: the type is the first 4 bytes the CRC covers
    const uint32_t len = (uint32_t)zlen;
    A.chunk[0] = len >> 24; A.chunk[1] = len >> 16; A.chunk[2] = len >> 8; A.chunk[3] = len;
    A.chunk[4] = 'I'; A.chunk[5] = 'D'; A.chunk[6] = 'A'; A.chunk[7] = 'T';
}

constexpr int kCrcSeg = 256;

// Slicing-by-8 tables (zlib crc32 "braid" precursor): t8[k][n] = CRC of byte n followed by k zeros.
struct Crc8Tab {
    uint32_t t[8][256];
};

constexpr Crc8Tab make_crc8() {
    Crc8Tab c{};
    for (uint32_t n = 0; n < 256; ++n) {
        uint32_t r = n;
        for (int k = 0; k < 8; ++k) r = (r & 1) ? kCrcPoly ^ (r >> 1) : r >> 1;
        c.t[0][n] = r;
    }
    for (int k = 1; k < 8; ++k)
        for (uint32_t n = 0; n < 256; ++n) c.t[k][n] = (c.t[k - 1][n] >> 8) ^ c.t[0][c.t[k - 1][n] & 0xFF];
    return c;
}

__constant__ Crc8Tab c_crc8 = make_crc8();

// CRC-32 of chunk type + data = bytes [4, 8 + zlen) of the chunk buffer: one 256-byte segment per
// lane, 8 bytes per step through the slicing tables in LDS, each segment's CRC shifted to the end
// of the data by x^(8n) mod P, XOR-combined within the workgroup and once per workgroup in memory.
__global__ void __launch_bounds__(256) k_png_crc(PngArgs A) {
    __shared__ uint32_t t[8][256];
    __shared__ uint32_t s_x[4];
    for (int i = threadIdx.x; i < 8 * 256; i += 256) t[i >> 8][i & 255] = c_crc8.t[i >> 8][i & 255];
    __syncthreads();
    const int64_t n = 4 + png_zlen(A);
    const uint8_t* d = A.chunk + 4;                 // 4-byte aligned (chunk is 256-aligned)
    const int64_t s = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t b0 = s * kCrcSeg;
    uint32_t v = 0;
    if (b0 < n) {
        const int64_t b1 = min(n, b0 + kCrcSeg);
        uint32_t r = 0xFFFFFFFFu;
        int64_t i = b0;
        for (; i + 8 <= b1; i += 8) {
            const uint32_t w0 = *reinterpret_cast<const uint32_t*>(d + i) ^ r;
            const uint32_t w1 = *reinterpret_cast<const uint32_t*>(d + i + 4);
            r = t[7][w0 & 0xFF] ^ t[6][(w0 >> 8) & 0xFF] ^ t[5][(w0 >> 16) & 0xFF] ^ t[4][w0 >> 24] ^
                t[3][w1 & 0xFF] ^ t[2][(w1 >> 8) & 0xFF] ^ t[1][(w1 >> 16) & 0xFF] ^ t[0][w1 >> 24];
        }
        for (; i < b1; ++i) r = t[0][(r ^ d[i]) & 0xFF] ^ (r >> 8);
        v = multmodp(x2nmodp((uint64_t)(n - b1), 3), ~r);
    }
    for (int o = 32; o > 0; o >>= 1) v ^= __shfl_xor(v, o, 64);
    if ((threadIdx.x & 63) == 0) s_x[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t x = s_x[0] ^ s_x[1] ^ s_x[2] ^ s_x[3];
        if (x) atomicXor(A.crc_out, x);
    }
}

__global__ void k_png_finish(PngArgs A) {
    const uint32_t crc = *A.crc_out;
    uint8_t* c = A.chunk + 8 + png_zlen(A);
    c[0] = crc >> 24; c[1] = crc >> 16; c[2] = crc >> 8; c[3] = crc;
}

// =====================================================================================
// Deflate (RFC 1951) on the device: the IDAT payload of the rendered-region and mask PNGs.
// ImageIO's PNG writer filters rows adaptively and deflates them; pixels are the parity bar,
// so the filter choice and the LZ77 parse are ours (PNG decoders accept any):
//   D1 k_png_filter     one workgroup per row: the five PNG filters, pick the minimum sum of
//                       |signed residual| (libpng's heuristic), write filter byte + row; Adler
//                       partials
//   D2 k_png_lz_parse   one lane per 32-byte segment (staged in LDS with one row of look-back):
//                       greedy LZ77 over
//                       the distances image rows repeat at (1, bpp, 2*bpp, one row up; matches
//                       may reach back into earlier segments, never past the segment end);
//                       tokens + symbol histograms
//   D3 k_png_tables     length-limited (15-bit) Huffman codes for literal/length and distance
//                       symbols from the two histograms, the run-length coded code-length
//                       header (7-bit code) — one dynamic block for the whole image
//   D4 k_png_lz_bits    bits per segment -> exclusive scan -> bit offsets
//   D5 k_png_lz_write   one lane per segment writes its tokens' codes LSB-first into words
//                       (boundary words ORed), the header and EOB are ORed in by D5's lane 0
//   D6 k_png_zcopy      words -> zlib stream bytes in the IDAT chunk; then Adler-32 and CRC-32
// If the dynamic stream would be longer than stored blocks (noise), the stored encoding is used.
// =====================================================================================
constexpr int kSeg = 32;                   // bytes of filtered stream per parse lane
constexpr int kMaxBits = 15;

struct DeflateTabs {
    uint16_t len_sym[259];   // match length -> literal/length symbol (257..285)
    uint8_t len_xbits[29];
    uint16_t len_base[29];
    uint8_t dist_code[512];  // zlib's _dist_code: d-1 < 256 -> [d-1], else [256 + ((d-1) >> 7)]
    uint8_t dist_xbits[30];
    uint16_t dist_base[30];
};

constexpr DeflateTabs make_deflate_tabs() {
    DeflateTabs t{};
    const uint16_t lb[29] = {3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31, 35, 43, 51, 59, 67, 83, 99,
                             115, 131, 163, 195, 227, 258};
    const uint8_t lx[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
    for (int i = 0; i < 29; ++i) { t.len_base[i] = lb[i]; t.len_xbits[i] = lx[i]; }
    for (int l = 0; l < 259; ++l) {
        int s = 0;
        for (int i = 0; i < 29; ++i)
            if (l >= lb[i]) s = i;
        t.len_sym[l] = (uint16_t)(257 + (l >= 3 ? s : 0));
    }
    t.len_sym[258] = 285;
    const uint16_t db[30] = {1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193, 257, 385, 513, 769, 1025,
                             1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
    const uint8_t dx[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12,
                            13, 13};
    for (int i = 0; i < 30; ++i) { t.dist_base[i] = db[i]; t.dist_xbits[i] = dx[i]; }
    for (int d = 1; d <= 256; ++d) {
        int s = 0;
        for (int i = 0; i < 30; ++i)
            if (d >= db[i]) s = i;
        t.dist_code[d - 1] = (uint8_t)s;
    }
    for (int k = 0; k < 256; ++k) {          // d-1 = k << 7 .. (k << 7) + 127, d > 256
        const int d = (k << 7) + 1;
        int s = 0;
        for (int i = 0; i < 30; ++i)
            if (d >= db[i]) s = i;
        t.dist_code[256 + k] = (uint8_t)(k < 2 ? t.dist_code[(k << 7)] : s);
    }
    return t;
}

__constant__ DeflateTabs c_dfl = make_deflate_tabs();

__device__ __forceinline__ int dist_sym(uint32_t d) {   // 1 <= d <= 32768
    return (d - 1) < 256 ? c_dfl.dist_code[d - 1] : c_dfl.dist_code[256 + ((d - 1) >> 7)];
}

struct DflTables;

struct DflArgs {
    PngArgs P;
    uint8_t* flt;              // [raw] filtered stream
    uint32_t* tokens;          // [raw]: segment s owns [s*kSeg, ...)
    uint16_t* ntok;            // [nseg]
    uint32_t* lhist;           // [286]
    uint32_t* dhist;           // [30]
    const struct DflTables* tab;   // codes, lengths, header (built on the host)
    uint32_t* seg_bits;        // [nseg] -> exclusive offsets after the scan
    uint32_t* tot;             // [2] token bits total (scan), deflate bytes
    uint32_t* words;           // [out words] deflate stream
    unsigned long long* row_sums;  // [H][2] Adler partials per row
    int64_t nseg, out_words;
    int32_t bpp;
};

// Raw (unfiltered) byte i of image row y (0 <= i < rowlen - 1).
__device__ __forceinline__ uint32_t row_byte(const PngArgs& A, int y, int i) {
    if (A.kind == kRgb) {
        const int px = i / 3, comp = i - px * 3;
        return (A.argb[(int64_t)y * A.W + px] >> (16 - 8 * comp)) & 0xFF;
    }
    if (A.kind == kIdx8) return mask_bit(A, i, y);
    uint32_t b = 0;
    for (int k = 0; k < 8; ++k) b = (b << 1) | (i * 8 + k < A.W ? mask_bit(A, i * 8 + k, y) : 0u);
    return b;
}

__device__ __forceinline__ uint32_t paeth(uint32_t a, uint32_t b, uint32_t c) {
    const int p = (int)a + (int)b - (int)c;
    const int pa = abs(p - (int)a), pb = abs(p - (int)b), pc = abs(p - (int)c);
    return (pa <= pb && pa <= pc) ? a : (pb <= pc ? b : c);
}

// D1 works on kPngRowsPerWg consecutive rows per workgroup (the row above each is the previous
// row's, still in LDS: H + H / 4 row loads instead of 2 H).  LDS per workgroup, for rows of
// rb = rowlen - 1 bytes: two row buffers (this row, the row above) and, when they fit, the five
// candidate residual rows, each of stride align4(rb) + 4 behind 4 bytes of zeros (the left
// neighbours of the first pixel are 0; the stash rows keep the filter byte there).
constexpr int kPngRowsPerWg = 4;
__host__ __device__ constexpr int64_t png_row_stride(int64_t rb) { return ((rb + 3) & ~(int64_t)3) + 4; }
constexpr int64_t kPngFilterLdsMax = 150 * 1024;
__host__ __device__ constexpr bool png_filter_stash(int64_t rb) { return 7 * png_row_stride(rb) <= kPngFilterLdsMax; }
__host__ __device__ constexpr int64_t png_filter_lds(int64_t rb) {
    return (png_filter_stash(rb) ? 7 : 2) * png_row_stride(rb);
}

__device__ __forceinline__ uint32_t byte_at(uint32_t w, int k) { return (w >> (8 * k)) & 0xFF; }

// Bytewise x - y mod 256 of four packed bytes (SWAR).
__device__ __forceinline__ uint32_t sub8(uint32_t x, uint32_t y) {
    return ((x | 0x80808080u) - (y & 0x7F7F7F7Fu)) ^ ((x ^ ~y) & 0x80808080u);
}

// Paeth predictors of two bytes held as 16-bit halves (values 0..255), packed 16-bit arithmetic
// (v_pk_*): pa = |b - c|, pb = |a - c|, pc = |a + b - 2c|; a when pa <= min(pb, pc), else b when
// pb <= pc, else c -- the PNG rule, selected by the sign masks of two differences.
typedef short omr_s16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t paeth_pairs(uint32_t a, uint32_t b, uint32_t c) {
    const omr_s16x2 va = __builtin_bit_cast(omr_s16x2, a), vb = __builtin_bit_cast(omr_s16x2, b),
                    vc = __builtin_bit_cast(omr_s16x2, c);
    const omr_s16x2 d1 = vb - vc, d2 = va - vc;
    const omr_s16x2 pa = __builtin_elementwise_abs(d1), pb = __builtin_elementwise_abs(d2),
                    pc = __builtin_elementwise_abs(d1 + d2);
    const omr_s16x2 m = __builtin_elementwise_min(pb, pc);
    uint32_t na = __builtin_bit_cast(uint32_t, (omr_s16x2)((m - pa) >> 15));   // ~0: not a
    uint32_t nb = __builtin_bit_cast(uint32_t, (omr_s16x2)((pc - pb) >> 15));  // ~0: c over b
    // opaque masks: otherwise the selects below become a compare + v_cndmask per 16-bit half
    // (plus the extracts and a v_perm to rejoin them) instead of one v_bitop3 each
    asm("" : "+v"(na), "+v"(nb));
    const uint32_t bc = (nb & c) | (~nb & b);
    return (na & bc) | (~na & a);
}

// Paeth predictor of 4 row bytes (even and odd bytes as two 16-bit pairs); checked against the
// per-byte rule on every (a, b, c) byte triple.
__device__ __forceinline__ uint32_t paeth4(uint32_t A, uint32_t B, uint32_t C) {
    constexpr uint32_t M = 0x00FF00FFu;
    const uint32_t e = paeth_pairs(A & M, B & M, C & M);
    const uint32_t o = paeth_pairs((A >> 8) & M, (B >> 8) & M, (C >> 8) & M);
    return e | (o << 8);
}

// The five PNG filter residuals of 4 row bytes: dword X of this row, B of the row above, A / C the
// same bytes bpp to the left.  None / Sub / Up / Average in SWAR, Paeth on 16-bit pairs.
__device__ __forceinline__ void png_residuals(uint32_t X, uint32_t A, uint32_t B, uint32_t C, uint32_t (&r)[5]) {
    r[0] = X;
    r[1] = sub8(X, A);
    r[2] = sub8(X, B);
    r[3] = sub8(X, (A & B) + (((A ^ B) & 0xFEFEFEFEu) >> 1));    // floor((a + b) / 2) per byte
    r[4] = sub8(X, paeth4(A, B, C));
}

// Sum over the 4 bytes of |(int8) byte| (libpng's minimum-sum heuristic): |(r ^ 0x80) - 0x80| per
// byte, one v_sad_u8.
__device__ __forceinline__ uint32_t abs_sum8(uint32_t r, uint32_t acc) {
    return __builtin_amdgcn_sad_u8(r ^ 0x80808080u, 0x80808080u, acc);
}

// Row yy of image A into the LDS row buffer `row` (rb bytes, zero tail to the dword; yy < 0: zeros).
__device__ __forceinline__ void png_load_row(const PngArgs& A, int yy, int rb, uint8_t* row) {
    uint32_t* rw = reinterpret_cast<uint32_t*>(row);
    const int nw = (rb + 3) >> 2;
    if (yy < 0) {
        for (int j = threadIdx.x; j < nw; j += 256) rw[j] = 0;
        return;
    }
    if (A.kind == kRgb && (A.W & 3) == 0) {        // four pixels (one 16-byte load) -> three dwords
        const uint4* src = reinterpret_cast<const uint4*>(A.argb + (int64_t)yy * A.W);
        for (int q = threadIdx.x; q < (A.W >> 2); q += 256) {
            const uint4 v = src[q];
            rw[3 * q] = __builtin_amdgcn_perm(v.y, v.x, 0x06000102u);       // r0 g0 b0 r1
            rw[3 * q + 1] = __builtin_amdgcn_perm(v.z, v.y, 0x05060001u);   // g1 b1 r2 g2
            rw[3 * q + 2] = __builtin_amdgcn_perm(v.w, v.z, 0x04050600u);   // b2 r3 g3 b3
        }
        return;                                    // rb = 3 W: no tail
    }
    if (A.kind == kRgb) {
        for (int px = threadIdx.x; px < A.W; px += 256) {
            const uint32_t v = A.argb[(int64_t)yy * A.W + px];
            row[3 * px] = (uint8_t)(v >> 16); row[3 * px + 1] = (uint8_t)(v >> 8); row[3 * px + 2] = (uint8_t)v;
        }
    } else {
        for (int i = threadIdx.x; i < rb; i += 256) row[i] = (uint8_t)row_byte(A, yy, i);
    }
    for (int i = rb + threadIdx.x; i < 4 * nw; i += 256) row[i] = 0;
}

// D1: rows y0 .. y0 + nrows - 1 of image A, one workgroup: each row's filter byte + filtered bytes
// at flt + y * rowlen, its Adler partials at rs[2 (y - y0)], rs[2 (y - y0) + 1].  Per row one pass
// computes the five residual rows (4 bytes per lane step) with their |residual| sums and keeps them
// in LDS; the row leaves from the chosen one with aligned dword stores (the partial first / last
// dword, shared with the neighbouring rows, byte by byte).  Rows too wide for the stash recompute
// the chosen filter and store bytes.
__device__ void png_filter_rows(const PngArgs& A, int bpp, int y0, int nrows, uint8_t* __restrict__ flt,
                                unsigned long long* __restrict__ rs, uint8_t* lds) {
    __shared__ uint32_t s_sum[5][4];
    __shared__ int s_f;
    __shared__ unsigned long long s_ad[2][4];
    const int rb = (int)A.rowlen - 1;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int stride = (int)png_row_stride(rb);
    const int nw = (rb + 3) >> 2;
    const bool stash = png_filter_stash(rb);
    uint8_t* rowbuf[2] = {lds + 4, lds + 4 + stride};
    uint8_t* st0 = lds + 2 * stride + 4;           // stash row f at st0 + f * stride
    for (int k = threadIdx.x; k < (stash ? 7 : 2); k += 256)
        *reinterpret_cast<uint32_t*>(lds + k * stride) = 0;     // the pads
    png_load_row(A, y0 - 1, rb, rowbuf[0]);
    const int lsh = 4 - bpp;                       // bytes i-bpp .. i-bpp+3 = alignbyte(w[j], w[j-1], 4-bpp)
    for (int r = 0; r < nrows; ++r) {
        const int y = y0 + r;
        uint8_t* cur = rowbuf[(r + 1) & 1];
        const uint8_t* prev = rowbuf[r & 1];
        png_load_row(A, y, rb, cur);
        __syncthreads();
        const uint32_t* cw = reinterpret_cast<const uint32_t*>(cur);    // cw[-1]: the zero pad
        const uint32_t* pw = reinterpret_cast<const uint32_t*>(prev);
        uint32_t sm[5] = {0, 0, 0, 0, 0};
        for (int j = threadIdx.x; j < nw; j += 256) {
            const uint32_t X = cw[j], Bv = pw[j];
            const uint32_t Av = __builtin_amdgcn_alignbyte(X, cw[j - 1], lsh);
            const uint32_t Cv = __builtin_amdgcn_alignbyte(Bv, pw[j - 1], lsh);
            uint32_t rr[5];
            png_residuals(X, Av, Bv, Cv, rr);
            const int valid = rb - 4 * j;
            const uint32_t vm = valid >= 4 ? 0xFFFFFFFFu : (1u << (8 * valid)) - 1u;
#pragma unroll
            for (int f = 0; f < 5; ++f) {
                sm[f] = abs_sum8(rr[f] & vm, sm[f]);
                if (stash) reinterpret_cast<uint32_t*>(st0 + f * stride)[j] = rr[f];
            }
        }
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            uint32_t v = sm[k];
            for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
            if (lane == 0) s_sum[k][wv] = v;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t best = 0xFFFFFFFFu;
            int bf = 0;
            for (int k = 0; k < 5; ++k) {
                const uint32_t v = s_sum[k][0] + s_sum[k][1] + s_sum[k][2] + s_sum[k][3];
                if (v < best) { best = v; bf = k; }
            }
            s_f = bf;
            if (stash) st0[bf * stride - 1] = (uint8_t)bf;   // v[0] = the filter byte, v[j] = residual j-1
        }
        __syncthreads();
        const int f = s_f;
        const int64_t row0 = (int64_t)y * A.rowlen;
        unsigned long long s1 = 0, s2 = 0;
        if (stash) {
            // global dwords [row0 / 4, (row0 + rowlen - 1) / 4]: v[jj] (jj = byte - row0) read from the
            // stash row as an unaligned dword (two aligned reads + alignbyte)
            const uint8_t* vrow = st0 + f * stride - 1;           // v[jj] = vrow[jj]
            const int64_t g0 = row0 >> 2, g1 = (row0 + A.rowlen - 1) >> 2;
            const uint32_t* vw = reinterpret_cast<const uint32_t*>(st0 + f * stride - 4);   // aligned, vw[0] = pad
            uint32_t* gw = reinterpret_cast<uint32_t*>(flt);
            for (int64_t g = g0 + threadIdx.x; g <= g1; g += 256) {
                const int64_t jj = 4 * g - row0;                  // v index of the dword's first byte
                if (jj >= 0 && jj + 4 <= A.rowlen) {
                    // st0[jj - 1 .. jj + 2] = bytes 4 + jj - 1 .. of vw
                    const int64_t q = jj + 3;                     // byte offset from vw[0]
                    const uint32_t w = __builtin_amdgcn_alignbyte(vw[(q >> 2) + 1], vw[q >> 2], (uint32_t)(q & 3));
                    gw[g] = w;
                    const uint32_t sv = __builtin_amdgcn_sad_u8(w, 0u, 0u);
                    s1 += sv;
                    s2 += (unsigned long long)(A.raw - row0 - jj) * sv - __builtin_amdgcn_udot4(w, 0x03020100u, 0u, false);
                } else {
                    for (int k = 0; k < 4; ++k) {
                        const int64_t t = jj + k;
                        if (t >= 0 && t < A.rowlen) {
                            const uint32_t v = vrow[t];
                            flt[row0 + t] = (uint8_t)v;
                            s1 += v;
                            s2 += (unsigned long long)(A.raw - row0 - t) * v;
                        }
                    }
                }
            }
        } else {
            for (int j = threadIdx.x; j < nw; j += 256) {
                const uint32_t X = cw[j], Bv = pw[j];
                const uint32_t Av = __builtin_amdgcn_alignbyte(X, cw[j - 1], lsh);
                const uint32_t Cv = __builtin_amdgcn_alignbyte(Bv, pw[j - 1], lsh);
                uint32_t rr[5];
                png_residuals(X, Av, Bv, Cv, rr);
                const uint32_t w = rr[f];
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const int i = 4 * j + k;
                    if (i < rb) {
                        const uint32_t v = byte_at(w, k);
                        flt[row0 + 1 + i] = (uint8_t)v;
                        s1 += v;
                        s2 += (unsigned long long)(A.raw - row0 - 1 - i) * v;
                    }
                }
            }
            if (threadIdx.x == 0) {
                flt[row0] = (uint8_t)f;
                s1 += (unsigned long long)f;
                s2 += (unsigned long long)(A.raw - row0) * (unsigned long long)f;
            }
        }
        for (int o = 32; o > 0; o >>= 1) {
            s1 += __shfl_down(s1, o, 64);
            s2 += __shfl_down(s2, o, 64);
        }
        if (lane == 0) { s_ad[0][wv] = s1; s_ad[1][wv] = s2; }
        __syncthreads();                             // also: the stash / row buffers are free again
        if (threadIdx.x == 0) {                      // per-row Adler partials
            rs[2 * r] = s_ad[0][0] + s_ad[0][1] + s_ad[0][2] + s_ad[0][3];
            rs[2 * r + 1] = s_ad[1][0] + s_ad[1][1] + s_ad[1][2] + s_ad[1][3];
        }
    }
}

__global__ void __launch_bounds__(256) k_png_filter(DflArgs D) {
    extern __shared__ __attribute__((aligned(16))) uint8_t s_rows[];
    const int y0 = blockIdx.x * kPngRowsPerWg;
    png_filter_rows(D.P, D.bpp, y0, min(kPngRowsPerWg, D.P.H - y0), D.flt, D.row_sums + 2 * y0, s_rows);
}

// Sum of the per-row Adler partials into A.sums (one workgroup; both encodings carry flt).
__global__ void __launch_bounds__(256) k_png_adler_rows(DflArgs D) {
    __shared__ unsigned long long s_ad[2][4];
    unsigned long long s1 = 0, s2 = 0;
    for (int y = threadIdx.x; y < D.P.H; y += 256) { s1 += D.row_sums[2 * y]; s2 += D.row_sums[2 * y + 1]; }
    for (int o = 32; o > 0; o >>= 1) {
        s1 += __shfl_down(s1, o, 64);
        s2 += __shfl_down(s2, o, 64);
    }
    if ((threadIdx.x & 63) == 0) { s_ad[0][threadIdx.x >> 6] = s1; s_ad[1][threadIdx.x >> 6] = s2; }
    __syncthreads();
    if (threadIdx.x == 0) {
        D.P.sums[0] = s_ad[0][0] + s_ad[0][1] + s_ad[0][2] + s_ad[0][3];
        D.P.sums[1] = s_ad[1][0] + s_ad[1][1] + s_ad[1][2] + s_ad[1][3];
    }
}

constexpr int kParseLanes = 128;            // segments (lanes) per parse workgroup

// Token slot k of segment s (image-local): segments in blocks of kParseLanes, token-major inside a
// block, so the lanes of a wave store (D2) and load (D4/D5) one token index at consecutive
// addresses instead of 128 bytes apart.  A stream's token buffer holds align(nseg, 128) * kSeg.
__device__ __forceinline__ int64_t tok_at(int64_t s, int k) {
    return ((s / kParseLanes) * kSeg + k) * kParseLanes + (s % kParseLanes);
}
__host__ __device__ constexpr int64_t tok_slots(int64_t nseg) {
    return (nseg + kParseLanes - 1) / kParseLanes * kParseLanes * kSeg;
}
constexpr int kMaxBack = 31 * 1024;         // LDS look-back window (bytes)

// A token: a literal byte (bit 31 clear), or a match: bit 31 | lsym - 257 (bits 0-4) | dsym << 5
// (bits 5-9) | the length's extra-bits value << 10 (5 bits) | the distance's extra-bits value << 15
// (13 bits).  D4 / D5 then code it with the two code tables alone; the extra-bit counts follow
// from the symbols (RFC 1951 3.2.5).
__host__ __device__ constexpr int len_xbits_of(int ls) { return (ls < 8 || ls == 28) ? 0 : (ls - 4) >> 2; }
__host__ __device__ constexpr int dist_xbits_of(int ds) { return ds < 4 ? 0 : (ds - 2) >> 1; }
__device__ __forceinline__ uint32_t pack_match(const DeflateTabs& T, uint32_t l, uint32_t d) {
    const uint32_t ls = T.len_sym[l] - 257u;
    const uint32_t ds = (d - 1) < 256 ? T.dist_code[d - 1] : T.dist_code[256 + ((d - 1) >> 7)];
    return 0x80000000u | ls | (ds << 5) | ((l - T.len_base[ls]) << 10) | ((d - T.dist_base[ds]) << 15);
}

// Bit q of the result: byte beg+q equals byte beg+q-d, for q < n (the segment's bytes), from the
// segment's 32 bytes x[] (registers) and the 36 staged bytes from beg-d rounded down to a dword.
__device__ __forceinline__ uint32_t eq_mask(const uint32_t (&x)[8], const uint32_t* sw, int64_t a) {
    const uint32_t* q = sw + (a >> 2);
    const int sh = (int)(a & 3);
    uint32_t m = 0;
    uint32_t lo = q[0];
#pragma unroll
    for (int i = 0; i < 8; i += 2) {
        uint32_t acc = 0;
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const uint32_t hi = q[i + k + 1];
            const uint32_t y = __builtin_amdgcn_alignbyte(hi, lo, sh);
            lo = hi;
            const uint32_t e = x[i + k] ^ y;                  // zero bytes: equal
            const uint32_t z = ~(((e & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | e | 0x7F7F7F7Fu);   // 0x80 per zero byte
            // the four flags (bytes of 0 / 1) weighted 1, 2, 4, 8 (<< 4 for the second dword) by one dot4
            acc = __builtin_amdgcn_udot4((z >> 7) & 0x01010101u, k ? 0x80402010u : 0x08040201u, acc, false);
        }
        m |= acc << (4 * i);
    }
    return m;
}

// D2 in three pieces, shared by the single-image parse (tokens stored), the batched histogram
// pass and the batched encoder (both re-parse instead of storing tokens, round 5):
//   lz_stage         the workgroup stages its kParseLanes * kSeg bytes of filtered stream plus the
//                    look-back window (one image row, <= 31 KiB) in LDS
//   lz_seg_prepare   one lane per kSeg-byte segment: for each candidate distance (1, bpp, 2*bpp,
//                    one row up) a 32-bit mask of "byte == byte d back", built with dword compares
//   lz_seg_tokens    greedy LZ77 from the masks: the match length at q is the run of ones from bit
//                    q; the first candidate with the longest match wins (the tokens of a byte-by-
//                    byte compare loop); every token goes to tok(t, position, candidate or -1)
// flt is the image's filtered stream (16-byte aligned); the staged window covers [wbeg, bend).
__device__ __forceinline__ void lz_stage(const uint8_t* __restrict__ flt, int64_t raw, int64_t blk, int32_t back,
                                         uint8_t* s_win, int64_t& wbeg, int64_t& bend) {
    const int64_t bbeg = blk * kParseLanes * kSeg;
    bend = min(raw, bbeg + (int64_t)kParseLanes * kSeg);
    wbeg = max((int64_t)0, bbeg - back);                        // back is a multiple of 16
    const int64_t n16 = (bend - wbeg) / 16;
    const uint4* g16 = reinterpret_cast<const uint4*>(flt + wbeg);
    for (int64_t i = threadIdx.x; i < n16; i += blockDim.x) reinterpret_cast<uint4*>(s_win)[i] = g16[i];
    for (int64_t i = wbeg + n16 * 16 + threadIdx.x; i < bend; i += blockDim.x) s_win[i - wbeg] = flt[i];
}

struct LzSeg {
    uint32_t m[4];      // equal-byte masks per candidate distance
    uint32_t dl[4];     // the candidate distances
    int nd, n;          // candidates, segment bytes
    int64_t beg;        // stream offset of the segment
};

__device__ __forceinline__ void lz_seg_prepare(const uint8_t* s_win, int64_t wbeg, int64_t s, int64_t raw,
                                               int64_t rowlen, int bpp, int32_t back, LzSeg& L) {
    const uint8_t* f = s_win - wbeg;            // f[p] for p in [wbeg, bend)
    const uint32_t* sw = reinterpret_cast<const uint32_t*>(s_win);
    const int64_t beg = s * kSeg;
    L.beg = beg;
    const int n = (int)(min(raw, beg + kSeg) - beg);
    L.n = n;
    const uint32_t nmask = n >= 32 ? 0xFFFFFFFFu : (1u << n) - 1u;
    uint32_t x[8];
    {
        const uint4* o = reinterpret_cast<const uint4*>(s_win + (beg - wbeg));   // 16-byte aligned
        const uint4 u0 = o[0], u1 = o[1];
        x[0] = u0.x; x[1] = u0.y; x[2] = u0.z; x[3] = u0.w;
        x[4] = u1.x; x[5] = u1.y; x[6] = u1.z; x[7] = u1.w;
    }
    // candidates in the compare order of the byte-wise parse: 1, bpp, 2 bpp (not for bpp 1,
    // where bpp repeats distance 1), one row up
    L.nd = bpp == 1 ? 2 : 4;
    L.dl[0] = 1u;
    L.dl[1] = bpp == 1 ? (uint32_t)rowlen : (uint32_t)bpp;
    L.dl[2] = (uint32_t)(2 * bpp);
    L.dl[3] = (uint32_t)rowlen;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        L.m[k] = 0;
        if (k >= L.nd) continue;
        const int64_t d = L.dl[k];
        if (d > back) continue;                              // past the staged look-back
        if (beg - d >= wbeg) {
            L.m[k] = eq_mask(x, sw, beg - d - wbeg) & nmask;
        } else {                                             // the window's first bytes
            uint32_t mm = 0;
            for (int q = 0; q < n; ++q)
                if (beg + q - d >= wbeg && f[beg + q] == f[beg + q - d]) mm |= 1u << q;
            L.m[k] = mm;
        }
    }
}

template <typename Tok>
__device__ __forceinline__ void lz_seg_tokens(const LzSeg& L, const uint8_t* s_win, int64_t wbeg,
                                              const DeflateTabs& T, Tok&& tok) {
    const uint8_t* f = s_win - wbeg;
    // positions where some candidate's run of equal bytes reaches 3: the only places a match can
    // start; the bytes in between are literals and skip the candidate evaluation
    uint32_t A = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        if (k >= L.nd) break;
        A |= L.m[k] & (L.m[k] >> 1) & (L.m[k] >> 2);
    }
    int p = 0;
    while (p < L.n) {
        const uint32_t ap = p < 32 ? A >> p : 0u;
        const int q = ap ? p + __builtin_ctz(ap) : L.n;        // the next match start (or the end)
        for (; p < q; ++p) tok((uint32_t)f[L.beg + p], p, -1);
        if (p >= L.n) break;
        int best = 0, bk = 0;
        uint32_t bd = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (k >= L.nd) break;
            const uint32_t v = L.m[k] >> p;
            const int l = v == 0xFFFFFFFFu ? 32 : __builtin_ctz(~v);   // run of equal bytes from p
            if (l > best) { best = l; bd = L.dl[k]; bk = k; }
        }
        if (best >= 3) {
            tok(pack_match(T, (uint32_t)best, bd), p, bk);
            p += best;
        } else {
            tok((uint32_t)f[L.beg + p], p, -1);
            ++p;
        }
    }
}

static_assert(sizeof(DeflateTabs) % 2 == 0 && alignof(DeflateTabs) == 2, "DeflateTabs copies as u16");
__device__ __forceinline__ void lz_load_tabs(DeflateTabs& T) {
    const uint16_t* src = reinterpret_cast<const uint16_t*>(&c_dfl);
    uint16_t* dst = reinterpret_cast<uint16_t*>(&T);
    for (int i = threadIdx.x; i < (int)(sizeof(DeflateTabs) / 2); i += blockDim.x) dst[i] = src[i];
}

// Parse block `blk` of one image with the tokens stored (the single-image pipeline): tokens / ntok
// its segments' token slots (tok_at) and counts, lhist / dhist its symbol histograms.
__device__ void png_lz_parse_block(const uint8_t* __restrict__ flt, int64_t raw, int64_t rowlen, int bpp,
                                   int64_t nseg, int64_t blk, int32_t back, uint32_t* __restrict__ tokens,
                                   uint16_t* __restrict__ ntok, uint32_t* __restrict__ lhist,
                                   uint32_t* __restrict__ dhist, uint8_t* s_win) {
    __shared__ uint32_t lh[286], dh[30];
    __shared__ DeflateTabs T;
    for (int i = threadIdx.x; i < 286; i += kParseLanes) lh[i] = 0;
    if (threadIdx.x < 30) dh[threadIdx.x] = 0;
    lz_load_tabs(T);
    int64_t wbeg, bend;
    lz_stage(flt, raw, blk, back, s_win, wbeg, bend);
    __syncthreads();
    const int64_t s = blk * kParseLanes + threadIdx.x;
    if (s < nseg) {
        LzSeg L;
        lz_seg_prepare(s_win, wbeg, s, raw, rowlen, bpp, back, L);
        int nt = 0;
        lz_seg_tokens(L, s_win, wbeg, T, [&](uint32_t t, int, int) {
            tokens[tok_at(s, nt++)] = t;
            if (t & 0x80000000u) {
                atomicAdd(&lh[257 + (t & 31)], 1u);
                atomicAdd(&dh[(t >> 5) & 31], 1u);
            } else {
                atomicAdd(&lh[t], 1u);
            }
        });
        ntok[s] = (uint16_t)nt;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < 286; i += kParseLanes)
        if (lh[i]) atomicAdd(&lhist[i], lh[i]);
    if (threadIdx.x < 30 && dh[threadIdx.x]) atomicAdd(&dhist[threadIdx.x], dh[threadIdx.x]);
}

__global__ void __launch_bounds__(kParseLanes) k_png_lz_parse(DflArgs D, int32_t back) {
    extern __shared__ __attribute__((aligned(16))) uint8_t s_win[];
    png_lz_parse_block(D.flt, D.P.raw, D.P.rowlen, D.bpp, D.nseg, blockIdx.x, back, D.tokens, D.ntok, D.lhist,
                       D.dhist, s_win);
}

// ---- D3 on the device: the code is a function of two small histograms (286 + 30 counts); one
// workgroup builds it between D2 and D4, so an encode needs no host round trip mid-pipeline.
// The parallel steps (ranking, depths, length assignment, canonical codes) use every lane; the
// two-queue merge, the Kraft repair and the run-length header are short serial loops on lane 0.

// Exclusive scan over the workgroup (blockDim.x a multiple of 64, s_wave[blockDim.x / 64]).
__device__ __forceinline__ uint32_t pngb_block_excl_scan(uint32_t v, uint32_t* s_wave, uint32_t& total) {
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

// Measurement build only (tools/ab_build.sh <name> -DOMR_PNG_T3_PROBE): block 0's shader-clock
// stamps at the phases of the table build, read back by omr_png_t3_probe (tools/png_batch_probe.py).
#ifdef OMR_PNG_T3_PROBE
__device__ unsigned long long g_t3[32];
#define T3MARK(i) do { if (blockIdx.x == 0 && threadIdx.x == 0) g_t3[i] = __builtin_amdgcn_s_memtime(); } while (0)
// P4 phases of one workgroup in the middle of the grid, in g_t3[16 + i]
#define T4MARK(i) do { if (blockIdx.x == gridDim.x / 2 && threadIdx.x == 0) g_t3[16 + (i)] = __builtin_amdgcn_s_memtime(); } while (0)
extern "C" int omr_png_t3_probe(unsigned long long* out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_t3), sizeof(g_t3)) == hipSuccess ? 0 : 1;
}
#else
#define T3MARK(i) do {} while (0)
#define T4MARK(i) do {} while (0)
#endif

// The table block D4/D5 read: codes, lengths and the block header bits.
struct DflTables {
    uint16_t lcode[286];
    uint16_t dcode[30];
    uint8_t llen[286];
    uint8_t dlen[30];
    uint32_t hdr[96];        // header bits LSB-first; hdr[95] = bit count
};

constexpr int kHuffMaxSym = 288;
constexpr int kHuffNodes = kHuffMaxSym + 2;   // W.wt index of node m (the first merged node)
constexpr int kHuffThreads = 320;       // one symbol per thread (286 + 30 + 19 symbols: <= 286)
struct HuffWork {                       // LDS scratch of one tree
    alignas(16) uint32_t f[kHuffMaxSym];   // symbol frequencies
    uint32_t wt[2 * kHuffMaxSym + 8];   // leaf weights (sorted) + 2 x INF; merged nodes from kHuffNodes
    int16_t ord[kHuffMaxSym];           // used symbols by (frequency, symbol)
    int16_t parent[2 * kHuffMaxSym];
    uint8_t len[kHuffMaxSym];
    int bl[17];                         // leaves per code length
    int next[17];
    int wcnt[kHuffThreads / 64][16];    // per wave: symbols of each code length
    int m;
};
static_assert(sizeof(HuffWork::wt) >= 8 * (kHuffMaxSym + 1) && offsetof(HuffWork, wt) % 16 == 0,
              "the rank keys (u64, n + 1) fit W.wt, 16-byte aligned");

// Code lengths (<= maxbits) of the n symbols in W.f -> W.len, by the two-queue Huffman
// construction (leaves sorted by (freq, symbol)), then miniz's tdefl_huffman_enforce_max_code_size:
// clamp, then drop one max-length code and split the longest shorter code until the Kraft sum is
// exactly 2^maxbits; the longest codes go to the least frequent symbols.  Fewer than two used
// symbols get two 1-bit codes (RFC 1951 3.2.7 allows the unused one).  Every thread calls it.
__device__ void huff_lengths_dev(HuffWork& W, int n, int maxbits) {
    const int tid = threadIdx.x, nt = blockDim.x;
    if (tid == 0) W.m = 0;
    if (tid < 17) W.bl[tid] = 0;
    __syncthreads();
    if (n == 286) T3MARK(8);
    // rank among the used symbols in (frequency, symbol) order: with key = f << 9 | symbol (all
    // ones for an unused symbol) a rank is one 64-bit compare per symbol, two keys per broadcast
    // read (round 6: a third of the compares-and-selects of the (f, j < i) test)
    uint64_t* key = reinterpret_cast<uint64_t*>(W.wt);          // free until the merge
    for (int i = tid; i < n + 1; i += nt) {
        const uint32_t fi = i < n ? W.f[i] : 0u;
        key[i] = fi ? ((uint64_t)fi << 9) | (uint32_t)i : ~0ull;
    }
    __syncthreads();
    for (int i = tid; i < n; i += nt) {
        const uint64_t ki = key[i];
        W.len[i] = 0;
        if (ki != ~0ull) {
            int r = 0;
            const uint4* k2 = reinterpret_cast<const uint4*>(key);
#pragma unroll 4
            for (int j = 0; j < n; j += 2) {        // keys j, j + 1 (key[n] is all ones)
                const uint4 v = k2[j >> 1];
                r += (((uint64_t)v.y << 32) | v.x) < ki ? 1 : 0;
                r += (((uint64_t)v.w << 32) | v.z) < ki ? 1 : 0;
            }
            W.ord[r] = (int16_t)i;
            atomicAdd(&W.m, 1);
        }
    }
    __syncthreads();
    const int m = W.m;
    if (m < 2) {
        if (tid == 0) {
            const int a = m == 1 ? W.ord[0] : 0;
            W.len[a] = 1;
            W.len[a == 0 ? 1 : 0] = 1;
        }
        __syncthreads();
        return;
    }
    // leaves, two INF entries after them, and INF in every node slot (a node not yet merged)
    for (int k = tid; k < kHuffNodes + m + 1; k += nt)
        W.wt[k] = k < m ? W.f[W.ord[k]] : 0xFFFFFFFFu;
    __syncthreads();
    if (n == 286) T3MARK(9);
    if (tid == 0) {                                 // two queues: sorted leaves, merged nodes
        // Serial: each merge reads the two queue heads as two adjacent pairs -- leaves past m and
        // nodes not yet merged read INF, so the reads are unconditional and go out together --
        // and selects without branches.  A leaf wins ties, as wt[li] <= wt[qi] does.
        int li = 0, qi = m, qn = m;
        const uint32_t* nodes = W.wt + kHuffNodes - m;   // nodes[q]: node q (q >= m)
        for (int c = 0; c < m - 1; ++c) {
            const uint32_t a = W.wt[li], b = W.wt[li + 1];
            const uint32_t q0 = nodes[qi], q1 = nodes[qi + 1];
            const bool la = a <= q0;                 // first: leaf li, else node qi
            const int p0 = la ? li : qi;
            const uint32_t w0 = la ? a : q0;
            const uint32_t c1 = la ? b : a, c2 = la ? q0 : q1;   // the second's two candidates
            const bool lb = c1 <= c2;                // second: a leaf, else a node
            const int p1 = la ? (lb ? li + 1 : qi) : (lb ? li : qi + 1);
            const uint32_t w1 = lb ? c1 : c2;
            li += (la ? 1 : 0) + (lb ? 1 : 0);
            qi += (la ? 0 : 1) + (lb ? 0 : 1);
            W.wt[kHuffNodes + qn - m] = w0 + w1;
            W.parent[p0] = W.parent[p1] = (int16_t)qn;
            ++qn;
        }
    }
    __syncthreads();
    if (n == 286) T3MARK(10);
    const int root = 2 * m - 2;
    for (int k = tid; k < m; k += nt) {             // leaf depth: walk up to the root
        int d = 0;
        for (int x = k; x != root; x = W.parent[x]) ++d;
        atomicAdd(&W.bl[min(d, maxbits)], 1);
    }
    __syncthreads();
    if (n == 286) T3MARK(11);
    if (tid == 0) {                                 // Kraft repair after the clamp (in registers)
        int bl[16];
#pragma unroll
        for (int b = 0; b < 16; ++b) bl[b] = W.bl[b];
        uint32_t total = 0;
#pragma unroll
        for (int b = 1; b < 16; ++b)
            if (b <= maxbits) total += (uint32_t)bl[b] << (maxbits - b);
        while (total != (1u << maxbits)) {
#pragma unroll
            for (int b = 1; b < 16; ++b)
                if (b == maxbits) bl[b]--;
            bool done = false;
#pragma unroll
            for (int b = 14; b > 0; --b)
                if (!done && b < maxbits && bl[b]) { bl[b]--; bl[b + 1] += 2; done = true; }
            --total;
        }
#pragma unroll
        for (int b = 0; b < 16; ++b) W.bl[b] = bl[b];
    }
    __syncthreads();
    for (int k = tid; k < m; k += nt) {             // rank k -> length (least frequent longest)
        int cum = 0, b = maxbits;
        for (; b > 1; --b) {
            cum += W.bl[b];
            if (k < cum) break;
        }
        W.len[W.ord[k]] = (uint8_t)b;
    }
    __syncthreads();
    if (n == 286) T3MARK(12);
}

// Canonical codes of W.len (RFC 1951 3.2.2), bit-reversed for LSB-first packing; every thread
// (kHuffThreads, one symbol each).  A symbol's rank among the symbols of its length: ballots
// per length inside its wave, plus the counts of the waves before it.
__device__ void huff_canon_dev(HuffWork& W, int n, uint16_t* code) {
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int l = tid < n ? W.len[tid] : 0;
    const uint64_t lt = (1ull << lane) - 1;
    int rk = 0;
#pragma unroll
    for (int b = 1; b < 16; ++b) {
        const uint64_t mk = __ballot(l == b);
        if (lane == 0) W.wcnt[wv][b] = __popcll(mk);
        if (l == b) rk = __popcll(mk & lt);
    }
    __syncthreads();
    if (tid == 0) {
        int c = 0, prev = 0;
        for (int b = 1; b < 16; ++b) {
            c = (c + prev) << 1;
            W.next[b] = c;
            prev = 0;
            for (int w = 0; w < kHuffThreads / 64; ++w) prev += W.wcnt[w][b];
        }
    }
    __syncthreads();
    if (tid < n) {
        if (!l) {
            code[tid] = 0;
        } else {
            for (int w = 0; w < wv; ++w) rk += W.wcnt[w][l];
            const uint32_t v = (uint32_t)(W.next[l] + rk);
            code[tid] = (uint16_t)(__brev(v) >> (32 - l));
        }
    }
    __syncthreads();
}

// D3: one workgroup.  hist = [286 literal/length][30 distance] counts from D2.
__device__ void png_build_tables(const uint32_t* __restrict__ hist, DflTables* __restrict__ T) {
    __shared__ HuffWork W;
    __shared__ DflTables t;
    __shared__ uint8_t seq[286 + 30];
    __shared__ uint8_t rs[286 + 30], rx[286 + 30];   // run-length symbols and their extra bits
    __shared__ int s_nr, s_hlit, s_hdist;
    const int tid = threadIdx.x;
    T3MARK(0);
    for (int i = tid; i < 286; i += kHuffThreads) W.f[i] = hist[i] + (i == 256 ? 1u : 0u);   // + EOB
    huff_lengths_dev(W, 286, kMaxBits);
    T3MARK(1);
    for (int i = tid; i < 286; i += kHuffThreads) t.llen[i] = W.len[i];
    huff_canon_dev(W, 286, t.lcode);
    T3MARK(2);
    if (tid < 30) W.f[tid] = hist[286 + tid];
    huff_lengths_dev(W, 30, kMaxBits);
    if (tid < 30) t.dlen[tid] = W.len[tid];
    huff_canon_dev(W, 30, t.dcode);
    T3MARK(3);
    // zlib trees.c scan_tree over the lengths, one thread per run of equal lengths (round 6; the
    // serial walk on lane 0 took ~107k cycles): runs found by a neighbour compare and compacted by
    // a scan, each run's entries counted, scanned and written at their positions -- the same
    // entries in the same order as the walk (a zero run: chunks of min(rest, 138) while >= 3
    // remain; a non-zero run: the length, then 16 for min(rest - 1, 6) more, while >= 4 remain;
    // single entries for the rest).  Entries <= ns <= 316 < kHuffThreads.
    __shared__ uint32_t s_wave[kHuffThreads / 64];
    __shared__ int16_t run_at[286 + 30 + 1];
    __shared__ int s_hclen;
    if (tid == 0) {
        int hlit = 286, hdist = 30;
        while (hlit > 257 && t.llen[hlit - 1] == 0) --hlit;
        while (hdist > 1 && t.dlen[hdist - 1] == 0) --hdist;
        s_hlit = hlit; s_hdist = hdist;
    }
    __syncthreads();
    const int ns = s_hlit + s_hdist;
    if (tid < ns) seq[tid] = tid < s_hlit ? t.llen[tid] : t.dlen[tid - s_hlit];
    __syncthreads();
    {
        const bool st = tid < ns && (tid == 0 || seq[tid] != seq[tid - 1]);
        uint32_t nruns;
        const uint32_t ri = pngb_block_excl_scan(st ? 1u : 0u, s_wave, nruns);
        if (st) run_at[ri] = (int16_t)tid;
        if (tid == 0) run_at[nruns] = (int16_t)ns;
        __syncthreads();
        const bool own = tid < (int)nruns;
        const int r0 = own ? run_at[tid] : 0, len = own ? run_at[tid + 1] - r0 : 0;
        const int v = own ? seq[r0] : 0;
        auto walk = [&](auto&& emit) {               // the run's entries, in the walk's order
            int rem = len;
            if (v == 0) {
                while (rem >= 3) {
                    const int k = min(rem, 138);
                    emit(k >= 11 ? 18 : 17, k >= 11 ? k - 11 : k - 3);
                    rem -= k;
                }
            } else {
                while (rem >= 4) {
                    const int k = min(rem - 1, 6);
                    emit(v, 0);
                    emit(16, k - 3);
                    rem -= 1 + k;
                }
            }
            for (; rem > 0; --rem) emit(v, 0);
        };
        uint32_t cnt = 0;
        walk([&](int, int) { ++cnt; });
        uint32_t nr_all;
        uint32_t at = pngb_block_excl_scan(cnt, s_wave, nr_all);
        walk([&](int sym, int x) { rs[at] = (uint8_t)sym; rx[at] = (uint8_t)x; ++at; });
        if (tid == 0) s_nr = (int)nr_all;
    }
    if (tid < 19) W.f[tid] = 0;
    __syncthreads();
    T3MARK(4);
    const int nr = s_nr;
    for (int i = tid; i < nr; i += kHuffThreads) atomicAdd(&W.f[rs[i]], 1u);
    huff_lengths_dev(W, 19, 7);
    __shared__ uint16_t ccode[19];
    huff_canon_dev(W, 19, ccode);
    T3MARK(5);
    // The block header, LSB-first: BFINAL, BTYPE, HLIT, HDIST, HCLEN (17 bits), HCLEN 3-bit
    // code-length-code lengths, then every run-length entry's code + extra bits at its scanned bit
    // offset -- each field ORed into its (at most two) words in parallel.
    static constexpr uint8_t kOrd[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
    for (int i = tid; i < 96; i += kHuffThreads) t.hdr[i] = 0;
    if (tid == 0) {
        int hclen = 19;
        while (hclen > 4 && W.len[kOrd[hclen - 1]] == 0) --hclen;
        s_hclen = hclen;
    }
    __syncthreads();
    const int hclen = s_hclen;
    const uint32_t hbits = 17 + 3 * (uint32_t)hclen;
    auto put_at = [&](uint32_t pos, uint32_t v) {    // v < 2^17
        const uint64_t sh = (uint64_t)v << (pos & 31);
        atomicOr(&t.hdr[pos >> 5], (uint32_t)sh);
        if ((uint32_t)(sh >> 32)) atomicOr(&t.hdr[(pos >> 5) + 1], (uint32_t)(sh >> 32));
    };
    uint32_t ev = 0, en = 0;
    if (tid < nr) {
        const int sym = rs[tid];
        const int xb = sym == 16 ? 2 : sym == 17 ? 3 : sym == 18 ? 7 : 0;
        ev = ccode[sym] | ((uint32_t)rx[tid] << W.len[sym]);
        en = (uint32_t)(W.len[sym] + xb);
    }
    uint32_t ebits;
    const uint32_t eoff = hbits + pngb_block_excl_scan(en, s_wave, ebits);
    if (en) put_at(eoff, ev);
    if (tid < hclen) put_at(17 + 3 * (uint32_t)tid, W.len[kOrd[tid]]);
    if (tid == 0) {
        put_at(0, 1u | (2u << 1) | ((uint32_t)(s_hlit - 257) << 3) | ((uint32_t)(s_hdist - 1) << 8) |
                      ((uint32_t)(hclen - 4) << 13));
        t.hdr[95] = hbits + ebits;
    }
    __syncthreads();
    T3MARK(6);
    const uint32_t* src = reinterpret_cast<const uint32_t*>(&t);
    uint32_t* dst = reinterpret_cast<uint32_t*>(T);
    for (int i = tid; i < (int)(sizeof(DflTables) / 4); i += kHuffThreads) dst[i] = src[i];
    T3MARK(7);
}

__global__ void __launch_bounds__(kHuffThreads) k_png_tables(const uint32_t* __restrict__ hist, DflTables* __restrict__ T) {
    png_build_tables(hist, T);
}

// ---- D3 on the host (the default): the same construction in C++ between D2 and D4 (one
// 1.3 KB histogram read back, one 1 KB table upload).  Measured faster per encode than the
// single-workgroup device build above, which ctx->png_device_d3 selects.
// Code lengths (<= maxbits) by the two-queue Huffman construction (leaves sorted by (freq,
// symbol)), then miniz's tdefl_huffman_enforce_max_code_size: clamp, then drop one max-length
// code and split the longest shorter code until the Kraft sum is exactly 2^maxbits; the longest
// codes go to the least frequent symbols.  Fewer than two used symbols get two 1-bit codes
// (RFC 1951 3.2.7 allows the unused one).
static void huff_lengths_host(const uint32_t* freq, int n, int maxbits, uint8_t* len) {
    std::vector<int> ord;
    for (int i = 0; i < n; ++i) {
        len[i] = 0;
        if (freq[i]) ord.push_back(i);
    }
    std::stable_sort(ord.begin(), ord.end(), [&](int a, int b) { return freq[a] < freq[b]; });
    const int m = (int)ord.size();
    if (m < 2) {
        const int a = m == 1 ? ord[0] : 0;
        len[a] = 1;
        len[a == 0 ? 1 : 0] = 1;
        return;
    }
    std::vector<uint64_t> wt(2 * m);
    std::vector<int> parent(2 * m), depth(2 * m);
    for (int i = 0; i < m; ++i) wt[i] = freq[ord[i]];
    int li = 0, qi = m, qn = m;
    for (int c = 0; c < m - 1; ++c) {
        int pick[2];
        for (int k = 0; k < 2; ++k) pick[k] = (li < m && (qi >= qn || wt[li] <= wt[qi])) ? li++ : qi++;
        wt[qn] = wt[pick[0]] + wt[pick[1]];
        parent[pick[0]] = parent[pick[1]] = qn++;
    }
    const int root = qn - 1;
    depth[root] = 0;
    int bl[64] = {0};
    for (int node = root - 1; node >= 0; --node) {
        depth[node] = depth[parent[node]] + 1;
        if (node < m) bl[std::min(depth[node], maxbits)]++;
    }
    uint32_t total = 0;
    for (int b = maxbits; b > 0; --b) total += (uint32_t)bl[b] << (maxbits - b);
    while (total != (1u << maxbits)) {
        bl[maxbits]--;
        for (int b = maxbits - 1; b > 0; --b)
            if (bl[b]) { bl[b]--; bl[b + 1] += 2; break; }
        --total;
    }
    int k = 0;
    for (int b = maxbits; b >= 1; --b)
        for (int c = 0; c < bl[b]; ++c) len[ord[k++]] = (uint8_t)b;
}

// Canonical codes (RFC 1951 3.2.2), bit-reversed for LSB-first packing.
static void canon_host(const uint8_t* len, int n, uint16_t* code) {
    int bl[16] = {0}, next[16] = {0};
    for (int i = 0; i < n; ++i) bl[len[i]]++;
    bl[0] = 0;
    int c = 0;
    for (int b = 1; b < 16; ++b) { c = (c + bl[b - 1]) << 1; next[b] = c; }
    for (int i = 0; i < n; ++i) {
        if (!len[i]) { code[i] = 0; continue; }
        uint32_t v = (uint32_t)next[len[i]]++, r = 0;
        for (int b = 0; b < len[i]; ++b) r |= ((v >> b) & 1u) << (len[i] - 1 - b);
        code[i] = (uint16_t)r;
    }
}

static void build_dynamic_block(const uint32_t* lhist, const uint32_t* dhist, DflTables& T) {
    uint32_t lf[286], df[30];
    for (int i = 0; i < 286; ++i) lf[i] = lhist[i] + (i == 256 ? 1u : 0u);   // + EOB
    for (int i = 0; i < 30; ++i) df[i] = dhist[i];
    huff_lengths_host(lf, 286, kMaxBits, T.llen);
    huff_lengths_host(df, 30, kMaxBits, T.dlen);
    canon_host(T.llen, 286, T.lcode);
    canon_host(T.dlen, 30, T.dcode);
    int hlit = 286, hdist = 30;
    while (hlit > 257 && T.llen[hlit - 1] == 0) --hlit;
    while (hdist > 1 && T.dlen[hdist - 1] == 0) --hdist;
    std::vector<uint8_t> seq(T.llen, T.llen + hlit);
    seq.insert(seq.end(), T.dlen, T.dlen + hdist);
    std::vector<std::pair<uint8_t, uint8_t>> rle;        // (symbol, extra) — zlib trees.c scan_tree
    const int ns = (int)seq.size();
    for (int i = 0; i < ns;) {
        const int v = seq[i];
        int r = 1;
        while (i + r < ns && seq[i + r] == v) ++r;
        if (v == 0 && r >= 3) {
            const int k = std::min(r, 138);
            rle.push_back(k >= 11 ? std::make_pair((uint8_t)18, (uint8_t)(k - 11)) : std::make_pair((uint8_t)17, (uint8_t)(k - 3)));
            i += k;
        } else if (v != 0 && r >= 4) {
            const int k = std::min(r - 1, 6);
            rle.push_back({(uint8_t)v, 0});
            rle.push_back({16, (uint8_t)(k - 3)});
            i += 1 + k;
        } else {
            rle.push_back({(uint8_t)v, 0});
            ++i;
        }
    }
    uint32_t cf[19] = {0};
    for (auto& e : rle) cf[e.first]++;
    uint8_t clen[19];
    uint16_t ccode[19];
    huff_lengths_host(cf, 19, 7, clen);
    canon_host(clen, 19, ccode);
    static const uint8_t kOrd[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
    int hclen = 19;
    while (hclen > 4 && clen[kOrd[hclen - 1]] == 0) --hclen;
    std::memset(T.hdr, 0, sizeof(T.hdr));
    uint32_t nb = 0;
    auto put = [&](uint32_t v, int n) {
        for (int b = 0; b < n; ++b, ++nb)
            if ((v >> b) & 1u) T.hdr[nb >> 5] |= 1u << (nb & 31);
    };
    put(1, 1);                           // BFINAL
    put(2, 2);                           // BTYPE = 10 (dynamic)
    put((uint32_t)(hlit - 257), 5);
    put((uint32_t)(hdist - 1), 5);
    put((uint32_t)(hclen - 4), 4);
    for (int i = 0; i < hclen; ++i) put(clen[kOrd[i]], 3);
    for (auto& e : rle) {
        put(ccode[e.first], clen[e.first]);
        if (e.first == 16) put(e.second, 2);
        else if (e.first == 17) put(e.second, 3);
        else if (e.first == 18) put(e.second, 7);
    }
    T.hdr[95] = nb;
}

__device__ __forceinline__ uint32_t token_bits(uint32_t t, const uint8_t* llen, const uint8_t* dlen) {
    if (!(t & 0x80000000u)) return llen[t];
    const int ls = (int)(t & 31), ds = (int)((t >> 5) & 31);
    return llen[257 + ls] + len_xbits_of(ls) + dlen[ds] + dist_xbits_of(ds);
}

// The codes of one packed token, LSB-first through put(value, bits).
template <typename Put>
__device__ __forceinline__ void put_token(uint32_t t, const uint16_t* lcode, const uint8_t* llen, const uint16_t* dcode,
                                          const uint8_t* dlen, Put& put) {
    if (!(t & 0x80000000u)) {
        put(lcode[t], llen[t]);
        return;
    }
    const int ls = (int)(t & 31), ds = (int)((t >> 5) & 31);
    put(lcode[257 + ls], llen[257 + ls]);
    const int lx = len_xbits_of(ls), dx = dist_xbits_of(ds);
    if (lx) put((t >> 10) & 31u, lx);
    put(dcode[ds], dlen[ds]);
    if (dx) put((t >> 15) & 0x1FFFu, dx);
}

__global__ void __launch_bounds__(256) k_png_lz_bits(DflArgs D) {
    __shared__ uint8_t llen[286], dlen[30];
    for (int i = threadIdx.x; i < 286; i += 256) llen[i] = D.tab->llen[i];
    if (threadIdx.x < 30) dlen[threadIdx.x] = D.tab->dlen[threadIdx.x];
    __syncthreads();
    const int64_t s = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (s >= D.nseg) return;
    const int nt = D.ntok[s];
    uint32_t b = 0;
    for (int i = 0; i < nt; ++i) b += token_bits(D.tokens[tok_at(s, i)], llen, dlen);
    D.seg_bits[s] = b;
}

// Zero the deflate words the stream will occupy (bounded by the device-side total).
__global__ void __launch_bounds__(256) k_png_zero_words(DflArgs D) {
    const uint32_t total = D.tab->hdr[95] + D.tot[0] + 15;
    const int64_t nw = min((int64_t)(total + 31) / 32 + 1, D.out_words);
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nw; i += (int64_t)gridDim.x * 256) D.words[i] = 0;
}

__global__ void __launch_bounds__(256) k_png_lz_write(DflArgs D) {
    __shared__ uint8_t llen[286], dlen[30];
    __shared__ uint16_t lcode[286], dcode[30];
    for (int i = threadIdx.x; i < 286; i += 256) { llen[i] = D.tab->llen[i]; lcode[i] = D.tab->lcode[i]; }
    if (threadIdx.x < 30) { dlen[threadIdx.x] = D.tab->dlen[threadIdx.x]; dcode[threadIdx.x] = D.tab->dcode[threadIdx.x]; }
    __syncthreads();
    const uint32_t hb = D.tab->hdr[95];
    const int64_t s = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (s == 0) {
        for (uint32_t i = 0; i < (hb + 31) / 32; ++i) atomicOr(&D.words[i], D.tab->hdr[i]);
        const uint32_t eob = hb + D.tot[0];
        const uint32_t v = lcode[256], n = llen[256], wi = eob >> 5, sh = eob & 31;
        atomicOr(&D.words[wi], v << sh);
        if (sh + n > 32) atomicOr(&D.words[wi + 1], v >> (32 - sh));
        D.tot[1] = (eob + n + 7) / 8;     // deflate bytes
    }
    if (s >= D.nseg) return;
    const int nt = D.ntok[s];
    uint32_t pos = hb + D.seg_bits[s];
    uint64_t acc = 0;
    int nacc = (int)(pos & 31);
    uint32_t wpos = pos >> 5;
    bool first = true;
    auto put = [&](uint32_t v, int n) {        // LSB-first into a 64-bit accumulator
        acc |= (uint64_t)(v & ((1u << n) - 1)) << nacc;
        nacc += n;
        if (nacc >= 32) {
            if (first) atomicOr(&D.words[wpos], (uint32_t)acc);
            else D.words[wpos] = (uint32_t)acc;
            first = false;
            ++wpos;
            acc >>= 32;
            nacc -= 32;
        }
    };
    for (int i = 0; i < nt; ++i) put_token(D.tokens[tok_at(s, i)], lcode, llen, dcode, dlen, put);
    if (nacc > 0) atomicOr(&D.words[wpos], (uint32_t)acc);
}

// Stored or dynamic: the zlib stream length of each, the shorter wins (noise: stored).
__global__ void k_png_select(DflArgs D) {
    const int64_t zdyn = 2 + (int64_t)D.tot[1] + 4;
    const bool stored = zdyn >= D.P.zlen;
    const int64_t zlen = stored ? D.P.zlen : zdyn;
    D.P.meta[0] = zlen;
    D.P.meta[1] = stored ? 1 : 0;
    D.P.meta[2] = 8 + zlen + 4;
}

// Deflate bytes -> IDAT chunk: [len][IDAT][78 01][deflate ...][adler][crc] (dynamic stream only).
__global__ void __launch_bounds__(256) k_png_zcopy(DflArgs D) {
    if (D.P.meta[1]) return;
    const int64_t nbytes = D.tot[1];
    uint8_t* z = D.P.chunk + 8;
    const uint8_t* src = reinterpret_cast<const uint8_t*>(D.words);
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nbytes + 2; i += (int64_t)gridDim.x * 256)
        z[i] = i == 0 ? 0x78 : i == 1 ? 0x01 : src[i - 2];
}

// The IDAT chunk length, and with `copy` the chunk, land in the context's fine-grained pinned
// buffer: [len u64][pad 8][chunk].
constexpr int64_t kPngLandBytes = 256 * 1024;
__global__ void __launch_bounds__(256) k_png_chunk_to_host(PngArgs A, uint8_t* __restrict__ host, int copy) {
    const int64_t len = A.meta[2];
    const int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 16;
    if (i == 0) *reinterpret_cast<int64_t*>(host) = len;
    if (!copy || i >= len) return;
    uint8_t* dst = host + 16;
    if (i + 16 <= len) {
        *reinterpret_cast<uint4*>(dst + i) = *reinterpret_cast<const uint4*>(A.chunk + i);
    } else {
        for (int64_t j = i; j < len; ++j) dst[j] = A.chunk[j];
    }
}

static void put32(std::vector<uint8_t>& v, uint32_t x) {
    v.push_back(x >> 24); v.push_back(x >> 16); v.push_back(x >> 8); v.push_back(x);
}

static void put_chunk(std::vector<uint8_t>& v, const char* type, const uint8_t* data, uint32_t n) {
    put32(v, n);
    const size_t start = v.size();
    v.insert(v.end(), type, type + 4);
    v.insert(v.end(), data, data + n);
    put32(v, host_crc(v.data() + start, 4 + n));
}

struct PngPlan {
    int64_t rowlen, raw, nblk, zlen, chunk_bytes;
};

static PngPlan png_plan(int kind, int W, int H) {
    PngPlan p;
    const int64_t rowbytes = kind == kRgb ? 3ll * W : kind == kIdx8 ? W : (W + 7) / 8;
    p.rowlen = 1 + rowbytes;
    p.raw = p.rowlen * H;
    p.nblk = (p.raw + kStored - 1) / kStored;
    if (p.nblk == 0) p.nblk = 1;
    p.zlen = 2 + 5 * p.nblk + p.raw + 4;
    p.chunk_bytes = 8 + p.zlen + 4;
    return p;
}

// Scratch layout of one PNG encode (ws + off): deflate working buffers after the chunk.
struct PngLayout {
    size_t sums, crc, meta, chunk, flt, tokens, ntok, lhist, dhist, tab, segb, tot, words, rows, scan,
        total;
    int64_t nseg, out_words;
};

static PngLayout png_layout(int kind, int W, int H) {
    const PngPlan P = png_plan(kind, W, H);
    PngLayout L{};
    L.nseg = (P.raw + kSeg - 1) / kSeg;
    L.out_words = (P.raw * 15 + 7) / 32 + 256;          // every byte a 15-bit literal + header
    size_t o = 0;
    auto take = [&](size_t b) { const size_t r = o; o = align_up(o + b, 256); return r; };
    L.sums = take(16);
    L.crc = take(4);
    L.meta = take(32);
    L.chunk = take((size_t)P.chunk_bytes);
    L.flt = take((size_t)P.raw);
    L.tokens = take((size_t)tok_slots(L.nseg) * 4);
    L.ntok = take((size_t)L.nseg * 2);
    L.lhist = take((286 + 30) * 4);                 // lhist then dhist, contiguous
    L.dhist = L.lhist + 286 * 4;
    L.tab = take(sizeof(DflTables));
    L.segb = take((size_t)L.nseg * 4);
    L.tot = take(8);
    L.words = take((size_t)L.out_words * 4);
    L.rows = take((size_t)H * 16);
    L.scan = take(scan_scratch_bytes(L.nseg));
    L.total = o;
    return L;
}

// Encode on the device; scratch at ws + off.  Host-side prefix (signature, IHDR, PLTE/tRNS)
// and IEND are assembled here; the IDAT chunk comes back from the device.
static omr_status encode_png_ws(Ctx* ctx, int kind, const uint32_t* d_argb, const uint8_t* d_bits, int W,
                                int H, int fh, int fv, const uint8_t* rgba, size_t off, uint8_t* out,
                                size_t cap, size_t* out_len) {
    const PngPlan P = png_plan(kind, W, H);
    const PngLayout L = png_layout(kind, W, H);
    uint8_t* ws = static_cast<uint8_t*>(ctx->ws) + off;
    std::vector<uint8_t> pre;
    const uint8_t sig[8] = {0x89, 'P', 'N', 'G', 0x0D, 0x0A, 0x1A, 0x0A};
    pre.insert(pre.end(), sig, sig + 8);
    uint8_t ihdr[13];
    ihdr[0] = W >> 24; ihdr[1] = W >> 16; ihdr[2] = W >> 8; ihdr[3] = W;
    ihdr[4] = H >> 24; ihdr[5] = H >> 16; ihdr[6] = H >> 8; ihdr[7] = H;
    ihdr[8] = kind == kIdx1 ? 1 : 8;
    ihdr[9] = kind == kRgb ? 2 : 3;   // truecolour / indexed
    ihdr[10] = ihdr[11] = ihdr[12] = 0;
    put_chunk(pre, "IHDR", ihdr, 13);
    if (kind != kRgb) {
        const uint8_t plte[6] = {0, 0, 0, rgba[0], rgba[1], rgba[2]};
        put_chunk(pre, "PLTE", plte, 6);
        const uint8_t trns[2] = {0, rgba[3]};
        put_chunk(pre, "tRNS", trns, 2);
    }
    static const uint8_t iend[12] = {0, 0, 0, 0, 'I', 'E', 'N', 'D', 0xAE, 0x42, 0x60, 0x82};
    PngArgs A;
    A.argb = d_argb;
    A.bits = d_bits;
    A.chunk = ws + L.chunk;
    A.sums = reinterpret_cast<unsigned long long*>(ws + L.sums);
    A.crc_out = reinterpret_cast<uint32_t*>(ws + L.crc);
    A.kind = kind;
    A.W = W;
    A.H = H;
    A.flip_h = fh;
    A.flip_v = fv;
    A.rowlen = P.rowlen;
    A.raw = P.raw;
    A.nblk = P.nblk;
    A.zlen = P.zlen;
    DflArgs D;
    D.P = A;
    D.flt = ws + L.flt;
    D.tokens = reinterpret_cast<uint32_t*>(ws + L.tokens);
    D.ntok = reinterpret_cast<uint16_t*>(ws + L.ntok);
    D.lhist = reinterpret_cast<uint32_t*>(ws + L.lhist);
    D.dhist = reinterpret_cast<uint32_t*>(ws + L.dhist);
    D.tab = reinterpret_cast<const DflTables*>(ws + L.tab);
    D.seg_bits = reinterpret_cast<uint32_t*>(ws + L.segb);
    D.tot = reinterpret_cast<uint32_t*>(ws + L.tot);
    D.words = reinterpret_cast<uint32_t*>(ws + L.words);
    D.row_sums = reinterpret_cast<unsigned long long*>(ws + L.rows);
    D.nseg = L.nseg;
    D.out_words = L.out_words;
    D.bpp = kind == kRgb ? 3 : 1;
    A.meta = reinterpret_cast<int64_t*>(ws + L.meta);
    D.P = A;
    OMR_HIP(ctx, hipMemsetAsync(ws + L.sums, 0, 256, ctx->stream));
    OMR_HIP(ctx, hipMemsetAsync(ws + L.crc, 0, 4, ctx->stream));
    OMR_HIP(ctx, hipMemsetAsync(ws + L.lhist, 0, L.dhist + 30 * 4 - L.lhist, ctx->stream));
    const unsigned gseg = (unsigned)((L.nseg + 255) / 256);
    const size_t rows_lds = align_up((size_t)png_filter_lds(P.rowlen - 1) + 16, 16);   // + the last stash read
    if (rows_lds > (size_t)kPngFilterLdsMax + 64) return fail(ctx, OMR_INVALID_ARGUMENT, "PNG row too wide");
    if (P.chunk_bytes >= ((int64_t)1 << 31)) return fail(ctx, OMR_INVALID_ARGUMENT, "PNG image too large");
    if (rows_lds > (size_t)60 * 1024)
        OMR_HIP(ctx, hipFuncSetAttribute(reinterpret_cast<const void*>(k_png_filter),
                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)rows_lds + 1024));
    hipLaunchKernelGGL(k_png_filter, dim3((unsigned)((H + kPngRowsPerWg - 1) / kPngRowsPerWg)), dim3(256), rows_lds,
                       ctx->stream, D);
    const int32_t back = (int32_t)align_up((size_t)std::min<int64_t>(std::max<int64_t>(P.rowlen, 2 * D.bpp), kMaxBack), 16);
    hipLaunchKernelGGL(k_png_lz_parse, dim3((unsigned)((L.nseg + kParseLanes - 1) / kParseLanes)), dim3(kParseLanes),
                       (size_t)back + (size_t)kParseLanes * kSeg, ctx->stream, D, back);
    if (ctx->png_device_d3) {
        // D3 on the device: the code from the two histograms, no host round trip
        hipLaunchKernelGGL(k_png_tables, dim3(1), dim3(kHuffThreads), 0, ctx->stream, D.lhist,
                           reinterpret_cast<DflTables*>(ws + L.tab));
        OMR_HIP(ctx, hipGetLastError());
    } else {
        // D3 on the host: the two histograms to the host, the code back (pinned ring)
        uint32_t hist[286 + 30];
        OMR_HIP(ctx, hipMemcpyAsync(hist, ws + L.lhist, sizeof(hist), hipMemcpyDeviceToHost, ctx->stream));
        OMR_HIP(ctx, hipStreamSynchronize(ctx->stream));
        DflTables T;
        build_dynamic_block(hist, hist + 286, T);
        omr_status sst = stage_h2d(ctx, ws + L.tab, &T, sizeof(T));
        if (sst) return sst;
    }
    hipLaunchKernelGGL(k_png_lz_bits, dim3(gseg), dim3(256), 0, ctx->stream, D);
    OMR_HIP(ctx, hipGetLastError());
    omr_status st = device_exclusive_scan(ctx, D.seg_bits, D.seg_bits, L.nseg, D.tot,
                                          reinterpret_cast<uint32_t*>(ws + L.scan));
    if (st) return st;
    hipLaunchKernelGGL(k_png_zero_words, dim3((unsigned)std::min<int64_t>((L.out_words + 255) / 256, 4096)), dim3(256),
                       0, ctx->stream, D);
    hipLaunchKernelGGL(k_png_lz_write, dim3(gseg), dim3(256), 0, ctx->stream, D);
    // stored vs dynamic decided on the device; both paths are queued, the unchosen one exits
    hipLaunchKernelGGL(k_png_select, dim3(1), dim3(1), 0, ctx->stream, D);
    const unsigned gl = (unsigned)std::min<int64_t>((P.zlen + 255) / 256, (int64_t)ctx->cu_count * 8);
    hipLaunchKernelGGL(k_png_layout, dim3(gl), dim3(256), 0, ctx->stream, A, D.flt);
    hipLaunchKernelGGL(k_png_zcopy, dim3(gl), dim3(256), 0, ctx->stream, D);
    hipLaunchKernelGGL(k_png_adler_rows, dim3(1), dim3(256), 0, ctx->stream, D);
    hipLaunchKernelGGL(k_png_adler, dim3(1), dim3(1), 0, ctx->stream, A);
    const int64_t segs = (4 + P.zlen + kCrcSeg - 1) / kCrcSeg;   // stored length: the longest
    hipLaunchKernelGGL(k_png_crc, dim3((unsigned)((segs + 255) / 256)), dim3(256), 0, ctx->stream, A);
    hipLaunchKernelGGL(k_png_finish, dim3(1), dim3(1), 0, ctx->stream, A);
    OMR_HIP(ctx, hipGetLastError());
    // Small chunks (masks) land with their length in pinned host memory: one stream sync.  Big
    // ones (rendered RGB tiles): the length lands first, then one DMA copy of exactly the chunk
    // (a kernel writing MBs over PCIe into host memory plus a host memcpy was slower).
    const bool land = P.chunk_bytes <= kPngLandBytes;
    st = ensure_host_out(ctx, land ? (size_t)P.chunk_bytes + 16 : 16);
    if (st) return st;
    const int64_t land_bytes = land ? P.chunk_bytes : 0;
    hipLaunchKernelGGL(k_png_chunk_to_host, dim3((unsigned)((land_bytes + 16 * 256 - 1) / (16 * 256) + 1)), dim3(256),
                       0, ctx->stream, A, ctx->h_out, land ? 1 : 0);
    OMR_HIP(ctx, hipGetLastError());
    OMR_HIP(ctx, hipStreamSynchronize(ctx->stream));
    const int64_t chunk_bytes = *reinterpret_cast<volatile int64_t*>(ctx->h_out);
    const size_t total = pre.size() + (size_t)chunk_bytes + sizeof(iend);
    if (out_len) *out_len = total;
    if (!out || cap < total) return fail(ctx, OMR_BUFFER_TOO_SMALL, "PNG output buffer too small");
    std::memcpy(out, pre.data(), pre.size());
    if (land) {
        std::memcpy(out + pre.size(), ctx->h_out + 16, (size_t)chunk_bytes);
    } else {
        OMR_HIP(ctx, hipMemcpyAsync(out + pre.size(), A.chunk, (size_t)chunk_bytes, hipMemcpyDeviceToHost, ctx->stream));
        OMR_HIP(ctx, hipStreamSynchronize(ctx->stream));
    }
    std::memcpy(out + pre.size() + chunk_bytes, iend, sizeof(iend));
    return OMR_OK;
}

static size_t png_scratch(int kind, int W, int H) { return png_layout(kind, W, H).total; }

// =====================================================================================
// Batched PNG (rounds 4-5): N images — rendered RGB tiles of one size, or shape masks of any size —
// through one launch per stage, every grid spanning all images, and the N files packed in device
// memory with per-image status (the batch form of the per-request ImageIO.write calls,
// ImageRegionRequestHandler.java:597-599, and of every mask, ShapeMaskRequestHandler.java:185-203):
//   P1 k_pngb_filter   one wave per band of image rows (wave form, RGB tiles), else one
//                      workgroup per 4 rows (D1)
//   P2 k_pngb_parse    one lane per 32-byte segment, 128 per workgroup (D2): candidate masks in
//                      registers from global loads, greedy parse over the match starts, a 12-byte
//                      parse trace per segment (no token buffer), per-block symbol counts and
//                      the per-image histograms
//   P3 k_pngb_tables   one workgroup per image: length-limited Huffman code + block header (D3
//                      on the device: no host round trip; N workgroups run side by side)
//   P3b k_pngb_block_offsets  one workgroup per image: every parse block's code bits from its
//                      symbol counts x the code lengths, scanned into bit offsets
//   P4 k_pngb_encode   one workgroup per 256 segments: the tokens again from the traces and the
//                      stream bytes, each lane's codes into its LDS column, an in-group scan,
//                      the columns shifted into the group's words, whole words stored, the
//                      group's two partial words kept aside
//   P5 k_pngb_fixup    one lane per group: the words groups share, ORed from the kept parts
//   P5b k_pngb_meta    one workgroup per image: stream length, stored vs dynamic, Adler-32 from
//                      the row partials
//   P6 k_pngb_offsets  one workgroup: files' offsets in the output (16-byte aligned), status
//   P8 k_pngb_emit     16 output bytes per lane: prefix chunks, IDAT header, zlib stream (deflate
//                      words funnel-shifted, or stored blocks of the filtered stream), Adler,
//                      IEND — aligned 16-byte stores
//   P8+P9 k_pngb_emit_crc  (round 6, the default) P8 with each wave's 4 KiB strip CRCed from the
//                      registers it stores (16-byte braid over the lanes); P9b k_pngb_crc_combine
//                      moves every strip's CRC to the range end by x^(8n) powers and XORs them
//   P9 k_pngb_crc      (OMR_PNG_CRC_P9=1: after the plain P8) braided CRC-32 re-reading the file:
//                      one wave per 16 KiB strip, coalesced dword loads, strips combined by powers
//   P10 k_pngb_finish  one lane per image: the CRC bytes
// =====================================================================================
constexpr int kPngbGroup = 256;                 // segments per P4/P7 group
constexpr int kPngbEmitBytes = 16 * 256;        // output bytes per P8 workgroup (separate P9)
// P8 with the IDAT CRC fused (round 6, the default): each wave emits one strip of the file and
// CRCs the IDAT-range bytes of it from the registers it stored (k_pngb_emit_crc), P9b combines the
// strips' CRCs (k_pngb_crc_combine), so the file is not read back from HBM by a separate CRC pass.
// 4 KiB strips (round 6 A/B, profiles/r06/ab_png_crc_strip.txt): at 256 C2 tiles per call 4, 8 and
// 16 KiB run alike (P8+P9b 0.343-0.348 ms); on the smaller batches of the probe's other cases 4 KiB
// is 6 % faster (more waves, shorter CRC chains per lane).
#ifndef OMR_PNG_CRC_STRIP_KIB
#define OMR_PNG_CRC_STRIP_KIB 4
#endif
constexpr int kPngbEmitCrcStrip = OMR_PNG_CRC_STRIP_KIB * 1024;   // bytes a wave emits and CRCs (steps of 1 KiB)
constexpr int kPngbEmitCrcBytes = 4 * kPngbEmitCrcStrip;   // file bytes per workgroup (4 waves)
// Direct mode (round 6, the default; env OMR_PNG_DIRECT=0 for the forms below): P5b / P6 run before
// P4, which codes into the files in place; P8 then stores only the bytes around the streams and
// P9 CRCs the files (k_pngb_crc).
static bool png_direct() {
    static const bool v = [] { const char* e = std::getenv("OMR_PNG_DIRECT"); return !(e && std::atoi(e) == 0); }();
    return v;
}
// env OMR_PNG_CRC_P9=1 (with OMR_PNG_DIRECT=0): the round-5 form (P8 4 KiB per workgroup, then
// the separate P9 pass); otherwise P8 with the CRC fused (k_pngb_emit_crc)
static bool png_crc_separate() {
    static const bool v = [] { const char* e = std::getenv("OMR_PNG_CRC_P9"); return e && std::atoi(e) != 0; }();
    return v;
}
constexpr int kPngbCrcBytes = 256 * 256;        // CRC range bytes per P9 workgroup
constexpr int kPngbMaxSide = 4096;
constexpr int kCrcPowLo = 4096, kCrcPowHi = 2048;

struct PngImg {
    const uint32_t* argb;      // kRgb: pixels, row stride W
    const uint8_t* bits;       // kIdx1 / kIdx8: MSB-first mask bits
    int32_t kind, W, H, flip_h, flip_v, bpp;
    int32_t row0, pblk0, grp0, pre_len;         // first global row / parse block / group; prefix bytes
    int32_t rblk0, pad2;                        // first D1 workgroup (kPngRowsPerWg rows each)
    int32_t back, pad;                          // parse look-back (bytes, multiple of 16)
    int64_t rowlen, raw, nseg, nblk;            // row bytes + 1, filtered stream bytes, segments, stored blocks
    int64_t flt, seg0, words;                   // filtered stream offset (bytes), first segment, first word
    int64_t tok0;                               // first token slot (tok_at layout)
    int64_t eblk0, cblk0;                       // first P8 / P9 workgroup
    uint8_t pre[72];                            // signature, IHDR (+ PLTE, tRNS)
};

struct PngMeta {
    int64_t zlen, file_len, off;               // zlib stream bytes; file bytes; offset in the output (-1: none)
    uint32_t adler, crc, hbits, tot_bits;       // Adler-32, CRC-32 (XOR-accumulated), header bits, codes' bits
    int32_t stored, status, pad0, pad1;
};

struct PngBatch {
    const PngImg* img;
    int32_t n, uniform;                         // uniform: every image has the same geometry
    int32_t rblk_per, pblk_per, grp_per, eblk_per, cblk_per;   // per-image counts when uniform
    int32_t total_grp, fw_bands;                // fw_bands: row bands per image of the wave-form D1
    const int32_t* rblk0;                       // [n] first D1 workgroup etc. (binary search when not uniform)
    const int32_t* pblk0;
    const int32_t* grp0;
    const int32_t* eblk0;
    const int32_t* cblk0;
    uint8_t* flt;
    uint16_t* bh;                               // [parse blocks][316] symbol counts of each parse block
    uint32_t* poff;                             // [parse blocks] bit offset of each parse block's codes
    uint32_t* img_bits;                         // [n] stream bits: header + codes + EOB
    uint32_t* blk_b0;                           // [groups] first bit of the P4 group (kPngbGroup segments) in its stream
    uint32_t* blk_b1;                           // [groups] one past its last bit
    uint32_t* blk_cf;                           // [groups] its first (partial) word
    uint32_t* blk_cl;                           // [groups] its last (partial) word
    int32_t total_pblk, pad3;
    int64_t total_segs;
    uint32_t* trace;                            // [3][segments] parse traces (S, M, D)
    uint32_t* hist;                             // [n][316]
    DflTables* tab;                             // [n]
    PngMeta* meta;                              // [n]
    unsigned long long* row_sums;               // [rows][2]
    uint32_t* words;                            // deflate streams
    uint8_t* out;
    uint64_t out_cap;
    uint64_t* d_offsets;
    uint32_t* d_lengths;
    int32_t* d_status;
    const uint32_t* crc_pow;                    // [kCrcPowAll] (k_png_crc_pow)
    uint32_t* strip_crc;                        // [P8 workgroups][4] raw CRC of each P8+P9 strip at its end
    int32_t direct, pad4;                       // P4 codes straight into the files (png_direct())
};

// Image owning global item `x` of a stage whose per-image first items are `first` (sorted).
__device__ __forceinline__ int pngb_image(const PngBatch& B, const int32_t* first, int32_t per, int64_t x) {
    if (B.uniform) return (int)(x / per);
    int lo = 0, hi = B.n - 1;
    while (lo < hi) {                           // last image whose first item <= x
        const int mid = (lo + hi + 1) >> 1;
        if (first[mid] <= x) lo = mid; else hi = mid - 1;
    }
    return lo;
}

// Where P4 / P5 put image I's deflate words, and the bit offset of the stream in them: the words
// buffer (bit 0), or -- direct mode (round 6) -- the file itself: the stream starts at file byte
// pre_len + 10 (after the IDAT length and type and the zlib header), so the words are the file's
// aligned dwords from a = (pre_len + 10) mod 4 bytes before it, and bit 8a is the stream's bit 0.
// The file offsets (P5b, P6) are known before P4: they follow from P3b's stream lengths.
__device__ __forceinline__ uint32_t* pngb_stream_words(const PngBatch& B, const PngImg& I, const PngMeta& M,
                                                       uint32_t& bo) {
    if (!B.direct) {
        bo = 0;
        return B.words + I.words;
    }
    const int a = (I.pre_len + 10) & 3;
    bo = 8u * (uint32_t)a;
    return reinterpret_cast<uint32_t*>(B.out + M.off + I.pre_len + 10 - a);
}

__device__ __forceinline__ PngArgs pngb_args(const PngImg& I) {
    PngArgs A{};
    A.argb = I.argb;
    A.bits = I.bits;
    A.kind = I.kind;
    A.W = I.W;
    A.H = I.H;
    A.flip_h = I.flip_h;
    A.flip_v = I.flip_v;
    A.rowlen = I.rowlen;
    A.raw = I.raw;
    A.nblk = I.nblk;
    return A;
}

// x^-1 mod P (zlib's reflected form: bit 31 is x^0): with P = x Q + 1, x Q = P + 1 = 1 mod P, so
// x^-1 = Q = x^31 + x^25 + x^22 + x^21 + x^15 + x^11 + x^10 + x^9 + x^7 + x^6 + x^4 + x^3 + x + 1
constexpr uint32_t kCrcXInv = (1u << 0) | (1u << 6) | (1u << 9) | (1u << 10) | (1u << 16) | (1u << 20) |
                              (1u << 21) | (1u << 22) | (1u << 24) | (1u << 25) | (1u << 27) | (1u << 28) |
                              (1u << 30) | (1u << 31);
static_assert(multmodp_c(1u << 30, kCrcXInv) == 1u << 31, "x * x^-1 == 1 mod P");
constexpr int kCrcPowR = kCrcPowLo + kCrcPowHi;   // x^(8 r), r < 256
constexpr int kCrcInvR = kCrcPowR + 256;          // x^(-8 r), r < 256
constexpr int kCrcInvA = kCrcInvR + 256;          // x^(-8 256 a), a < 64
constexpr int kCrcPowAll = kCrcInvA + 64;

// x^(8*256*j) mod P: [0, 4096) for j, [4096, 6144) for j * 4096; then x^(8 r) and x^(-8 r) for
// r < 256 and x^(-8*256*a) for a < 64 (one lane per entry).
__global__ void __launch_bounds__(256) k_png_crc_pow(uint32_t* __restrict__ pw) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= kCrcPowAll) return;
    if (i < kCrcPowR) {
        const uint64_t j = i < kCrcPowLo ? (uint64_t)i : (uint64_t)(i - kCrcPowLo) * kCrcPowLo;
        pw[i] = x2nmodp(j * 256, 3);
        return;
    }
    const bool inv = i >= kCrcInvR;
    const uint64_t e = i < kCrcInvR ? (uint64_t)(i - kCrcPowR) : i < kCrcInvA ? (uint64_t)(i - kCrcInvR)
                                                                             : (uint64_t)(i - kCrcInvA) * 256;
    if (!inv) { pw[i] = x2nmodp(e, 3); return; }
    uint32_t xi8 = kCrcXInv;                      // x^-8 = (x^-1)^8
    for (int k = 0; k < 3; ++k) xi8 = multmodp(xi8, xi8);
    uint32_t p = 1u << 31, b = xi8;
    for (uint64_t n = e; n; n >>= 1) {            // (x^-8)^e by squaring
        if (n & 1) p = multmodp(b, p);
        b = multmodp(b, b);
    }
    pw[i] = p;
}

__global__ void __launch_bounds__(256) k_pngb_filter(PngBatch B) {
    extern __shared__ __attribute__((aligned(16))) uint8_t s_rows[];
    const int i = pngb_image(B, B.rblk0, B.rblk_per, blockIdx.x);
    const PngImg& I = B.img[i];
    const int y0 = ((int)blockIdx.x - (B.uniform ? i * B.rblk_per : I.rblk0)) * kPngRowsPerWg;
    png_filter_rows(pngb_args(I), I.bpp, y0, min(kPngRowsPerWg, I.H - y0), B.flt + I.flt,
                    B.row_sums + 2 * ((int64_t)I.row0 + y0), s_rows);
}

// XCD-aware order of a grid's blocks (round 6): workgroup g runs on XCD g mod 8, so handing XCD x
// the x-th contiguous eighth of the blocks puts a block and the one before it -- whose bytes its
// look-back windows re-read -- on the same XCD, in the same L2.
#ifndef OMR_PNG_XCD_ORDER
#define OMR_PNG_XCD_ORDER 1
#endif
__device__ __forceinline__ int64_t xcd_block(int64_t g, int64_t total) {
    if (!OMR_PNG_XCD_ORDER) return g;
    constexpr int64_t X = 8;
    const int64_t q = total / X, r = total % X, x = g % X, k = g / X;
    return x < r ? x * (q + 1) + k : r * (q + 1) + (x - r) * q + k;
}

// D1, wave form (round 5): for a uniform batch of RGB images with W % 4 == 0 and W <= 1024 (the
// rendered tiles), one wave filters a band of kFilterBandRows rows.  Lane l holds pixel quads
// q = l + 64 m (4 px = 3 dwords of RGB, one coalesced 16-byte load), the row above stays in
// registers from the previous row, the left neighbours come from lane l - 1 (or lane 63 of quad
// block m - 1) by a lane shift, the five residual sums reduce inside the wave -- no LDS, no
// workgroup barrier.  The chosen row leaves as aligned dwords (alignbyte of two neighbouring
// residual dwords; the filter byte and the partial dwords shared with the neighbouring rows byte
// by byte) and the band's Adler partials go to its first row's slot (the others 0: P5 sums every
// row).  Same filter choice (minimum sum of |residual|, lowest filter on ties) and bytes as
// png_filter_rows.
constexpr int kFilterBandRows = 8;

// Residual f (wave-uniform) of 4 row bytes: png_residuals' entry f alone.
__device__ __forceinline__ uint32_t png_residual(int f, uint32_t X, uint32_t A, uint32_t B, uint32_t C) {
    switch (f) {
    case 0: return X;
    case 1: return sub8(X, A);
    case 2: return sub8(X, B);
    case 3: return sub8(X, (A & B) + (((A ^ B) & 0xFEFEFEFEu) >> 1));
    default: return sub8(X, paeth4(A, B, C));
    }
}

// v_writelane_b32: the uniform value v into lane `lane` of old (LLVM's intrinsic).
__device__ int png_lane_write(int v, int lane, int old) __asm("llvm.amdgcn.writelane.i32");

// Dword j + 1 of a row held as w[t] = dword lane + 64 t: lane l + 1's w (DPP wave_shl:1), lane 63
// lane 0's of the next step (`nxt`, read out to a scalar and written into lane 63).
__device__ __forceinline__ uint32_t next_lane_dword(uint32_t w, uint32_t nxt) {
    const int dn = __builtin_amdgcn_mov_dpp((int)w, 0x130, 0xF, 0xF, true);
    return (uint32_t)png_lane_write(__builtin_amdgcn_readlane((int)nxt, 0), 63, dn);
}

// Sum over the wave's 64 lanes, returned in a scalar register (every lane active): sums of 16 by
// four DPP adds (quad swaps, half-row and row mirrors), then the four rows' lanes read out.
__device__ __forceinline__ uint32_t wave_sum_dpp(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);    // quad_perm [1,0,3,2]
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);    // quad_perm [2,3,0,1]
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, false);   // row_half_mirror
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x140, 0xF, 0xF, false);   // row_mirror
    return (uint32_t)(__builtin_amdgcn_readlane((int)v, 0) + __builtin_amdgcn_readlane((int)v, 16) +
                      __builtin_amdgcn_readlane((int)v, 32) + __builtin_amdgcn_readlane((int)v, 48));
}

template <int V> struct FltIdx { static constexpr int value = V; };

__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// LDS per wave: two rows (this one and the one above) of 3 * 64 * M dwords behind a zero dword
// (the left neighbour of the row's first dword).
template <int M> __host__ __device__ constexpr int fw_row_dwords() { return 3 * 64 * M + 1; }
template <int M> __host__ __device__ constexpr size_t fw_lds_bytes() { return (size_t)4 * 2 * fw_row_dwords<M>() * 4; }

#ifndef OMR_PNG_FW_WAVES
#define OMR_PNG_FW_WAVES 5
#endif
// FULL: W == 256 * M (the 1024-wide tiles at M = 4), so every lane's quads and dwords lie inside
// the row: no per-dword guards, and the compiler keeps the sums in v_sad_u8's accumulator and
// batches the LDS reads across dwords.
template <int M, bool FULL>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(OMR_PNG_FW_WAVES))) k_pngb_filter_wave(PngBatch B) {
    extern __shared__ __attribute__((aligned(16))) uint32_t s_fw[];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t wid = xcd_block(blockIdx.x, gridDim.x) * 4 + wv;   // (XCD order: the band above on the same L2)
    const int i = (int)(wid / B.fw_bands);
    if (i >= B.n) return;
    const PngImg& I = B.img[i];
    const int y0 = (int)(wid - (int64_t)i * B.fw_bands) * kFilterBandRows;
    const int y1 = min(I.H, y0 + kFilterBandRows);
    const int W = I.W, nq = W >> 2, nd = 3 * nq, rb = 3 * W;
    const uint32_t* __restrict__ argb = I.argb;
    uint8_t* __restrict__ flt = B.flt + I.flt;
    const int64_t rowlen = I.rowlen, raw = I.raw;
    constexpr int S = fw_row_dwords<M>();
    uint32_t* bufA = s_fw + wv * 2 * S;
    uint32_t* bufB = bufA + S;
    if (lane == 0) { bufA[0] = 0u; bufB[0] = 0u; }
    auto load_raw = [&](int y, uint4 (&v)[M]) {
#pragma unroll
        for (int m = 0; m < M; ++m) {
            const int q = lane + 64 * m;
            v[m] = make_uint4(0, 0, 0, 0);
            if (y >= 0 && (FULL || q < nq)) v[m] = reinterpret_cast<const uint4*>(argb + (int64_t)y * W)[q];
        }
    };
    auto put_row = [&](const uint4 (&v)[M], uint32_t* row) {   // RGB dwords of the row at row[1 + j]
#pragma unroll
        for (int m = 0; m < M; ++m) {
            const int q = lane + 64 * m;
            if (FULL || q < nq) {
                row[1 + 3 * q] = __builtin_amdgcn_perm(v[m].y, v[m].x, 0x06000102u);       // r0 g0 b0 r1
                row[2 + 3 * q] = __builtin_amdgcn_perm(v[m].z, v[m].y, 0x05060001u);       // g1 b1 r2 g2
                row[3 + 3 * q] = __builtin_amdgcn_perm(v[m].w, v[m].z, 0x04050600u);       // b2 r3 g3 b3
            }
        }
    };
    uint4 nxt[M];
    load_raw(y0 - 1, nxt);
    uint32_t* prev = bufA;
    uint32_t* cur = bufB;
    put_row(nxt, prev);
    load_raw(y0, nxt);
    unsigned long long s1 = 0, s2 = 0;
    for (int y = y0; y < y1; ++y) {
        put_row(nxt, cur);
        if (y + 1 < y1) load_raw(y + 1, nxt);                 // the next row's loads fly meanwhile
        wave_lds_sync();
        // pass 1: the five |residual| sums; lane l takes row dwords j = l + 64 t (conflict-free LDS)
        uint32_t sm[5] = {0, 0, 0, 0, 0};
#pragma unroll
        for (int t = 0; t < 3 * M; ++t) {
            const int j = lane + 64 * t;
            if (FULL || j < nd) {
                const uint32_t X = cur[1 + j], Bv = prev[1 + j];
                const uint32_t Av = __builtin_amdgcn_alignbyte(X, cur[j], 1);
                const uint32_t Cv = __builtin_amdgcn_alignbyte(Bv, prev[j], 1);
                uint32_t r[5];
                png_residuals(X, Av, Bv, Cv, r);
#pragma unroll
                for (int f = 0; f < 5; ++f) sm[f] = abs_sum8(r[f], sm[f]);
            }
            if (FULL) __builtin_amdgcn_sched_barrier(0);      // one dword's reads at a time (VGPRs)
        }
        int f = 0;                                             // scalar: sums by DPP, read out
        uint32_t best = 0xFFFFFFFFu;
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            const uint32_t v = wave_sum_dpp(sm[k]);
            if (v < best) { best = v; f = k; }                 // lowest filter on ties
        }
        // pass 2: the chosen residual row (one straight-line copy per filter, picked once per row)
        uint32_t c[3 * M];
        auto pass2 = [&](auto F) {
#pragma unroll
            for (int t = 0; t < 3 * M; ++t) {
                const int j = lane + 64 * t;
                c[t] = 0u;
                if (FULL || j < nd) {
                    const uint32_t X = cur[1 + j], Bv = prev[1 + j];
                    const uint32_t Av = __builtin_amdgcn_alignbyte(X, cur[j], 1);
                    const uint32_t Cv = __builtin_amdgcn_alignbyte(Bv, prev[j], 1);
                    c[t] = png_residual(decltype(F)::value, X, Av, Bv, Cv);
                }
            }
        };
        switch (f) {
        case 0: pass2(FltIdx<0>{}); break;
        case 1: pass2(FltIdx<1>{}); break;
        case 2: pass2(FltIdx<2>{}); break;
        case 3: pass2(FltIdx<3>{}); break;
        default: pass2(FltIdx<4>{}); break;
        }
        const int64_t ypos = (int64_t)y * rowlen;              // the row's offset in the stream
        const int64_t row0 = I.flt + ypos;                     // ... and in B.flt (16-aligned base)
        const int u = (int)((-row0 - 1) & 3);                  // residual byte u sits at an aligned address
        uint32_t* gw = reinterpret_cast<uint32_t*>(B.flt + row0 + u + 1);   // out dword J
        const int jfull = (rb - u) >> 2;                       // out dwords J < jfull lie inside the row
        const unsigned long long rbase = (unsigned long long)(raw - ypos - 1);
        uint32_t a1 = 0, aj = 0, ad = 0;                      // this row's Adler partials in 32 bits
#pragma unroll
        for (int t = 0; t < 3 * M; ++t) {
            const int j = lane + 64 * t;
            const uint32_t hi = next_lane_dword(c[t], t + 1 < 3 * M ? c[t + 1] : 0u);   // residual dword j + 1
            if (FULL || j < nd) {
                const uint32_t w = c[t];
                if ((FULL && t < 3 * M - 1) || j < jfull) gw[j] = __builtin_amdgcn_alignbyte(hi, w, u);
                const uint32_t sv = __builtin_amdgcn_sad_u8(w, 0u, 0u);
                a1 += sv;
                aj += (uint32_t)j * sv;                        // <= 767 * 12 * 1020 per lane and row
                ad = __builtin_amdgcn_udot4(w, 0x03020100u, ad, false);
                // bytes outside the whole out dwords: the row's first u, its last (rb - u) & 3
                // (FULL: only dword 0 and the row's last dword can hold such bytes)
                if ((!FULL || t == 0 || t == 3 * M - 1) && (4 * j < u || 4 * j + 3 >= u + 4 * jfull)) {
                    for (int b = 0; b < 4; ++b) {
                        const int tt = 4 * j + b;
                        if (tt < u || tt >= u + 4 * jfull) flt[ypos + 1 + tt] = (uint8_t)byte_at(w, b);
                    }
                }
            }
        }
        s1 += a1;                                              // sum (raw - pos) * byte over the row
        s2 += rbase * a1 - 4ull * aj - ad;
        if (lane == 0) {
            flt[ypos] = (uint8_t)f;
            s1 += (unsigned long long)f;
            s2 += (unsigned long long)(raw - ypos) * (unsigned long long)f;
        }
        wave_lds_sync();                                       // every lane is done with `prev`
        uint32_t* tmp = prev;
        prev = cur;
        cur = tmp;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        s1 += __shfl_xor(s1, o, 64);
        s2 += __shfl_xor(s2, o, 64);
    }
    unsigned long long* rs = B.row_sums + 2 * ((int64_t)I.row0 + y0);
    if (lane < 2 * (y1 - y0)) rs[lane] = lane == 0 ? s1 : lane == 1 ? s2 : 0ull;
}

// P2: the parse of one block: the image's symbol histograms (eight LDS copies, lane & 7, two
// 16-bit counts per dword, so the common literals' atomics spread over eight addresses) and each segment's parse trace -- token
// starts S, match starts M, the matches' candidate indices D (2 bits each, <= 10 per segment) --
// so that P4 codes the segment without parsing it again.
// P2 (round 5): no LDS staging.  A lane's 32 stream bytes, the 8 before them and the 36 one row
// up come from global memory (consecutive lanes read consecutive segments: coalesced; the row
// above was read by a block one row back, an L2 hit), and every candidate's "byte == byte d back"
// mask is built in registers.  The greedy parse then visits only match starts (positions where
// some candidate's run reaches 3: there a match always starts); everything between is literals,
// counted by a static walk over the 32 bytes.  Symbol counts go to lane-private u8 counters in
// LDS -- [bin / 4][lane & 31]: a lane's adds hit its own bank, no conflicts; at most 4 lanes x 32
// symbols share a counter, so u8 never wraps.
// P2 match symbols from a per-workgroup (candidate, length) table instead of pack_match's four
// table reads and the per-lane candidate distance select (round 6)
#ifndef OMR_PNG_PARSE_PM
#define OMR_PNG_PARSE_PM 1
#endif
constexpr int kPmLen = 33;
#ifndef OMR_PNG_HIST_B128
#define OMR_PNG_HIST_B128 1
#endif                      // lengths 0..32 (tokens stay inside their segment)
#ifndef OMR_PNG_LIT_FLAT
#define OMR_PNG_LIT_FLAT 1
#endif
constexpr int kHistRows = 316 / 4 + 1;          // dwords of four u8 counters per copy

__device__ __forceinline__ uint32_t eq_mask_q(const uint32_t (&x)[8], const uint32_t (&q)[9], int sh) {
    uint32_t m = 0;
#pragma unroll
    for (int i = 0; i < 8; i += 2) {
        uint32_t acc = 0;
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const uint32_t y = __builtin_amdgcn_alignbyte(q[i + k + 1], q[i + k], sh);
            const uint32_t e = x[i + k] ^ y;                  // zero bytes: equal
            const uint32_t z = ~(((e & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | e | 0x7F7F7F7Fu);   // 0x80 per zero byte
            acc = __builtin_amdgcn_udot4((z >> 7) & 0x01010101u, k ? 0x80402010u : 0x08040201u, acc, false);
        }
        m |= acc << (4 * i);
    }
    return m;
}

// LDS-only workgroup barrier: orders the LDS traffic (the counters) without waiting for the
// wave's outstanding global stores, which __syncthreads' workgroup fence would.
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

__global__ void __launch_bounds__(kParseLanes) k_pngb_parse(PngBatch B) {
    __shared__ __attribute__((aligned(16))) uint32_t lh[kHistRows * 32];                 // u8 counters [bin / 4][copy]
#if OMR_PNG_PARSE_PM
    __shared__ uint32_t pm[4 * kPmLen];     // (candidate, length) -> the match's two symbols
#else
    __shared__ DeflateTabs T;
#endif
    const int64_t gblk = xcd_block(blockIdx.x, B.total_pblk);
    const int i = pngb_image(B, B.pblk0, B.pblk_per, gblk);
    const PngImg& I = B.img[i];
    const int64_t blk = gblk - (B.uniform ? (int64_t)i * B.pblk_per : I.pblk0);
    const int64_t s = blk * kParseLanes + threadIdx.x;
    const bool live = s < I.nseg;
    const uint8_t* f = B.flt + I.flt;                       // 16-byte aligned, >= 64 bytes of slack after
    const int64_t beg = s * kSeg, rowlen = I.rowlen;
    // every global load first (the segment, the 8 bytes before it, 36 bytes one row up), so one
    // memory latency covers them and the table copy below
    uint32_t x[8] = {}, p0 = 0, p1 = 0, up[9] = {};
    const bool row_ok = live && rowlen <= I.back && beg >= rowlen;
    if (live) {
        const uint4* o = reinterpret_cast<const uint4*>(f + beg);
        const uint4 u0 = o[0], u1 = o[1];
        x[0] = u0.x; x[1] = u0.y; x[2] = u0.z; x[3] = u0.w;
        x[4] = u1.x; x[5] = u1.y; x[6] = u1.z; x[7] = u1.w;
        if (beg >= 8) {
            const uint2 u = *reinterpret_cast<const uint2*>(f + beg - 8);
            p0 = u.x;
            p1 = u.y;
        }
        if (row_ok) {
            const uint32_t* ua = reinterpret_cast<const uint32_t*>(f + ((beg - rowlen) & ~(int64_t)3));
#pragma unroll
            for (int j = 0; j < 9; ++j) up[j] = ua[j];
        }
    }
    for (int k = threadIdx.x; k < kHistRows * 32; k += kParseLanes) lh[k] = 0;
#if OMR_PNG_PARSE_PM
    {   // 257 + length symbol | (286 + distance symbol) << 16 of every (candidate, length <= 32)
        const uint32_t dl0[4] = {1u, I.bpp == 1 ? (uint32_t)rowlen : (uint32_t)I.bpp, (uint32_t)(2 * I.bpp),
                                 (uint32_t)rowlen};
        for (int e = threadIdx.x; e < 4 * kPmLen; e += kParseLanes) {
            const int k = e / kPmLen, l = e % kPmLen;
            uint32_t v = 0;
            if (l >= 3) {
                const uint32_t t = pack_match(c_dfl, (uint32_t)l, dl0[k]);
                v = (257u + (t & 31u)) | ((286u + ((t >> 5) & 31u)) << 16);
            }
            pm[e] = v;
        }
    }
#else
    lz_load_tabs(T);
#endif
    uint32_t* const hl = lh + (threadIdx.x & 31);
    auto count = [&](uint32_t t) {                          // one symbol into this lane's counters
        atomicAdd(hl + ((t >> 2) << 5), 1u << ((t << 3) & 31u));
    };
    uint32_t S = 0, M = 0, D = 0;
    __syncthreads();
    if (live) {
        const int n = (int)min((int64_t)kSeg, I.raw - beg);
        const uint32_t nmask = n >= 32 ? 0xFFFFFFFFu : (1u << n) - 1u;
        // candidates in the compare order of the byte-wise parse: 1, bpp, 2 bpp (not for bpp 1,
        // where bpp repeats distance 1), one row up (bpp <= 4: every candidate but the row is
        // within 8 bytes)
        const int nd = I.bpp == 1 ? 2 : 4;
        const uint32_t dl[4] = {1u, I.bpp == 1 ? (uint32_t)rowlen : (uint32_t)I.bpp, (uint32_t)(2 * I.bpp),
                                (uint32_t)rowlen};
        uint32_t m[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            m[k] = 0;
            if (k >= nd) continue;
            const int64_t d = dl[k];
            if (d > I.back) continue;                       // past the single path's look-back
            if (beg >= d) {
                uint32_t q[9];
                const int sh = (int)((-d) & 3);
                if (d <= 4) {                               // one dword back: p1, then the segment
                    q[0] = p1;
#pragma unroll
                    for (int j = 0; j < 8; ++j) q[j + 1] = x[j];
                } else if (d <= 8) {                        // two dwords back
                    q[0] = p0;
                    q[1] = p1;
#pragma unroll
                    for (int j = 0; j < 7; ++j) q[j + 2] = x[j];
                } else {                                    // one row up (d == rowlen)
#pragma unroll
                    for (int j = 0; j < 9; ++j) q[j] = up[j];
                }
                m[k] = eq_mask_q(x, q, sh) & nmask;
            } else if (d - beg < n) {                       // the image's first bytes
                uint32_t mm = 0;
                for (int q = (int)(d - beg); q < n; ++q)
                    if (f[beg + q] == f[beg + q - d]) mm |= 1u << q;
                m[k] = mm;
            }
        }
        uint32_t A = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) A |= m[k] & (m[k] >> 1) & (m[k] >> 2);
        uint32_t cov = 0;                                   // bytes inside matches
        int nm = 0, p = 0;
        while (p < 32) {
            const uint32_t ap = A >> p;
            if (!ap) break;
            p += __builtin_ctz(ap);                         // a match starts here
            int best = 0, bk = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t v = m[k] >> p;
                const int l = v == 0xFFFFFFFFu ? 32 : __builtin_ctz(~v);   // run of equal bytes from p
                if (l > best) { best = l; bk = k; }
            }
            S |= 1u << p;
            M |= 1u << p;
            D |= (uint32_t)bk << (2 * nm++);
            cov |= (best >= 32 ? 0xFFFFFFFFu : ((1u << best) - 1u)) << p;
#if OMR_PNG_PARSE_PM
            const uint32_t sy = pm[bk * kPmLen + best];     // one LDS read: both symbols
            count(sy & 0xFFFFu);
            count(sy >> 16);
#else
            const uint32_t t = pack_match(T, (uint32_t)best, dl[bk]);
            count(257 + (t & 31));
            count(286 + ((t >> 5) & 31));
#endif
            p += best;
        }
        const uint32_t lit = nmask & ~cov;
        S |= lit;
#if OMR_PNG_LIT_FLAT
        // every byte's add issued, a non-literal's with 0: no exec-mask branch per byte
#pragma unroll
        for (int q = 0; q < 32; ++q) {
            const uint32_t b = (x[q >> 2] >> (8 * (q & 3))) & 0xFFu;
            atomicAdd(hl + ((b >> 2) << 5), ((lit >> q) & 1u) << ((b << 3) & 31u));
        }
#else
#pragma unroll
        for (int q = 0; q < 32; ++q)
            if (lit & (1u << q)) count((x[q >> 2] >> (8 * (q & 3))) & 0xFFu);
#endif
    }
    lds_barrier();
    // per-block counts: bins 4r..4r+3 summed over the 32 copies of row r (u16 pairs: <= 32 x 128);
    // the image histogram is summed from them by k_pngb_hist (no per-block global atomics)
    uint16_t* bh = B.bh + (size_t)gblk * 316;               // <= 4096 symbols per block: u16
    for (int r = threadIdx.x; r < kHistRows; r += kParseLanes) {
        uint32_t ev = 0, od = 0;
#if OMR_PNG_HIST_B128
        // four copies per 16-byte read (rotated by the row: 8 lanes cover the 32 banks); even bytes
        // by a mask, odd ones by a v_perm, two dwords per v_add3
        const uint4* row4 = reinterpret_cast<const uint4*>(lh + r * 32);
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            const uint4 v = row4[(c + r) & 7];
            ev += (v.x & 0x00FF00FFu) + (v.y & 0x00FF00FFu);
            ev += (v.z & 0x00FF00FFu) + (v.w & 0x00FF00FFu);
            od += __builtin_amdgcn_perm(0u, v.x, 0x0C030C01u) + __builtin_amdgcn_perm(0u, v.y, 0x0C030C01u);
            od += __builtin_amdgcn_perm(0u, v.z, 0x0C030C01u) + __builtin_amdgcn_perm(0u, v.w, 0x0C030C01u);
        }
#else
#pragma unroll 8
        for (int c = 0; c < 32; ++c) {
            const uint32_t v = lh[r * 32 + ((c + r) & 31)];  // rotated start: rows spread over banks
            ev += v & 0x00FF00FFu;
            od += (v >> 8) & 0x00FF00FFu;
        }
#endif
        const uint32_t cnt[4] = {ev & 0xFFFFu, od & 0xFFFFu, ev >> 16, od >> 16};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int k = 4 * r + j;
            if (k < 316) bh[k] = (uint16_t)cnt[j];
        }
    }
    if (live) {
        const int64_t gs = I.seg0 + s;
        B.trace[gs] = S;
        B.trace[B.total_segs + gs] = M;
        B.trace[2 * B.total_segs + gs] = D;
    }
}

// P2b: the image histograms from the per-block counts: kHistParts workgroups per image, each
// summing its share of the image's parse blocks (coalesced 632-byte rows), one atomic per bin.
constexpr int kHistParts = 16;
__global__ void __launch_bounds__(320) k_pngb_hist(PngBatch B) {
    const int i = blockIdx.x / kHistParts, part = blockIdx.x % kHistParts;
    const PngImg& I = B.img[i];
    const int64_t p0 = B.uniform ? (int64_t)i * B.pblk_per : I.pblk0;
    const int npb = (int)((I.nseg + kParseLanes - 1) / kParseLanes);
    const int j0 = (int)((int64_t)npb * part / kHistParts), j1 = (int)((int64_t)npb * (part + 1) / kHistParts);
    const int k = threadIdx.x;
    if (k >= 316 || j0 >= j1) return;
    const uint16_t* bh = B.bh + (size_t)p0 * 316 + k;
    uint32_t v = 0;
#pragma unroll 8
    for (int j = j0; j < j1; ++j) v += bh[(size_t)j * 316];
    if (v) atomicAdd(&B.hist[(size_t)i * 316 + k], v);
}

// P3b: one workgroup per image, after the code is known: each parse block's code bits are its
// symbol counts times the code lengths (extra bits included), an exclusive scan over the image's
// blocks from the header's end gives every block's first bit -- so P4 needs no inter-block
// communication at all.
#ifndef OMR_PNG_BOFF_WAVE
#define OMR_PNG_BOFF_WAVE 1
#endif
#if OMR_PNG_BOFF_WAVE
// (round 6) A wave per parse block: the lanes read the block's 632-byte count row together (three
// coalesced loads instead of 158 row-strided ones per lane), multiply by the code lengths held in
// registers and sum by DPP; four blocks' loads in flight per wave, 16 waves, chunks of 1024 blocks
// scanned by the workgroup.
constexpr int kBoffThreads = 1024, kBoffChunk = 1024;
__global__ void __launch_bounds__(kBoffThreads) k_pngb_block_offsets(PngBatch B) {
    __shared__ uint32_t s_bits[kBoffChunk];
    __shared__ uint32_t s_wave[kBoffThreads / 64];
    __shared__ uint32_t s_carry;
    const int i = blockIdx.x;
    const PngImg& I = B.img[i];
    const DflTables* T = B.tab + i;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    constexpr int kWaves = kBoffThreads / 64;
    auto cost_of = [&](int k) -> uint32_t {                    // code bits of symbol k (extra bits included)
        if (k >= 316) return 0u;
        if (k < 257) return T->llen[k];
        if (k < 286) return T->llen[k] + len_xbits_of(k - 257);
        return T->dlen[k - 286] + dist_xbits_of(k - 286);
    };
    uint32_t ce[3], co[3];                                    // lane's dwords lane + 64 m: symbols 2d, 2d + 1
#pragma unroll
    for (int m = 0; m < 3; ++m) {
        const int d = lane + 64 * m;
        ce[m] = cost_of(2 * d);
        co[m] = cost_of(2 * d + 1);
    }
    const uint32_t hb = T->hdr[95];
    if (threadIdx.x == 0) s_carry = hb;
    const int64_t p0 = B.uniform ? (int64_t)i * B.pblk_per : I.pblk0;
    const int npb = (int)((I.nseg + kParseLanes - 1) / kParseLanes);
    for (int j0 = 0; j0 < npb; j0 += kBoffChunk) {
        const int nj = min(kBoffChunk, npb - j0);
        for (int b = wv * 4; b < nj; b += 4 * kWaves) {        // four blocks per wave step
            uint32_t v[4][3];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const uint32_t* c2 = reinterpret_cast<const uint32_t*>(B.bh + (size_t)(p0 + j0 + min(b + u, nj - 1)) * 316);
#pragma unroll
                for (int m = 0; m < 3; ++m) v[u][m] = (m < 2 || lane < 158 - 128) ? c2[lane + 64 * m] : 0u;
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                uint32_t acc = 0;
#pragma unroll
                for (int m = 0; m < 3; ++m) acc += (v[u][m] & 0xFFFFu) * ce[m] + (v[u][m] >> 16) * co[m];
                const uint32_t tot = wave_sum_dpp(acc);
                if (lane == 0 && b + u < nj) s_bits[b + u] = tot;
            }
        }
        __syncthreads();
        const int j = j0 + (int)threadIdx.x;
        const uint32_t bits = (int)threadIdx.x < nj ? s_bits[threadIdx.x] : 0u;
        uint32_t tot;
        const uint32_t ex = pngb_block_excl_scan(bits, s_wave, tot);
        const uint32_t base = s_carry;
        if (j < npb) B.poff[p0 + j] = base + ex;
        __syncthreads();
        if (threadIdx.x == 0) s_carry = base + tot;
        __syncthreads();
    }
    if (threadIdx.x == 0) B.img_bits[i] = s_carry + T->llen[256];   // + EOB
}
#else
constexpr int kBoffThreads = 256;
__global__ void __launch_bounds__(256) k_pngb_block_offsets(PngBatch B) {
    __shared__ uint32_t cost[316];
    __shared__ uint32_t s_wave[4];
    __shared__ uint32_t s_carry;
    const int i = blockIdx.x;
    const PngImg& I = B.img[i];
    const DflTables* T = B.tab + i;
    for (int k = threadIdx.x; k < 316; k += 256) {
        uint32_t c;
        if (k < 257) c = T->llen[k];
        else if (k < 286) c = T->llen[k] + len_xbits_of(k - 257);
        else c = T->dlen[k - 286] + dist_xbits_of(k - 286);
        cost[k] = c;
    }
    const uint32_t hb = T->hdr[95];
    if (threadIdx.x == 0) s_carry = hb;
    __syncthreads();
    const int64_t p0 = B.uniform ? (int64_t)i * B.pblk_per : I.pblk0;
    const int npb = (int)((I.nseg + kParseLanes - 1) / kParseLanes);
    for (int j0 = 0; j0 < npb; j0 += 256) {
        const int j = j0 + threadIdx.x;
        uint32_t bits = 0;
        if (j < npb) {
            const uint32_t* c2 = reinterpret_cast<const uint32_t*>(B.bh + (size_t)(p0 + j) * 316);   // 4-aligned
            for (int k = 0; k < 158; ++k) {
                const uint32_t v = c2[k];
                bits += (v & 0xFFFFu) * cost[2 * k] + (v >> 16) * cost[2 * k + 1];
            }
        }
        uint32_t tot;
        const uint32_t ex = pngb_block_excl_scan(bits, s_wave, tot);
        const uint32_t base = s_carry;
        if (j < npb) B.poff[p0 + j] = base + ex;
        __syncthreads();
        if (threadIdx.x == 0) s_carry = base + tot;
        __syncthreads();
    }
    if (threadIdx.x == 0) B.img_bits[i] = s_carry + T->llen[256];   // + EOB
}

#endif

// The tokens of a segment from its parse trace (P2): t as lz_seg_tokens produced them.
template <typename Byte, typename Tok>
__device__ __forceinline__ void trace_tokens(uint32_t S, uint32_t M, uint32_t D, int n, Byte&& seg,
                                             const uint32_t (&dl)[4], const DeflateTabs& T, Tok&& tok) {
    while (S) {
        const int p = __builtin_ctz(S);
        S &= S - 1;
        const int q = S ? __builtin_ctz(S) : n;
        if ((M >> p) & 1u) {
            tok(pack_match(T, (uint32_t)(q - p), dl[D & 3u]));
            D >>= 2;
        } else {
            tok(seg(p));
        }
    }
}

// The encoder's walk of a segment's parse trace: the tokens of trace_tokens, coded through
// put(value, bits), two adjacent literals at a time (their codes, <= 15 bits each, joined into one
// put): literal runs -- most of a photographic tile -- take half the iterations.
template <typename Byte, typename Put>
__device__ __forceinline__ void trace_codes(uint32_t S, uint32_t M, uint32_t D, int n, Byte&& seg,
                                            const uint32_t (&dl)[4], const DeflateTabs& T, const uint32_t* lc,
                                            const uint32_t* dc, Put& put) {
    while (S) {
        const int p = __builtin_ctz(S);
        S &= S - 1;
        if ((M >> p) & 1u) {
            const int q = S ? __builtin_ctz(S) : n;
            put_token_packed(pack_match(T, (uint32_t)(q - p), dl[D & 3u]), lc, dc, put);
            D >>= 2;
            continue;
        }
        const uint32_t e1 = lc[seg(p)];
        if (p < 31 && ((S & ~M) >> (p + 1)) & 1u) {             // the next byte is a literal too
            S &= S - 1;
            const uint32_t e2 = lc[seg(p + 1)];
            const uint32_t n1 = e1 >> 16;
            put((e1 & 0xFFFFu) | ((e2 & 0xFFFFu) << n1), (int)(n1 + (e2 >> 16)));
        } else {
            put(e1 & 0xFFFFu, (int)(e1 >> 16));
        }
    }
}

// P4's pass-1 walk without branches (round 6; OMR_PNG_ENC_FLAT=0 builds the trace_codes form):
// every step takes one token -- a match, or one or two literals -- and puts its whole code at
// once.  A match's code comes from one 8-byte table entry per (distance candidate, length) --
// the four candidate distances are the image's, a length is <= 32 (tokens stay inside their
// segment) -- holding the length code + extra bits, then the distance code + extra bits (<= 48
// bits), and the bit count in bits 58-63.  The literal and match values are both formed and one
// selected, so a wave with literals in some lanes and matches in others runs one path instead of
// both under masks (the branchy walk ran ~140 instructions per step).
constexpr int kMcLen = 33;                       // match table: [candidate][length 0..32]
template <typename Byte, typename Put>
__device__ __forceinline__ void trace_codes_flat(uint32_t S, uint32_t M, uint32_t D, int n, Byte&& seg,
                                                 const uint64_t* mc, const uint32_t* lc, Put& put) {
    while (S) {
        const int p = __builtin_ctz(S);
        S &= S - 1;
        const int q = S ? __builtin_ctz(S) : n;
        const bool ism = (M >> p) & 1u;
        const uint64_t me = mc[(D & 3u) * kMcLen + (uint32_t)(q - p)];
        const uint32_t e1 = lc[seg(p)];
        // a literal followed by a literal (the next byte starts a token that is no match)
        const bool pair = !ism && q < n && !((M >> q) & 1u);
        const uint32_t e2 = lc[seg(pair ? q : p)];
        const uint32_t n1 = e1 >> 16, n2 = pair ? e2 >> 16 : 0u;
        const uint64_t lv = (e1 & 0xFFFFu) | (pair ? (e2 & 0xFFFFu) << n1 : 0u);
        put(ism ? me & 0xFFFFFFFFFFFFull : lv, ism ? (uint32_t)(me >> 58) : n1 + n2);
        S = pair ? S & (S - 1) : S;
        D = ism ? D >> 2 : D;
    }
}

// The same walk taking up to four literals in a row per step (OMR_PNG_ENC_FLAT=2, the default):
// the four bytes from p come out of the lane's stream column as one word (two reads and an
// alignbyte), their four codes are read, and those past the run of literals get length 0 -- a
// literal-heavy segment (most of a photographic tile) takes 8 steps instead of 16.  Codes of a
// step: up to 4 x 15 bits, or a match's <= 48.
template <typename Word4, typename Put>
__device__ __forceinline__ void trace_codes_quad(uint32_t S, uint32_t M, uint32_t D, int n, Word4&& seg4,
                                                 const uint64_t* mc, const uint32_t* lc, Put& put) {
    const uint32_t L = S & ~M;                      // literal starts
    while (S) {
        const int p = __builtin_ctz(S);
        const bool ism = (M >> p) & 1u;
        // literals in a row from p, at most 4 (L holds no bit at or past n)
        const int k = ism ? 1 : min(4, (int)__builtin_ctz(~(L >> p) | 0x10u));
        const uint32_t Sn = S & ~(((2u << (k - 1)) - 1u) << p);   // the next tokens
        const int q = Sn ? __builtin_ctz(Sn) : n;
        const uint64_t me = mc[(D & 3u) * kMcLen + (uint32_t)(q - p)];
        const uint32_t b4 = seg4(p);
        const uint32_t e0 = lc[b4 & 255u], e1 = lc[(b4 >> 8) & 255u], e2 = lc[(b4 >> 16) & 255u], e3 = lc[b4 >> 24];
        const uint32_t n0 = e0 >> 16, n1 = k > 1 ? e1 >> 16 : 0u, n2 = k > 2 ? e2 >> 16 : 0u, n3 = k > 3 ? e3 >> 16 : 0u;
        const uint32_t p01 = (e0 & 0xFFFFu) | (k > 1 ? (e1 & 0xFFFFu) << n0 : 0u);
        const uint32_t p23 = (k > 2 ? e2 & 0xFFFFu : 0u) | (k > 3 ? (e3 & 0xFFFFu) << n2 : 0u);
        const uint64_t lv = (uint64_t)p01 | ((uint64_t)p23 << (n0 + n1));
        put(ism ? me & 0xFFFFFFFFFFFFull : lv, ism ? (uint32_t)(me >> 58) : n0 + n1 + n2 + n3);
        S = Sn;
        D = ism ? D >> 2 : D;
    }
}

__global__ void __launch_bounds__(kHuffThreads) k_pngb_tables(PngBatch B) {
    png_build_tables(B.hist + (size_t)blockIdx.x * 316, B.tab + blockIdx.x);
}

// P4: one workgroup per group of kPngbGroup segments (two parse blocks): its bit range comes
// from P3b, so groups run independently.
// LDS for 8 bits per stream byte + header; a group whose codes need more (<= 16 bits per byte:
// high-entropy data) ORs its interior words straight into memory (the slow path).
constexpr int kEncWords = kPngbGroup * kSeg * 8 / 32 + 96 + 4;
#ifndef OMR_PNG_ENC_SCR
#define OMR_PNG_ENC_SCR 10
#endif
// Words of codes a lane keeps in LDS: 10 (320 bits, 10 bits per stream byte; round 6).  A lane
// past them codes its tokens again in pass 2 with a word-by-word atomic put, and its wave (and
// the workgroup's barrier) waits for it: at 8 words (256 bits) enough C2 segments passed that P4
// ran 1.03 ms per 256 tiles, at 10 or 12 words 0.73-0.75 (profiles/r06/ab_png_encode_scr.txt).
constexpr int kEncScr = OMR_PNG_ENC_SCR;
#ifndef OMR_PNG_ENC_LDS_T
#define OMR_PNG_ENC_LDS_T 0
#endif
#ifndef OMR_PNG_ENC_FLAT
#define OMR_PNG_ENC_FLAT 2
#endif
static_assert(kPngbGroup == 2 * kParseLanes, "P4 groups are two parse blocks");

// The codes of one packed token through put(value, bits), with the code tables packed as
// code | length << 16: a literal is one put, a match two (its extra bits ride above each code).
template <typename Put>
__device__ __forceinline__ void put_token_packed(uint32_t t, const uint32_t* lc, const uint32_t* dc, Put& put) {
    if (!(t & 0x80000000u)) {
        const uint32_t e = lc[t];
        put(e & 0xFFFFu, (int)(e >> 16));
        return;
    }
    const int ls = (int)(t & 31), ds = (int)((t >> 5) & 31);
    const uint32_t le = lc[257 + ls], de = dc[ds];
    const int ll = (int)(le >> 16), dn = (int)(de >> 16);
    put((le & 0xFFFFu) | (((t >> 10) & 31u) << ll), ll + len_xbits_of(ls));          // <= 20 bits
    put((de & 0xFFFFu) | (((t >> 15) & 0x1FFFu) << dn), dn + dist_xbits_of(ds));     // <= 28 bits
}

__global__ void __launch_bounds__(kPngbGroup) k_pngb_encode(PngBatch B) {
    // the group's stream bytes, [dword][lane] (pass 1: a lane reads only its own column, each
    // read on its own bank), then in the same LDS the group's code words (pass 2)
    __shared__ __attribute__((aligned(16))) uint32_t s_buf[kEncWords];
    static_assert(kEncWords * 4 >= kPngbGroup * kSeg, "stream bytes fit the word buffer");
#if OMR_PNG_ENC_LDS_T
    __shared__ DeflateTabs T;
#else
    // (round 6) the deflate tables from constant memory: they serve only the (candidate, length)
    // table build and the rare long-lane re-code, and their 1.2 KiB of LDS lets a seventh
    // workgroup onto the CU
    const DeflateTabs& T = c_dfl;
#endif
    __shared__ uint32_t lc[286], dc[30];                        // code | length << 16
    __shared__ uint32_t scr[(kEncScr + 2) * kPngbGroup];        // [word][lane]: each lane's codes from bit 0
                                                                // (+2 rows: pass 1's spill, see put)
    __shared__ uint32_t s_end[2];                               // slow path: the group's first / last word
    __shared__ uint32_t s_wave[kPngbGroup / 64];
#if OMR_PNG_ENC_FLAT
    __shared__ uint64_t mc[4 * kMcLen];                         // match codes (trace_codes_flat)
#endif
    const int i = pngb_image(B, B.grp0, B.grp_per, blockIdx.x);
    const PngImg& I = B.img[i];
    const int64_t gfirst = B.uniform ? (int64_t)i * B.grp_per : I.grp0;
    const int64_t blk = (int64_t)blockIdx.x - gfirst;
    const int64_t g = blockIdx.x;                               // this workgroup's group
    const DflTables* Tb = B.tab + i;
    T4MARK(0);
    // the group's bit range from P3b: its first parse block's offset (the header opens group 0)
    // to the next group's (or the stream's end)
    const int64_t p0 = B.uniform ? (int64_t)i * B.pblk_per : I.pblk0;
    const int npb = (int)((I.nseg + kParseLanes - 1) / kParseLanes);
    // stored blocks win for this image (P5b decides the same from the same bits): nothing to code;
    // direct mode: nor for a file without a slot in the output
    if (2 + ((int64_t)B.img_bits[i] + 7) / 8 + 4 >= 2 + 5 * I.nblk + I.raw + 4) return;
    if (B.direct && B.meta[i].off < 0) return;
    uint32_t bo;                                                // the stream's bit 0 in the words
    uint32_t* w = pngb_stream_words(B, I, B.meta[i], bo);
    // (group 0 owns the bits below bo too: zero here, the zlib header's bytes are stored by P8)
    const uint32_t c0 = B.poff[p0 + 2 * blk] + bo;              // first code bit of the group
    const uint32_t b0 = blk == 0 ? 0u : c0;
    const uint32_t b1 = (2 * blk + 2 < npb ? B.poff[p0 + 2 * blk + 2] : B.img_bits[i]) + bo;
    const uint32_t w0 = b0 >> 5, w1 = (b1 - 1) >> 5, nwl = w1 - w0;
    uint32_t* const sw = s_buf;
    for (int k = threadIdx.x; k < 286; k += kPngbGroup) lc[k] = (uint32_t)Tb->lcode[k] | (uint32_t)Tb->llen[k] << 16;
    if (threadIdx.x < 30) dc[threadIdx.x] = (uint32_t)Tb->dcode[threadIdx.x] | (uint32_t)Tb->dlen[threadIdx.x] << 16;
    bool big = false;                                           // set after pass 1, workgroup-uniform
    // local word li of the group's code run: LDS, or (slow path) its first / last word in LDS and
    // the rest in memory.  orw for words other lanes (or groups) share; stw for a lane's own.
    auto orw = [&](uint32_t li, uint32_t v) {
        if (!big) atomicOr(&sw[li], v);
        else if (li == 0) atomicOr(&s_end[0], v);
        else if (li == nwl) atomicOr(&s_end[1], v);
        else atomicOr(&w[w0 + li], v);
    };
    auto stw = [&](uint32_t li, uint32_t v) {
        if (!big) sw[li] = v;
        else if (li == 0 || li == nwl) orw(li, v);
        else w[w0 + li] = v;
    };
#if OMR_PNG_ENC_LDS_T
    lz_load_tabs(T);
#endif
    const int64_t s = blk * kPngbGroup + threadIdx.x;
    const bool live = s < I.nseg;
    uint32_t x[kSeg / 4] = {};                                  // the lane's 32 stream bytes
    uint32_t S = 0, M = 0, D = 0;                               // its parse trace (P2)
    if (live) {                                                 // (P2 left >= 64 bytes of slack past each stream)
        const int64_t gs = I.seg0 + s;
        S = B.trace[gs];
        M = B.trace[B.total_segs + gs];
        D = B.trace[2 * B.total_segs + gs];
        const uint4* o = reinterpret_cast<const uint4*>(B.flt + I.flt + s * kSeg);
        const uint4 u0 = o[0], u1 = o[1];
        x[0] = u0.x; x[1] = u0.y; x[2] = u0.z; x[3] = u0.w;
        x[4] = u1.x; x[5] = u1.y; x[6] = u1.z; x[7] = u1.w;
#pragma unroll
        for (int k = 0; k < kSeg / 4; ++k) s_buf[k * kPngbGroup + threadIdx.x] = x[k];
    }
    __syncthreads();
    T4MARK(1);
    const bool last = s == I.nseg - 1;                          // the EOB code follows its tokens
    int n = 0;
    const uint32_t dl[4] = {1u, I.bpp == 1 ? (uint32_t)I.rowlen : (uint32_t)I.bpp, (uint32_t)(2 * I.bpp),
                            (uint32_t)I.rowlen};               // lz_seg_prepare's candidates
    auto seg_byte = [&](int p) { return (s_buf[(p >> 2) * kPngbGroup + threadIdx.x] >> (8 * (p & 3))) & 0xFFu; };
    uint32_t nb = 0;
#if OMR_PNG_ENC_FLAT
    if (threadIdx.x < 4 * kMcLen) {                             // (lc, dc, T are staged: barrier above)
        const int k = threadIdx.x / kMcLen, l = threadIdx.x % kMcLen;
        uint64_t e = 0;
        if (l >= 3) {
            const uint32_t t = pack_match(T, (uint32_t)l, dl[k]);
            const int ls = (int)(t & 31), ds = (int)((t >> 5) & 31);
            const uint32_t le = lc[257 + ls], de = dc[ds];
            const uint32_t lb = (le >> 16) + (uint32_t)len_xbits_of(ls), db = (de >> 16) + (uint32_t)dist_xbits_of(ds);
            const uint64_t lv = (le & 0xFFFFu) | (((t >> 10) & 31u) << (le >> 16));
            const uint64_t dv = (de & 0xFFFFu) | (((t >> 15) & 0x1FFFu) << (de >> 16));
            e = lv | (dv << lb) | ((uint64_t)(lb + db) << 58);
        }
        mc[threadIdx.x] = e;
    }
    __syncthreads();
    // pass 1: the lane's codes from bit 0 into its scratch column (a lane whose codes pass
    // kEncScr words only counts them and codes again in pass 2); codes of up to 48 bits, the
    // pending bits (< 32) in a 64-bit accumulator, at most two words out per put
    if (live) {
        n = (int)min((int64_t)kSeg, I.raw - s * kSeg);
        uint64_t acc = 0;
        uint32_t nacc = 0, nw = 0;
        // every put stores the three words its bits can reach, unconditionally (a partial word
        // is stored again, more complete, by the next put; rows past the lane's last word hold
        // zeros or nothing pass 2 reads).  From word kEncScr - 1 on the stores stay at rows 7-9:
        // such a lane passes kEncScr words, and pass 2 codes it again from its stream bytes.
        auto put = [&](uint64_t v, uint32_t bits) {
            const uint64_t lo = acc | (v << nacc);
            const uint32_t hi = (uint32_t)((v >> 1) >> (63 - nacc));          // bits past 64 (0 when nacc = 0)
            const uint32_t tot = nacc + bits, wn = tot >> 5;                  // whole words done: 0 .. 2
            uint32_t* col = scr + min(nw, (uint32_t)kEncScr - 1) * kPngbGroup + threadIdx.x;
            col[0] = (uint32_t)lo;
            col[kPngbGroup] = (uint32_t)(lo >> 32);
            col[2 * kPngbGroup] = hi;
            const uint32_t a0 = wn == 0 ? (uint32_t)lo : wn == 1 ? (uint32_t)(lo >> 32) : hi;
            const uint32_t a1 = wn == 0 ? (uint32_t)(lo >> 32) : wn == 1 ? hi : 0u;
            acc = ((uint64_t)a1 << 32) | a0;
            nw += wn;
            nacc = tot & 31u;
        };
#if OMR_PNG_ENC_FLAT == 2
        auto seg4 = [&](int p) {                                // stream bytes p .. p + 3 of the lane
            const int d = p >> 2;
            const uint32_t lo = s_buf[d * kPngbGroup + threadIdx.x];
            const uint32_t hi = s_buf[min(d + 1, kSeg / 4 - 1) * kPngbGroup + threadIdx.x];   // (past the segment: unused)
            return __builtin_amdgcn_alignbyte(hi, lo, (uint32_t)(p & 3));
        };
        trace_codes_quad(S, M, D, n, seg4, mc, lc, put);
        (void)seg_byte;
#else
        trace_codes_flat(S, M, D, n, seg_byte, mc, lc, put);
#endif
        if (last) put(lc[256] & 0xFFFFu, lc[256] >> 16);
        if (nacc > 0 && nw < (uint32_t)kEncScr) scr[nw * kPngbGroup + threadIdx.x] = (uint32_t)acc;
        nb = 32 * nw + nacc;
    }
#else
    // pass 1: the lane's codes from bit 0 into its scratch column (a lane whose codes pass
    // kEncScr words only counts them and codes again in pass 2)
    if (live) {
        n = (int)min((int64_t)kSeg, I.raw - s * kSeg);
        uint64_t acc = 0;
        int nacc = 0;
        uint32_t nw = 0;
        auto put = [&](uint32_t v, int bits) {
            acc |= (uint64_t)v << nacc;
            nacc += bits;
            if (nacc >= 32) {
                if (nw < (uint32_t)kEncScr) scr[nw * kPngbGroup + threadIdx.x] = (uint32_t)acc;
                ++nw;
                acc >>= 32;
                nacc -= 32;
            }
        };
        trace_codes(S, M, D, n, seg_byte, dl, T, lc, dc, put);
        if (last) put(lc[256] & 0xFFFFu, (int)(lc[256] >> 16));
        if (nacc > 0 && nw < (uint32_t)kEncScr) scr[nw * kPngbGroup + threadIdx.x] = (uint32_t)acc;
        nb = 32 * nw + (uint32_t)nacc;
    }
#endif
    // a lane whose codes passed its scratch column codes them again in pass 2, from its stream
    // bytes kept in that column (the stream buffer becomes the word buffer; the scan's barriers
    // order these copies before it is zeroed)
    if (nb > 32u * kEncScr) {
#pragma unroll
        for (int k = 0; k < kSeg / 4; ++k) scr[k * kPngbGroup + threadIdx.x] = x[k];
    }
    T4MARK(2);
    uint32_t total;
    const uint32_t ex = pngb_block_excl_scan(nb, s_wave, total);
    const uint32_t hb = Tb->hdr[95];
    (void)total;                                                // == b1 - c0 (the same codes)
    // the slow path when the group's words pass the LDS buffer (> 8 bits per stream byte)
    big = nwl >= (uint32_t)kEncWords;
    if (!big) {
        for (uint32_t k = threadIdx.x; k <= nwl; k += kPngbGroup) sw[k] = 0;
    } else {                                                    // slow path: interior words in memory
        if (threadIdx.x < 2) s_end[threadIdx.x] = 0;
        for (uint32_t k = w0 + 1 + threadIdx.x; k < w1; k += kPngbGroup) w[k] = 0;
        __threadfence_block();                                  // the zeroed words before any OR
    }
    __syncthreads();
    T4MARK(3);
    if (blk == 0 && threadIdx.x == 0) {                         // the block header, from bit bo
        const uint32_t nh = (hb + 31) / 32;
        uint32_t prev = 0;
        for (uint32_t k = 0; k < (hb + bo + 31) / 32; ++k) {
            const uint32_t v = k < nh ? Tb->hdr[k] : 0u;
            orw(k, bo ? (v << bo) | (prev >> (32 - bo)) : v);
            prev = v;
        }
    }
    if (live && nb) {
        const uint32_t pos = c0 + ex - 32 * w0;                 // bit position in sw
        const uint32_t sh = pos & 31, wb = pos >> 5;
        if (nb <= 32u * kEncScr) {
            // pass 2: the scratch column shifted into place; the first and last output words
            // are shared with the neighbouring lanes, the rest are this lane's alone
            const uint32_t nsrc = (nb + 31) >> 5, nout = (sh + nb + 31) >> 5;
            uint32_t prev = 0;
            for (uint32_t k = 0; k < nout; ++k) {
                const uint32_t v = k < nsrc ? scr[k * kPngbGroup + threadIdx.x] : 0u;
                const uint32_t o = sh ? (v << sh) | (prev >> (32 - sh)) : v;
                prev = v;
                if (k == 0 || k == nout - 1) orw(wb + k, o);
                else stw(wb + k, o);
            }
        } else {                                                // long codes: code the tokens again
            auto byte = [&](int p) { return (scr[(p >> 2) * kPngbGroup + threadIdx.x] >> (8 * (p & 3))) & 0xFFu; };
            uint64_t acc = 0;
            int nacc = (int)sh;
            uint32_t wpos = wb;
            auto put = [&](uint32_t v, int bits) {
                acc |= (uint64_t)v << nacc;
                nacc += bits;
                if (nacc >= 32) {
                    orw(wpos, (uint32_t)acc);
                    ++wpos;
                    acc >>= 32;
                    nacc -= 32;
                }
            };
            trace_codes(S, M, D, n, byte, dl, T, lc, dc, put);
            if (last) put(lc[256] & 0xFFFFu, (int)(lc[256] >> 16));
            if (nacc > 0) orw(wpos, (uint32_t)acc);
        }
    }
    __syncthreads();
    T4MARK(4);
    // whole words inside [b0, b1) go out; the first and last (shared with the neighbouring
    // blocks) are kept for P5
    const uint32_t cf = big ? s_end[0] : sw[0], cl = nwl ? (big ? s_end[1] : sw[nwl]) : 0u;
    if (!big) {
        for (uint32_t k = w0 + threadIdx.x; k <= w1; k += kPngbGroup)
            if (b0 <= 32 * k && b1 >= 32 * k + 32) w[k] = sw[k - w0];
    } else if (threadIdx.x == 0) {                              // the interior is in memory already
        if (b0 == 32 * w0) w[w0] = cf;                         // (never both ends inside one word here)
        if (b1 == 32 * w1 + 32) w[w1] = cl;
    }
    if (threadIdx.x == 0) {
        B.blk_b0[g] = b0;
        B.blk_b1[g] = b1;
        B.blk_cf[g] = cf;
        B.blk_cl[g] = cl;
    }
    T4MARK(5);
}

// P5: the words two or more blocks share.  Block g handles the partial word its stream ends in,
// when it is the first block touching that word, ORing the first words of the blocks that
// follow while they start inside it.
__global__ void __launch_bounds__(256) k_pngb_fixup(PngBatch B) {
    const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (g >= B.total_grp) return;
    const int i = pngb_image(B, B.grp0, B.grp_per, g);
    const PngImg& I = B.img[i];
    const int64_t gend = (B.uniform ? (int64_t)i * B.grp_per : I.grp0) + (I.nseg + kPngbGroup - 1) / kPngbGroup;
    if (2 + ((int64_t)B.img_bits[i] + 7) / 8 + 4 >= 2 + 5 * I.nblk + I.raw + 4) return;   // stored: P4 skipped
    const uint32_t b0 = B.blk_b0[g], b1 = B.blk_b1[g], w0 = b0 >> 5, w1 = (b1 - 1) >> 5;
    if ((b1 & 31) == 0 || !(w1 > w0 || (b0 & 31) == 0)) return;
    if (B.direct && B.meta[i].off < 0) return;
    uint32_t v = w1 == w0 ? B.blk_cf[g] : B.blk_cl[g];
    for (int64_t j = g + 1; j < gend && B.blk_b0[j] < 32 * (w1 + 1); ++j) v |= B.blk_cf[j];
    uint32_t bo;
    pngb_stream_words(B, I, B.meta[i], bo)[w1] = v;
}

// P5b: one workgroup per image: stream length, stored vs dynamic, Adler-32.
__global__ void __launch_bounds__(256) k_pngb_meta(PngBatch B) {
    __shared__ unsigned long long s_ad[2][4];
    const int i = blockIdx.x;
    const PngImg& I = B.img[i];
    const int64_t glast = (B.uniform ? (int64_t)i * B.grp_per : I.grp0) + (I.nseg + kPngbGroup - 1) / kPngbGroup - 1;
    const uint32_t total = B.img_bits[i];                      // header + codes + EOB
    (void)glast;
    const int64_t zdyn = 2 + ((int64_t)total + 7) / 8 + 4, zstored = 2 + 5 * I.nblk + I.raw + 4;
    const bool stored = zdyn >= zstored;
    unsigned long long s1 = 0, s2 = 0;
    for (int y = threadIdx.x; y < I.H; y += 256) {
        s1 += B.row_sums[2 * ((int64_t)I.row0 + y)];
        s2 += B.row_sums[2 * ((int64_t)I.row0 + y) + 1];
    }
    for (int o = 32; o > 0; o >>= 1) {
        s1 += __shfl_down(s1, o, 64);
        s2 += __shfl_down(s2, o, 64);
    }
    if ((threadIdx.x & 63) == 0) { s_ad[0][threadIdx.x >> 6] = s1; s_ad[1][threadIdx.x >> 6] = s2; }
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned long long a1 = s_ad[0][0] + s_ad[0][1] + s_ad[0][2] + s_ad[0][3];
        const unsigned long long a2 = s_ad[1][0] + s_ad[1][1] + s_ad[1][2] + s_ad[1][3];
        const uint64_t a = (1 + a1) % 65521, b = ((uint64_t)I.raw % 65521 + a2 % 65521) % 65521;
        const uint32_t hb = B.tab[i].hdr[95];
        PngMeta& M = B.meta[i];
        M.zlen = stored ? zstored : zdyn;
        M.file_len = I.pre_len + 8 + M.zlen + 4 + 12;
        M.off = -1;
        M.adler = (uint32_t)((b << 16) | a);
        M.crc = 0;
        M.hbits = hb;
        M.tot_bits = total - hb;
        M.stored = stored ? 1 : 0;
        M.status = OMR_OK;
    }
}

// P6: one workgroup: each file's offset (16-byte aligned slots, in image order) and status.
__global__ void __launch_bounds__(1024) k_pngb_offsets(PngBatch B) {
    __shared__ unsigned long long s_wave[16];
    __shared__ unsigned long long s_carry;
    if (threadIdx.x == 0) s_carry = 0;
    __syncthreads();
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    for (int i0 = 0; i0 < B.n; i0 += 1024) {
        const int i = i0 + threadIdx.x;
        const bool ok = i < B.n && B.meta[i].status == OMR_OK;   // a failed image takes no slot
        const unsigned long long v = ok ? ((unsigned long long)B.meta[i].file_len + 15ull) & ~15ull : 0ull;
        unsigned long long x = v;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const unsigned long long y = __shfl_up(x, o, 64);
            if (lane >= o) x += y;
        }
        if (lane == 63) s_wave[wid] = x;
        __syncthreads();
        if (wid == 0) {
            unsigned long long t = lane < 16 ? s_wave[lane] : 0ull;
#pragma unroll
            for (int o = 1; o < 16; o <<= 1) {
                const unsigned long long y = __shfl_up(t, o, 64);
                if (lane >= o) t += y;
            }
            if (lane < 16) s_wave[lane] = t;
        }
        __syncthreads();
        const unsigned long long base = s_carry, ex = base + (wid ? s_wave[wid - 1] : 0ull) + x - v;
        if (i < B.n) {
            PngMeta& M = B.meta[i];
            const bool fits = ok && ex + v <= B.out_cap; // the whole 16-byte slot (P8 stores 16 B)
            M.off = fits ? (int64_t)ex : -1;
            M.status = !ok ? M.status : fits ? OMR_OK : OMR_BUFFER_TOO_SMALL;
            if (B.d_offsets) B.d_offsets[i] = fits ? ex : 0ull;
            if (B.d_lengths) B.d_lengths[i] = fits ? (uint32_t)M.file_len : 0u;
            if (B.d_status) B.d_status[i] = M.status;
        }
        __syncthreads();
        if (threadIdx.x == 0) s_carry = base + s_wave[15];
        __syncthreads();
    }
}

__constant__ uint8_t c_iend[12] = {0, 0, 0, 0, 'I', 'E', 'N', 'D', 0xAE, 0x42, 0x60, 0x82};

// Byte k of image I's file (P8's general path).
__device__ uint32_t pngb_file_byte(const PngBatch& B, const PngImg& I, const PngMeta& M, int64_t k) {
    const int64_t P = I.pre_len;
    if (k < P) return I.pre[k];
    k -= P;
    if (k < 4) return (uint32_t)(M.zlen >> (24 - 8 * k)) & 0xFF;
    if (k < 8) return (uint32_t)"IDAT"[k - 4];
    k -= 8;
    if (k < M.zlen) {
        if (k == 0) return 0x78;                       // CMF/FLG: deflate, 32K window, check bits
        if (k == 1) return 0x01;
        if (k >= M.zlen - 4) return (M.adler >> (8 * (M.zlen - 1 - k))) & 0xFF;
        const int64_t d = k - 2;
        if (!M.stored) return reinterpret_cast<const uint8_t*>(B.words + I.words)[d];
        const int64_t b = d / (kStored + 5), o = d - b * (kStored + 5);
        if (o >= 5) return B.flt[I.flt + b * kStored + (o - 5)];
        const uint32_t len = (uint32_t)min((int64_t)kStored, I.raw - b * kStored);
        switch (o) {
        case 0: return b == I.nblk - 1 ? 1u : 0u;       // BFINAL, BTYPE=00
        case 1: return len & 0xFF;
        case 2: return (len >> 8) & 0xFF;
        case 3: return (~len) & 0xFF;
        default: return ((~len) >> 8) & 0xFF;
        }
    }
    k -= M.zlen;
    if (k < 4) return 0;                               // CRC: P10
    k -= 4;
    return k < 12 ? c_iend[k] : 0u;
}

// The 16 bytes of image I's file at k0 outside the dynamic stream's interior (chunk headers,
// zlib header and Adler, stored blocks, CRC and IEND), byte by byte: a rare path, kept out of line
// so it does not inflate the callers' registers.
__device__ __noinline__ uint4 pngb_file_chunk_bytes(const PngBatch& B, const PngImg& I, const PngMeta& M, int64_t k0) {
    uint32_t o[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        uint32_t v = 0;
        for (int b = 0; b < 4; ++b) {
            const int64_t k = k0 + 4 * j + b;
            if (k < M.file_len) v |= pngb_file_byte(B, I, M, k) << (8 * b);
        }
        o[j] = v;
    }
    return make_uint4(o[0], o[1], o[2], o[3]);
}

// The 16 bytes of image I's file at k0 (P8's body).
__device__ __forceinline__ uint4 pngb_file_chunk(const PngBatch& B, const PngImg& I, const PngMeta& M, int64_t k0) {
    const int64_t d0 = k0 - I.pre_len - 10;            // deflate byte of k0 (dynamic stream)
    if (!M.stored && d0 >= 0 && k0 + 16 <= I.pre_len + 8 + M.zlen - 4) {
        const uint32_t* w = B.words + I.words + (d0 >> 2);
        const int sh = (int)(d0 & 3) * 8;
        uint32_t x[5], o[4];
#pragma unroll
        for (int j = 0; j < 5; ++j) x[j] = w[j];
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = sh ? (x[j] >> sh) | (x[j + 1] << (32 - sh)) : x[j];
        return make_uint4(o[0], o[1], o[2], o[3]);
    }
    return pngb_file_chunk_bytes(B, I, M, k0);
}

// P8: 16 bytes of one file per lane, one aligned 16-byte store (the form with a separate P9).
__global__ void __launch_bounds__(256) k_pngb_emit(PngBatch B) {
    const int i = pngb_image(B, B.eblk0, B.eblk_per, blockIdx.x);
    const PngImg& I = B.img[i];
    const PngMeta& M = B.meta[i];
    const int64_t lb = (int64_t)blockIdx.x - (B.uniform ? (int64_t)i * B.eblk_per : I.eblk0);
    const int64_t k0 = (lb * 256 + threadIdx.x) * 16;
    if (M.off < 0 || k0 >= M.file_len) return;
    *reinterpret_cast<uint4*>(B.out + M.off + k0) = pngb_file_chunk(B, I, M, k0);
}

// P8 in direct mode: the file's bytes around the stream P4 / P5 already coded in place -- the prefix
// chunks, IDAT length and type, zlib header, Adler-32, IEND (the CRC is P10's) -- by byte stores
// from each image's first workgroup; a stored-blocks file whole, 16 bytes per lane, as k_pngb_emit,
// over the image's kEmitDirectWgs workgroups (grid: images x kEmitDirectWgs -- a grid of every
// file's 4 KiB pieces, nearly all idle here, cost 0.06 ms of dispatch per 256 tiles).
constexpr int kEmitDirectWgs = 16;
__global__ void __launch_bounds__(256) k_pngb_emit_direct(PngBatch B) {
    const int i = blockIdx.x / kEmitDirectWgs, lb = blockIdx.x % kEmitDirectWgs;
    const PngImg& I = B.img[i];
    const PngMeta& M = B.meta[i];
    if (M.off < 0) return;
    if (M.stored) {
        for (int64_t k0 = ((int64_t)lb * 256 + threadIdx.x) * 16; k0 < M.file_len; k0 += kEmitDirectWgs * 256 * 16)
            *reinterpret_cast<uint4*>(B.out + M.off + k0) = pngb_file_chunk(B, I, M, k0);
        return;
    }
    if (lb != 0) return;
    uint8_t* f = B.out + M.off;
    const int64_t head = I.pre_len + 10, tail = I.pre_len + 8 + M.zlen - 4;   // Adler on
    for (int64_t k = threadIdx.x; k < head; k += 256) f[k] = (uint8_t)pngb_file_byte(B, I, M, k);
    for (int64_t k = tail + threadIdx.x; k < M.file_len; k += 256) f[k] = (uint8_t)pngb_file_byte(B, I, M, k);
}

// P9 tables (round 5): braid[b][v] = raw CRC of byte v at position b of a 4-byte word followed
// by 255 - b zero bytes (the state then sits at the same lane's next word, 256 bytes on: zlib's
// "braided" CRC with 64 lanes of one word); last[b][v] the same without the trailing 252 bytes
// (slicing-by-4: the state at the end of the word); lane[k] = x^(32 (63 - k)) mod P, the shift
// from lane k's last word end to the end of its strip.
struct CrcBraid {
    uint32_t braid[4][256];
    uint32_t last[4][256];
    uint32_t lane[64];
};

constexpr CrcBraid make_crc_braid() {
    CrcBraid c{};
    uint32_t t[256] = {};                      // t[n]: CRC of byte n followed by k zero bytes
    for (uint32_t n = 0; n < 256; ++n) {
        uint32_t r = n;
        for (int k = 0; k < 8; ++k) r = (r & 1) ? kCrcPoly ^ (r >> 1) : r >> 1;
        t[n] = r;
    }
    uint32_t t0[256] = {};
    for (int n = 0; n < 256; ++n) t0[n] = t[n];
    for (int k = 0; k <= 255; ++k) {           // t = k zero bytes after the byte
        for (int b = 0; b < 4; ++b) {
            if (k == 3 - b)
                for (int n = 0; n < 256; ++n) c.last[b][n] = t[n];
            if (k == 255 - b)
                for (int n = 0; n < 256; ++n) c.braid[b][n] = t[n];
        }
        for (int n = 0; n < 256; ++n) t[n] = (t[n] >> 8) ^ t0[t[n] & 0xFF];
    }
    uint32_t x32 = 1u << 31;                   // x^0
    uint32_t x8 = 1u << 30;                    // x^1 -> x^8 by squaring three times
    for (int i = 0; i < 3; ++i) x8 = multmodp_c(x8, x8);
    const uint32_t x32step = multmodp_c(multmodp_c(x8, x8), multmodp_c(x8, x8));   // x^32
    for (int k = 63; k >= 0; --k) {            // lane[63] = x^0, lane[62] = x^32, ...
        c.lane[k] = x32;
        x32 = multmodp_c(x32step, x32);
    }
    return c;
}

__constant__ CrcBraid c_braid = make_crc_braid();

__device__ __forceinline__ uint32_t load_u32_any(const uint8_t* p) {   // unaligned 32-bit load
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    const uint32_t* q = reinterpret_cast<const uint32_t*>(a & ~(uintptr_t)3);
    const int sh = (int)(a & 3) * 8;
    const uint32_t w0 = q[0];
    return sh ? (w0 >> sh) | (q[1] << (32 - sh)) : w0;
}

// P9: CRC-32 of 'IDAT' + zlib stream (n = 4 + zlen bytes of the output file).  Each wave owns a
// strip of kCrcStrip bytes, strips counted back from the end of the range (strip g ends g strips
// before it; the first strip may start before the range, those bytes read as 0, which leaves a
// zero-initialised CRC unchanged).  Lane k reads the word at strip + 256 j + 4 k (a wave reads 256
// contiguous bytes per step: coalesced) and keeps a braided state (braid tables); the last step
// leaves lane k's state at its word end, the lane constant shifts it to the strip end, the wave
// XOR-reduces, and lane 0 shifts the strip's CRC to the range end (x^(8 * kCrcStrip * g)) and
// XORs it into the file's CRC.  The init / final inversions add ~(x^(8n) * 0xFFFFFFFF) once.
constexpr int kCrcStrip = 64 * 256;            // bytes per wave (64 steps of 256)
static_assert(kPngbCrcBytes == 4 * kCrcStrip, "P9: four strips per workgroup");

__global__ void __launch_bounds__(256) k_pngb_crc(PngBatch B) {
    __shared__ uint32_t sb[4][256], sl[4][256];
    for (int k = threadIdx.x; k < 4 * 256; k += 256) {
        sb[k >> 8][k & 255] = c_braid.braid[k >> 8][k & 255];
        sl[k >> 8][k & 255] = c_braid.last[k >> 8][k & 255];
    }
    __syncthreads();
    const int i = pngb_image(B, B.cblk0, B.cblk_per, blockIdx.x);
    const PngImg& I = B.img[i];
    const PngMeta& M = B.meta[i];
    if (M.off < 0) return;
    const int lane = threadIdx.x & 63;
    const int64_t g = ((int64_t)blockIdx.x - (B.uniform ? (int64_t)i * B.cblk_per : I.cblk0)) * 4 + (threadIdx.x >> 6);
    const int64_t n = 4 + M.zlen;
    const int64_t s0 = n - kCrcStrip * (g + 1);           // strip start, relative to the range
    if (s0 + kCrcStrip <= 0) return;                      // wave-uniform: past the range's start
    const uint8_t* base = B.out + M.off + I.pre_len + 4;
    // the strip's words are read as aligned dwords (one coalesced 256-byte read per wave and step)
    // and realigned with the next lane's dword (lane 63: lane 0's of the next step)
    const uintptr_t sa = reinterpret_cast<uintptr_t>(base) + (uintptr_t)s0;   // may lie below base
    const uint32_t* aw = reinterpret_cast<const uint32_t*>(sa & ~(uintptr_t)3);
    const int sh = (int)(sa & 3);
    const int64_t arel = s0 - sh;                         // range offset of aw[0]
    uint32_t q = 0;
    // an inner strip (s0 >= 0, not the last: every byte its 17 x 4 loads reach lies in the range)
    // runs without the range tests (round 6: one wave-uniform branch per strip)
    auto walk = [&](auto inner_c) {
        constexpr bool kInner = decltype(inner_c)::value;
#pragma unroll 1
        for (int j0 = 0; j0 < 64; j0 += 16) {
            uint32_t cw[17];
#pragma unroll
            for (int t = 0; t < 17; ++t) {                // 17 loads in flight; bytes outside the range read 0
                const int64_t r = arel + 256 * (j0 + t) + 4 * lane;
                cw[t] = (kInner || (r > -4 && r < n)) ? aw[64 * (j0 + t) + lane] : 0u;
            }
#pragma unroll
            for (int t = 0; t < 16; ++t) {
                uint32_t w = __builtin_amdgcn_alignbyte(next_lane_dword(cw[t], cw[t + 1]), cw[t], sh);
                if (!kInner) {
                    const int64_t rel = s0 + 256 * (j0 + t) + 4 * lane;   // range offset of the word
                    if (rel < 0) w = rel <= -4 ? 0u : w & (0xFFFFFFFFu << (8 * (int)(-rel)));   // bytes before the range: 0
                }
                const uint32_t x = q ^ w;
                if (j0 + t < 63) {
                    q = sb[0][x & 255] ^ sb[1][(x >> 8) & 255] ^ sb[2][(x >> 16) & 255] ^ sb[3][x >> 24];
                } else {
                    q = sl[0][x & 255] ^ sl[1][(x >> 8) & 255] ^ sl[2][(x >> 16) & 255] ^ sl[3][x >> 24];
                }
            }
        }
    };
    if (s0 >= 0 && g > 0) walk(FltIdx<1>{});
    else walk(FltIdx<0>{});
    uint32_t v = q ? multmodp(c_braid.lane[lane], q) : 0u;
    for (int o = 32; o > 0; o >>= 1) v ^= __shfl_xor(v, o, 64);
    if (lane == 0) {
        const uint64_t jj = (uint64_t)g * (kCrcStrip / 256);   // x^(8 * 256 * jj)
        if (v && jj) {
            v = multmodp(B.crc_pow[jj & (kCrcPowLo - 1)], v);
            if (jj >= kCrcPowLo) v = multmodp(B.crc_pow[kCrcPowLo + (jj / kCrcPowLo)], v);
        }
        if (g == 0) v ^= ~multmodp(x2nmodp((uint64_t)n, 3), 0xFFFFFFFFu);
        if (v) atomicXor(&B.meta[i].crc, v);
    }
}

// P8+P9 tables: hop[b][v] = raw CRC of byte v at position b of a 4-byte word followed by 3 - b +
// 1008 zero bytes (the state then sits at the same lane's next 16-byte chunk, 1 KiB on); lane16[k]
// = x^(8 (1008 - 16 k)), the shift from the end of lane k's last chunk to the end of its strip.
struct CrcHop {
    uint32_t hop[4][256];
    uint32_t lane16[64];
};
constexpr CrcHop make_crc_hop() {
    CrcHop c{};
    uint32_t t[256] = {}, t0[256] = {};
    for (uint32_t n = 0; n < 256; ++n) {
        uint32_t r = n;
        for (int k = 0; k < 8; ++k) r = (r & 1) ? kCrcPoly ^ (r >> 1) : r >> 1;
        t[n] = t0[n] = r;
    }
    for (int k = 0; k <= 1011; ++k) {          // t = CRC of byte n followed by k zero bytes
        for (int b = 0; b < 4; ++b)
            if (k == 1011 - b)
                for (int n = 0; n < 256; ++n) c.hop[b][n] = t[n];
        for (int n = 0; n < 256; ++n) t[n] = (t[n] >> 8) ^ t0[t[n] & 0xFF];
    }
    uint32_t x8 = 1u << 30;                    // x^1 -> x^8
    for (int i = 0; i < 3; ++i) x8 = multmodp_c(x8, x8);
    const uint32_t x32 = multmodp_c(multmodp_c(x8, x8), multmodp_c(x8, x8));
    const uint32_t x128 = multmodp_c(multmodp_c(x32, x32), multmodp_c(x32, x32));          // x^(8*16)
    uint32_t p = 1u << 31;                     // lane 63: x^0
    for (int k = 63; k >= 0; --k) {
        c.lane16[k] = p;
        p = multmodp_c(x128, p);
    }
    return c;
}
__constant__ CrcHop c_hop = make_crc_hop();

// P8 + P9 fused (round 6, the default): each wave emits a strip of the file (lane t, step
// s: the 16 bytes at strip + 1 KiB s + 16 t -- one coalesced 1 KiB store per step) and CRCs it
// from the same registers: lane t's 16 bytes are four words through slicing-by-4 tables, the
// fourth with a table that also hops the state over the other lanes' 1008 bytes to its next chunk
// (a 16-byte braid); no LDS staging, no barrier after the tables.  Bytes outside the IDAT range
// ['IDAT', end of the zlib stream) read as 0.  The strip's raw CRC sits at the strip end E; it is
// moved to the range end R1 (x^(8 (R1 - E)) from the power tables, or x^(-8 (E - R1)) for the
// strip holding R1, whose trailing bytes read as 0) in P9b, which XORs it into the file's CRC; P10
// stores it.  The file is not read back from HBM (P9 re-read it: 482 MB per 256 C2 tiles).
__global__ void __launch_bounds__(256) k_pngb_emit_crc(PngBatch B) {
    constexpr int kSteps = kPngbEmitCrcStrip / 1024;
    __shared__ uint32_t sl[4][256], sh[4][256];
    const int i = pngb_image(B, B.eblk0, B.eblk_per, blockIdx.x);
    const PngImg& I = B.img[i];
    const PngMeta& M = B.meta[i];
    const int64_t lb = (int64_t)blockIdx.x - (B.uniform ? (int64_t)i * B.eblk_per : I.eblk0);
    const int64_t F0 = lb * kPngbEmitCrcBytes;          // file offset of the workgroup's bytes
    if (M.off < 0 || F0 >= M.file_len) return;          // workgroup-uniform
    for (int k = threadIdx.x; k < 4 * 256; k += 256) {
        sl[k >> 8][k & 255] = c_braid.last[k >> 8][k & 255];
        sh[k >> 8][k & 255] = c_hop.hop[k >> 8][k & 255];
    }
    __syncthreads();                                    // the CRC tables
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t S0 = F0 + (int64_t)wv * kPngbEmitCrcStrip, E = S0 + kPngbEmitCrcStrip;
    if (S0 >= M.file_len) return;                       // wave-uniform (P9b skips the strip too)
    const int64_t R0 = I.pre_len + 4, R1 = I.pre_len + 8 + M.zlen;   // CRC range: 'IDAT' + zlib stream
    const bool any = !(E <= R0 || S0 >= R1);            // wave-uniform: the strip holds range bytes
    // range limits relative to this lane's first byte of the strip (clamped: a strip is 16 KiB)
    const int64_t p0 = S0 + 16 * lane;
    const int32_t lo = (int32_t)max<int64_t>(min<int64_t>(R0 - p0, 1 << 20), -(1 << 20));
    const int32_t hi = (int32_t)max<int64_t>(min<int64_t>(R1 - p0, 1 << 20), -(1 << 20));
    auto T = [&](const uint32_t (*t)[256], uint32_t x) {
        return t[0][x & 255] ^ t[1][(x >> 8) & 255] ^ t[2][(x >> 16) & 255] ^ t[3][x >> 24];
    };
    uint32_t q = 0;
#pragma unroll 4
    for (int st = 0; st < kSteps; ++st) {
        const int64_t k0 = p0 + 1024 * st;
        uint4 v = make_uint4(0, 0, 0, 0);
        if (k0 < M.file_len) {
            v = pngb_file_chunk(B, I, M, k0);
            *reinterpret_cast<uint4*>(B.out + M.off + k0) = v;
        }
        if (any) {
            uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int32_t r = 1024 * st + 4 * j;    // word offset from p0
                if (r < lo) w[j] = r + 4 <= lo ? 0u : w[j] & (0xFFFFFFFFu << (8 * (lo - r)));     // before the range
                if (r + 4 > hi) w[j] = r >= hi ? 0u : w[j] & (0xFFFFFFFFu >> (8 * (r + 4 - hi))); // after it
                q = (j < 3 || st == kSteps - 1) ? T(sl, q ^ w[j]) : T(sh, q ^ w[j]);
            }
        }
    }
    uint32_t c = 0;
    if (any) {
        c = q ? multmodp(c_hop.lane16[lane], q) : 0u;
        for (int o = 32; o > 0; o >>= 1) c ^= __shfl_xor(c, o, 64);
    }
    // the strip's raw CRC at its end; P9b moves it to the range end (one thread per strip, so the
    // GF(2) products run on every lane instead of on lane 0 of each wave)
    if (lane == 0) B.strip_crc[(int64_t)blockIdx.x * 4 + wv] = c;
}

// P9b: every strip's CRC moved to its file's range end R1 -- x^(8 (R1 - E)), or x^(-8 (E - R1))
// for the strip holding R1 -- plus the init / final inversions once per file, XORed into the CRC.
__global__ void __launch_bounds__(256) k_pngb_crc_combine(PngBatch B, int64_t n_strips) {
    const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const bool live = g < n_strips;
    const int64_t blk = live ? g >> 2 : (n_strips - 1) >> 2;
    const int i = pngb_image(B, B.eblk0, B.eblk_per, blk);
    const PngImg& I = B.img[i];
    const PngMeta& M = B.meta[i];
    const int64_t lb = blk - (B.uniform ? (int64_t)i * B.eblk_per : I.eblk0);
    const int64_t S0 = lb * kPngbEmitCrcBytes + (g & 3) * (int64_t)kPngbEmitCrcStrip, E = S0 + kPngbEmitCrcStrip;
    const int64_t R0 = I.pre_len + 4, R1 = I.pre_len + 8 + M.zlen;
    // strips the emit skipped contribute 0 (no early return: the wave reduces below)
    const bool used = live && !(M.off < 0 || S0 >= M.file_len || E <= R0 || S0 >= R1);
    uint32_t c = used ? B.strip_crc[g] : 0u;
    if (c) {
        if (E <= R1) {                                  // x^(8 d), d = R1 - E = 256 jj + r
            const uint64_t d = (uint64_t)(R1 - E), jj = d >> 8, r = d & 255;
            if (r) c = multmodp(B.crc_pow[kCrcPowR + r], c);
            if (jj & (kCrcPowLo - 1)) c = multmodp(B.crc_pow[jj & (kCrcPowLo - 1)], c);
            if (jj >= kCrcPowLo) c = multmodp(B.crc_pow[kCrcPowLo + (jj / kCrcPowLo)], c);
        } else {                                        // the strip holding R1: x^(-8 t), t < the strip
            const uint64_t t = (uint64_t)(E - R1), a = t >> 8, r = t & 255;
            if (r) c = multmodp(B.crc_pow[kCrcInvR + r], c);
            if (a) c = multmodp(B.crc_pow[kCrcInvA + a], c);
        }
    }
    if (used && E >= R1) {                              // the init / final inversions: x^(8 n) from the tables
        const uint64_t n = (uint64_t)(R1 - R0), jj = n >> 8, r = n & 255;   // (x2nmodp's 21 dependent
        uint32_t x = B.crc_pow[kCrcPowR + r];                                // constant loads cost 40 us)
        if (jj & (kCrcPowLo - 1)) x = multmodp(B.crc_pow[jj & (kCrcPowLo - 1)], x);
        if (jj >= kCrcPowLo) x = multmodp(B.crc_pow[kCrcPowLo + (jj / kCrcPowLo)], x);
        c ^= ~multmodp(x, 0xFFFFFFFFu);
    }
    // one atomic per wave when its 64 strips are one file's (all but the waves at file seams):
    // 256 files' CRC words otherwise take every strip's atomic in turn
    const int i0 = __shfl(i, 0, 64);
    if (__ballot(i != i0) == 0) {
        for (int o = 32; o > 0; o >>= 1) c ^= __shfl_xor(c, o, 64);
        if ((threadIdx.x & 63) == 0 && c) atomicXor(&B.meta[i].crc, c);
    } else if (c) {
        atomicXor(&B.meta[i].crc, c);
    }
}
static_assert(kPngbEmitCrcStrip / 256 <= 64, "P8+P9: the inverse-power table covers a strip");

// P10: the CRC bytes after the zlib stream.
__global__ void __launch_bounds__(256) k_pngb_finish(PngBatch B) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= B.n) return;
    const PngMeta& M = B.meta[i];
    if (M.off < 0) return;
    uint8_t* c = B.out + M.off + B.img[i].pre_len + 8 + M.zlen;
    const uint32_t crc = M.crc;
    c[0] = crc >> 24; c[1] = crc >> 16; c[2] = crc >> 8; c[3] = crc;
}

// One image of a batch as the host describes it.
struct PngImgHost {
    const uint32_t* argb;
    const uint8_t* bits;
    int kind, W, H, flip_h, flip_v;
    uint8_t rgba[4];
};

static int png_prefix(int kind, int W, int H, const uint8_t* rgba, uint8_t* pre) {
    std::vector<uint8_t> v;
    const uint8_t sig[8] = {0x89, 'P', 'N', 'G', 0x0D, 0x0A, 0x1A, 0x0A};
    v.insert(v.end(), sig, sig + 8);
    uint8_t ihdr[13];
    ihdr[0] = W >> 24; ihdr[1] = W >> 16; ihdr[2] = W >> 8; ihdr[3] = W;
    ihdr[4] = H >> 24; ihdr[5] = H >> 16; ihdr[6] = H >> 8; ihdr[7] = H;
    ihdr[8] = kind == kIdx1 ? 1 : 8;
    ihdr[9] = kind == kRgb ? 2 : 3;   // truecolour / indexed
    ihdr[10] = ihdr[11] = ihdr[12] = 0;
    put_chunk(v, "IHDR", ihdr, 13);
    if (kind != kRgb) {
        const uint8_t plte[6] = {0, 0, 0, rgba[0], rgba[1], rgba[2]};
        put_chunk(v, "PLTE", plte, 6);
        const uint8_t trns[2] = {0, rgba[3]};
        put_chunk(v, "tRNS", trns, 2);
    }
    std::memcpy(pre, v.data(), v.size());
    return (int)v.size();
}

static omr_status ensure_crc_pow(Ctx* ctx) {
    if (ctx->d_crc_pow) return OMR_OK;
    OMR_HIP(ctx, hipMalloc(&ctx->d_crc_pow, sizeof(uint32_t) * kCrcPowAll));
    hipLaunchKernelGGL(k_png_crc_pow, dim3((kCrcPowAll + 255) / 256), dim3(256), 0, ctx->stream,
                       ctx->d_crc_pow);
    OMR_HIP(ctx, hipGetLastError());
    return OMR_OK;
}

// Geometry, grids and scratch layout of one batch (no pointers yet): plan_png_batch, then the
// caller sizes the workspace, then launch_png_batch.
struct PngBatchPlan {
    std::vector<PngImg> I;
    std::vector<int32_t> firsts;
    int64_t rows = 0, rblk = 0, pblk = 0, grp = 0, eblk = 0, cblk = 0, segs = 0, toks = 0, flt = 0, words = 0;
    size_t rows_lds = 16, parse_lds = 16;
    bool uniform = true;
    size_t o_img, o_first, o_flt, o_bh, o_poff, o_blk, o_trace, o_hist, o_tab, o_meta, o_rows, o_words, o_scrc;
    size_t scratch = 0;
};

static omr_status plan_png_batch(Ctx* ctx, const PngImgHost* im, int n, PngBatchPlan& L) {
    L.I.assign(n, PngImg{});
    L.firsts.assign(5 * (size_t)n, 0);
    for (int i = 0; i < n; ++i) {
        const PngImgHost& h = im[i];
        const PngPlan P = png_plan(h.kind, h.W, h.H);
        PngImg& d = L.I[i];
        d.kind = h.kind;
        d.W = h.W;
        d.H = h.H;
        d.flip_h = h.flip_h;
        d.flip_v = h.flip_v;
        d.bpp = h.kind == kRgb ? 3 : 1;
        d.rowlen = P.rowlen;
        d.raw = P.raw;
        d.nblk = P.nblk;
        d.nseg = (P.raw + kSeg - 1) / kSeg;
        d.back = (int32_t)align_up((size_t)std::min<int64_t>(std::max<int64_t>(P.rowlen, 2 * d.bpp), kMaxBack), 16);
        d.pre_len = png_prefix(h.kind, h.W, h.H, h.rgba, d.pre);
        const int64_t npb = (d.nseg + kParseLanes - 1) / kParseLanes, ng = (d.nseg + kPngbGroup - 1) / kPngbGroup;
        const int64_t max_file = d.pre_len + 8 + P.zlen + 4 + 12;
        const int64_t eb = png_direct() || png_crc_separate() ? kPngbEmitBytes : kPngbEmitCrcBytes;
        const int64_t ne = (max_file + eb - 1) / eb;
        const int64_t nc = (4 + P.zlen + kPngbCrcBytes - 1) / kPngbCrcBytes;
        if (L.rows + h.H > INT32_MAX || L.pblk + npb > INT32_MAX || L.grp + ng > INT32_MAX ||
            L.eblk + ne > INT32_MAX || L.cblk + nc > INT32_MAX)
            return fail(ctx, OMR_INVALID_ARGUMENT, "PNG batch too large");
        d.row0 = (int32_t)L.rows;
        d.rblk0 = (int32_t)L.rblk;
        d.pblk0 = (int32_t)L.pblk;
        d.grp0 = (int32_t)L.grp;
        d.eblk0 = L.eblk;
        d.cblk0 = L.cblk;
        d.seg0 = L.segs;
        d.tok0 = L.toks;
        d.flt = L.flt;
        d.words = L.words;
        L.firsts[i] = d.rblk0;
        L.firsts[n + i] = d.pblk0;
        L.firsts[2 * (size_t)n + i] = d.grp0;
        L.firsts[3 * (size_t)n + i] = (int32_t)d.eblk0;
        L.firsts[4 * (size_t)n + i] = (int32_t)d.cblk0;
        L.rows += h.H;
        L.rblk += (h.H + kPngRowsPerWg - 1) / kPngRowsPerWg;
        L.pblk += npb;
        L.grp += ng;
        L.eblk += ne;
        L.cblk += nc;
        L.segs += d.nseg;
        L.toks += tok_slots(d.nseg);
        L.flt += (int64_t)align_up((size_t)P.raw, 16);
        L.words += (int64_t)align_up((size_t)(P.raw / 2 + 128), 4);     // <= 16 bits per byte + header
        L.rows_lds = std::max(L.rows_lds, align_up((size_t)png_filter_lds(P.rowlen - 1) + 16, 16));
        if (i && (h.kind != im[0].kind || h.W != im[0].W || h.H != im[0].H)) L.uniform = false;
    }
    size_t o = 0;
    auto take = [&](size_t b) { const size_t r = o; o = align_up(o + b, 256); return r; };
    L.o_img = take(sizeof(PngImg) * n);
    L.o_first = take(sizeof(int32_t) * 5 * n);
    L.o_flt = take((size_t)L.flt + 64);              // P2 reads up to 48 bytes past an image's stream
    L.o_bh = take((size_t)L.pblk * 316 * 2);
    L.o_poff = take((size_t)L.pblk * 4 + (size_t)n * 4);
    L.o_blk = take((size_t)L.grp * 16);
    L.o_trace = take((size_t)L.segs * 12);
    L.o_hist = take((size_t)n * 316 * 4);
    L.o_tab = take(sizeof(DflTables) * n);
    L.o_meta = take(sizeof(PngMeta) * n);
    L.o_rows = take((size_t)L.rows * 16);
    L.o_words = take((size_t)L.words * 4 + 64);
    L.o_scrc = take((size_t)L.eblk * 16);
    L.scratch = o;
    return OMR_OK;
}

// Encode images[0..n) into d_out (asynchronous on the context stream).  Scratch: the workspace
// from ws_off on, already sized to ws_off + L.scratch (it must not hold the inputs).
static omr_status launch_png_batch(Ctx* ctx, PngBatchPlan& L, const PngImgHost* im, int n, size_t ws_off,
                                   uint8_t* d_out, size_t out_cap, uint64_t* d_offsets, uint32_t* d_lengths,
                                   int32_t* d_status) {
    if (n <= 0) return OMR_OK;
    omr_status st = ensure_crc_pow(ctx);
    if (st) return st;
    for (int i = 0; i < n; ++i) {
        L.I[i].argb = im[i].argb;
        L.I[i].bits = im[i].bits;
    }
    std::vector<PngImg>& I = L.I;
    std::vector<int32_t>& firsts = L.firsts;
    const int64_t pblk = L.pblk, grp = L.grp, eblk = L.eblk, cblk = L.cblk;
    const size_t rows_lds = L.rows_lds, parse_lds = L.parse_lds;
    const bool uniform = L.uniform;
    auto at = [&](size_t rel) { return ws_off + rel; };
    const size_t o_img = at(L.o_img), o_first = at(L.o_first), o_flt = at(L.o_flt),
                 o_blk = at(L.o_blk), o_hist = at(L.o_hist), o_tab = at(L.o_tab), o_meta = at(L.o_meta),
                 o_rows = at(L.o_rows), o_words = at(L.o_words), o_scrc = at(L.o_scrc);
    uint8_t* ws = static_cast<uint8_t*>(ctx->ws);
    PngBatch Bt{};
    Bt.img = reinterpret_cast<const PngImg*>(ws + o_img);
    Bt.n = n;
    Bt.uniform = uniform ? 1 : 0;
    Bt.rblk_per = (im[0].H + kPngRowsPerWg - 1) / kPngRowsPerWg;
    Bt.pblk_per = n > 1 ? I[1].pblk0 : (int32_t)pblk;
    Bt.grp_per = n > 1 ? I[1].grp0 : (int32_t)grp;
    Bt.eblk_per = n > 1 ? (int32_t)I[1].eblk0 : (int32_t)eblk;
    Bt.cblk_per = n > 1 ? (int32_t)I[1].cblk0 : (int32_t)cblk;
    Bt.total_grp = (int32_t)grp;
    const int32_t* fd = reinterpret_cast<const int32_t*>(ws + o_first);
    Bt.rblk0 = fd;
    Bt.pblk0 = fd + n;
    Bt.grp0 = fd + 2 * (size_t)n;
    Bt.eblk0 = fd + 3 * (size_t)n;
    Bt.cblk0 = fd + 4 * (size_t)n;
    Bt.flt = ws + o_flt;
    Bt.bh = reinterpret_cast<uint16_t*>(ws + at(L.o_bh));
    Bt.poff = reinterpret_cast<uint32_t*>(ws + at(L.o_poff));
    Bt.img_bits = Bt.poff + pblk;
    Bt.blk_b0 = reinterpret_cast<uint32_t*>(ws + o_blk);
    Bt.blk_b1 = Bt.blk_b0 + grp;
    Bt.blk_cf = Bt.blk_b1 + grp;
    Bt.blk_cl = Bt.blk_cf + grp;
    Bt.total_pblk = (int32_t)pblk;
    Bt.total_segs = L.segs;
    Bt.trace = reinterpret_cast<uint32_t*>(ws + at(L.o_trace));
    Bt.hist = reinterpret_cast<uint32_t*>(ws + o_hist);
    Bt.tab = reinterpret_cast<DflTables*>(ws + o_tab);
    Bt.meta = reinterpret_cast<PngMeta*>(ws + o_meta);
    Bt.row_sums = reinterpret_cast<unsigned long long*>(ws + o_rows);
    Bt.words = reinterpret_cast<uint32_t*>(ws + o_words);
    Bt.out = d_out;
    Bt.out_cap = out_cap;
    Bt.d_offsets = d_offsets;
    Bt.d_lengths = d_lengths;
    Bt.d_status = d_status;
    Bt.crc_pow = ctx->d_crc_pow;
    Bt.strip_crc = reinterpret_cast<uint32_t*>(ws + o_scrc);
    Bt.direct = png_direct() ? 1 : 0;
    st = stage_h2d2(ctx, ws + o_img, I.data(), sizeof(PngImg) * n, ws + o_first, firsts.data(),
                    sizeof(int32_t) * 5 * n);
    if (st) return st;
    OMR_HIP(ctx, hipMemsetAsync(ws + o_hist, 0, (size_t)n * 316 * 4, ctx->stream));
    if (rows_lds > (size_t)60 * 1024)
        OMR_HIP(ctx, hipFuncSetAttribute(reinterpret_cast<const void*>(k_pngb_filter),
                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)rows_lds + 1024));
    if (parse_lds > (size_t)40 * 1024) {
        OMR_HIP(ctx, hipFuncSetAttribute(reinterpret_cast<const void*>(k_pngb_parse),
                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)parse_lds + 2048));
    }
    hipStream_t s = ctx->stream;
    // D1: the wave form for uniform batches of RGB tiles up to 1024 wide (OMR_PNG_FILTER_WAVE=0: the
    // workgroup form, for measurement)
    const char* fw_env = std::getenv("OMR_PNG_FILTER_WAVE");        // read per call: tests A/B it
    const bool wave_filter = !(fw_env && *fw_env == '0');
    const int W0 = im[0].W, H0 = im[0].H;
    const int fw_m = (W0 / 4 + 63) / 64;
    // kernel timing (omr_ctx_enable_kernel_timing): kinds 20.. per stage, for bench.py's roofline
    // of the batched PNG pipeline
    {
        KernelTimer t_filter(ctx, 20);
        if (wave_filter && uniform && im[0].kind == kRgb && W0 % 4 == 0 && W0 <= 1024) {
            Bt.fw_bands = (H0 + kFilterBandRows - 1) / kFilterBandRows;
            const unsigned blocks = (unsigned)(((int64_t)n * Bt.fw_bands + 3) / 4);
            const bool full = W0 == 256 * fw_m;                // every lane's quads inside the row
            switch (fw_m * 2 + (full ? 1 : 0)) {
            case 2: hipLaunchKernelGGL((k_pngb_filter_wave<1, false>), dim3(blocks), dim3(256), fw_lds_bytes<1>(), s, Bt); break;
            case 3: hipLaunchKernelGGL((k_pngb_filter_wave<1, true>), dim3(blocks), dim3(256), fw_lds_bytes<1>(), s, Bt); break;
            case 4: hipLaunchKernelGGL((k_pngb_filter_wave<2, false>), dim3(blocks), dim3(256), fw_lds_bytes<2>(), s, Bt); break;
            case 5: hipLaunchKernelGGL((k_pngb_filter_wave<2, true>), dim3(blocks), dim3(256), fw_lds_bytes<2>(), s, Bt); break;
            case 6: hipLaunchKernelGGL((k_pngb_filter_wave<3, false>), dim3(blocks), dim3(256), fw_lds_bytes<3>(), s, Bt); break;
            case 7: hipLaunchKernelGGL((k_pngb_filter_wave<3, true>), dim3(blocks), dim3(256), fw_lds_bytes<3>(), s, Bt); break;
            case 8: hipLaunchKernelGGL((k_pngb_filter_wave<4, false>), dim3(blocks), dim3(256), fw_lds_bytes<4>(), s, Bt); break;
            default: hipLaunchKernelGGL((k_pngb_filter_wave<4, true>), dim3(blocks), dim3(256), fw_lds_bytes<4>(), s, Bt); break;
            }
        } else {
            hipLaunchKernelGGL(k_pngb_filter, dim3((unsigned)L.rblk), dim3(256), rows_lds, s, Bt);
        }
    }
    {
        KernelTimer t(ctx, 21);
        hipLaunchKernelGGL(k_pngb_parse, dim3((unsigned)pblk), dim3(kParseLanes), parse_lds, s, Bt);
        hipLaunchKernelGGL(k_pngb_hist, dim3((unsigned)(n * kHistParts)), dim3(320), 0, s, Bt);
    }
    {
        KernelTimer t(ctx, 22);
        hipLaunchKernelGGL(k_pngb_tables, dim3((unsigned)n), dim3(kHuffThreads), 0, s, Bt);
        hipLaunchKernelGGL(k_pngb_block_offsets, dim3((unsigned)n), dim3(kBoffThreads), 0, s, Bt);
    }
    if (Bt.direct) {
        // P5b, P6 (the files' lengths and offsets), P4 into the files, P5, P8 around the
        // streams, P9, P10 (timer kinds: 24 meta + offsets, 23 encode, 25 fixup + emit, 26 CRC)
        {
            KernelTimer t(ctx, 24);
            hipLaunchKernelGGL(k_pngb_meta, dim3((unsigned)n), dim3(256), 0, s, Bt);
            hipLaunchKernelGGL(k_pngb_offsets, dim3(1), dim3(1024), 0, s, Bt);
        }
        {
            KernelTimer t(ctx, 23);
            hipLaunchKernelGGL(k_pngb_encode, dim3((unsigned)grp), dim3(kPngbGroup), 0, s, Bt);
        }
        {
            KernelTimer t(ctx, 25);
            hipLaunchKernelGGL(k_pngb_fixup, dim3((unsigned)((grp + 255) / 256)), dim3(256), 0, s, Bt);
            hipLaunchKernelGGL(k_pngb_emit_direct, dim3((unsigned)(n * kEmitDirectWgs)), dim3(256), 0, s, Bt);
        }
        {
            KernelTimer t(ctx, 26);
            hipLaunchKernelGGL(k_pngb_crc, dim3((unsigned)cblk), dim3(256), 0, s, Bt);
            hipLaunchKernelGGL(k_pngb_finish, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, Bt);
        }
        OMR_HIP(ctx, hipGetLastError());
        return OMR_OK;
    }
    {
        KernelTimer t(ctx, 23);
        hipLaunchKernelGGL(k_pngb_encode, dim3((unsigned)grp), dim3(kPngbGroup), 0, s, Bt);
    }
    {
        KernelTimer t(ctx, 24);
        hipLaunchKernelGGL(k_pngb_fixup, dim3((unsigned)((grp + 255) / 256)), dim3(256), 0, s, Bt);
        hipLaunchKernelGGL(k_pngb_meta, dim3((unsigned)n), dim3(256), 0, s, Bt);
        hipLaunchKernelGGL(k_pngb_offsets, dim3(1), dim3(1024), 0, s, Bt);
    }
    {
        KernelTimer t(ctx, 25);
        if (png_crc_separate()) hipLaunchKernelGGL(k_pngb_emit, dim3((unsigned)eblk), dim3(256), 0, s, Bt);
        else hipLaunchKernelGGL(k_pngb_emit_crc, dim3((unsigned)eblk), dim3(256), 0, s, Bt);   // P8 + P9
    }
    KernelTimer t_crc(ctx, 26);
    if (png_crc_separate()) hipLaunchKernelGGL(k_pngb_crc, dim3((unsigned)cblk), dim3(256), 0, s, Bt);
    else hipLaunchKernelGGL(k_pngb_crc_combine, dim3((unsigned)((eblk * 4 + 255) / 256)), dim3(256), 0, s, Bt,
                            (int64_t)(eblk * 4));
    hipLaunchKernelGGL(k_pngb_finish, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, Bt);
    OMR_HIP(ctx, hipGetLastError());
    return OMR_OK;
}

// One image through the batched pipeline (n = 1; round 5): the single-request entry points use the
// same kernels as the batch -- device Huffman tables, no token buffers, one sync -- so a tile's
// file is the batch's byte for byte.  Workspace from `base`: [file slot][meta][batch scratch].
__global__ void __launch_bounds__(256) k_png_file_to_host(const uint8_t* __restrict__ src,
                                                          const uint32_t* __restrict__ d_len,
                                                          const int32_t* __restrict__ d_stat, uint8_t* __restrict__ host) {
    const uint32_t len = *d_stat == OMR_OK ? *d_len : 0u;
    const uint64_t i = ((uint64_t)blockIdx.x * 256 + threadIdx.x) * 16;
    if (i == 0) {
        reinterpret_cast<uint32_t*>(host)[0] = len;
        reinterpret_cast<int32_t*>(host)[1] = *d_stat;
    }
    if (i >= len) return;
    uint8_t* dst = host + 16;
    if (i + 16 <= len) {
        *reinterpret_cast<uint4*>(dst + i) = *reinterpret_cast<const uint4*>(src + i);
    } else {
        for (uint64_t j = i; j < len; ++j) dst[j] = src[j];
    }
}

struct PngSingleLayout {
    size_t o_out, o_meta, o_scr, fcap, total;
};

static omr_status png_single_layout(Ctx* ctx, const PngImgHost& im, size_t base, PngBatchPlan& L, PngSingleLayout& S) {
    omr_status st = plan_png_batch(ctx, &im, 1, L);
    if (st) return st;
    S.fcap = align_up(omr_png_max_bytes(im.W, im.H, im.kind == kRgb ? 3 : 1), 256);
    S.o_out = align_up(base, 256);
    S.o_meta = S.o_out + S.fcap;
    S.o_scr = S.o_meta + 256;
    S.total = S.o_scr + L.scratch;
    return OMR_OK;
}

// The caller has sized the workspace to S.total (a host-input caller stages its pixels below base).
static omr_status png_single_batched(Ctx* ctx, PngImgHost im, PngBatchPlan& L, const PngSingleLayout& S,
                                     uint8_t* out, size_t cap, size_t* out_len) {
    uint8_t* ws = static_cast<uint8_t*>(ctx->ws);
    uint64_t* d_off = reinterpret_cast<uint64_t*>(ws + S.o_meta);
    uint32_t* d_len = reinterpret_cast<uint32_t*>(ws + S.o_meta + 8);
    int32_t* d_st = reinterpret_cast<int32_t*>(ws + S.o_meta + 12);
    omr_status st = launch_png_batch(ctx, L, &im, 1, S.o_scr, ws + S.o_out, S.fcap, d_off, d_len, d_st);
    if (st) return st;
    st = ensure_host_out(ctx, S.fcap + 16);
    if (st) return st;
    hipLaunchKernelGGL(k_png_file_to_host, dim3((unsigned)((S.fcap + 16 * 256 - 1) / (16 * 256))), dim3(256), 0,
                       ctx->stream, ws + S.o_out, d_len, d_st, ctx->h_out);
    OMR_HIP(ctx, hipGetLastError());
    OMR_HIP(ctx, hipStreamSynchronize(ctx->stream));
    const uint32_t len = reinterpret_cast<volatile uint32_t*>(ctx->h_out)[0];
    const int32_t fst = reinterpret_cast<volatile int32_t*>(ctx->h_out)[1];
    if (fst != OMR_OK || len == 0) return fail(ctx, fst ? fst : OMR_INTERNAL, "PNG: the encode failed on the device");
    if (out_len) *out_len = len;
    if (!out || cap < len) return fail(ctx, OMR_BUFFER_TOO_SMALL, "PNG output buffer too small");
    std::memcpy(out, ctx->h_out + 16, len);
    return OMR_OK;
}

}  // namespace omr

using namespace omr;

extern "C" {

size_t omr_png_max_bytes(int32_t width, int32_t height, int32_t channels) {
    if (width <= 0 || height <= 0) return 256;
    const int kind = channels >= 3 ? kRgb : kIdx8;
    return 256 + (size_t)png_plan(kind, width, height).chunk_bytes;
}

omr_status omr_encode_png_device(omr_ctx* ctx, const uint32_t* d_argb, int32_t width, int32_t height, uint8_t* out,
                                 size_t cap, size_t* out_len) {
    if (!ctx) return OMR_INVALID_ARGUMENT;
    if (width <= 0 || height <= 0 || !d_argb) return fail(ctx, OMR_INVALID_ARGUMENT, "bad PNG input");
    OMR_HIP(ctx, hipSetDevice(ctx->device));
    if (width <= kPngbMaxSide && height <= kPngbMaxSide && ctx->png_single_batched) {
        const PngImgHost im{d_argb, nullptr, kRgb, width, height, 0, 0, {0, 0, 0, 0}};
        PngBatchPlan L;
        PngSingleLayout S;
        omr_status st = png_single_layout(ctx, im, 0, L, S);
        if (!st) st = ensure_workspace(ctx, S.total);
        return st ? st : png_single_batched(ctx, im, L, S, out, cap, out_len);
    }
    omr_status st = ensure_workspace(ctx, png_scratch(kRgb, width, height));
    if (st) return st;
    return encode_png_ws(ctx, kRgb, d_argb, nullptr, width, height, 0, 0, nullptr, 0, out, cap, out_len);
}

omr_status omr_encode_png(omr_ctx* ctx, const uint32_t* argb, int32_t width, int32_t height, uint8_t* out,
                          size_t cap, size_t* out_len) {
    if (!ctx) return OMR_INVALID_ARGUMENT;
    if (width <= 0 || height <= 0 || !argb) return fail(ctx, OMR_INVALID_ARGUMENT, "bad PNG input");
    OMR_HIP(ctx, hipSetDevice(ctx->device));
    const size_t img = align_up((size_t)width * height * 4, 256);
    if (width <= kPngbMaxSide && height <= kPngbMaxSide && ctx->png_single_batched) {
        PngImgHost im{nullptr, nullptr, kRgb, width, height, 0, 0, {0, 0, 0, 0}};
        PngBatchPlan L;
        PngSingleLayout S;
        omr_status st = png_single_layout(ctx, im, img, L, S);
        if (!st) st = ensure_workspace(ctx, S.total);          // before the pixels are staged
        if (st) return st;
        im.argb = static_cast<const uint32_t*>(ctx->ws);
        OMR_HIP(ctx, hipMemcpyAsync(ctx->ws, argb, (size_t)width * height * 4, hipMemcpyHostToDevice, ctx->stream));
        return png_single_batched(ctx, im, L, S, out, cap, out_len);
    }
    omr_status st = ensure_workspace(ctx, img + png_scratch(kRgb, width, height));
    if (st) return st;
    uint32_t* d = static_cast<uint32_t*>(ctx->ws);
    OMR_HIP(ctx, hipMemcpyAsync(d, argb, (size_t)width * height * 4, hipMemcpyHostToDevice, ctx->stream));
    return encode_png_ws(ctx, kRgb, d, nullptr, width, height, 0, 0, nullptr, img, out, cap, out_len);
}

omr_status omr_encode_png_batch_device(omr_ctx* ctx, const uint32_t* d_argb, int64_t tile_stride_px, int32_t n_tiles,
                                       int32_t width, int32_t height, uint8_t* d_out, size_t out_cap,
                                       uint64_t* d_offsets, uint32_t* d_lengths, int32_t* d_status) {
    if (!ctx) return OMR_INVALID_ARGUMENT;
    if (n_tiles < 0 || width <= 0 || height <= 0 || width > kPngbMaxSide || height > kPngbMaxSide)
        return fail(ctx, OMR_INVALID_ARGUMENT, "bad PNG batch size (tiles up to 4096 x 4096)");
    if (n_tiles == 0) return OMR_OK;
    if (!d_argb || !d_out) return fail(ctx, OMR_INVALID_ARGUMENT, "null PNG batch buffer");
    const int64_t px = (int64_t)width * height, stride = tile_stride_px ? tile_stride_px : px;
    if (stride < px) return fail(ctx, OMR_INVALID_ARGUMENT, "tile stride below width*height");
    OMR_HIP(ctx, hipSetDevice(ctx->device));
    std::vector<PngImgHost> im(n_tiles);
    for (int i = 0; i < n_tiles; ++i) im[i] = {d_argb + stride * i, nullptr, kRgb, width, height, 0, 0, {0, 0, 0, 0}};
    PngBatchPlan L;
    omr_status st = plan_png_batch(ctx, im.data(), n_tiles, L);
    if (st) return st;
    st = ensure_workspace(ctx, L.scratch);
    if (st) return st;
    return launch_png_batch(ctx, L, im.data(), n_tiles, 0, d_out, out_cap, d_offsets, d_lengths, d_status);
}

size_t omr_png_batch_max_bytes(int32_t width, int32_t height, int32_t channels, int32_t n) {
    if (n <= 0) return 0;
    return (size_t)n * align_up(omr_png_max_bytes(width, height, channels), 16);
}

omr_status omr_render_shape_mask_png_batch(omr_ctx* ctx, const omr_mask_job* jobs, int32_t n, uint8_t* out,
                                           size_t cap, uint64_t* offsets, uint32_t* lengths, int32_t* status) {
    if (!ctx) return OMR_INVALID_ARGUMENT;
    if (n < 0 || (n && (!jobs || !offsets || !lengths || !status)))
        return fail(ctx, OMR_INVALID_ARGUMENT, "bad mask batch arguments");
    if (n == 0) return OMR_OK;
    if (!out && cap) return fail(ctx, OMR_INVALID_ARGUMENT, "null output buffer");
    OMR_HIP(ctx, hipSetDevice(ctx->device));
    // Per mask: the single call's checks (each one the reference's 404, ShapeMaskVerticle.java:119-128)
    // and its packed-buffer flip (w % 8 == 0 with a flip, :175-181); masks whose stream would not fit
    // the batch's 32-bit bit offsets go through the single-mask path after the batch.
    std::vector<PngImgHost> im;
    std::vector<int> idx, big;
    std::vector<std::vector<uint8_t>> flipped(n);
    std::vector<size_t> boff;
    size_t bits_total = 0;
    for (int i = 0; i < n; ++i) {
        const omr_mask_job& j = jobs[i];
        offsets[i] = 0;
        lengths[i] = 0;
        status[i] = OMR_OK;
        const int64_t npx = (int64_t)j.width * j.height;
        if (j.width <= 0 || j.height <= 0 || npx > INT32_MAX || !j.bits || (int64_t)j.n_bytes * 8 < npx) {
            status[i] = OMR_NOT_FOUND;
            continue;
        }
        const uint8_t* bits = j.bits;
        int fh = j.flip_h ? 1 : 0, fv = j.flip_v ? 1 : 0;
        if (j.width % 8 == 0 && (fh || fv) && !(ctx->sem & OMR_SEM_MASK_PIXEL_FLIP)) {
            if ((int64_t)j.n_bytes < npx) {        // ArrayIndexOutOfBoundsException in the packed flip
                status[i] = OMR_NOT_FOUND;
                continue;
            }
            std::vector<uint8_t>& f = flipped[i];
            f.assign(j.n_bytes, 0);
            for (int64_t y = 0; y < j.height; ++y) {
                const int64_t drow = (fv ? j.height - 1 - y : y) * j.width;
                for (int64_t x = 0; x < j.width; ++x) f[drow + (fh ? j.width - 1 - x : x)] = j.bits[y * j.width + x];
            }
            bits = f.data();
            fh = fv = 0;
        }
        const int kind = j.width % 8 == 0 ? kIdx1 : kIdx8;
        const PngPlan P = png_plan(kind, j.width, j.height);
        // > 2^31 bits worst case, or a row too wide for the batch filter's LDS: the single path
        // (which answers the too-wide row for this mask alone)
        if (P.raw > ((int64_t)1 << 27) ||
            align_up((size_t)png_filter_lds(P.rowlen - 1) + 16, 16) > (size_t)kPngFilterLdsMax + 64) {
            big.push_back(i);
            continue;
        }
        PngImgHost h{nullptr, bits, kind, j.width, j.height, fh, fv, {j.rgba[0], j.rgba[1], j.rgba[2], j.rgba[3]}};
        im.push_back(h);
        idx.push_back(i);
        boff.push_back(bits_total);
        bits_total += align_up((size_t)((npx + 7) / 8), 16);
    }
    const int m = (int)im.size();
    size_t used = 0;
    if (m) {
        PngBatchPlan L;
        omr_status st = plan_png_batch(ctx, im.data(), m, L);
        if (st) return st;
        size_t dcap = 0;
        for (int k = 0; k < m; ++k) dcap += align_up(omr_png_max_bytes(im[k].W, im[k].H, 1), 16);
        dcap = std::min(dcap, cap & ~(size_t)15);      // whole 16-byte slots inside the caller's buffer
        const size_t o_bits = 0, o_out = align_up(bits_total, 256), o_meta = o_out + align_up(dcap, 256);
        const size_t o_scr = o_meta + align_up((size_t)m * 16, 256);
        st = ensure_workspace(ctx, o_scr + L.scratch);
        if (st) return st;
        st = ensure_host_out(ctx, std::max(bits_total, (size_t)m * 16));
        if (st) return st;
        uint8_t* ws = static_cast<uint8_t*>(ctx->ws);
        for (int k = 0; k < m; ++k) {
            const size_t nb = (size_t)(((int64_t)im[k].W * im[k].H + 7) / 8);
            std::memcpy(ctx->h_out + boff[k], im[k].bits, nb);
            im[k].bits = ws + o_bits + boff[k];
        }
        OMR_HIP(ctx, hipMemcpyAsync(ws + o_bits, ctx->h_out, bits_total, hipMemcpyHostToDevice, ctx->stream));
        uint64_t* d_off = reinterpret_cast<uint64_t*>(ws + o_meta);
        uint32_t* d_len = reinterpret_cast<uint32_t*>(d_off + m);
        int32_t* d_st = reinterpret_cast<int32_t*>(d_len + m);
        st = launch_png_batch(ctx, L, im.data(), m, o_scr, ws + o_out, dcap, d_off, d_len, d_st);
        if (st) return st;
        OMR_HIP(ctx, hipMemcpyAsync(ctx->h_out, d_off, (size_t)m * 16, hipMemcpyDeviceToHost, ctx->stream));
        OMR_HIP(ctx, hipStreamSynchronize(ctx->stream));
        const uint64_t* h_off = reinterpret_cast<const uint64_t*>(ctx->h_out);
        const uint32_t* h_len = reinterpret_cast<const uint32_t*>(h_off + m);
        const int32_t* h_st = reinterpret_cast<const int32_t*>(h_len + m);
        for (int k = 0; k < m; ++k) {
            const int i = idx[k];
            status[i] = h_st[k];
            if (h_st[k] == OMR_OK) {
                offsets[i] = h_off[k];
                lengths[i] = h_len[k];
                used = std::max<size_t>(used, align_up(h_off[k] + h_len[k], 16));
            }
        }
        if (used) OMR_HIP(ctx, hipMemcpy(out, ws + o_out, used, hipMemcpyDeviceToHost));
    }
    for (int i : big) {                                 // rare: huge masks one at a time, appended
        size_t len = 0;
        const omr_mask_job& j = jobs[i];
        const omr_status st = omr_render_shape_mask_png(ctx, j.bits, j.n_bytes, j.width, j.height, j.rgba, j.flip_h,
                                                        j.flip_v, used < cap ? out + used : nullptr,
                                                        used < cap ? cap - used : 0, &len);
        status[i] = st;
        if (st == OMR_OK) {
            offsets[i] = used;
            lengths[i] = (uint32_t)len;
            used = align_up(used + len, 16);
        } else if (st != OMR_BUFFER_TOO_SMALL && st != OMR_NOT_FOUND && st != OMR_INVALID_ARGUMENT) {
            return st;                                  // a device failure fails the call
        }
    }
    return OMR_OK;
}

omr_status omr_render_shape_mask_png(omr_ctx* ctx, const uint8_t* bits, size_t n_bytes, int32_t width,
                                     int32_t height, const uint8_t rgba[4], int32_t flip_h, int32_t flip_v,
                                     uint8_t* out, size_t cap, size_t* out_len) {
    if (!ctx) return OMR_INVALID_ARGUMENT;
    if (!rgba) return fail(ctx, OMR_INVALID_ARGUMENT, "null fill colour");
    // Every exception the reference raises inside renderShapeMask fails its future, which
    // ShapeMaskVerticle.java:119-128 answers with 404 ("Cannot render Mask").
    if (width <= 0 || height <= 0) return fail(ctx, OMR_NOT_FOUND, "Attempted to flip image with 0 size");
    const int64_t npx = (int64_t)width * height;
    if (npx > INT32_MAX) return fail(ctx, OMR_NOT_FOUND, "width*height overflows a Java int");
    if (!bits) return fail(ctx, OMR_NOT_FOUND, "NullPointerException: null mask bytes");
    if ((int64_t)n_bytes * 8 < npx) return fail(ctx, OMR_NOT_FOUND, "mask shorter than width*height bits");
    // width % 8 == 0: the reference skips the unpack (:175-178) and flips the still-packed buffer as
    // one byte per pixel (:179-181, :145-150) unless OMR_SEM_MASK_PIXEL_FLIP asks for the pixel flip
    std::vector<uint8_t> packed_flip;
    if (width % 8 == 0 && (flip_h || flip_v) && !(ctx->sem & OMR_SEM_MASK_PIXEL_FLIP)) {
        if ((int64_t)n_bytes < npx)
            return fail(ctx, OMR_NOT_FOUND, "ArrayIndexOutOfBoundsException: flip of the packed mask reads " +
                                                std::to_string(npx) + " bytes of " + std::to_string(n_bytes));
        packed_flip.assign(n_bytes, 0);   // new byte[src.length]; bytes past width*height stay 0
        for (int64_t y = 0; y < height; ++y) {
            const int64_t drow = (flip_v ? height - 1 - y : y) * width;
            for (int64_t x = 0; x < width; ++x) packed_flip[drow + (flip_h ? width - 1 - x : x)] = bits[y * width + x];
        }
        bits = packed_flip.data();        // rendered as packed bits, no further flip
        flip_h = flip_v = 0;
    }
    OMR_HIP(ctx, hipSetDevice(ctx->device));
    const int kind = width % 8 == 0 ? kIdx1 : kIdx8;   // bitsPerPixel 1 or 8 (:174-178)
    const PngPlan P1 = png_plan(kind, width, height);
    if (ctx->png_single_batched && P1.raw <= ((int64_t)1 << 27) &&
        align_up((size_t)png_filter_lds(P1.rowlen - 1) + 16, 16) <= (size_t)kPngFilterLdsMax + 64) {
        // the batch of one (the mask bits go to the workspace below base; packed flip done above)
        const size_t nbits = align_up((size_t)((npx + 7) / 8), 256);
        PngImgHost im{nullptr, nullptr, kind, width, height, flip_h ? 1 : 0, flip_v ? 1 : 0,
                      {rgba[0], rgba[1], rgba[2], rgba[3]}};
        PngBatchPlan L;
        PngSingleLayout S;
        omr_status st = png_single_layout(ctx, im, nbits, L, S);
        if (!st) st = ensure_workspace(ctx, S.total);
        if (st) return st;
        im.bits = static_cast<const uint8_t*>(ctx->ws);
        OMR_HIP(ctx, hipMemcpyAsync(ctx->ws, bits, (size_t)((npx + 7) / 8), hipMemcpyHostToDevice, ctx->stream));
        return png_single_batched(ctx, im, L, S, out, cap, out_len);
    }
    const size_t nb = align_up(n_bytes, 256);
    omr_status st = ensure_workspace(ctx, nb + png_scratch(kind, width, height));
    if (st) return st;
    uint8_t* d_bits = static_cast<uint8_t*>(ctx->ws);
    OMR_HIP(ctx, hipMemcpyAsync(d_bits, bits, n_bytes, hipMemcpyHostToDevice, ctx->stream));
    return encode_png_ws(ctx, kind, nullptr, d_bits, width, height, flip_h ? 1 : 0, flip_v ? 1 : 0, rgba, nb, out,
                         cap, out_len);
}

}  // extern "C"
