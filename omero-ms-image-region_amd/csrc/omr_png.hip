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

__device__ __forceinline__ uint32_t raw_byte(const PngArgs& A, int64_t i) {
    const int64_t row = i / A.rowlen, col = i - row * A.rowlen;
    if (col == 0) return 0;
    const int64_t c = col - 1;
    if (A.kind == kRgb) {
        const int64_t px = c / 3;
        const uint32_t p = A.argb[row * A.W + px];
        return (p >> (16 - 8 * (c - px * 3))) & 0xFF;
    }
    if (A.kind == kIdx8) return mask_bit(A, (int)c, (int)row);
    uint32_t b = 0;
    for (int k = 0; k < 8; ++k) b = (b << 1) | mask_bit(A, (int)(c * 8 + k), (int)row);
    return b;
}

// One lane per zlib-stream byte (header, stored-block headers, payload) + Adler partials.
__global__ void __launch_bounds__(256) k_png_layout(PngArgs A) {
    if (A.meta[1] == 0) return;                     // the dynamic stream was chosen
    unsigned long long s1 = 0, s2 = 0;
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
                const int64_t i = b * kStored + (o - 5);
                v = raw_byte(A, i);
                s1 += v;
                s2 += (unsigned long long)(A.raw - i) * v;
            }
        }
        z[j] = (uint8_t)v;
    }
    // block reduction of the Adler partials
    for (int o = 32; o > 0; o >>= 1) {
        s1 += __shfl_down(s1, o, 64);
        s2 += __shfl_down(s2, o, 64);
    }
    if ((threadIdx.x & 63) == 0 && (s1 | s2)) {
        atomicAdd(&A.sums[0], s1);
        atomicAdd(&A.sums[1], s2);
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

// LDS: the raw bytes of this row and the row above (2 * (rowlen - 1) bytes, dynamic); every
// filter residual is then computed from LDS.
__global__ void __launch_bounds__(256) k_png_filter(DflArgs D) {
    extern __shared__ __attribute__((aligned(16))) uint8_t s_rows[];
    __shared__ uint32_t s_sum[5][4];
    __shared__ int s_f;
    const PngArgs& A = D.P;
    const int y = blockIdx.x;
    const int rb = (int)A.rowlen - 1, bpp = D.bpp;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint8_t* cur = s_rows;
    uint8_t* prev = s_rows + rb;
    if (A.kind == kRgb) {                         // one ARGB load per pixel and row
        for (int px = threadIdx.x; px < A.W; px += 256) {
            const uint32_t v = A.argb[(int64_t)y * A.W + px];
            cur[3 * px] = (uint8_t)(v >> 16); cur[3 * px + 1] = (uint8_t)(v >> 8); cur[3 * px + 2] = (uint8_t)v;
            const uint32_t u = y > 0 ? A.argb[(int64_t)(y - 1) * A.W + px] : 0u;
            prev[3 * px] = (uint8_t)(u >> 16); prev[3 * px + 1] = (uint8_t)(u >> 8); prev[3 * px + 2] = (uint8_t)u;
        }
    } else {
        for (int i = threadIdx.x; i < rb; i += 256) {
            cur[i] = (uint8_t)row_byte(A, y, i);
            prev[i] = y > 0 ? (uint8_t)row_byte(A, y - 1, i) : (uint8_t)0;
        }
    }
    __syncthreads();
    uint32_t sm[5] = {0, 0, 0, 0, 0};
    auto filt = [&](int i, uint32_t (&f)[5]) {
        const uint32_t x = cur[i];
        const uint32_t a = i >= bpp ? cur[i - bpp] : 0u;
        const uint32_t b = prev[i];
        const uint32_t c = i >= bpp ? prev[i - bpp] : 0u;
        f[0] = x;
        f[1] = (x - a) & 0xFF;
        f[2] = (x - b) & 0xFF;
        f[3] = (x - ((a + b) >> 1)) & 0xFF;
        f[4] = (x - paeth(a, b, c)) & 0xFF;
    };
    for (int i = threadIdx.x; i < rb; i += 256) {
        uint32_t f[5];
        filt(i, f);
#pragma unroll
        for (int k = 0; k < 5; ++k) sm[k] += min(f[k], 256u - f[k]);
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
    }
    __syncthreads();
    const int f = s_f;
    const int64_t row0 = (int64_t)y * A.rowlen;
    unsigned long long s1 = 0, s2 = 0;
    if (threadIdx.x == 0) {
        D.flt[row0] = (uint8_t)f;
        s1 += (unsigned long long)f;
        s2 += (unsigned long long)(A.raw - row0) * (unsigned long long)f;
    }
    for (int i = threadIdx.x; i < rb; i += 256) {
        uint32_t fv[5];
        filt(i, fv);
        const uint32_t v = fv[f];
        const int64_t idx = row0 + 1 + i;
        D.flt[idx] = (uint8_t)v;
        s1 += v;
        s2 += (unsigned long long)(A.raw - idx) * v;
    }
    for (int o = 32; o > 0; o >>= 1) {
        s1 += __shfl_down(s1, o, 64);
        s2 += __shfl_down(s2, o, 64);
    }
    __shared__ unsigned long long s_ad[2][4];
    if (lane == 0) { s_ad[0][wv] = s1; s_ad[1][wv] = s2; }
    __syncthreads();
    if (threadIdx.x == 0) {      // per-row Adler partials; summed by k_png_adler_rows
        D.row_sums[2 * y] = s_ad[0][0] + s_ad[0][1] + s_ad[0][2] + s_ad[0][3];
        D.row_sums[2 * y + 1] = s_ad[1][0] + s_ad[1][1] + s_ad[1][2] + s_ad[1][3];
    }
}

// Sum of the per-row Adler partials into A.sums (one workgroup; dynamic stream only).
__global__ void __launch_bounds__(256) k_png_adler_rows(DflArgs D) {
    if (D.P.meta[1]) return;
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
constexpr int kMaxBack = 31 * 1024;         // LDS look-back window (bytes)

// One lane per kSeg-byte segment; the workgroup first stages its 32 KiB of filtered stream plus
// the look-back window (one image row, <= 31 KiB) in LDS, so the greedy parse's byte compares
// are LDS reads instead of dependent global loads.
__global__ void __launch_bounds__(kParseLanes) k_png_lz_parse(DflArgs D, int32_t back) {
    extern __shared__ __attribute__((aligned(16))) uint8_t s_win[];
    __shared__ uint32_t lh[286], dh[30];
    for (int i = threadIdx.x; i < 286; i += kParseLanes) lh[i] = 0;
    if (threadIdx.x < 30) dh[threadIdx.x] = 0;
    const int64_t bbeg = (int64_t)blockIdx.x * kParseLanes * kSeg;
    const int64_t bend = min(D.P.raw, bbeg + (int64_t)kParseLanes * kSeg);
    const int64_t wbeg = max((int64_t)0, bbeg - back);          // back is a multiple of 16
    const int64_t n16 = (bend - wbeg) / 16;
    const uint4* g16 = reinterpret_cast<const uint4*>(D.flt + wbeg);
    for (int64_t i = threadIdx.x; i < n16; i += kParseLanes) reinterpret_cast<uint4*>(s_win)[i] = g16[i];
    for (int64_t i = wbeg + n16 * 16 + threadIdx.x; i < bend; i += kParseLanes) s_win[i - wbeg] = D.flt[i];
    __syncthreads();
    const int64_t s = (int64_t)blockIdx.x * kParseLanes + threadIdx.x;
    if (s < D.nseg) {
        const uint8_t* f = s_win - wbeg;            // f[p] for p in [wbeg, bend)
        const int64_t beg = s * kSeg, end = min(D.P.raw, beg + kSeg);
        const int64_t rowlen = D.P.rowlen;
        const int64_t cand[4] = {1, D.bpp, 2 * D.bpp, rowlen};
        const int nc = D.bpp == 1 ? 2 : 3;
        uint32_t* tok = D.tokens + beg;
        int nt = 0;
        int64_t p = beg;
        while (p < end) {
            const int64_t lim = min((int64_t)258, end - p);
            int64_t best = 0, bd = 0;
            const uint32_t x0 = f[p];
            for (int k = 0; k < 4; ++k) {
                if (k >= nc && k != 3) continue;
                const int64_t d = cand[k];
                if (d > p - wbeg || d > back) continue;   // inside the staged window
                if (f[p - d] != x0) continue;
                int64_t l = 1;
                while (l < lim && f[p + l] == f[p - d + l]) ++l;
                if (l > best) { best = l; bd = d; }
                if (best == lim) break;
            }
            if (best >= 3) {
                tok[nt++] = 0x80000000u | (uint32_t)(best - 3) | ((uint32_t)(bd - 1) << 8);
                atomicAdd(&lh[c_dfl.len_sym[best]], 1u);
                atomicAdd(&dh[dist_sym((uint32_t)bd)], 1u);
                p += best;
            } else {
                tok[nt++] = x0;
                atomicAdd(&lh[x0], 1u);
                ++p;
            }
        }
        D.ntok[s] = (uint16_t)nt;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < 286; i += kParseLanes)
        if (lh[i]) atomicAdd(&D.lhist[i], lh[i]);
    if (threadIdx.x < 30 && dh[threadIdx.x]) atomicAdd(&D.dhist[threadIdx.x], dh[threadIdx.x]);
}

// ---- D3 on the device: the code is a function of two small histograms (286 + 30 counts); one
// workgroup builds it between D2 and D4, so an encode needs no host round trip mid-pipeline.
// The parallel steps (ranking, depths, length assignment, canonical codes) use every lane; the
// two-queue merge, the Kraft repair and the run-length header are short serial loops on lane 0.

// The table block D4/D5 read: codes, lengths and the block header bits.
struct DflTables {
    uint16_t lcode[286];
    uint16_t dcode[30];
    uint8_t llen[286];
    uint8_t dlen[30];
    uint32_t hdr[96];        // header bits LSB-first; hdr[95] = bit count
};

constexpr int kHuffMaxSym = 288;
constexpr int kHuffThreads = 320;       // one symbol per thread (286 + 30 + 19 symbols: <= 286)
struct HuffWork {                       // LDS scratch of one tree
    alignas(16) uint32_t f[kHuffMaxSym];   // symbol frequencies
    uint32_t wt[2 * kHuffMaxSym];       // leaf weights (sorted), then merged nodes
    int16_t ord[kHuffMaxSym];           // used symbols by (frequency, symbol)
    int16_t parent[2 * kHuffMaxSym];
    uint8_t len[kHuffMaxSym];
    int bl[17];                         // leaves per code length
    int next[17];
    int wcnt[kHuffThreads / 64][16];    // per wave: symbols of each code length
    int m;
};

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
    for (int i = tid; i < n; i += nt) {
        const uint32_t fi = W.f[i];
        W.len[i] = 0;
        if (fi) {                                   // rank among the used symbols (stable order)
            int r = 0;
            const int n4 = n & ~3;
            const uint4* f4 = reinterpret_cast<const uint4*>(W.f);
#pragma unroll 4
            for (int j = 0; j < n4; j += 4) {       // four broadcast reads per LDS access
                const uint4 v = f4[j >> 2];
                r += (v.x != 0u && (v.x < fi || (v.x == fi && j < i))) ? 1 : 0;
                r += (v.y != 0u && (v.y < fi || (v.y == fi && j + 1 < i))) ? 1 : 0;
                r += (v.z != 0u && (v.z < fi || (v.z == fi && j + 2 < i))) ? 1 : 0;
                r += (v.w != 0u && (v.w < fi || (v.w == fi && j + 3 < i))) ? 1 : 0;
            }
            for (int j = n4; j < n; ++j) {
                const uint32_t fj = W.f[j];
                r += (fj != 0u && (fj < fi || (fj == fi && j < i))) ? 1 : 0;
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
    for (int k = tid; k < m; k += nt) W.wt[k] = W.f[W.ord[k]];
    __syncthreads();
    if (tid == 0) {                                 // two queues: sorted leaves, merged nodes
        // the two heads of each queue are read together (one LDS round trip per merge); a leaf
        // wins ties, as wt[li] <= wt[qi] does
        constexpr uint32_t kInf = 0xFFFFFFFFu;       // weights stay below it (< 2^31 bytes)
        int li = 0, qi = m, qn = m;
        for (int c = 0; c < m - 1; ++c) {
            const uint32_t a = li < m ? W.wt[li] : kInf, b = li + 1 < m ? W.wt[li + 1] : kInf;
            const uint32_t q0 = qi < qn ? W.wt[qi] : kInf, q1 = qi + 1 < qn ? W.wt[qi + 1] : kInf;
            int p0, p1;
            uint32_t w0, w1;
            if (a <= q0) {                          // first: leaf li; second: leaf li+1 or node qi
                p0 = li; w0 = a;
                if (b <= q0) { p1 = li + 1; w1 = b; li += 2; }
                else { p1 = qi; w1 = q0; li += 1; qi += 1; }
            } else {                                // first: node qi; second: leaf li or node qi+1
                p0 = qi; w0 = q0;
                if (a <= q1) { p1 = li; w1 = a; li += 1; qi += 1; }
                else { p1 = qi + 1; w1 = q1; qi += 2; }
            }
            W.wt[qn] = w0 + w1;
            W.parent[p0] = W.parent[p1] = (int16_t)qn;
            ++qn;
        }
    }
    __syncthreads();
    const int root = 2 * m - 2;
    for (int k = tid; k < m; k += nt) {             // leaf depth: walk up to the root
        int d = 0;
        for (int x = k; x != root; x = W.parent[x]) ++d;
        atomicAdd(&W.bl[min(d, maxbits)], 1);
    }
    __syncthreads();
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
__global__ void __launch_bounds__(kHuffThreads) k_png_tables(const uint32_t* __restrict__ hist, DflTables* __restrict__ T) {
    __shared__ HuffWork W;
    __shared__ DflTables t;
    __shared__ uint8_t seq[286 + 30];
    __shared__ uint8_t rs[286 + 30], rx[286 + 30];   // run-length symbols and their extra bits
    __shared__ int s_nr, s_hlit, s_hdist;
    const int tid = threadIdx.x;
    for (int i = tid; i < 286; i += kHuffThreads) W.f[i] = hist[i] + (i == 256 ? 1u : 0u);   // + EOB
    huff_lengths_dev(W, 286, kMaxBits);
    for (int i = tid; i < 286; i += kHuffThreads) t.llen[i] = W.len[i];
    huff_canon_dev(W, 286, t.lcode);
    if (tid < 30) W.f[tid] = hist[286 + tid];
    huff_lengths_dev(W, 30, kMaxBits);
    if (tid < 30) t.dlen[tid] = W.len[tid];
    huff_canon_dev(W, 30, t.dcode);
    if (tid == 0) {                                 // zlib trees.c scan_tree over the lengths
        int hlit = 286, hdist = 30;
        while (hlit > 257 && t.llen[hlit - 1] == 0) --hlit;
        while (hdist > 1 && t.dlen[hdist - 1] == 0) --hdist;
        for (int i = 0; i < hlit; ++i) seq[i] = t.llen[i];
        for (int i = 0; i < hdist; ++i) seq[hlit + i] = t.dlen[i];
        const int ns = hlit + hdist;
        int nr = 0;
        for (int i = 0; i < ns;) {
            const int v = seq[i];
            int r = 1;
            while (i + r < ns && seq[i + r] == v) ++r;
            if (v == 0 && r >= 3) {
                const int k = min(r, 138);
                rs[nr] = k >= 11 ? 18 : 17;
                rx[nr++] = (uint8_t)(k >= 11 ? k - 11 : k - 3);
                i += k;
            } else if (v != 0 && r >= 4) {
                const int k = min(r - 1, 6);
                rs[nr] = (uint8_t)v; rx[nr++] = 0;
                rs[nr] = 16; rx[nr++] = (uint8_t)(k - 3);
                i += 1 + k;
            } else {
                rs[nr] = (uint8_t)v; rx[nr++] = 0;
                ++i;
            }
        }
        s_nr = nr; s_hlit = hlit; s_hdist = hdist;
    }
    if (tid < 19) W.f[tid] = 0;
    __syncthreads();
    const int nr = s_nr;
    for (int i = tid; i < nr; i += kHuffThreads) atomicAdd(&W.f[rs[i]], 1u);
    huff_lengths_dev(W, 19, 7);
    __shared__ uint16_t ccode[19];
    huff_canon_dev(W, 19, ccode);
    for (int i = tid; i < 96; i += kHuffThreads) t.hdr[i] = 0;
    // each run-length entry's code + extra bits (LSB-first: the code, then the extra), in parallel
    __shared__ uint16_t ev[286 + 30];
    __shared__ uint8_t en[286 + 30];
    for (int i = tid; i < nr; i += kHuffThreads) {
        const int sym = rs[i];
        const int xb = sym == 16 ? 2 : sym == 17 ? 3 : sym == 18 ? 7 : 0;
        ev[i] = (uint16_t)(ccode[sym] | ((uint32_t)rx[i] << W.len[sym]));
        en[i] = (uint8_t)(W.len[sym] + xb);
    }
    __syncthreads();
    if (tid == 0) {                                 // block header, LSB-first
        static constexpr uint8_t kOrd[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
        int hclen = 19;
        while (hclen > 4 && W.len[kOrd[hclen - 1]] == 0) --hclen;
        uint32_t nb = 0;
        uint64_t acc = 0;                           // pending bits, LSB-first; whole words out
        auto put = [&](uint32_t v, int n) {
            acc |= (uint64_t)(v & ((1u << n) - 1u)) << (nb & 31);   // n <= 14
            nb += n;
            if ((nb >> 5) != ((nb - n) >> 5)) { t.hdr[(nb - n) >> 5] = (uint32_t)acc; acc >>= 32; }
        };
        put(1, 1);                                  // BFINAL
        put(2, 2);                                  // BTYPE = 10 (dynamic)
        put((uint32_t)(s_hlit - 257), 5);
        put((uint32_t)(s_hdist - 1), 5);
        put((uint32_t)(hclen - 4), 4);
        for (int i = 0; i < hclen; ++i) put(W.len[kOrd[i]], 3);
        for (int i = 0; i < nr; ++i) put(ev[i], en[i]);
        if (nb & 31) t.hdr[nb >> 5] = (uint32_t)acc;
        t.hdr[95] = nb;
    }
    __syncthreads();
    const uint32_t* src = reinterpret_cast<const uint32_t*>(&t);
    uint32_t* dst = reinterpret_cast<uint32_t*>(T);
    for (int i = tid; i < (int)(sizeof(DflTables) / 4); i += kHuffThreads) dst[i] = src[i];
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
    const uint32_t l = (t & 0xFF) + 3, d = ((t >> 8) & 0x7FFF) + 1;
    const int ls = c_dfl.len_sym[l], ds = dist_sym(d);
    return llen[ls] + c_dfl.len_xbits[ls - 257] + dlen[ds] + c_dfl.dist_xbits[ds];
}

__global__ void __launch_bounds__(256) k_png_lz_bits(DflArgs D) {
    __shared__ uint8_t llen[286], dlen[30];
    for (int i = threadIdx.x; i < 286; i += 256) llen[i] = D.tab->llen[i];
    if (threadIdx.x < 30) dlen[threadIdx.x] = D.tab->dlen[threadIdx.x];
    __syncthreads();
    const int64_t s = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (s >= D.nseg) return;
    const uint32_t* tok = D.tokens + s * kSeg;
    const int nt = D.ntok[s];
    uint32_t b = 0;
    for (int i = 0; i < nt; ++i) b += token_bits(tok[i], llen, dlen);
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
    const uint32_t* tok = D.tokens + s * kSeg;
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
    for (int i = 0; i < nt; ++i) {
        const uint32_t t = tok[i];
        if (!(t & 0x80000000u)) {
            put(lcode[t], llen[t]);
        } else {
            const uint32_t l = (t & 0xFF) + 3, d = ((t >> 8) & 0x7FFF) + 1;
            const int ls = c_dfl.len_sym[l], ds = dist_sym(d);
            put(lcode[ls], llen[ls]);
            if (c_dfl.len_xbits[ls - 257]) put(l - c_dfl.len_base[ls - 257], c_dfl.len_xbits[ls - 257]);
            put(dcode[ds], dlen[ds]);
            if (c_dfl.dist_xbits[ds]) put(d - c_dfl.dist_base[ds], c_dfl.dist_xbits[ds]);
        }
    }
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
    L.tokens = take((size_t)P.raw * 4);
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
    const size_t rows_lds = align_up(2 * (size_t)(P.rowlen - 1), 16);
    if (rows_lds > (size_t)150 * 1024) return fail(ctx, OMR_INVALID_ARGUMENT, "PNG row too wide");
    if (P.chunk_bytes >= ((int64_t)1 << 31)) return fail(ctx, OMR_INVALID_ARGUMENT, "PNG image too large");
    if (rows_lds > (size_t)60 * 1024)
        OMR_HIP(ctx, hipFuncSetAttribute(reinterpret_cast<const void*>(k_png_filter),
                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)rows_lds + 1024));
    hipLaunchKernelGGL(k_png_filter, dim3((unsigned)H), dim3(256), rows_lds, ctx->stream, D);
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
    hipLaunchKernelGGL(k_png_layout, dim3(gl), dim3(256), 0, ctx->stream, A);
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
    omr_status st = ensure_workspace(ctx, img + png_scratch(kRgb, width, height));
    if (st) return st;
    uint32_t* d = static_cast<uint32_t*>(ctx->ws);
    OMR_HIP(ctx, hipMemcpyAsync(d, argb, (size_t)width * height * 4, hipMemcpyHostToDevice, ctx->stream));
    return encode_png_ws(ctx, kRgb, d, nullptr, width, height, 0, 0, nullptr, img, out, cap, out_len);
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
    const size_t nb = align_up(n_bytes, 256);
    omr_status st = ensure_workspace(ctx, nb + png_scratch(kind, width, height));
    if (st) return st;
    uint8_t* d_bits = static_cast<uint8_t*>(ctx->ws);
    OMR_HIP(ctx, hipMemcpyAsync(d_bits, bits, n_bytes, hipMemcpyHostToDevice, ctx->stream));
    return encode_png_ws(ctx, kind, nullptr, d_bits, width, height, flip_h ? 1 : 0, flip_v ? 1 : 0, rgba, nb, out,
                         cap, out_len);
}

}  // extern "C"
