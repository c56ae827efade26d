// omr_png.hip — K5 PNG encode and K6 shape-mask raster.
//
// K5 replaces ImageIO.write(image, "png", output) for rendered regions
// (ImageRegionRequestHandler.java:583-600): 24-bit RGB (the DirectColorModel view drops
// alpha, :576-578).  K6 replaces ShapeMaskRequestHandler.renderShapeMask(Color, byte[], w, h)
// (:165-221): MSB-first bit mask -> (flip) -> 2-entry palette PNG (index 0 transparent,
// index 1 = fill colour; 1-bit rows when width % 8 == 0, else 8-bit, :174-198).
//
// PNG is compared decoded (pixels), so the zlib stream uses stored deflate blocks: every
// output byte is a pure function of its index, written by one lane; Adler-32 is a parallel
// 64-bit reduction; CRC-32 is per-segment CRCs combined with x^(8n) mod P multiplications
// (XOR-reduction), so the whole IDAT chunk is built on the device.
#include "omr_device.h"

namespace omr {

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
    int64_t zlen;            // zlib stream length (2 + 5*nblk + raw + 4)
};

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
    uint8_t* t = A.chunk + 8 + A.zlen - 4;
    t[0] = adler >> 24; t[1] = adler >> 16; t[2] = adler >> 8; t[3] = adler;
}

constexpr int kCrcSeg = 128;

// CRC-32 of chunk type + data = bytes [4, 8 + zlen) of the chunk buffer: one 128-byte segment
// per lane (a short serial table walk), each segment's CRC shifted to the end of the data by
// x^(8n) mod P, XOR-combined within the workgroup and once per workgroup in memory.
__global__ void __launch_bounds__(256) k_png_crc(PngArgs A) {
    __shared__ uint32_t t[256];
    __shared__ uint32_t s_x[4];
    t[threadIdx.x] = c_crc.t[threadIdx.x];
    __syncthreads();
    const int64_t n = 4 + A.zlen;
    const uint8_t* d = A.chunk + 4;
    const int64_t s = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t b0 = s * kCrcSeg;
    uint32_t v = 0;
    if (b0 < n) {
        const int64_t b1 = min(n, b0 + kCrcSeg);
        uint32_t r = 0xFFFFFFFFu;
        for (int64_t i = b0; i < b1; ++i) r = t[(r ^ d[i]) & 0xFF] ^ (r >> 8);
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
    uint8_t* c = A.chunk + 8 + A.zlen;
    c[0] = crc >> 24; c[1] = crc >> 16; c[2] = crc >> 8; c[3] = crc;
    const uint32_t len = (uint32_t)A.zlen;
    A.chunk[0] = len >> 24; A.chunk[1] = len >> 16; A.chunk[2] = len >> 8; A.chunk[3] = len;
    A.chunk[4] = 'I'; A.chunk[5] = 'D'; A.chunk[6] = 'A'; A.chunk[7] = 'T';
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

// Encode on the device; scratch at ws + off.  Host-side prefix (signature, IHDR, PLTE/tRNS)
// and IEND are assembled here; the IDAT chunk comes back from the device.
static omr_status encode_png_ws(Ctx* ctx, int kind, const uint32_t* d_argb, const uint8_t* d_bits, int W,
                                int H, int fh, int fv, const uint8_t* rgba, size_t off, uint8_t* out,
                                size_t cap, size_t* out_len) {
    const PngPlan P = png_plan(kind, W, H);
    uint8_t* ws = static_cast<uint8_t*>(ctx->ws) + off;
    unsigned long long* sums = reinterpret_cast<unsigned long long*>(ws);
    uint32_t* crc = reinterpret_cast<uint32_t*>(ws + 16);
    uint8_t* chunk = ws + 256;
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
    const size_t total = pre.size() + (size_t)P.chunk_bytes + sizeof(iend);
    if (out_len) *out_len = total;
    if (!out || cap < total) return fail(ctx, OMR_BUFFER_TOO_SMALL, "PNG output buffer too small");
    PngArgs A;
    A.argb = d_argb;
    A.bits = d_bits;
    A.chunk = chunk;
    A.sums = sums;
    A.crc_out = crc;
    A.kind = kind;
    A.W = W;
    A.H = H;
    A.flip_h = fh;
    A.flip_v = fv;
    A.rowlen = P.rowlen;
    A.raw = P.raw;
    A.nblk = P.nblk;
    A.zlen = P.zlen;
    OMR_HIP(ctx, hipMemsetAsync(ws, 0, 256, ctx->stream));
    const int64_t need = (P.zlen + 255) / 256;
    const unsigned g = (unsigned)std::min<int64_t>(need, (int64_t)ctx->cu_count * 8);
    hipLaunchKernelGGL(k_png_layout, dim3(g), dim3(256), 0, ctx->stream, A);
    hipLaunchKernelGGL(k_png_adler, dim3(1), dim3(1), 0, ctx->stream, A);
    const int64_t segs = (4 + P.zlen + kCrcSeg - 1) / kCrcSeg;
    hipLaunchKernelGGL(k_png_crc, dim3((unsigned)((segs + 255) / 256)), dim3(256), 0, ctx->stream, A);
    hipLaunchKernelGGL(k_png_finish, dim3(1), dim3(1), 0, ctx->stream, A);
    OMR_HIP(ctx, hipGetLastError());
    std::memcpy(out, pre.data(), pre.size());
    OMR_HIP(ctx, hipMemcpyAsync(out + pre.size(), chunk, (size_t)P.chunk_bytes, hipMemcpyDeviceToHost, ctx->stream));
    OMR_HIP(ctx, hipStreamSynchronize(ctx->stream));
    std::memcpy(out + pre.size() + P.chunk_bytes, iend, sizeof(iend));
    return OMR_OK;
}

static size_t png_scratch(int kind, int W, int H) { return 256 + align_up((size_t)png_plan(kind, W, H).chunk_bytes, 256); }

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
    if (width <= 0 || height <= 0) return fail(ctx, OMR_INVALID_ARGUMENT, "Attempted to flip image with 0 size");
    const int64_t npx = (int64_t)width * height;
    if (!bits || (int64_t)n_bytes * 8 < npx) return fail(ctx, OMR_INVALID_ARGUMENT, "mask shorter than width*height bits");
    if (!rgba) return fail(ctx, OMR_INVALID_ARGUMENT, "null fill colour");
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
