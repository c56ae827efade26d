// omr_tiff.cpp — TIFF output of the render path (host writer).
//
// Replaces the jai-imageio TIFFImageWriter branch of ImageRegionRequestHandler.render
// (:584-596): the 24-bit DirectColorModel view of the ARGB buffer (ImageUtil, alpha dropped)
// written as a baseline, uncompressed, big-endian ("MM") RGB TIFF with 8-bit samples in
// strips of >= 8 KiB.  The writer is host-only: it is a byte shuffle of the rendered tile
// with no arithmetic, so the device path hands it the ARGB with one D2H copy.
#include <vector>

#include "omr_internal.h"

namespace {

void put16(std::vector<uint8_t>& b, uint32_t v) { b.push_back((uint8_t)(v >> 8)); b.push_back((uint8_t)v); }
void put32(std::vector<uint8_t>& b, uint32_t v) { put16(b, v >> 16); put16(b, v & 0xFFFF); }

size_t tiff_size(int W, int H, int* rows_per_strip, int* n_strips) {
    const size_t row = (size_t)W * 3;
    int rps = (int)std::max<size_t>(1, 8192 / std::max<size_t>(row, 1));
    rps = std::max(rps, 1);
    if (rps > H) rps = H;
    const int ns = (H + rps - 1) / rps;
    *rows_per_strip = rps;
    *n_strips = ns;
    const int n_tags = 10;
    // header 8 + IFD (2 + 12*n + 4) + BitsPerSample 6 + strip offsets/counts 8*ns + pixels
    return 8 + 2 + 12 * n_tags + 4 + 6 + (size_t)ns * 8 + row * H;
}

omr_status write_tiff(const uint32_t* argb, int W, int H, uint8_t* out, size_t cap, size_t* out_len) {
    int rps, ns;
    const size_t total = tiff_size(W, H, &rps, &ns);
    if (out_len) *out_len = total;
    if (!out || cap < total) return OMR_BUFFER_TOO_SMALL;
    std::vector<uint8_t> b;
    b.reserve(total);
    b.push_back('M'); b.push_back('M'); put16(b, 42); put32(b, 8);
    const int n_tags = 10;
    const uint32_t ifd_end = 8 + 2 + 12 * n_tags + 4;
    const uint32_t bps_off = ifd_end;
    const uint32_t offs_off = bps_off + 6;
    const uint32_t cnts_off = offs_off + 4 * ns;
    const uint32_t pix_off = cnts_off + 4 * ns;
    auto tag = [&](uint16_t id, uint16_t type, uint32_t count, uint32_t value) {
        put16(b, id); put16(b, type); put32(b, count);
        if (type == 3 && count == 1) { put16(b, value); put16(b, 0); }
        else put32(b, value);
    };
    put16(b, n_tags);
    tag(256, 4, 1, (uint32_t)W);                  // ImageWidth
    tag(257, 4, 1, (uint32_t)H);                  // ImageLength
    tag(258, 3, 3, bps_off);                      // BitsPerSample 8,8,8
    tag(259, 3, 1, 1);                            // Compression: none
    tag(262, 3, 1, 2);                            // PhotometricInterpretation: RGB
    if (ns == 1) tag(273, 4, 1, pix_off);         // StripOffsets
    else tag(273, 4, (uint32_t)ns, offs_off);
    tag(277, 3, 1, 3);                            // SamplesPerPixel
    tag(278, 4, 1, (uint32_t)rps);                // RowsPerStrip
    if (ns == 1) tag(279, 4, 1, (uint32_t)((size_t)W * 3 * H));   // StripByteCounts
    else tag(279, 4, (uint32_t)ns, cnts_off);
    tag(284, 3, 1, 1);                            // PlanarConfiguration: chunky
    put32(b, 0);                                  // no next IFD
    put16(b, 8); put16(b, 8); put16(b, 8);
    for (int s = 0; s < ns; ++s) put32(b, pix_off + (uint32_t)((size_t)s * rps * W * 3));
    for (int s = 0; s < ns; ++s) {
        const int rows = std::min(rps, H - s * rps);
        put32(b, (uint32_t)((size_t)rows * W * 3));
    }
    std::memcpy(out, b.data(), b.size());
    uint8_t* px = out + b.size();
    const size_t n = (size_t)W * H;
    for (size_t i = 0; i < n; ++i) {
        const uint32_t p = argb[i];
        px[3 * i] = (uint8_t)(p >> 16);
        px[3 * i + 1] = (uint8_t)(p >> 8);
        px[3 * i + 2] = (uint8_t)p;
    }
    return OMR_OK;
}

}  // namespace

using namespace omr;

extern "C" {

size_t omr_tiff_max_bytes(int32_t width, int32_t height) {
    if (width <= 0 || height <= 0) return 0;
    int rps, ns;
    return tiff_size(width, height, &rps, &ns);
}

omr_status omr_encode_tiff(omr_ctx* ctx, const uint32_t* argb, int32_t width, int32_t height,
                           uint8_t* out, size_t cap, size_t* out_len) {
    if (!argb || width <= 0 || height <= 0 || width > 65535 || height > 65535) {
        if (ctx) fail(ctx, OMR_INVALID_ARGUMENT, "TIFF: bad image");
        return OMR_INVALID_ARGUMENT;
    }
    const omr_status st = write_tiff(argb, width, height, out, cap, out_len);
    if (st && ctx) fail(ctx, st, "TIFF output buffer too small");
    return st;
}

omr_status omr_encode_tiff_device(omr_ctx* ctx, const uint32_t* d_argb, int32_t width, int32_t height,
                                  uint8_t* out, size_t cap, size_t* out_len) {
    if (!ctx) return OMR_INVALID_ARGUMENT;
    if (!d_argb || width <= 0 || height <= 0 || width > 65535 || height > 65535)
        return fail(ctx, OMR_INVALID_ARGUMENT, "TIFF: bad image");
    OMR_HIP(ctx, hipSetDevice(ctx->device));
    std::vector<uint32_t> host((size_t)width * height);
    OMR_HIP(ctx, hipMemcpyAsync(host.data(), d_argb, host.size() * 4, hipMemcpyDeviceToHost, ctx->stream));
    OMR_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return omr_encode_tiff(ctx, host.data(), width, height, out, cap, out_len);
}

}  // extern "C"
