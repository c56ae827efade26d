// omr_host.cpp — host-side request helpers of the drop-in (no device work).
// These mirror the reference's static/handler helpers that turn a request into kernel
// parameters; they stay on the CPU exactly as in the reference.
#include <algorithm>
#include <cctype>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "omr/omr.h"

namespace {

// Integer.parseInt(s, 16) for the two-character substrings splitHTMLColor feeds it.
bool parse_hex2(const std::string& s, int32_t& out) {
    auto dig = [](char c) -> int {
        if (c >= '0' && c <= '9') return c - '0';
        if (c >= 'a' && c <= 'f') return c - 'a' + 10;
        if (c >= 'A' && c <= 'F') return c - 'A' + 10;
        return -1;
    };
    if (s.size() != 2) return false;
    if (s[0] == '-' || s[0] == '+') {
        const int d = dig(s[1]);
        if (d < 0) return false;
        out = s[0] == '-' ? -d : d;
        return true;
    }
    const int a = dig(s[0]), b = dig(s[1]);
    if (a < 0 || b < 0) return false;
    out = a * 16 + b;
    return true;
}

// Java int arithmetic: two's-complement wrap-around (JLS 15.17.1 / 15.18.2), which is
// undefined behaviour on int32_t in C++, so go through uint32_t.
inline int32_t jadd(int32_t a, int32_t b) { return (int32_t)((uint32_t)a + (uint32_t)b); }
inline int32_t jsub(int32_t a, int32_t b) { return (int32_t)((uint32_t)a - (uint32_t)b); }
inline int32_t jmul(int32_t a, int32_t b) { return (int32_t)((uint32_t)a * (uint32_t)b); }

}  // namespace

extern "C" {

// ImageRegionRequestHandler.splitHTMLColor (:865-890), including its 3/4-character bug:
// `color += ch + ch` adds two chars as ints and appends the decimal number (:873).
omr_status omr_split_html_color(const char* color, int32_t rgba_out[4]) {
    if (!color || !rgba_out) return OMR_INVALID_ARGUMENT;
    std::string c(color);
    if (c.size() == 3 || c.size() == 4) {
        std::string s;
        for (unsigned char ch : c) s += std::to_string((int)ch + (int)ch);
        c = s;
    }
    if (c.size() == 6) c += "FF";
    if (c.size() != 8) return OMR_INVALID_ARGUMENT;
    int32_t v[4];
    for (int i = 0; i < 4; ++i)
        if (!parse_hex2(c.substr(2 * i, 2), v[i])) return OMR_INVALID_ARGUMENT;
    for (int i = 0; i < 4; ++i) rgba_out[i] = v[i];
    return OMR_OK;
}

// ShapeMaskRequestHandler.renderShapeMask(Mask) fill colour (:97-106).  The mask's own
// colour goes through java.awt.Color(int rgb), which reads 0x??RRGGBB and forces alpha
// 255; default yellow; a request colour overrides (Color(r,g,b,a) rejects components
// outside 0..255 with IllegalArgumentException).
omr_status omr_shape_mask_fill_color(int32_t has_mask_fill, int32_t mask_fill_color,
                                     const char* request_color, uint8_t rgba_out[4]) {
    if (!rgba_out) return OMR_INVALID_ARGUMENT;
    int32_t r = 255, g = 255, b = 0, a = 255;
    if (has_mask_fill) {
        r = (mask_fill_color >> 16) & 0xFF;
        g = (mask_fill_color >> 8) & 0xFF;
        b = mask_fill_color & 0xFF;
        a = 255;
    }
    if (request_color) {
        int32_t v[4];
        if (omr_split_html_color(request_color, v) != OMR_OK) return OMR_INVALID_ARGUMENT;
        for (int i = 0; i < 4; ++i)
            if (v[i] < 0 || v[i] > 255) return OMR_INVALID_ARGUMENT;
        r = v[0]; g = v[1]; b = v[2]; a = v[3];
    }
    rgba_out[0] = (uint8_t)r; rgba_out[1] = (uint8_t)g; rgba_out[2] = (uint8_t)b; rgba_out[3] = (uint8_t)a;
    return OMR_OK;
}

// getRegionDef (:789-832) + truncateRegionDef (:751-758) + flipRegionDef (:770-780).
omr_status omr_get_region_def(int32_t mode, const omr_region* request, int32_t resolution,
                              const int32_t* level_sizes, int32_t n_levels, int32_t tile_size_x,
                              int32_t tile_size_y, int32_t max_tile_length, int32_t flip_h,
                              int32_t flip_v, omr_region* out) {
    if (!out || !level_sizes || n_levels <= 0) return OMR_INVALID_ARGUMENT;
    const int32_t res = resolution < 0 ? 0 : resolution;
    if (res >= n_levels) return OMR_INVALID_ARGUMENT;   // List.get out of range
    const int32_t size_x = level_sizes[2 * res], size_y = level_sizes[2 * res + 1];
    omr_region rd{0, 0, 0, 0};
    if (mode == 0) {
        if (!request) return OMR_INVALID_ARGUMENT;
        int32_t tsx = request->width, tsy = request->height;
        if (tsx == 0) tsx = tile_size_x;
        if (tsx > max_tile_length) tsx = max_tile_length;
        if (tsy == 0) tsy = tile_size_y;
        if (tsy > max_tile_length) tsy = max_tile_length;
        rd.width = tsx;
        rd.height = tsy;
        rd.x = jmul(request->x, tsx);
        rd.y = jmul(request->y, tsy);
    } else if (mode == 1) {
        if (!request) return OMR_INVALID_ARGUMENT;
        rd = *request;
    } else {
        rd = omr_region{0, 0, size_x, size_y};
        *out = rd;
        return OMR_OK;
    }
    rd.width = std::min(rd.width, jsub(size_x, rd.x));
    rd.height = std::min(rd.height, jsub(size_y, rd.y));
    if (flip_h) rd.x = jsub(jsub(size_x, rd.width), rd.x);
    if (flip_v) rd.y = jsub(jsub(size_y, rd.height), rd.y);
    *out = rd;
    return OMR_OK;
}

int32_t omr_resolution_level(int32_t n_levels, int32_t resolution) { return jsub(jsub(n_levels, resolution), 1); }

// checkPlaneDef (:651-681).
omr_status omr_check_plane_def(omr_region* rd, int32_t size_x, int32_t size_y) {
    if (!rd) return OMR_OK;
    if (jadd(rd->width, rd->x) > size_x) rd->width = jsub(size_x, rd->x);
    if (jadd(rd->height, rd->y) > size_y) rd->height = jsub(size_y, rd->y);
    return OMR_OK;
}

// LutReader input formats (LutProviderImpl.java:42-58 reads every *.lut under the script
// repository): ImageJ binary (768 B, or 800 B with a 32-byte "ICOL" header) and text
// tables (one row per index: "r g b" or "index r g b", optional header line).
omr_status omr_parse_lut(const uint8_t* data, size_t n, uint8_t lut_out[768]) {
    if (!data || !lut_out) return OMR_INVALID_ARGUMENT;
    if (n == 768) { std::memcpy(lut_out, data, 768); return OMR_OK; }
    if (n == 800 && std::memcmp(data, "ICOL", 4) == 0) { std::memcpy(lut_out, data + 32, 768); return OMR_OK; }
    std::vector<int> rows[3];
    size_t i = 0;
    while (i < n) {
        size_t j = i;
        while (j < n && data[j] != '\n') ++j;
        std::vector<long> nums;
        size_t k = i;
        bool bad = false;
        while (k < j) {
            while (k < j && (data[k] == ' ' || data[k] == '\t' || data[k] == ',' || data[k] == '\r')) ++k;
            if (k >= j) break;
            if (!std::isdigit(data[k])) { bad = true; break; }
            long v = 0;   // saturates: anything above 255 is rejected below
            while (k < j && std::isdigit(data[k])) v = std::min(v * 10 + (data[k++] - '0'), 1000000L);
            nums.push_back(v);
        }
        if (!bad && (nums.size() == 3 || nums.size() == 4)) {
            const size_t o = nums.size() - 3;
            for (int c = 0; c < 3; ++c) {
                if (nums[o + c] > 255) return OMR_INVALID_ARGUMENT;
                rows[c].push_back((int)nums[o + c]);
            }
        }
        i = j + 1;
    }
    if (rows[0].size() != 256) return OMR_INVALID_ARGUMENT;
    for (int c = 0; c < 3; ++c)
        for (int v = 0; v < 256; ++v) lut_out[c * 256 + v] = (uint8_t)rows[c][v];
    return OMR_OK;
}

}  // extern "C"
