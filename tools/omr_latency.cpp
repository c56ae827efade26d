// omr_latency — native per-request latency of the hot path through the C ABI, as a JNI/Panama
// caller on a Vert.x worker thread would see it (no Python in the loop).
//
// One request = ImageRegionRequestHandler.render for a C2 tile (4-channel uint16 1024^2,
// big-endian, rgb model, windows 0:65535,1755:51199,3218:26623,100:4000, colours
// 0000FF,00FF00,FF0000,FFFFFF): bindings filled per request (updateSettings, :689-741), then
//   render  : omr_render_packed_int_device + omr_ctx_synchronize   (renderAsPackedInt, :559)
//   jpeg    : render + omr_encode_jpeg_device to a host buffer      (+ compressToStream, :580-582)
//   fused   : omr_render_jpeg (the same request in one call: render inside the JPEG's first kernel)
// with the planes already in HBM.  Prints one JSON object: p50 / p90 / mean in ms.
// Then C3 (BASELINE configs[2]: 3-channel uint16 512x512x64 big-endian stacks, p=intmax|0:63 and
// intmean): omr_render_projected_device requests issued back to back on one context (the
// projection glue, ImageRegionRequestHandler.java:506-575), seven windows of >= 50 ms each with
// one stream sync per window: the median window rate in requests/s (no Python in the loop).
//
// Usage: omr_latency [iters] [device]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "omr/omr.h"

namespace {

constexpr int kTile = 1024, kChannels = 4;

struct Stats {
    double p50, p90, mean;
};

Stats stats(std::vector<double> v) {
    std::sort(v.begin(), v.end());
    double s = 0;
    for (double x : v) s += x;
    return {v[v.size() / 2], v[v.size() * 9 / 10], s / v.size()};
}

void fill_bindings(omr_channel_binding* ch) {
    static const double win[kChannels][2] = {{0, 65535}, {1755, 51199}, {3218, 26623}, {100, 4000}};
    static const char* col[kChannels] = {"0000FF", "00FF00", "FF0000", "FFFFFF"};
    for (int c = 0; c < kChannels; ++c) {
        omr_channel_binding& b = ch[c];
        std::memset(&b, 0, sizeof(b));
        b.active = 1;
        b.family = OMR_FAMILY_LINEAR;
        b.coefficient = 1.0;
        b.input_start = (double)(float)win[c][0];   // Float windows (ImageRegionCtx.java:313)
        b.input_end = (double)(float)win[c][1];
        b.global_min = 0;
        b.global_max = 65535;
        int32_t rgba[4];
        omr_split_html_color(col[c], rgba);
        for (int i = 0; i < 4; ++i) b.rgba[i] = (uint8_t)rgba[i];
        b.lut = nullptr;
    }
}

bool ok(omr_status st, omr_ctx* ctx, const char* what) {
    if (st == OMR_OK) return true;
    std::fprintf(stderr, "%s failed: %d %s\n", what, (int)st, ctx ? omr_last_error(ctx) : "");
    return false;
}

}  // namespace

int main(int argc, char** argv) {
    const int iters = argc > 1 ? std::atoi(argv[1]) : 200;
    const int device = argc > 2 ? std::atoi(argv[2]) : 0;
    omr_ctx* ctx = nullptr;
    if (!ok(omr_ctx_create(device, &ctx), nullptr, "omr_ctx_create")) return 1;
    const size_t plane = (size_t)kTile * kTile * 2;
    std::vector<uint16_t> host(kTile * kTile);
    uint32_t seed = 20261015u;
    void* d_planes[kChannels];
    for (int c = 0; c < kChannels; ++c) {
        for (auto& v : host) { seed = seed * 1664525u + 1013904223u; v = (uint16_t)(seed >> 16); }
        if (hipMalloc(&d_planes[c], plane) != hipSuccess) return 1;
        if (hipMemcpy(d_planes[c], host.data(), plane, hipMemcpyHostToDevice) != hipSuccess) return 1;
    }
    uint32_t* d_argb = nullptr;
    if (hipMalloc(&d_argb, (size_t)kTile * kTile * 4) != hipSuccess) return 1;
    const size_t cap = omr_jpeg_max_bytes(kTile, kTile);
    std::vector<uint8_t> jpeg(cap);
    const omr_quantum_def q{0, 255, 255, OMR_MODEL_RGB};
    omr_channel_binding ch[kChannels];
    using clk = std::chrono::steady_clock;
    auto render = [&]() {
        fill_bindings(ch);
        return omr_render_packed_int_device(ctx, &q, ch, kChannels, (const void* const*)d_planes, 0,
                                            OMR_PIXELS_UINT16, 1, kTile, kTile, 0, 0, d_argb);
    };
    std::vector<double> t_render, t_jpeg;
    size_t jlen = 0;
    for (int i = 0; i < iters + 5; ++i) {
        const auto t0 = clk::now();
        if (!ok(render(), ctx, "render") || !ok(omr_ctx_synchronize(ctx), ctx, "synchronize")) return 1;
        const double ms = std::chrono::duration<double, std::milli>(clk::now() - t0).count();
        if (i >= 5) t_render.push_back(ms);
    }
    for (int i = 0; i < iters + 5; ++i) {
        const auto t0 = clk::now();
        if (!ok(render(), ctx, "render")) return 1;
        if (!ok(omr_encode_jpeg_device(ctx, d_argb, kTile, kTile, 0.9f, jpeg.data(), cap, &jlen), ctx, "jpeg"))
            return 1;
        const double ms = std::chrono::duration<double, std::milli>(clk::now() - t0).count();
        if (i >= 5) t_jpeg.push_back(ms);
    }
    std::vector<double> t_fused;
    size_t flen = 0;
    for (int i = 0; i < iters + 5; ++i) {
        const auto t0 = clk::now();
        fill_bindings(ch);
        if (!ok(omr_render_jpeg(ctx, &q, ch, kChannels, (const void* const*)d_planes, 0, OMR_PIXELS_UINT16, 1, kTile,
                                kTile, 0, 0, 0.9f, jpeg.data(), cap, &flen), ctx, "render_jpeg"))
            return 1;
        const double ms = std::chrono::duration<double, std::milli>(clk::now() - t0).count();
        if (i >= 5) t_fused.push_back(ms);
    }
    if (flen != jlen) { std::fprintf(stderr, "fused JPEG length %zu != %zu\n", flen, jlen); return 1; }
    // ---- C3: projection glue requests back to back
    constexpr int kS = 512, kZ = 64, kC = 3;
    void* d_stacks[kC];
    std::vector<uint16_t> stack((size_t)kS * kS * kZ);
    for (int c = 0; c < kC; ++c) {
        for (auto& v : stack) { seed = seed * 1664525u + 1013904223u; v = (uint16_t)(seed >> 16); }
        if (hipMalloc(&d_stacks[c], stack.size() * 2) != hipSuccess) return 1;
        if (hipMemcpy(d_stacks[c], stack.data(), stack.size() * 2, hipMemcpyHostToDevice) != hipSuccess) return 1;
    }
    double c3_rate[2];
    for (int a = 0; a < 2; ++a) {
        const int alg = a == 0 ? OMR_PROJECTION_MAX : OMR_PROJECTION_MEAN;
        auto c3 = [&]() {
            fill_bindings(ch);
            return omr_render_projected_device(ctx, &q, ch, kC, (const void* const*)d_stacks, OMR_PIXELS_UINT16, 1, kS,
                                               kS, kZ, alg, 0, kZ - 1, 1, 0, 0, d_argb);
        };
        for (int i = 0; i < 200; ++i)
            if (!ok(c3(), ctx, "render_projected")) return 1;
        if (!ok(omr_ctx_synchronize(ctx), ctx, "synchronize")) return 1;
        std::vector<double> rates;
        for (int w = 0; w < 7; ++w) {
            const auto t0 = clk::now();
            long n = 0;
            double el = 0;
            do {
                for (int i = 0; i < 32; ++i)
                    if (!ok(c3(), ctx, "render_projected")) return 1;
                n += 32;
                el = std::chrono::duration<double>(clk::now() - t0).count();
            } while (el < 0.05);
            if (!ok(omr_ctx_synchronize(ctx), ctx, "synchronize")) return 1;
            rates.push_back(n / std::chrono::duration<double>(clk::now() - t0).count());
        }
        std::sort(rates.begin(), rates.end());
        c3_rate[a] = rates[rates.size() / 2];
    }
    for (int c = 0; c < kC; ++c) (void)hipFree(d_stacks[c]);
    const Stats r = stats(t_render), j = stats(t_jpeg), f = stats(t_fused);
    std::printf("{\"iters\": %d, \"render_device_resident\": {\"p50_ms\": %.4f, \"p90_ms\": %.4f, \"mean_ms\": %.4f}, "
                "\"render_to_jpeg_host\": {\"p50_ms\": %.4f, \"p90_ms\": %.4f, \"mean_ms\": %.4f, \"jpeg_bytes\": %zu}, "
                "\"render_jpeg_one_call\": {\"p50_ms\": %.4f, \"p90_ms\": %.4f, \"mean_ms\": %.4f}, "
                "\"c3_requests_per_s\": {\"max\": %.1f, \"mean\": %.1f, "
                "\"method\": \"median of 7 windows >= 50 ms, one context, no Python\"}}\n",
                iters, r.p50, r.p90, r.mean, j.p50, j.p90, j.mean, jlen, f.p50, f.p90, f.mean, c3_rate[0], c3_rate[1]);
    for (int c = 0; c < kChannels; ++c) (void)hipFree(d_planes[c]);
    (void)hipFree(d_argb);
    omr_ctx_destroy(ctx);
    return 0;
}
