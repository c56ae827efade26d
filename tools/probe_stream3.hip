// probe_stream3.hip — K2 streaming-pattern ceiling, round 1 second sweep (not product code).
// 256 tiles x 4 planes x 1024^2 uint16 in (2 MiB per plane), 4 MiB ARGB out per tile.
// Full grid, each lane owns CPT chunks of 8 pixels: 4*CPT 16-B loads issued before any store.
// Variants: chunks per lane, block size, non-temporal loads / stores, read-only and write-only
// halves, and an XCD-aware block order.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int CPT, int BLK, int NTL, int NTS, int XCD>
__global__ void __launch_bounds__(BLK) k_mix(const uint8_t* __restrict__ in, uint32_t* __restrict__ out,
                                             uint32_t total, uint32_t cpt, uint32_t nblk) {
    uint32_t b = blockIdx.x;
    if (XCD) {   // blocks are dealt round-robin to the 8 XCDs: give each XCD a contiguous span
        const uint32_t per = nblk / 8;
        b = (b % 8) * per + b / 8;
    }
    u32x4 d[CPT][4];
    uint32_t gs[CPT];
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
        const uint32_t g = min(b * BLK * CPT + k * BLK + threadIdx.x, total - 1);
        gs[k] = g;
        const uint32_t tile = g / cpt, rem = g - tile * cpt;
        const uint8_t* base = in + (size_t)tile * 4 * (1 << 21) + (size_t)rem * 16;
#pragma unroll
        for (int a = 0; a < 4; ++a) {
            const u32x4* p = (const u32x4*)(base + ((size_t)a << 21));
            d[k][a] = NTL ? __builtin_nontemporal_load(p) : *p;
        }
    }
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
        const u32x4 x = d[k][0] ^ d[k][1] ^ d[k][2] ^ d[k][3];
        const u32x4 y = x + 1;
        u32x4* o = (u32x4*)(out + (size_t)gs[k] * 8);
        if (NTS) { __builtin_nontemporal_store(x, o); __builtin_nontemporal_store(y, o + 1); }
        else { o[0] = x; o[1] = y; }
    }
}

template <int CPT>
__global__ void __launch_bounds__(256) k_read(const uint8_t* __restrict__ in, uint32_t* __restrict__ out,
                                              uint32_t total, uint32_t cpt) {
    u32x4 acc = {0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
        const uint32_t g = min(blockIdx.x * 256 * CPT + k * 256 + threadIdx.x, total - 1);
        const uint32_t tile = g / cpt, rem = g - tile * cpt;
        const uint8_t* base = in + (size_t)tile * 4 * (1 << 21) + (size_t)rem * 16;
#pragma unroll
        for (int a = 0; a < 4; ++a) acc ^= *(const u32x4*)(base + ((size_t)a << 21));
    }
    if (acc[0] == 0x12345678u && acc[1] == 0x9abcdef0u) out[threadIdx.x] = acc[2];
}

template <int CPT, int NTS>
__global__ void __launch_bounds__(256) k_write(uint32_t* __restrict__ out, uint32_t total) {
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
        const uint32_t g = blockIdx.x * 256 * CPT + k * 256 + threadIdx.x;
        if (g >= total) return;
        const u32x4 x = {g, g + 1, g + 2, g + 3};
        u32x4* o = (u32x4*)(out + (size_t)g * 8);
        if (NTS) { __builtin_nontemporal_store(x, o); __builtin_nontemporal_store(x, o + 1); }
        else { o[0] = x; o[1] = x; }
    }
}

int main() {
    const int tiles = 256;
    const size_t in_bytes = (size_t)tiles * 4 * (1 << 21), out_bytes = (size_t)tiles * (1 << 22);
    uint8_t* in; uint32_t* out;
    hipMalloc(&in, in_bytes); hipMalloc(&out, out_bytes);
    hipMemset(in, 1, in_bytes); hipMemset(out, 0, out_bytes);
    const uint32_t cpt = (1 << 20) / 8, total = cpt * tiles;
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    auto run = [&](const char* name, double bytes, auto launch) {
        for (int i = 0; i < 5; ++i) launch();
        hipEventRecord(e0);
        for (int i = 0; i < 40; ++i) launch();
        hipEventRecord(e1); hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        printf("%-40s %8.4f ms/launch  %8.1f GB/s\n", name, ms / 40, bytes / (ms / 40 * 1e-3) / 1e9);
        fflush(stdout);
    };
    const double mix = (double)(in_bytes + out_bytes);
#define MIX(CPT, BLK, NTL, NTS, XCD)                                                                   \
    {                                                                                                  \
        const uint32_t nblk = (total + BLK * CPT - 1) / (BLK * CPT);                                   \
        char n[96];                                                                                    \
        snprintf(n, 96, "mix cpt=%d blk=%d ntl=%d nts=%d xcd=%d", CPT, BLK, NTL, NTS, XCD);             \
        run(n, mix, [&] { hipLaunchKernelGGL((k_mix<CPT, BLK, NTL, NTS, XCD>), dim3(nblk), dim3(BLK), 0, 0, \
                                             in, out, total, cpt, nblk); });                          \
    }
    for (int rep = 0; rep < 2; ++rep) {
        MIX(2, 256, 0, 0, 0)
        MIX(2, 256, 0, 1, 0)
        MIX(2, 256, 1, 1, 0)
        MIX(1, 256, 0, 0, 0)
        MIX(4, 256, 0, 0, 0)
        MIX(4, 256, 0, 1, 0)
        MIX(2, 512, 0, 0, 0)
        MIX(2, 1024, 0, 0, 0)
        MIX(2, 256, 0, 0, 1)
        MIX(4, 256, 0, 0, 1)
    }
    run("read-only cpt=2 (in_bytes)", (double)in_bytes, [&] {
        hipLaunchKernelGGL((k_read<2>), dim3((total + 511) / 512), dim3(256), 0, 0, in, out, total, cpt); });
    run("read-only cpt=4 (in_bytes)", (double)in_bytes, [&] {
        hipLaunchKernelGGL((k_read<4>), dim3((total + 1023) / 1024), dim3(256), 0, 0, in, out, total, cpt); });
    run("write-only cpt=2 (out_bytes)", (double)out_bytes, [&] {
        hipLaunchKernelGGL((k_write<2, 0>), dim3((total + 511) / 512), dim3(256), 0, 0, out, total); });
    run("write-only cpt=2 nt (out_bytes)", (double)out_bytes, [&] {
        hipLaunchKernelGGL((k_write<2, 1>), dim3((total + 511) / 512), dim3(256), 0, 0, out, total); });
    run("hipMemcpy D2D out_bytes (r+w)", 2.0 * out_bytes, [&] {
        hipMemcpyAsync(out, in, out_bytes, hipMemcpyDeviceToDevice, 0); });
    return 0;
}
