// probe_stream.hip — HBM ceiling for K2's access pattern (not product code).
// Same geometry as k_render<u16,4ch>: persistent grid, 8 px/lane, 4 x 16-B loads + 2 x 16-B
// stores per lane, with trivial compute; plus a plain D2D copy for reference.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int NT, int STORE_MODE>
__global__ void __launch_bounds__(256) k_probe(const uint8_t* __restrict__ in, uint32_t* __restrict__ out,
                                               uint32_t total, uint32_t cpt) {
    for (uint32_t g = blockIdx.x * 256 + threadIdx.x; g < total; g += gridDim.x * 256) {
        const uint32_t tile = g / cpt, rem = g - tile * cpt;
        const uint8_t* base = in + (size_t)tile * 4 * (1 << 21) + (size_t)rem * 16;
        u32x4 a = NT ? __builtin_nontemporal_load((const u32x4*)base) : *(const u32x4*)base;
        u32x4 b = NT ? __builtin_nontemporal_load((const u32x4*)(base + (1 << 21))) : *(const u32x4*)(base + (1 << 21));
        u32x4 c = NT ? __builtin_nontemporal_load((const u32x4*)(base + (2 << 21))) : *(const u32x4*)(base + (2 << 21));
        u32x4 d = NT ? __builtin_nontemporal_load((const u32x4*)(base + (3 << 21))) : *(const u32x4*)(base + (3 << 21));
        u32x4 x = a ^ b ^ c ^ d;
        uint32_t* o = out + (size_t)g * 8;
        u32x4 y = x + 1;
        if (STORE_MODE == 0) { *(u32x4*)o = x; *(u32x4*)(o + 4) = y; }
        else { __builtin_nontemporal_store(x, (u32x4*)o); __builtin_nontemporal_store(y, (u32x4*)(o + 4)); }
    }
}

int main() {
    const int tiles = 256;
    const size_t in_bytes = (size_t)tiles * 4 * (1 << 21), out_bytes = (size_t)tiles * (1 << 22);
    uint8_t* in; uint32_t* out;
    hipMalloc(&in, in_bytes); hipMalloc(&out, out_bytes);
    hipMemset(in, 1, in_bytes); hipMemset(out, 0, out_bytes);
    hipDeviceProp_t p; hipGetDeviceProperties(&p, 0);
    const uint32_t cpt = (1 << 20) / 8, total = cpt * tiles;
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    auto run = [&](const char* name, auto launch) {
        for (int i = 0; i < 3; ++i) launch();
        hipEventRecord(e0);
        for (int i = 0; i < 10; ++i) launch();
        hipEventRecord(e1); hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        printf("%-34s %8.3f ms/launch  %8.1f GB/s\n", name, ms / 10, (in_bytes + out_bytes) / (ms / 10 * 1e-3) / 1e9);
    };
    for (int bpc : {4, 8, 16}) {
        const int grid = p.multiProcessorCount * bpc;
        char n[64];
        snprintf(n, 64, "k2-pattern plain  grid=%d", grid);
        run(n, [&] { hipLaunchKernelGGL((k_probe<0, 0>), dim3(grid), dim3(256), 0, 0, in, out, total, cpt); });
        snprintf(n, 64, "k2-pattern nt-load grid=%d", grid);
        run(n, [&] { hipLaunchKernelGGL((k_probe<1, 0>), dim3(grid), dim3(256), 0, 0, in, out, total, cpt); });
        snprintf(n, 64, "k2-pattern nt-ld+st grid=%d", grid);
        run(n, [&] { hipLaunchKernelGGL((k_probe<1, 1>), dim3(grid), dim3(256), 0, 0, in, out, total, cpt); });
    }
    const int full = (total + 255) / 256;
    run("k2-pattern plain  grid=full", [&] { hipLaunchKernelGGL((k_probe<0, 0>), dim3(full), dim3(256), 0, 0, in, out, total, cpt); });
    run("hipMemcpy D2D (in->out, out_bytes)", [&] { hipMemcpyAsync(out, in, out_bytes, hipMemcpyDeviceToDevice, 0); });
    printf("(copy line counts read+write of out_bytes as in+out only approximately)\n");
    return 0;
}
