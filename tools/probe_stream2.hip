// probe_stream2.hip — K2 memory-pattern variants (not product code).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// CPT chunks per thread (block covers CPT*256 consecutive chunks), optional LDS table preload.
template <int CPT, int TABLE>
__global__ void __launch_bounds__(256) k_full(const uint8_t* __restrict__ in, uint32_t* __restrict__ out,
                                              const uint32_t* __restrict__ tab, uint32_t total, uint32_t cpt) {
    __shared__ uint32_t s[1024];
    if (TABLE) {
        for (int i = threadIdx.x; i < 1024; i += 256) s[i] = tab[i];
        __syncthreads();
    }
    u32x4 a[CPT], b[CPT], c[CPT], d[CPT];
    uint32_t gs[CPT];
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
        const uint32_t g = blockIdx.x * 256 * CPT + k * 256 + threadIdx.x;
        gs[k] = g;
        if (g < total) {
            const uint32_t tile = g / cpt, rem = g - tile * cpt;
            const uint8_t* base = in + (size_t)tile * 4 * (1 << 21) + (size_t)rem * 16;
            a[k] = *(const u32x4*)base; b[k] = *(const u32x4*)(base + (1 << 21));
            c[k] = *(const u32x4*)(base + (2 << 21)); d[k] = *(const u32x4*)(base + (3 << 21));
        }
    }
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
        if (gs[k] >= total) continue;
        u32x4 x = a[k] ^ b[k] ^ c[k] ^ d[k];
        if (TABLE) x += s[x[0] & 1023];
        uint32_t* o = out + (size_t)gs[k] * 8;
        *(u32x4*)o = x; *(u32x4*)(o + 4) = x + 1;
    }
}

int main() {
    const int tiles = 256;
    const size_t in_bytes = (size_t)tiles * 4 * (1 << 21), out_bytes = (size_t)tiles * (1 << 22);
    uint8_t* in; uint32_t* out; uint32_t* tab;
    (void)hipMalloc(&in, in_bytes); (void)hipMalloc(&out, out_bytes); (void)hipMalloc(&tab, 4096);
    (void)hipMemset(in, 1, in_bytes); (void)hipMemset(out, 0, out_bytes); (void)hipMemset(tab, 0, 4096);
    const uint32_t cpt = (1 << 20) / 8, total = cpt * tiles;
    hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    auto run = [&](const char* name, auto launch) {
        for (int i = 0; i < 3; ++i) launch();
        (void)hipEventRecord(e0);
        for (int i = 0; i < 10; ++i) launch();
        (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
        float ms; (void)hipEventElapsedTime(&ms, e0, e1);
        printf("%-30s %8.3f ms/launch  %8.1f GB/s\n", name, ms / 10, (in_bytes + out_bytes) / (ms / 10 * 1e-3) / 1e9);
    };
#define RUN(C, T) run("cpt=" #C " table=" #T, [&] { hipLaunchKernelGGL((k_full<C, T>), dim3((total + 256 * C - 1) / (256 * C)), dim3(256), 0, 0, in, out, tab, total, cpt); })
    RUN(1, 0); RUN(2, 0); RUN(4, 0); RUN(1, 1); RUN(2, 1); RUN(4, 1); RUN(8, 1);
    return 0;
}
