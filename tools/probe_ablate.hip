// probe_ablate.hip — which part of K2 costs what (not product code).  Same geometry as
// k_render<u16, BE, NA=4, CPT=2>: 256 tiles of 4x1024^2 uint16 big-endian -> ARGB.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint32_t bsw(uint32_t d) { return __builtin_amdgcn_perm(d, d, 0x02030001u); }

struct P { double ws[4], a0[4]; float a0f[4], b0f[4]; };

template <int V>
__global__ void __launch_bounds__(256) k_ab(const uint8_t* __restrict__ in, uint32_t* __restrict__ out,
                                           const uint32_t* __restrict__ tab, uint32_t total, uint32_t cpt, P p) {
    __shared__ __attribute__((aligned(16))) uint32_t s[4 * 1024];
    const int n = (V == 5) ? 4 * 1024 : 4 * 256;
    for (int i = threadIdx.x; i < n; i += 256) s[i] = tab[i & 1023];
    u32x4 d[2][4];
    uint32_t gs[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const uint32_t g = blockIdx.x * 512 + k * 256 + threadIdx.x;
        gs[k] = g;
        const uint32_t tile = g / cpt, rem = g - tile * cpt;
        const uint8_t* base = in + (size_t)tile * 4 * (1 << 21) + (size_t)rem * 16;
#pragma unroll
        for (int a = 0; a < 4; ++a) d[k][a] = *(const u32x4*)(base + ((size_t)a << 21));
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        uint32_t acc[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] = 0;
#pragma unroll
        for (int a = 0; a < 4; ++a) {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                uint32_t w = bsw(d[k][a][j >> 1]);
                const uint32_t x = (j & 1) ? w >> 16 : w & 0xFFFF;
                uint32_t e;
                if (V == 0) { e = x; }
                else if (V == 1 || V == 2) {
                    const double dd = p.a0[a] * ((double)x - p.ws[a]);
                    const int v = min(max(__double2int_rz(floor(dd + 0.5)), 0), 255);
                    e = (V == 1) ? s[a * 256 + v] : (uint32_t)v * 0x100401u;
                } else if (V == 3) { e = s[a * 256 + (x >> 8)]; }
                else if (V == 4) {
                    const int v = min(max(__float2int_rd(fmaf((float)x, p.a0f[a], p.b0f[a])), 0), 255);
                    e = s[a * 256 + v];
                } else {   // V5: fp32 estimate + 16-B entry {c-1, c, c+1, L|U<<16} + selects
                    const int v = min(max(__float2int_rd(fmaf((float)x, p.a0f[a], p.b0f[a])), 0), 255);
                    const u32x4 t = *(const u32x4*)&s[(a * 256 + v) * 4];
                    const uint32_t L = t[3] & 0xFFFF, U = t[3] >> 16;
                    e = x < L ? t[0] : (x > U ? t[2] : t[1]);
                }
                acc[j] += e;
            }
        }
        uint32_t* o = out + (size_t)gs[k] * 8;
        *(u32x4*)o = u32x4{acc[0], acc[1], acc[2], acc[3]} | 0xFF000000u;
        *(u32x4*)(o + 4) = u32x4{acc[4], acc[5], acc[6], acc[7]} | 0xFF000000u;
    }
}

int main() {
    const int tiles = 256;
    const size_t in_bytes = (size_t)tiles * 4 * (1 << 21), out_bytes = (size_t)tiles * (1 << 22);
    uint8_t* in; uint32_t* out; uint32_t* tab;
    (void)hipMalloc(&in, in_bytes); (void)hipMalloc(&out, out_bytes); (void)hipMalloc(&tab, 4096 * 4);
    // pseudo-random 16-bit content so LDS indices vary like real data
    {
        uint32_t* h = (uint32_t*)malloc(1 << 24);
        uint32_t st = 12345;
        for (int i = 0; i < (1 << 22); ++i) { st = st * 1664525u + 1013904223u; h[i] = st; }
        for (size_t o = 0; o < in_bytes; o += (1 << 24)) (void)hipMemcpy(in + o, h, 1 << 24, hipMemcpyHostToDevice);
        free(h);
    }
    (void)hipMemset(tab, 7, 4096 * 4); (void)hipMemset(out, 0, out_bytes);
    P p;
    const double w[4][2] = {{0, 65535}, {1755, 51199}, {3218, 26623}, {100, 4000}};
    for (int a = 0; a < 4; ++a) {
        p.ws[a] = w[a][0]; p.a0[a] = 255.0 / (w[a][1] - w[a][0]);
        p.a0f[a] = (float)p.a0[a]; p.b0f[a] = (float)(0.5 - p.a0[a] * w[a][0]);
    }
    const uint32_t cpt = (1 << 20) / 8, total = cpt * tiles;
    hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    const char* names[] = {"V0 memory + int add (no LDS, no math)", "V1 DP quantize + LDS b32 (=K2 v4)",
                           "V2 DP quantize, no LDS", "V3 LDS b32, no math", "V4 fp32 estimate + LDS b32",
                           "V5 fp32 + LDS b128 + selects"};
    for (int v = 0; v < 6; ++v) {
        auto launch = [&] {
            switch (v) {
            case 0: hipLaunchKernelGGL(k_ab<0>, dim3(total / 512), dim3(256), 0, 0, in, out, tab, total, cpt, p); break;
            case 1: hipLaunchKernelGGL(k_ab<1>, dim3(total / 512), dim3(256), 0, 0, in, out, tab, total, cpt, p); break;
            case 2: hipLaunchKernelGGL(k_ab<2>, dim3(total / 512), dim3(256), 0, 0, in, out, tab, total, cpt, p); break;
            case 3: hipLaunchKernelGGL(k_ab<3>, dim3(total / 512), dim3(256), 0, 0, in, out, tab, total, cpt, p); break;
            case 4: hipLaunchKernelGGL(k_ab<4>, dim3(total / 512), dim3(256), 0, 0, in, out, tab, total, cpt, p); break;
            default: hipLaunchKernelGGL(k_ab<5>, dim3(total / 512), dim3(256), 0, 0, in, out, tab, total, cpt, p); break;
            }
        };
        for (int i = 0; i < 3; ++i) launch();
        (void)hipEventRecord(e0);
        for (int i = 0; i < 10; ++i) launch();
        (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
        float ms; (void)hipEventElapsedTime(&ms, e0, e1);
        printf("%-42s %8.3f ms  %8.1f GB/s\n", names[v], ms / 10, (in_bytes + out_bytes) / (ms / 10 * 1e-3) / 1e9);
    }
    return 0;
}
