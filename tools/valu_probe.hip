// valu_probe.hip — issue rate of the integer VALU forms the JPEG / PNG / C5 kernels are made of,
// and LDS table-lookup rates by access pattern (measurement tool, not product code).
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/valu_probe tools/valu_probe.hip && tools/valu_probe
//
// Each VALU case runs CH independent dependency chains of one instruction per lane (inline asm, so
// the count is exact) in every wave of a grid of 256 CUs x W waves; it reports SIMD cycles per
// wave-instruction = elapsed x clock x 1024 SIMDs / (waves x instructions).  The clock is read
// from the kernel's own s_memtime deltas against the event time.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

enum { OP_ADD, OP_XOR, OP_MUL24, OP_PERM, OP_CVT, OP_FREXP, OP_DOT2, OP_BFE, OP_ALIGNBIT, OP_ADD3, OP_LSHLADD,
       OP_FMA, OP_PKADD16, OP_CNDMASK, N_OPS };
static const char* kNames[N_OPS] = {"v_add_u32", "v_xor_b32", "v_mul_u32_u24", "v_perm_b32", "v_cvt_f32_i32",
                                    "v_frexp_exp_i32_f32", "v_dot2_u32_u16", "v_bfe_u32", "v_alignbit_b32",
                                    "v_add3_u32", "v_lshl_add_u32", "v_fma_f32", "v_pk_add_u16", "v_cndmask_b32"};

template <int OP, int CH>
__global__ void __launch_bounds__(256) k_valu(uint32_t* out, int iters, unsigned long long* clk) {
    uint32_t a[CH];
    const uint32_t k = threadIdx.x * 7 + 1;
#pragma unroll
    for (int c = 0; c < CH; ++c) a[c] = threadIdx.x + c;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int c = 0; c < CH; ++c) {
            if constexpr (OP == OP_ADD) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[c]) : "v"(k));
            if constexpr (OP == OP_XOR) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a[c]) : "v"(k));
            if constexpr (OP == OP_MUL24) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a[c]) : "v"(k));
            if constexpr (OP == OP_PERM) asm volatile("v_perm_b32 %0, %0, %1, %1" : "+v"(a[c]) : "v"(k));
            if constexpr (OP == OP_CVT) asm volatile("v_cvt_f32_i32 %0, %0" : "+v"(a[c]));
            if constexpr (OP == OP_FREXP) asm volatile("v_frexp_exp_i32_f32 %0, %0" : "+v"(a[c]));
            if constexpr (OP == OP_DOT2) asm volatile("v_dot2_u32_u16 %0, %0, %1, %0" : "+v"(a[c]) : "v"(k));
            if constexpr (OP == OP_BFE) asm volatile("v_bfe_u32 %0, %0, %1, 5" : "+v"(a[c]) : "v"(k));
            if constexpr (OP == OP_ALIGNBIT) asm volatile("v_alignbit_b32 %0, %0, %1, %1" : "+v"(a[c]) : "v"(k));
            if constexpr (OP == OP_ADD3) asm volatile("v_add3_u32 %0, %0, %1, %1" : "+v"(a[c]) : "v"(k));
            if constexpr (OP == OP_LSHLADD) asm volatile("v_lshl_add_u32 %0, %0, 1, %1" : "+v"(a[c]) : "v"(k));
            if constexpr (OP == OP_FMA) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(a[c]) : "v"(k));
            if constexpr (OP == OP_PKADD16) asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(a[c]) : "v"(k));
            if constexpr (OP == OP_CNDMASK) asm volatile("v_cmp_gt_u32 vcc, %0, %1\n\tv_cndmask_b32 %0, %0, %1, vcc" : "+v"(a[c]) : "v"(k) : "vcc");
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    uint32_t s = 0;
#pragma unroll
    for (int c = 0; c < CH; ++c) s += a[c];
    if (s == 0x12345678u) out[threadIdx.x] = s;          // keeps the chains live
    if (blockIdx.x == 0 && threadIdx.x == 0) *clk = t1 - t0;
}

// LDS lookups: every lane reads TAB-entry u16 tables at an index from a per-lane pattern.
//   mode 0: uniformly random index in [0, n)        mode 1: 75 % of lanes index 0, rest random
//   mode 2: random index in [0, 64) (one dword per bank: broadcast only)
template <int MODE>
__global__ void __launch_bounds__(256) k_lds(uint32_t* out, int iters, int n) {
    __shared__ uint16_t t[4096];
    for (int i = threadIdx.x; i < 4096; i += 256) t[i] = (uint16_t)(i * 37);
    __syncthreads();
    uint32_t x = threadIdx.x * 2654435761u + blockIdx.x, s = 0;
    for (int i = 0; i < iters; ++i) {
        uint32_t idx[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            x = x * 1664525u + 1013904223u;
            uint32_t r = (x >> 8) % (uint32_t)n;
            if (MODE == 1) r = ((x >> 4) & 3) ? 0u : r;
            if (MODE == 2) r = (x >> 8) & 127;
            idx[j] = r;
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) s += t[idx[j]];
    }
    if (s == 0x12345678u) out[threadIdx.x] = s;
}

template <int OP, int CH>
static double run_valu(int waves_per_simd, int iters, double* ghz) {
    uint32_t* out; unsigned long long* clk;
    CK(hipMalloc(&out, 4096)); CK(hipMalloc(&clk, 8));
    const int blocks = 256 * waves_per_simd;     // 4 waves per block = one per SIMD
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    hipLaunchKernelGGL((k_valu<OP, CH>), dim3(blocks), dim3(256), 0, 0, out, iters, clk);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL((k_valu<OP, CH>), dim3(blocks), dim3(256), 0, 0, out, iters, clk);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    unsigned long long c; CK(hipMemcpy(&c, clk, 8, hipMemcpyDeviceToHost));
    // s_memtime ticks at the shader clock on gfx950 (MI355X_MICROARCH.md constants table); one
    // block's loop time over the whole kernel's time bounds the clock from below
    *ghz = (double)c / (ms * 1e6);
    const double instr = (double)blocks * 4 * iters * CH;       // wave-instructions
    CK(hipFree(out)); CK(hipFree(clk));
    return ms * 1e-3 * 2.4e9 * 1024 / instr;                     // SIMD cycles per wave-instruction at 2.4 GHz
}

template <int OP>
static void valu_row(int iters) {
    double g1, g8, g8b;
    const double c1 = run_valu<OP, 8>(1, iters, &g1);
    const double c8 = run_valu<OP, 8>(8, iters / 4, &g8);
    const double c8b = run_valu<OP, 1>(8, iters, &g8b);
    printf("%-22s 1 wave/SIMD 8 chains: %5.2f cyc   8 waves/SIMD 8 chains: %5.2f cyc   8 waves/SIMD 1 chain: %5.2f cyc"
           "   (s_memtime/event GHz %.2f %.2f)\n", kNames[OP], c1, c8, c8b, g1, g8);
}

template <int MODE>
static void lds_row(int n) {
    uint32_t* out; CK(hipMalloc(&out, 4096));
    const int iters = 2000, blocks = 256 * 8;
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    hipLaunchKernelGGL((k_lds<MODE>), dim3(blocks), dim3(256), 0, 0, out, iters, n);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL((k_lds<MODE>), dim3(blocks), dim3(256), 0, 0, out, iters, n);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    const double reads = (double)blocks * 4 * iters * 8;          // wave-level ds_read_u16
    printf("LDS u16 lookup mode %d n=%4d: %5.2f CU cycles per wave-read (2 = conflict-free ds_read_b32)\n", MODE, n,
           ms * 1e-3 * 2.4e9 * 256 / reads);
    CK(hipFree(out));
}

int main() {
    const int it = 4000;
    valu_row<OP_ADD>(it); valu_row<OP_XOR>(it); valu_row<OP_MUL24>(it); valu_row<OP_PERM>(it);
    valu_row<OP_CVT>(it); valu_row<OP_FREXP>(it); valu_row<OP_DOT2>(it); valu_row<OP_BFE>(it);
    valu_row<OP_ALIGNBIT>(it); valu_row<OP_ADD3>(it); valu_row<OP_LSHLADD>(it); valu_row<OP_FMA>(it);
    valu_row<OP_PKADD16>(it); valu_row<OP_CNDMASK>(it);
    lds_row<0>(1024); lds_row<0>(256); lds_row<0>(64); lds_row<1>(1024); lds_row<2>(128);
    return 0;
}
