// issue_ubench.hip -- VALU issue cost per wave instruction on gfx950 at 1 and
// 8 waves per SIMD, wall-clock timed (HIP events, 2.4 GHz assumed).
// Question answered: does v_mad_u64_u32's carry-out SGPR (all writes to one
// pair) serialize independent MADs when a SIMD has a single wave?
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/issue_ubench tools/issue_ubench.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x)                                                                                      \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
            exit(1);                                                                               \
        }                                                                                          \
    } while (0)

// 8 independent 64-bit accumulators, 8 instructions per iteration
#define MADS_SAME                                                                     \
    "v_mad_u64_u32 %0, vcc, %8, %9, %0\n\t"                                           \
    "v_mad_u64_u32 %1, vcc, %8, %9, %1\n\t"                                           \
    "v_mad_u64_u32 %2, vcc, %8, %9, %2\n\t"                                           \
    "v_mad_u64_u32 %3, vcc, %8, %9, %3\n\t"                                           \
    "v_mad_u64_u32 %4, vcc, %8, %9, %4\n\t"                                           \
    "v_mad_u64_u32 %5, vcc, %8, %9, %5\n\t"                                           \
    "v_mad_u64_u32 %6, vcc, %8, %9, %6\n\t"                                           \
    "v_mad_u64_u32 %7, vcc, %8, %9, %7\n\t"
#define MADS_ROT                                                                      \
    "v_mad_u64_u32 %0, %8, %12, %13, %0\n\t"                                         \
    "v_mad_u64_u32 %1, %9, %12, %13, %1\n\t"                                         \
    "v_mad_u64_u32 %2, %10, %12, %13, %2\n\t"                                        \
    "v_mad_u64_u32 %3, %11, %12, %13, %3\n\t"                                        \
    "v_mad_u64_u32 %4, %8, %12, %13, %4\n\t"                                         \
    "v_mad_u64_u32 %5, %9, %12, %13, %5\n\t"                                         \
    "v_mad_u64_u32 %6, %10, %12, %13, %6\n\t"                                        \
    "v_mad_u64_u32 %7, %11, %12, %13, %7\n\t"
#define LSHLADD64                                                                     \
    "v_lshl_add_u64 %0, %8, 0, %0\n\t"                                                \
    "v_lshl_add_u64 %1, %8, 0, %1\n\t"                                                \
    "v_lshl_add_u64 %2, %8, 0, %2\n\t"                                                \
    "v_lshl_add_u64 %3, %8, 0, %3\n\t"                                                \
    "v_lshl_add_u64 %4, %8, 0, %4\n\t"                                                \
    "v_lshl_add_u64 %5, %8, 0, %5\n\t"                                                \
    "v_lshl_add_u64 %6, %8, 0, %6\n\t"                                                \
    "v_lshl_add_u64 %7, %8, 0, %7\n\t"

template <int KIND>
__global__ void __launch_bounds__(256) k_mad(uint64_t* out, uint32_t x, uint32_t y, int iters) {
    uint64_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6,
             a7 = a0 + 7;
    uint64_t s0, s1, s2, s3;
    const uint64_t z = ((uint64_t)y << 32) | x;
    for (int i = 0; i < iters; ++i) {
        if constexpr (KIND == 0)
            asm volatile(MADS_SAME MADS_SAME
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                         : "v"(x), "v"(y)
                         : "vcc");
        if constexpr (KIND == 1)
            asm volatile(MADS_ROT MADS_ROT
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7),
                           "=&s"(s0), "=&s"(s1), "=&s"(s2), "=&s"(s3)
                         : "v"(x), "v"(y));
        if constexpr (KIND == 2)
            asm volatile(LSHLADD64 LSHLADD64
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                         : "v"(z));
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

// 8 independent 32-bit chains
#define V32(I) I(0) I(1) I(2) I(3) I(4) I(5) I(6) I(7)
#define I_ADD(n) "v_add_u32 %" #n ", %" #n ", %8\n\t"
#define I_ADD3(n) "v_add3_u32 %" #n ", %" #n ", %8, %9\n\t"
#define I_MAD24(n) "v_mad_u32_u24 %" #n ", %" #n ", %8, %9\n\t"
#define I_MULLO(n) "v_mul_lo_u32 %" #n ", %" #n ", %8\n\t"
template <int KIND>
__global__ void __launch_bounds__(256) k_v32(uint32_t* out, uint32_t x, uint32_t y, int iters) {
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6,
             a7 = a0 + 7;
    for (int i = 0; i < iters; ++i) {
        if constexpr (KIND == 0)
            asm volatile(V32(I_ADD) V32(I_ADD)
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                         : "v"(x), "v"(y));
        if constexpr (KIND == 1)
            asm volatile(V32(I_ADD3) V32(I_ADD3)
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                         : "v"(x), "v"(y));
        if constexpr (KIND == 2)
            asm volatile(V32(I_MAD24) V32(I_MAD24)
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                         : "v"(x), "v"(y));
        if constexpr (KIND == 3)
            asm volatile(V32(I_MULLO) V32(I_MULLO)
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                         : "v"(x), "v"(y));
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

int main() {
    const int iters = 20000;
    void* out;
    CK(hipMalloc(&out, 8 << 20));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto run = [&](const char* name, void (*k)(void*, uint32_t, uint32_t, int), int waves_per_simd) {
        const int blocks = 256 * waves_per_simd;  // 256 threads = 4 waves = one per SIMD of a CU
        hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, 3u, 5u, 100);
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, 3u, 5u, iters);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double instr_per_simd = (double)iters * 16 * waves_per_simd;
        printf("{\"kind\": \"%s\", \"waves_per_simd\": %d, \"cycles_per_wave_instr\": %.2f}\n", name,
               waves_per_simd, ms * 1e-3 * 2.4e9 / instr_per_simd);
    };
    for (int w : {1, 2, 8}) {
        run("mad_u64_u32 sdst=vcc (8 indep)", (void (*)(void*, uint32_t, uint32_t, int))k_mad<0>, w);
        run("mad_u64_u32 sdst rotating 4 pairs", (void (*)(void*, uint32_t, uint32_t, int))k_mad<1>, w);
        run("lshl_add_u64 (8 indep)", (void (*)(void*, uint32_t, uint32_t, int))k_mad<2>, w);
        run("add_u32", (void (*)(void*, uint32_t, uint32_t, int))k_v32<0>, w);
        run("add3_u32", (void (*)(void*, uint32_t, uint32_t, int))k_v32<1>, w);
        run("mad_u32_u24", (void (*)(void*, uint32_t, uint32_t, int))k_v32<2>, w);
        run("mul_lo_u32", (void (*)(void*, uint32_t, uint32_t, int))k_v32<3>, w);
    }
    return 0;
}
