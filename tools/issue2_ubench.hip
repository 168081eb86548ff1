// issue2_ubench.hip -- single-wave VALU issue patterns on gfx950 (1 wave/SIMD),
// wall-clock timed: which back-to-back patterns issue fast and which stall.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/issue2_ubench tools/issue2_ubench.hip
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

#define R16(X) X X X X X X X X X X X X X X X X
#define OPS "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
template <int K>
__global__ void __launch_bounds__(256) k_pat(uint32_t* out, uint32_t x, uint32_t y, int iters) {
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6,
             a7 = a0 + 7;
    uint64_t m0 = a0, m1 = a1, m2 = a2, m3 = a3;
    for (int i = 0; i < iters; ++i) {
        if constexpr (K == 0)  // 8 chains, shared VGPR source
            asm volatile(R16("v_add_u32 %0, %0, %8\n\tv_add_u32 %1, %1, %8\n\tv_add_u32 %2, %2, %8\n\tv_add_u32 %3, %3, %8\n\t"
                             "v_add_u32 %4, %4, %8\n\tv_add_u32 %5, %5, %8\n\tv_add_u32 %6, %6, %8\n\tv_add_u32 %7, %7, %8\n\t")
                         : OPS : "v"(x));
        if constexpr (K == 1)  // 1 dependent chain
            asm volatile(R16("v_add_u32 %0, %0, %8\n\tv_add_u32 %0, %0, %8\n\tv_add_u32 %0, %0, %8\n\tv_add_u32 %0, %0, %8\n\t"
                             "v_add_u32 %0, %0, %8\n\tv_add_u32 %0, %0, %8\n\tv_add_u32 %0, %0, %8\n\tv_add_u32 %0, %0, %8\n\t")
                         : OPS : "v"(x));
        if constexpr (K == 2)  // 2 chains
            asm volatile(R16("v_add_u32 %0, %0, %8\n\tv_add_u32 %1, %1, %8\n\tv_add_u32 %0, %0, %8\n\tv_add_u32 %1, %1, %8\n\t"
                             "v_add_u32 %0, %0, %8\n\tv_add_u32 %1, %1, %8\n\tv_add_u32 %0, %0, %8\n\tv_add_u32 %1, %1, %8\n\t")
                         : OPS : "v"(x));
        if constexpr (K == 3)  // 8 chains, inline-constant source (one VGPR read)
            asm volatile(R16("v_add_u32 %0, 7, %0\n\tv_add_u32 %1, 7, %1\n\tv_add_u32 %2, 7, %2\n\tv_add_u32 %3, 7, %3\n\t"
                             "v_add_u32 %4, 7, %4\n\tv_add_u32 %5, 7, %5\n\tv_add_u32 %6, 7, %6\n\tv_add_u32 %7, 7, %7\n\t")
                         : OPS);
        if constexpr (K == 4)  // 8 chains, SGPR source
            asm volatile(R16("v_add_u32 %0, %8, %0\n\tv_add_u32 %1, %8, %1\n\tv_add_u32 %2, %8, %2\n\tv_add_u32 %3, %8, %3\n\t"
                             "v_add_u32 %4, %8, %4\n\tv_add_u32 %5, %8, %5\n\tv_add_u32 %6, %8, %6\n\tv_add_u32 %7, %8, %7\n\t")
                         : OPS : "s"(y));
        if constexpr (K == 5)  // dependent MAD chain
            asm volatile(R16("v_mad_u64_u32 %0, vcc, %4, %5, %0\n\t")
                         : "+v"(m0), "+v"(m1), "+v"(m2), "+v"(m3) : "v"(x), "v"(y) : "vcc");
        if constexpr (K == 6)  // 4 independent MAD chains
            asm volatile(R16("v_mad_u64_u32 %0, vcc, %4, %5, %0\n\tv_mad_u64_u32 %1, vcc, %4, %5, %1\n\t"
                             "v_mad_u64_u32 %2, vcc, %4, %5, %2\n\tv_mad_u64_u32 %3, vcc, %4, %5, %3\n\t")
                         : "+v"(m0), "+v"(m1), "+v"(m2), "+v"(m3) : "v"(x), "v"(y) : "vcc");
        if constexpr (K == 7)  // MAD alternating with VOP2 add (independent)
            asm volatile(R16("v_mad_u64_u32 %0, vcc, %4, %5, %0\n\tv_add_u32 %6, %6, %4\n\t"
                             "v_mad_u64_u32 %1, vcc, %4, %5, %1\n\tv_add_u32 %7, %7, %4\n\t")
                         : "+v"(m0), "+v"(m1), "+v"(m2), "+v"(m3) : "v"(x), "v"(y), "v"(a0), "v"(a1) : "vcc");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ (uint32_t)(m0 ^ m1 ^ m2 ^ m3);
}

int main() {
    const int iters = 2000;
    uint32_t* out;
    CK(hipMalloc(&out, 8 << 20));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto run = [&](const char* name, void (*k)(uint32_t*, uint32_t, uint32_t, int), int ninstr, int w) {
        const int blocks = 256 * w;
        hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, 3u, 5u, 10);
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, 3u, 5u, iters);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("{\"pattern\": \"%s\", \"waves_per_simd\": %d, \"cycles_per_wave_instr\": %.2f}\n", name, w,
               ms * 1e-3 * 2.4e9 / ((double)iters * ninstr * w));
    };
    for (int w : {1, 2}) {
        run("add x8 chains, shared vgpr src", k_pat<0>, 128, w);
        run("add 1 dependent chain", k_pat<1>, 128, w);
        run("add 2 chains", k_pat<2>, 128, w);
        run("add x8 chains, inline const", k_pat<3>, 128, w);
        run("add x8 chains, sgpr src", k_pat<4>, 128, w);
        run("mad64 dependent chain", k_pat<5>, 16, w);
        run("mad64 4 chains", k_pat<6>, 64, w);
        run("mad64/add alternating", k_pat<7>, 64, w);
    }
    return 0;
}
