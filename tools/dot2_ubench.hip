// dot2_ubench.hip -- the split-layout Fq2 product (fq2_split.h fq2_mul: one
// fq_dot2 column sum per lane) at two waves per SIMD, as the throughput kernels
// run it: V = 0 the compiler's product scan, V = 1 the hand-scheduled column sum
// (fq2_split.h BN_DOT2_ASM form).  Each lane runs `reps` dependent products
// x = x * y (two independent chains per lane, as the Fq6/Fq12 code interleaves
// pairs of products); the canonical residues go back out so the two forms can be
// compared word for word.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/dot2_ubench tools/dot2_ubench.hip
#include <stdio.h>
#include <stdlib.h>

#ifndef BN_DOT2_ASM
#define BN_DOT2_ASM 0
#endif
#include "../paritytech-bn_amd/csrc/fq.h"
#define BN_SPLIT 1
#include "../paritytech-bn_amd/csrc/tower.h"

#define CK(x)                                                                                      \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
            exit(1);                                                                               \
        }                                                                                          \
    } while (0)

using namespace bn;

__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2, 2)))
k_chain(uint32_t* io, size_t n, int reps) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Fq2<2> x, y, x2;
#pragma unroll
    for (int d = 0; d < 9; ++d) {
        x.c.v[d] = io[d * n + i];
        y.c.v[d] = io[(9 + d) * n + i];
        x2.c.v[d] = io[(18 + d) * n + i];
    }
#pragma unroll 1
    for (int r = 0; r < reps; ++r) {
        auto p = fq2_mul2(x, y, x2, y);
        x = widen<2>(p.a);
        x2 = widen<2>(p.b);
    }
    const Fq<1> a = fq_canonical(x.c), b = fq_canonical(x2.c);
#pragma unroll
    for (int d = 0; d < 9; ++d) {
        io[(27 + d) * n + i] = a.v[d];
        io[(36 + d) * n + i] = b.v[d];
    }
}

int main(int argc, char** argv) {
    const size_t n = argc > 1 ? strtoull(argv[1], 0, 0) : 131072;  // 2048 waves: two per SIMD
    const int reps = argc > 2 ? atoi(argv[2]) : 400;
    const size_t words = 45 * n;
    uint32_t* io;
    CK(hipMalloc(&io, words * 4));
    uint32_t* h = (uint32_t*)malloc(words * 4);
    uint64_t s = 99;
    for (size_t k = 0; k < 27 * n; ++k) {
        s = s * 6364136223846793005ull + 1442695040888963407ull;
        const size_t digit = (k / n) % 9;
        h[k] = (uint32_t)(s >> 35) & (digit == 8 ? 0x3fffffu : 0x1fffffffu);  // value < 2^254 < p
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipMemcpy(io, h, 27 * n * 4, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_chain, dim3((n + 511) / 512), dim3(512), 0, 0, io, n, 10);
    CK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int t = 0; t < 5; ++t) {
        CK(hipMemcpy(io, h, 27 * n * 4, hipMemcpyHostToDevice));
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(k_chain, dim3((n + 511) / 512), dim3(512), 0, 0, io, n, reps);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (ms < best) best = ms;
    }
    CK(hipMemcpy(h, io, words * 4, hipMemcpyDeviceToHost));
    uint64_t sum = 0;
    for (size_t k = 27 * n; k < 45 * n; ++k) sum = sum * 1000003ull + h[k];
    const double prods = (double)n * reps * 2;  // lane-products (one Fq2 coordinate each)
    const double cyc = best * 1e-3 * 2.4e9 * 1024 / (prods / 64);
    printf("{\"form\": \"%s\", \"n\": %zu, \"reps\": %d, \"ms\": %.3f, \"simd_cycles_per_wave_dot2\": %.1f, "
           "\"checksum\": \"%016llx\"}\n",
           BN_DOT2_ASM ? "asm column sum" : "compiler", n, reps, best, cyc, (unsigned long long)sum);
    return 0;
}
