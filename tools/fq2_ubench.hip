// fq2_ubench.hip -- Fq2 product variants at one wave per SIMD on MI355X:
// Karatsuba with lazy reduction (fq2_mul_lazy: 405 multiply-adds plus 64-bit
// adds/subtracts) vs schoolbook with lazy reduction (fq2_mul_sb: 486
// multiply-adds, no 64-bit add/subtract), as a dependent chain x = x*y per lane
// and as two independent chains; also checks that both give the same residues.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/fq2_ubench tools/fq2_ubench.hip
#include <stdio.h>
#include <stdlib.h>

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

template <int V>
__global__ void __launch_bounds__(256) k_chain(uint32_t* io, size_t n, int reps) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Fq2<2> x, y, x2;
#pragma unroll
    for (int d = 0; d < 9; ++d) {
        x.c0.v[d] = io[d * n + i];
        x.c1.v[d] = io[(9 + d) * n + i];
        y.c0.v[d] = io[(18 + d) * n + i];
        y.c1.v[d] = io[(27 + d) * n + i];
        x2.c0.v[d] = io[(36 + d) * n + i];
        x2.c1.v[d] = io[(45 + d) * n + i];
    }
#pragma unroll 1
    for (int r = 0; r < reps; ++r) {
        if constexpr (V == 0) x = fq2_fold(fq2_mul_lazy(x, y));
        if constexpr (V == 1) x = fq2_fold(fq2_mul_sb(x, y));
        if constexpr (V == 2) {
            x = fq2_fold(fq2_mul_lazy(x, y));
            x2 = fq2_fold(fq2_mul_lazy(x2, y));
        }
        if constexpr (V == 3) {
            x = fq2_fold(fq2_mul_sb(x, y));
            x2 = fq2_fold(fq2_mul_sb(x2, y));
        }
    }
    // canonical residues out, so the variants can be compared word for word
    const Fq<1> a = fq_canonical(x.c0), b = fq_canonical(x.c1), c = fq_canonical(x2.c0), d2 = fq_canonical(x2.c1);
#pragma unroll
    for (int d = 0; d < 9; ++d) {
        io[(54 + d) * n + i] = a.v[d];
        io[(63 + d) * n + i] = b.v[d];
        io[(72 + d) * n + i] = c.v[d];
        io[(81 + d) * n + i] = d2.v[d];
    }
}

int main(int argc, char** argv) {
    const size_t n = argc > 1 ? strtoull(argv[1], 0, 0) : 65536;
    const int reps = 1000;
    const size_t words = 90 * n;
    uint32_t* io;
    CK(hipMalloc(&io, words * 4));
    uint32_t* h = (uint32_t*)malloc(words * 4);
    uint32_t* r0 = (uint32_t*)malloc(words * 4);
    uint32_t* r1 = (uint32_t*)malloc(words * 4);
    uint64_t s = 99;
    for (size_t k = 0; k < 54 * n; ++k) {
        s = s * 6364136223846793005ull + 1442695040888963407ull;
        const size_t digit = (k / n) % 9;
        h[k] = (uint32_t)(s >> 35) & (digit == 8 ? 0x3fffffu : 0x1fffffffu);  // value < 2^254 < p
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto run = [&](const char* name, void (*k)(uint32_t*, size_t, int), double muls_per_rep, uint32_t* keep) {
        CK(hipMemcpy(io, h, 54 * n * 4, hipMemcpyHostToDevice));
        hipLaunchKernelGGL(k, dim3((n + 255) / 256), dim3(256), 0, 0, io, n, 10);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(io, h, 54 * n * 4, hipMemcpyHostToDevice));
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(k, dim3((n + 255) / 256), dim3(256), 0, 0, io, n, reps);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (keep) CK(hipMemcpy(keep, io, words * 4, hipMemcpyDeviceToHost));
        const double muls = (double)n * reps * muls_per_rep;
        const double cyc = ms * 1e-3 * 2.4e9 * 1024 / (muls / 64);  // SIMD cycles per wave-product at 2.4 GHz
        printf("{\"variant\": \"%s\", \"n\": %zu, \"ms\": %.3f, \"G_fq2mul_per_s\": %.2f, "
               "\"simd_cycles_per_wave_fq2mul\": %.1f}\n",
               name, n, ms, muls / ms / 1e6, cyc);
    };
    run("lazy Karatsuba chain", k_chain<0>, 1, r0);
    run("schoolbook chain", k_chain<1>, 1, r1);
    size_t diff = 0;
    for (size_t k = 54 * n; k < 72 * n; ++k) diff += r0[k] != r1[k];
    printf("{\"check\": \"chain results lazy vs schoolbook\", \"differing_words\": %zu}\n", diff);
    run("lazy Karatsuba x2 independent", k_chain<2>, 2, nullptr);
    run("schoolbook x2 independent", k_chain<3>, 2, nullptr);
    return diff != 0;
}
