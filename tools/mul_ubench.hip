// mul_ubench.hip -- Fq Montgomery product variants at one wave per SIMD on
// MI355X: a dependent chain x = x*y per lane, timed with HIP events.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/mul_ubench tools/mul_ubench.hip
#include <stdio.h>
#include <stdlib.h>

#include "../paritytech-bn_amd/csrc/fq.h"

#define CK(x)                                                                                      \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
            exit(1);                                                                               \
        }                                                                                          \
    } while (0)

using namespace bn;

// Variant S: each column's products summed in NACC independent partial
// accumulators (no chain through one register), carry added last.
template <int NACC, int A, int B>
__device__ __forceinline__ Fq<mul_bound(A, B)> mul_split(const Fq<A>& a, const Fq<B>& b) {
    uint32_t m[9];
    Fq<mul_bound(A, B)> r;
    uint64_t carry = 0;
#pragma unroll
    for (int k = 0; k < 17; ++k) {
        const int lo = k < 9 ? 0 : k - 8;
        const int hi = k < 9 ? k : 8;
        uint64_t s[NACC];
#pragma unroll
        for (int t = 0; t < NACC; ++t) s[t] = 0;
        int c = 0;
#pragma unroll
        for (int i = lo; i <= hi; ++i) {
            s[c % NACC] += (uint64_t)a.v[i] * b.v[k - i];
            ++c;
            if (i < k) {
                s[c % NACC] += (uint64_t)m[i] * kP29.v[k - i];
                ++c;
            }
        }
        uint64_t acc = carry;
#pragma unroll
        for (int t = 0; t < NACC; ++t) acc += s[t];
        if (k < 9) {
            m[k] = ((uint32_t)acc * BN_PINV29) & M29;
            acc += (uint64_t)m[k] * kP29.v[0];
        } else {
            r.v[k - 9] = (uint32_t)acc & M29;
        }
        carry = acc >> 29;
    }
    r.v[8] = (uint32_t)carry;
    return r;
}

template <int V>
__global__ void __launch_bounds__(256) k_chain(uint32_t* io, size_t n, int reps) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Fq<2> x, y, x2;
#pragma unroll
    for (int d = 0; d < 9; ++d) {
        x.v[d] = io[d * n + i];
        y.v[d] = io[(9 + d) * n + i];
        x2.v[d] = io[(18 + d) * n + i];
    }
#pragma unroll 1
    for (int r = 0; r < reps; ++r) {
        if constexpr (V == 0) x = fq_fold(fq_mul(x, y));
        if constexpr (V == 1) {
            x = fq_fold(fq_mul(x, y));
            x2 = fq_fold(fq_mul(x2, y));
        }
        if constexpr (V == 2) x = fq_fold(mul_split<2>(x, y));
        if constexpr (V == 3) x = fq_fold(mul_split<3>(x, y));
        if constexpr (V == 4) {
            x = fq_fold(mul_split<2>(x, y));
            x2 = fq_fold(mul_split<2>(x2, y));
        }
        if constexpr (V == 5) {  // 3 products, 2 independent
            x = fq_fold(fq_mul(x, y));
            x2 = fq_fold(fq_mul(x2, y));
            y = fq_fold(fq_mul(y, x));
        }
        if constexpr (V == 6) x = fq_fold(fq_mul(x, y));  // occupancy variant (launched at 2x n)
    }
#pragma unroll
    for (int d = 0; d < 9; ++d) io[(27 + d) * n + i] = x.v[d] ^ x2.v[d];
}

int main(int argc, char** argv) {
    const size_t n0 = argc > 1 ? strtoull(argv[1], 0, 0) : 65536;
    const int reps = 2000;
    uint32_t* io;
    CK(hipMalloc(&io, 36 * 2 * n0 * 4));
    uint32_t* h = (uint32_t*)malloc(36 * 2 * n0 * 4);
    uint64_t s = 99;
    for (size_t k = 0; k < 36 * 2 * n0; ++k) {
        s = s * 6364136223846793005ull + 1442695040888963407ull;
        h[k] = (uint32_t)(s >> 36) & 0x3fffff;  // small digits: valid Fq<1> for any digit slot
    }
    CK(hipMemcpy(io, h, 36 * 2 * n0 * 4, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto run = [&](const char* name, void (*k)(uint32_t*, size_t, int), size_t n, double muls_per_rep) {
        hipLaunchKernelGGL(k, dim3((n + 255) / 256), dim3(256), 0, 0, io, n, 10);
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(k, dim3((n + 255) / 256), dim3(256), 0, 0, io, n, reps);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double muls = (double)n * reps * muls_per_rep;
        // wave-cycles per product at 2.4 GHz over 1024 SIMDs
        const double cyc = ms * 1e-3 * 2.4e9 * 1024 / (muls / 64);
        printf("{\"variant\": \"%s\", \"n\": %zu, \"ms\": %.3f, \"Gmul_per_s\": %.2f, \"simd_cycles_per_wave_mul\": %.1f}\n",
               name, n, ms, muls / ms / 1e6, cyc);
    };
    run("fq_mul+fold chain", k_chain<0>, n0, 1);
    run("fq_mul+fold x2 independent", k_chain<1>, n0, 2);
    run("split2 chain", k_chain<2>, n0, 1);
    run("split3 chain", k_chain<3>, n0, 1);
    run("split2 x2 independent", k_chain<4>, n0, 2);
    run("fq_mul x3 (2 independent)", k_chain<5>, n0, 3);
    run("fq_mul chain, 2 waves/SIMD", k_chain<6>, 2 * n0, 1);
    return 0;
}
