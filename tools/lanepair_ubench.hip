// lanepair_ubench.hip -- go/no-go for a two-lanes-per-element Fq2 layout.
//
// With 2^16 pairings the engine runs exactly one wave per SIMD, and one wave
// alone issues a VALU instruction every ~4.5-5.3 cycles (profiles/
// r1_issue_ubench.jsonl), against ~2.4 (adds) and ~5.1 (multiply-add chains)
// with two waves.  Splitting every Fq2 over a lane pair doubles the wave count
// at the same total work.  In the normal basis {t, t^p}, t = (1+u)/2, the Fq2
// product is the same formula on both lanes:
//     c_own = (a_own*(b_own + b_other) + a_other*(b_own - b_other)) / 2,
// one 2-product Montgomery column sum per lane (the 1/2 is absorbed by holding
// values as x*R/2).  The partner's digits come over DPP quad_perm [1,0,3,2].
//
// Measured here: Fq2 products per second, one dependent-operand chain pair per
// element, for (a) the engine's schoolbook product, one lane per element, and
// (b) the lane-pair product, two lanes per element; both at 2^16 elements.
// Results are converted back to the standard basis and compared word for word.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/lanepair_ubench tools/lanepair_ubench.hip
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

// (a) engine layout: x = x*y and x2 = x2*y per lane; y passes a register fence
// each step so nothing that depends on it is hoisted out of the loop
__global__ void __launch_bounds__(256) k_base(uint32_t* io, size_t n, int reps) {
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
        fq2_fence(y);
        x = fq2_mul_sb(x, y);  // output bound 2: no fold needed
        x2 = fq2_mul_sb(x2, y);
    }
    const Fq<1> a = fq_canonical(x.c0), b = fq_canonical(x.c1), c = fq_canonical(x2.c0), d2 = fq_canonical(x2.c1);
#pragma unroll
    for (int d = 0; d < 9; ++d) {
        io[(54 + d) * n + i] = a.v[d];
        io[(63 + d) * n + i] = b.v[d];
        io[(72 + d) * n + i] = c.v[d];
        io[(81 + d) * n + i] = d2.v[d];
    }
}

BN_INLINE uint32_t partner(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
}
template <int B>
BN_INLINE Fq<B> partner(const Fq<B>& a) {
    Fq<B> r;
#pragma unroll
    for (int i = 0; i < 9; ++i) r.v[i] = partner(a.v[i]);
    return r;
}

// (a_own*s + a_oth*d) * 2^-261 mod p, product scanning as fq_mul; s digits
// < 2^30, d digits < 3*2^29, a digits < 2^29: a column stays below 54*2^58.
BN_INLINE Fq<2> dot2_mont(const Fq<2>& a, const Fq<2>& ao, const uint32_t s[9], const uint32_t d[9]) {
    uint32_t m[9];
    Fq<2> r;
    uint64_t acc = 0;
#pragma unroll
    for (int k = 0; k < 17; ++k) {
        const int lo = k < 9 ? 0 : k - 8;
        const int hi = k < 9 ? k : 8;
#pragma unroll
        for (int i = lo; i <= hi; ++i) {
            acc += (uint64_t)a.v[i] * s[k - i];
            acc += (uint64_t)ao.v[i] * d[k - i];
        }
#pragma unroll
        for (int i = lo; i <= hi; ++i)
            if (i < k) acc += (uint64_t)m[i] * kP29.v[k - i];
        if (k < 9) {
            m[k] = ((uint32_t)acc * BN_PINV29) & M29;
            acc += (uint64_t)m[k] * kP29.v[0];
        } else {
            r.v[k - 9] = (uint32_t)acc & M29;
        }
        acc >>= 29;
    }
    r.v[8] = (uint32_t)acc;
    return r;
}

// one lane's coordinate of a*b in the normal basis (values held as x*R/2)
BN_INLINE Fq<2> lp_mul(const Fq<2>& a, const Fq<2>& b) {
    const Fq<2> ao = partner(a), bo = partner(b);
    constexpr Limbs9 Q = kp_spread(3, 1);
    uint32_t s[9], d[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) {
        s[i] = b.v[i] + bo.v[i];
        d[i] = (b.v[i] + Q.v[i]) - bo.v[i];
    }
    return dot2_mont(a, ao, s, d);  // < T/R + p <= 2p
}

// (b) lane pair: lane 2e holds normal coordinate 0 of element e, lane 2e+1
// coordinate 1.  Standard -> normal: n0 = x0 + x1, n1 = x0 - x1; y enters
// halved so that N_k equals the normal coordinates of the standard chain.
__global__ void __launch_bounds__(256, 2) k_lanepair(uint32_t* io, size_t n, int reps) {
    const size_t l = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t i = l >> 1;
    const bool c1 = l & 1;
    if (i >= n) return;
    Fq<2> x0, x1, y0, y1, z0, z1;
#pragma unroll
    for (int d = 0; d < 9; ++d) {
        x0.v[d] = io[d * n + i];
        x1.v[d] = io[(9 + d) * n + i];
        y0.v[d] = io[(18 + d) * n + i];
        y1.v[d] = io[(27 + d) * n + i];
        z0.v[d] = io[(36 + d) * n + i];
        z1.v[d] = io[(45 + d) * n + i];
    }
    Fq<2> x = c1 ? fq_fold(fq_sub(x0, x1)) : fq_fold(fq_add(x0, x1));
    Fq<2> z = c1 ? fq_fold(fq_sub(z0, z1)) : fq_fold(fq_add(z0, z1));
    Fq<2> y = fq_fold(fq_half(c1 ? fq_fold(fq_sub(y0, y1)) : fq_fold(fq_add(y0, y1))));
#pragma unroll 1
    for (int r = 0; r < reps; ++r) {
        fq_fence(y);
        x = lp_mul(x, y);
        z = lp_mul(z, y);
    }
    // back to the standard basis: x0 = (n0 + n1)/2, x1 = (n0 - n1)/2
    const Fq<2> xo = partner(x), zo = partner(z);
    const Fq<1> a = fq_canonical(fq_half(c1 ? fq_fold(fq_sub(xo, x)) : fq_fold(fq_add(x, xo))));
    const Fq<1> b = fq_canonical(fq_half(c1 ? fq_fold(fq_sub(zo, z)) : fq_fold(fq_add(z, zo))));
    const size_t off = c1 ? 9 : 0;
#pragma unroll
    for (int d = 0; d < 9; ++d) {
        io[(54 + off + d) * n + i] = a.v[d];
        io[(72 + off + d) * n + i] = b.v[d];
    }
}

int main(int argc, char** argv) {
    const size_t n = argc > 1 ? strtoull(argv[1], 0, 0) : 65536;
    const int reps = argc > 2 ? atoi(argv[2]) : 1000;
    const size_t words = 90 * n;
    uint32_t* io;
    CK(hipMalloc(&io, words * 4));
    uint32_t* h = (uint32_t*)malloc(words * 4);
    uint32_t* r0 = (uint32_t*)malloc(words * 4);
    uint32_t* r1 = (uint32_t*)malloc(words * 4);
    uint64_t s = 7;
    for (size_t k = 0; k < 54 * n; ++k) {
        s = s * 6364136223846793005ull + 1442695040888963407ull;
        const size_t digit = (k / n) % 9;
        h[k] = (uint32_t)(s >> 35) & (digit == 8 ? 0x3fffffu : 0x1fffffffu);  // value < 2^254 < p
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto run = [&](const char* name, void (*k)(uint32_t*, size_t, int), size_t lanes, uint32_t* keep) {
        const dim3 grid((lanes + 255) / 256);
        CK(hipMemcpy(io, h, 54 * n * 4, hipMemcpyHostToDevice));
        hipLaunchKernelGGL(k, grid, dim3(256), 0, 0, io, n, 10);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(io, h, 54 * n * 4, hipMemcpyHostToDevice));
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(k, grid, dim3(256), 0, 0, io, n, reps);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        CK(hipMemcpy(keep, io, words * 4, hipMemcpyDeviceToHost));
        const double muls = (double)n * reps * 2;
        printf("{\"variant\": \"%s\", \"elements\": %zu, \"waves\": %zu, \"ms\": %.3f, \"G_fq2mul_per_s\": %.3f}\n",
               name, n, lanes / 64, ms, muls / ms / 1e6);
    };
    run("schoolbook, 1 lane per element", k_base, n, r0);
    run("normal-basis lane pair, 2 lanes per element", k_lanepair, 2 * n, r1);
    size_t diff = 0;
    for (size_t k = 54 * n; k < 90 * n; ++k) diff += r0[k] != r1[k];
    printf("{\"check\": \"lane pair vs schoolbook, standard-basis canonical words\", \"differing_words\": %zu}\n", diff);
    return diff != 0;
}
