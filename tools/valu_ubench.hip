// valu_ubench.hip -- VALU issue on gfx950 for the instruction shapes of the
// Fq2 column sums: v_mad_u64_u32 accumulate chains (dependency through the
// 64-bit addend), 1/2/4/8 interleaved chains, carry-out into one shared SGPR
// pair vs distinct pairs, MADs mixed with independent VOP2 ops, and the
// column shift / 64-bit add, at one and two waves per SIMD.  Wall-clock timed
// (HIP events, 2.4 GHz assumed), each pattern 64 instructions per iteration.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/valu_ubench tools/valu_ubench.hip
#include <hip/hip_runtime.h>
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

#define X4(s) s s s s
#define X8(s) X4(s) X4(s)
#define X16(s) X8(s) X8(s)
#define X32(s) X16(s) X16(s)
#define X64(s) X32(s) X32(s)

constexpr int kIters = 4096;

template <int K>
__global__ void __launch_bounds__(256) k_bench(uint32_t* out, uint32_t seed) {
    uint64_t a0 = seed, a1 = seed * 3u, a2 = seed * 5u, a3 = seed * 7u;
    uint64_t a4 = seed * 9u, a5 = seed * 11u, a6 = seed * 13u, a7 = seed * 15u;
    uint32_t x = seed ^ 0x1234u, y = seed ^ 0x5678u, z = seed + 11u;
    uint32_t u0 = seed, u1 = seed + 1, u2 = seed + 2, u3 = seed + 3;
#pragma unroll 1
    for (int it = 0; it < kIters; ++it) {
        if constexpr (K == 0) {  // one accumulate chain
            asm volatile(X64("v_mad_u64_u32 %0, vcc, %1, %2, %0\n") : "+v"(a0) : "v"(x), "v"(y) : "vcc");
        } else if constexpr (K == 1) {  // two interleaved chains
            asm volatile(X32("v_mad_u64_u32 %0, vcc, %2, %3, %0\n v_mad_u64_u32 %1, vcc, %2, %4, %1\n")
                         : "+v"(a0), "+v"(a1) : "v"(x), "v"(y), "v"(z) : "vcc");
        } else if constexpr (K == 2) {  // four interleaved chains
            asm volatile(X16("v_mad_u64_u32 %0, vcc, %4, %5, %0\n v_mad_u64_u32 %1, vcc, %4, %6, %1\n"
                             "v_mad_u64_u32 %2, vcc, %5, %6, %2\n v_mad_u64_u32 %3, vcc, %6, %4, %3\n")
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(x), "v"(y), "v"(z) : "vcc");
        } else if constexpr (K == 3) {  // eight interleaved chains
            asm volatile(X8("v_mad_u64_u32 %0, vcc, %8, %9, %0\n v_mad_u64_u32 %1, vcc, %8, %10, %1\n"
                            "v_mad_u64_u32 %2, vcc, %9, %10, %2\n v_mad_u64_u32 %3, vcc, %10, %8, %3\n"
                            "v_mad_u64_u32 %4, vcc, %8, %9, %4\n v_mad_u64_u32 %5, vcc, %8, %10, %5\n"
                            "v_mad_u64_u32 %6, vcc, %9, %10, %6\n v_mad_u64_u32 %7, vcc, %10, %8, %7\n")
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                         : "v"(x), "v"(y), "v"(z) : "vcc");
        } else if constexpr (K == 4) {  // four chains, carry-out to distinct SGPR pairs
            asm volatile(X16("v_mad_u64_u32 %0, s[90:91], %4, %5, %0\n v_mad_u64_u32 %1, s[92:93], %4, %6, %1\n"
                             "v_mad_u64_u32 %2, s[94:95], %5, %6, %2\n v_mad_u64_u32 %3, s[96:97], %6, %4, %3\n")
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(x), "v"(y), "v"(z)
                         : "s90", "s91", "s92", "s93", "s94", "s95", "s96", "s97");
        } else if constexpr (K == 5) {  // one chain, each MAD followed by an independent VOP2 add
            asm volatile(X32("v_mad_u64_u32 %0, vcc, %1, %2, %0\n v_add_u32 %3, %3, %1\n")
                         : "+v"(a0) : "v"(x), "v"(y), "v"(u0) : "vcc");
        } else if constexpr (K == 6) {  // two chains + VOP2 adds, 1:1
            asm volatile(X16("v_mad_u64_u32 %0, vcc, %2, %3, %0\n v_add_u32 %4, %4, %2\n"
                             "v_mad_u64_u32 %1, vcc, %2, %3, %1\n v_add_u32 %5, %5, %3\n")
                         : "+v"(a0), "+v"(a1) : "v"(x), "v"(y), "v"(u0), "v"(u1) : "vcc");
        } else if constexpr (K == 7) {  // independent VOP2 adds
            asm volatile(X16("v_add_u32 %0, %0, %4\n v_add_u32 %1, %1, %4\n v_add_u32 %2, %2, %4\n v_add_u32 %3, %3, %4\n")
                         : "+v"(u0), "+v"(u1), "+v"(u2), "+v"(u3) : "v"(x));
        } else if constexpr (K == 8) {  // dependent VOP2 add chain
            asm volatile(X64("v_add_u32 %0, %0, %1\n") : "+v"(u0) : "v"(x));
        } else if constexpr (K == 9) {  // column glue: 64-bit shift + 64-bit add, 4 independent pairs
            asm volatile(X8("v_lshrrev_b64 %0, 29, %0\n v_lshl_add_u64 %1, %1, 0, %0\n"
                            "v_lshrrev_b64 %2, 29, %2\n v_lshl_add_u64 %3, %3, 0, %2\n"
                            "v_lshrrev_b64 %0, 29, %0\n v_lshl_add_u64 %1, %1, 0, %0\n"
                            "v_lshrrev_b64 %2, 29, %2\n v_lshl_add_u64 %3, %3, 0, %2\n")
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3));
        } else if constexpr (K == 10) {  // v_mul_lo_u32 independent
            asm volatile(X16("v_mul_lo_u32 %0, %0, %4\n v_mul_lo_u32 %1, %1, %4\n v_mul_lo_u32 %2, %2, %4\n v_mul_lo_u32 %3, %3, %4\n")
                         : "+v"(u0), "+v"(u1), "+v"(u2), "+v"(u3) : "v"(x));
        } else if constexpr (K == 11) {  // v_add3_u32 independent (VOP3, 3 inputs)
            asm volatile(X16("v_add3_u32 %0, %0, %4, %5\n v_add3_u32 %1, %1, %4, %5\n v_add3_u32 %2, %2, %4, %5\n v_add3_u32 %3, %3, %4, %5\n")
                         : "+v"(u0), "+v"(u1), "+v"(u2), "+v"(u3) : "v"(x), "v"(y));
        }
    }
    if ((uint32_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ x ^ y ^ z ^ u0 ^ u1 ^ u2 ^ u3) == 0x12345679u) out[0] = 1;
}

static const char* kNames[] = {"mad64 1 chain",        "mad64 2 chains",          "mad64 4 chains",
                               "mad64 8 chains",       "mad64 4 chains, own sdst", "mad64 1 chain + add 1:1",
                               "mad64 2 chains + add", "add indep x4",            "add 1 dep chain",
                               "lshr64+lshl_add64 x2", "mul_lo_u32 indep x4",     "add3 indep x4"};

template <int K>
static void run(uint32_t* d, int waves_per_simd) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int blocks = 256 * waves_per_simd;
    k_bench<K><<<blocks, 256>>>(d, 7);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    k_bench<K><<<blocks, 256>>>(d, 7);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double instr = 64.0 * kIters;  // per wave
    printf("{\"pattern\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.4f, \"cycles_per_wave_instr\": %.2f, "
           "\"simd_cycles_per_instr\": %.2f}\n",
           kNames[K], waves_per_simd, ms, ms * 1e-3 * 2.4e9 / instr, ms * 1e-3 * 2.4e9 / instr / waves_per_simd);
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
}

template <int K>
static void all(uint32_t* d) {
    run<K>(d, 1);
    run<K>(d, 2);
    if constexpr (K < 11) all<K + 1>(d);
}

int main() {
    uint32_t* d;
    CK(hipMalloc(&d, 64));
    all<0>(d);
    CK(hipFree(d));
    return 0;
}
