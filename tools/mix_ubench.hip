// mix_ubench.hip -- how gfx950 issues MIXED VALU streams at two waves per SIMD
// (the pairing kernels' occupancy): the same multiset of v_mad_u64_u32 and
// VOP2 ops interleaved vs grouped, and the per-op price of the glue shapes the
// Fq column sums use (literal vs SGPR mask operand, VOP2 vs VOP3 select, DPP
// move, 64-bit shift).  Wall-clock timed (HIP events, 2.4 GHz assumed), each
// pattern 64 instructions per iteration.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/mix_ubench tools/mix_ubench.hip
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

#define X2(s) s s
#define X4(s) X2(s) X2(s)
#define X8(s) X4(s) X4(s)
#define X16(s) X8(s) X8(s)
#define X32(s) X16(s) X16(s)
#define X64(s) X32(s) X32(s)

constexpr int kIters = 4096;
#define MAD4 "v_mad_u64_u32 %0, vcc, %8, %9, %0\n v_mad_u64_u32 %1, vcc, %8, %10, %1\n" \
             "v_mad_u64_u32 %2, vcc, %9, %10, %2\n v_mad_u64_u32 %3, vcc, %10, %8, %3\n"
#define ADD4 "v_add_u32 %4, %4, %8\n v_add_u32 %5, %5, %9\n v_add_u32 %6, %6, %10\n v_add_u32 %7, %7, %8\n"
#define MA_ALT "v_mad_u64_u32 %0, vcc, %8, %9, %0\n v_add_u32 %4, %4, %8\n" \
               "v_mad_u64_u32 %1, vcc, %8, %10, %1\n v_add_u32 %5, %5, %9\n" \
               "v_mad_u64_u32 %2, vcc, %9, %10, %2\n v_add_u32 %6, %6, %10\n" \
               "v_mad_u64_u32 %3, vcc, %10, %8, %3\n v_add_u32 %7, %7, %8\n"
#define OUTS "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(u0), "+v"(u1), "+v"(u2), "+v"(u3)
#define INS "v"(x), "v"(y), "v"(z)

template <int K>
__global__ void __launch_bounds__(256) k_bench(uint32_t* out, uint32_t seed, uint32_t mask) {
    uint64_t a0 = seed, a1 = seed * 3u, a2 = seed * 5u, a3 = seed * 7u;
    uint32_t x = seed ^ 0x1234u, y = seed ^ 0x5678u, z = seed + 11u;
    uint32_t u0 = seed, u1 = seed + 1, u2 = seed + 2, u3 = seed + 3;
    const bool odd = (threadIdx.x & 1u) != 0;
    const uint64_t lm = __builtin_amdgcn_ballot_w64(odd);
#pragma unroll 1
    for (int it = 0; it < kIters; ++it) {
        if constexpr (K == 0) {  // MADs only, 4 chains
            asm volatile(X16(MAD4) : OUTS : INS : "vcc");
        } else if constexpr (K == 1) {  // MAD and VOP2 add alternating 1:1
            asm volatile(X8(MA_ALT) : OUTS : INS : "vcc");
        } else if constexpr (K == 2) {  // the same, grouped 4 + 4
            asm volatile(X8(MAD4 ADD4) : OUTS : INS : "vcc");
        } else if constexpr (K == 3) {  // the same, grouped 16 + 16
            asm volatile(X2(X4(MAD4) X4(ADD4)) : OUTS : INS : "vcc");
        } else if constexpr (K == 4) {  // VOP2 adds only
            asm volatile(X16(ADD4) : OUTS : INS : "vcc");
        } else if constexpr (K == 5) {  // v_and_b32 with a 32-bit literal (the M29 mask as emitted)
            asm volatile(X16("v_and_b32 %4, 0x1fffffff, %4\n v_and_b32 %5, 0x1fffffff, %5\n"
                             "v_and_b32 %6, 0x1fffffff, %6\n v_and_b32 %7, 0x1fffffff, %7\n")
                         : OUTS : INS : "vcc");
        } else if constexpr (K == 6) {  // v_and_b32 with the mask in an SGPR
            asm volatile(X16("v_and_b32 %4, %11, %4\n v_and_b32 %5, %11, %5\n"
                             "v_and_b32 %6, %11, %6\n v_and_b32 %7, %11, %7\n")
                         : OUTS : INS, "s"(mask) : "vcc");
        } else if constexpr (K == 7) {  // VOP2 select on vcc
            asm volatile("s_mov_b64 vcc, %11\n" X16("v_cndmask_b32 %4, %4, %8, vcc\n v_cndmask_b32 %5, %5, %9, vcc\n"
                             "v_cndmask_b32 %6, %6, %10, vcc\n v_cndmask_b32 %7, %7, %8, vcc\n")
                         : OUTS : INS, "s"(lm) : "vcc");
        } else if constexpr (K == 8) {  // VOP3 select on an SGPR pair
            asm volatile(X16("v_cndmask_b32_e64 %4, %4, %8, %11\n v_cndmask_b32_e64 %5, %5, %9, %11\n"
                             "v_cndmask_b32_e64 %6, %6, %10, %11\n v_cndmask_b32_e64 %7, %7, %8, %11\n")
                         : OUTS : INS, "s"(lm) : "vcc");
        } else if constexpr (K == 9) {  // DPP partner move
            asm volatile(X16("v_mov_b32_dpp %4, %8 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
                             "v_mov_b32_dpp %5, %9 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
                             "v_mov_b32_dpp %6, %10 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
                             "v_mov_b32_dpp %7, %8 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n")
                         : OUTS : INS : "vcc");
        } else if constexpr (K == 10) {  // 64-bit column shift, independent
            asm volatile(X16("v_lshrrev_b64 %0, 29, %0\n v_lshrrev_b64 %1, 29, %1\n"
                             "v_lshrrev_b64 %2, 29, %2\n v_lshrrev_b64 %3, 29, %3\n")
                         : OUTS : INS : "vcc");
        } else if constexpr (K == 11) {  // VOP2 sub with a literal (K*p digit - x)
            asm volatile(X16("v_sub_u32 %4, 0x1234567, %4\n v_sub_u32 %5, 0x1234567, %5\n"
                             "v_sub_u32 %6, 0x1234567, %6\n v_sub_u32 %7, 0x1234567, %7\n")
                         : OUTS : INS : "vcc");
        } else if constexpr (K == 12) {  // MAD + and(literal) 1:1 (the REDC digit glue)
            asm volatile(X8("v_mad_u64_u32 %0, vcc, %8, %9, %0\n v_and_b32 %4, 0x1fffffff, %4\n"
                            "v_mad_u64_u32 %1, vcc, %8, %10, %1\n v_and_b32 %5, 0x1fffffff, %5\n"
                            "v_mad_u64_u32 %2, vcc, %9, %10, %2\n v_and_b32 %6, 0x1fffffff, %6\n"
                            "v_mad_u64_u32 %3, vcc, %10, %8, %3\n v_and_b32 %7, 0x1fffffff, %7\n")
                         : OUTS : INS : "vcc");
        } else if constexpr (K == 13) {  // MAD + and(SGPR) 1:1
            asm volatile(X8("v_mad_u64_u32 %0, vcc, %8, %9, %0\n v_and_b32 %4, %11, %4\n"
                            "v_mad_u64_u32 %1, vcc, %8, %10, %1\n v_and_b32 %5, %11, %5\n"
                            "v_mad_u64_u32 %2, vcc, %9, %10, %2\n v_and_b32 %6, %11, %6\n"
                            "v_mad_u64_u32 %3, vcc, %10, %8, %3\n v_and_b32 %7, %11, %7\n")
                         : OUTS : INS, "s"(mask) : "vcc");
        } else if constexpr (K == 14) {  // 3 MADs : 1 add (the kernels' ratio, roughly)
            asm volatile(X16("v_mad_u64_u32 %0, vcc, %8, %9, %0\n v_mad_u64_u32 %1, vcc, %8, %10, %1\n"
                             "v_mad_u64_u32 %2, vcc, %9, %10, %2\n v_add_u32 %4, %4, %8\n")
                         : OUTS : INS : "vcc");
        } else if constexpr (K == 15) {  // v_add3_u32 vs two VOP2 adds: two adds here
            asm volatile(X16("v_add_u32 %4, %4, %8\n v_add_u32 %4, %4, %9\n"
                             "v_add_u32 %5, %5, %8\n v_add_u32 %5, %5, %9\n")
                         : OUTS : INS : "vcc");
        }
    }
    if ((uint32_t)(a0 ^ a1 ^ a2 ^ a3 ^ x ^ y ^ z ^ u0 ^ u1 ^ u2 ^ u3) == 0x12345679u) out[0] = 1;
}

static const char* kNames[] = {"mad only",          "mad+add alternating", "mad4+add4 grouped", "mad16+add16 grouped",
                               "add only",          "and literal",         "and sgpr",          "cndmask vop2 vcc",
                               "cndmask vop3 sgpr", "dpp mov",             "lshrrev_b64",       "sub literal",
                               "mad+and literal",   "mad+and sgpr",        "3 mad : 1 add",     "add pairs (add3 as 2 vop2)"};

template <int K>
static void run(uint32_t* d, int waves_per_simd) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int blocks = 256 * waves_per_simd;
    k_bench<K><<<blocks, 256>>>(d, 7, 0x1fffffffu);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    k_bench<K><<<blocks, 256>>>(d, 7, 0x1fffffffu);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double instr = 64.0 * kIters;  // per wave
    printf("{\"pattern\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.4f, \"simd_cycles_per_instr\": %.2f}\n", kNames[K],
           waves_per_simd, ms, ms * 1e-3 * 2.4e9 / instr / waves_per_simd);
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
}

template <int K>
static void all(uint32_t* d) {
    run<K>(d, 2);
    run<K>(d, 4);
    if constexpr (K < 15) all<K + 1>(d);
}

int main() {
    uint32_t* d;
    CK(hipMalloc(&d, 64));
    all<0>(d);
    CK(hipFree(d));
    return 0;
}
