// ubench.hip -- integer-VALU microbenchmarks on MI355X (gfx950) that set the
// roofline denominator for the pairing engine ("peak_MAD32_rate
// is measured, AMD does not publish it").  Prints one JSON object per line.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench tools/ubench.hip
//   ./tools/ubench
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "../paritytech-bn_amd/csrc/fq.h"

#define CK(x)                                                                      \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
            exit(1);                                                               \
        }                                                                          \
    } while (0)

// 8 independent v_mad_u64_u32 chains per lane
__global__ void k_mad_tput(uint64_t* out, uint32_t x, uint32_t y, int iters) {
    uint64_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    uint32_t xv = x + threadIdx.x, yv = y ^ blockIdx.x;
    uint64_t cc0;
    for (int i = 0; i < iters; ++i) {
        asm volatile(
            "v_mad_u64_u32 %0, %8, %9, %10, %0\n\t"
            "v_mad_u64_u32 %1, %8, %9, %10, %1\n\t"
            "v_mad_u64_u32 %2, %8, %9, %10, %2\n\t"
            "v_mad_u64_u32 %3, %8, %9, %10, %3\n\t"
            "v_mad_u64_u32 %4, %8, %9, %10, %4\n\t"
            "v_mad_u64_u32 %5, %8, %9, %10, %5\n\t"
            "v_mad_u64_u32 %6, %8, %9, %10, %6\n\t"
            "v_mad_u64_u32 %7, %8, %9, %10, %7\n\t"
            : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7), "=&s"(cc0)
            : "v"(xv), "v"(yv));
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
// 8 independent (mad + addc) chains per lane -- the FIPS inner step
__global__ void k_mac_tput(uint64_t* out, uint32_t x, uint32_t y, int iters) {
    uint64_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;
    uint32_t o0 = 0, o1 = 0, o2 = 0, o3 = 0;
    uint64_t c0, c1, c2, c3;
    uint32_t xv = x + threadIdx.x, yv = y ^ blockIdx.x;
    for (int i = 0; i < iters; ++i) {
        asm volatile(
            "v_mad_u64_u32 %0, %8, %12, %13, %0\n\t"
            "v_mad_u64_u32 %1, %9, %12, %13, %1\n\t"
            "v_mad_u64_u32 %2, %10, %12, %13, %2\n\t"
            "v_mad_u64_u32 %3, %11, %12, %13, %3\n\t"
            "v_addc_co_u32_e64 %4, %8, 0, %4, %8\n\t"
            "v_addc_co_u32_e64 %5, %9, 0, %5, %9\n\t"
            "v_addc_co_u32_e64 %6, %10, 0, %6, %10\n\t"
            "v_addc_co_u32_e64 %7, %11, 0, %7, %11\n\t"
            : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(o0), "+v"(o1), "+v"(o2), "+v"(o3),
              "=&s"(c0), "=&s"(c1), "=&s"(c2), "=&s"(c3)
            : "v"(xv), "v"(yv));
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ o0 ^ o1 ^ o2 ^ o3;
}
// one dependent v_mad_u64_u32 chain per lane: latency
__global__ void k_mad_lat(uint64_t* out, uint32_t x, int iters) {
    uint64_t a0 = threadIdx.x, cc;
    uint32_t xv = x + threadIdx.x;
    for (int i = 0; i < iters; ++i) {
        asm volatile(
            "v_mad_u64_u32 %0, %1, %2, %2, %0\n\t"
            "v_mad_u64_u32 %0, %1, %2, %2, %0\n\t"
            "v_mad_u64_u32 %0, %1, %2, %2, %0\n\t"
            "v_mad_u64_u32 %0, %1, %2, %2, %0\n\t"
            "v_mad_u64_u32 %0, %1, %2, %2, %0\n\t"
            "v_mad_u64_u32 %0, %1, %2, %2, %0\n\t"
            "v_mad_u64_u32 %0, %1, %2, %2, %0\n\t"
            "v_mad_u64_u32 %0, %1, %2, %2, %0\n\t"
            : "+v"(a0), "=&s"(cc)
            : "v"(xv));
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0;
}
__global__ void k_add_tput(uint64_t* out, uint32_t x, int iters) {
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    for (int i = 0; i < iters; ++i) {
        asm volatile(
            "v_add_co_u32 %0, vcc, %0, %8\n\t"
            "v_addc_co_u32 %1, vcc, %1, %8, vcc\n\t"
            "v_add_co_u32 %2, vcc, %2, %8\n\t"
            "v_addc_co_u32 %3, vcc, %3, %8, vcc\n\t"
            "v_add_co_u32 %4, vcc, %4, %8\n\t"
            "v_addc_co_u32 %5, vcc, %5, %8, vcc\n\t"
            "v_add_co_u32 %6, vcc, %6, %8\n\t"
            "v_addc_co_u32 %7, vcc, %7, %8, vcc\n\t"
            : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
            : "v"(x)
            : "vcc");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k_mullo_tput(uint64_t* out, uint32_t x, int iters) {
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    for (int i = 0; i < iters; ++i) {
        asm volatile(
            "v_mul_lo_u32 %0, %0, %8\n\t"
            "v_mul_lo_u32 %1, %1, %8\n\t"
            "v_mul_lo_u32 %2, %2, %8\n\t"
            "v_mul_lo_u32 %3, %3, %8\n\t"
            "v_mul_lo_u32 %4, %4, %8\n\t"
            "v_mul_lo_u32 %5, %5, %8\n\t"
            "v_mul_lo_u32 %6, %6, %8\n\t"
            "v_mul_lo_u32 %7, %7, %8\n\t"
            : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
            : "v"(x));
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k_fma64_tput(double* out, double x, int iters) {
    double a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    for (int i = 0; i < iters; ++i) {
        asm volatile(
            "v_fma_f64 %0, %0, %8, %8\n\t"
            "v_fma_f64 %1, %1, %8, %8\n\t"
            "v_fma_f64 %2, %2, %8, %8\n\t"
            "v_fma_f64 %3, %3, %8, %8\n\t"
            "v_fma_f64 %4, %4, %8, %8\n\t"
            "v_fma_f64 %5, %5, %8, %8\n\t"
            "v_fma_f64 %6, %6, %8, %8\n\t"
            "v_fma_f64 %7, %7, %8, %8\n\t"
            : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
            : "v"(x));
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}
// Fq Montgomery multiplication throughput: CHAINS independent x <- x*y chains per lane
template <int CHAINS>
__global__ void k_fqmul(bn::Fq* io, int iters) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    bn::Fq y = io[i];
    bn::Fq x[CHAINS];
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) {
        x[c] = y;
        x[c].v[0] ^= c;
    }
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int c = 0; c < CHAINS; ++c) x[c] = bn::fq_mul(x[c], y);
    }
    bn::Fq r = x[0];
#pragma unroll
    for (int c = 1; c < CHAINS; ++c) r = bn::fq_add(r, x[c]);
    io[i] = r;
}
__global__ void k_fqmul_check(const bn::Fq* a, const bn::Fq* b, bn::Fq* o, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) o[i] = bn::fq_mul(a[i], b[i]);
}
__global__ void k_clock(unsigned long long* out, int iters) {
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    uint64_t a = threadIdx.x, cc;
    uint32_t xv = threadIdx.x * 3 + 1;
    for (int i = 0; i < iters; ++i)
        asm volatile("v_mad_u64_u32 %0, %1, %2, %2, %0" : "+v"(a), "=&s"(cc) : "v"(xv));
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) {
        out[blockIdx.x * 2] = t1 - t0;
        out[blockIdx.x * 2 + 1] = r1 - r0;
    }
    if (a == 0x1234) out[0] = a;
}

template <typename F>
static float time_ms(F launch, int reps) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    launch();
    CK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < reps; ++r) {
        CK(hipEventRecord(e0));
        launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (ms < best) best = ms;
    }
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
    return best;
}

int main() {
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    int cus = prop.multiProcessorCount;
    printf("{\"device\": \"%s\", \"cus\": %d, \"clock_khz\": %d}\n", prop.gcnArchName, cus, prop.clockRate);
    uint64_t* buf;
    size_t maxthreads = (size_t)cus * 32 * 64 * 4;
    CK(hipMalloc(&buf, maxthreads * 16));
    const int iters = 4096;
    for (int wps : {1, 2, 4, 8}) {  // waves per SIMD
        int blocks = cus * wps;   // 256-thread blocks = 4 waves = one per SIMD
        double lanes = (double)blocks * 256;
        float ms = time_ms([&] { k_mad_tput<<<blocks, 256>>>(buf, 3, 5, iters); }, 5);
        double rate = lanes * iters * 8 / (ms * 1e-3);
        printf("{\"bench\": \"mad_u64_u32_tput\", \"waves_per_simd\": %d, \"ms\": %.4f, \"Gmad_per_s\": %.1f}\n", wps, ms, rate / 1e9);
        ms = time_ms([&] { k_mac_tput<<<blocks, 256>>>(buf, 3, 5, iters); }, 5);
        rate = lanes * iters * 4 / (ms * 1e-3);
        printf("{\"bench\": \"mad+addc_tput\", \"waves_per_simd\": %d, \"ms\": %.4f, \"Gmac_per_s\": %.1f}\n", wps, ms, rate / 1e9);
        ms = time_ms([&] { k_add_tput<<<blocks, 256>>>(buf, 3, iters); }, 5);
        rate = lanes * iters * 8 / (ms * 1e-3);
        printf("{\"bench\": \"add_co_tput\", \"waves_per_simd\": %d, \"ms\": %.4f, \"Gop_per_s\": %.1f}\n", wps, ms, rate / 1e9);
        ms = time_ms([&] { k_mullo_tput<<<blocks, 256>>>(buf, 3, iters); }, 5);
        rate = lanes * iters * 8 / (ms * 1e-3);
        printf("{\"bench\": \"mul_lo_u32_tput\", \"waves_per_simd\": %d, \"ms\": %.4f, \"Gop_per_s\": %.1f}\n", wps, ms, rate / 1e9);
        ms = time_ms([&] { k_fma64_tput<<<blocks, 256>>>((double*)buf, 1.0000001, iters); }, 5);
        rate = lanes * iters * 8 / (ms * 1e-3);
        printf("{\"bench\": \"fma_f64_tput\", \"waves_per_simd\": %d, \"ms\": %.4f, \"Gfma_per_s\": %.1f}\n", wps, ms, rate / 1e9);
        ms = time_ms([&] { k_mad_lat<<<blocks, 256>>>(buf, 3, iters); }, 5);
        rate = lanes * iters * 8 / (ms * 1e-3);
        printf("{\"bench\": \"mad_dependent_chain\", \"waves_per_simd\": %d, \"ms\": %.4f, \"Gmad_per_s\": %.1f}\n", wps, ms, rate / 1e9);
    }
    // Fq Montgomery multiplication
    const int fiters = 256;
    for (int wps : {1, 2, 4}) {
        int blocks = cus * wps;
        double lanes = (double)blocks * 256;
        float ms = time_ms([&] { k_fqmul<1><<<blocks, 256>>>((bn::Fq*)buf, fiters); }, 3);
        printf("{\"bench\": \"fq_mul\", \"chains\": 1, \"waves_per_simd\": %d, \"ms\": %.4f, \"Gmul_per_s\": %.2f}\n", wps, ms,
               lanes * fiters / (ms * 1e-3) / 1e9);
        ms = time_ms([&] { k_fqmul<2><<<blocks, 256>>>((bn::Fq*)buf, fiters); }, 3);
        printf("{\"bench\": \"fq_mul\", \"chains\": 2, \"waves_per_simd\": %d, \"ms\": %.4f, \"Gmul_per_s\": %.2f}\n", wps, ms,
               lanes * fiters * 2 / (ms * 1e-3) / 1e9);
        ms = time_ms([&] { k_fqmul<4><<<blocks, 256>>>((bn::Fq*)buf, fiters); }, 3);
        printf("{\"bench\": \"fq_mul\", \"chains\": 4, \"waves_per_simd\": %d, \"ms\": %.4f, \"Gmul_per_s\": %.2f}\n", wps, ms,
               lanes * fiters * 4 / (ms * 1e-3) / 1e9);
    }
    // effective clock
    {
        unsigned long long* ck;
        CK(hipMalloc(&ck, cus * 4 * 16));
        int blocks = cus * 4;
        k_clock<<<blocks, 256>>>(ck, 1 << 20);
        CK(hipDeviceSynchronize());
        unsigned long long* h = (unsigned long long*)malloc(blocks * 16);
        CK(hipMemcpy(h, ck, blocks * 16, hipMemcpyDeviceToHost));
        double f = 0;
        for (int b = 0; b < blocks; ++b) f += (double)h[2 * b] / (double)h[2 * b + 1] * 100.0;
        printf("{\"bench\": \"clock\", \"mhz_mean\": %.1f}\n", f / blocks);
    }
    return 0;
}
