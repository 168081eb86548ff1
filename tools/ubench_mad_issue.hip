// tools/ubench_mad_issue.hip -- profiles/r3j_mad_issue.txt
// Microbenchmark: issue rate and dependent latency of v_mad_u64_u32 on gfx950.
// One workgroup of W waves on one CU (W = 1: a lone wave on its SIMD; W = 8:
// two waves per SIMD).  Each wave runs R rounds of a chain of instructions and
// reports s_memtime cycles per instruction.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int R = 512;

template <int K>
__global__ void k_mad(uint64_t* out, uint32_t a0, uint32_t b0) {
    uint64_t acc[K];
    uint32_t a = a0 + threadIdx.x, b = b0 ^ threadIdx.x;
#pragma unroll
    for (int k = 0; k < K; ++k) acc[k] = k;
    const uint64_t t0 = __builtin_amdgcn_s_memtime(); const uint64_t r0 = __builtin_amdgcn_s_memrealtime();
#pragma unroll 1
    for (int r = 0; r < R; ++r) {
#pragma unroll
        for (int j = 0; j < 32 / K; ++j)
#pragma unroll
            for (int k = 0; k < K; ++k)
                { uint64_t cc; asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc[k]), "=s"(cc) : "v"(a), "v"(b)); }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime(); const uint64_t r1 = __builtin_amdgcn_s_memrealtime();
    uint64_t s = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) s += acc[k];
    if (threadIdx.x % 64 == 0) { out[threadIdx.x / 64] = t1 - t0; out[32 + threadIdx.x / 64] = r1 - r0; }
    if (s == 12345) out[63] = s;
}

// plain 32-bit add chains for comparison
template <int K>
__global__ void k_add(uint64_t* out, uint32_t a0, uint32_t b0) {
    uint32_t acc[K];
    uint32_t a = a0 + threadIdx.x;
#pragma unroll
    for (int k = 0; k < K; ++k) acc[k] = k;
    const uint64_t t0 = __builtin_amdgcn_s_memtime(); const uint64_t r0 = __builtin_amdgcn_s_memrealtime();
#pragma unroll 1
    for (int r = 0; r < R; ++r) {
#pragma unroll
        for (int j = 0; j < 32 / K; ++j)
#pragma unroll
            for (int k = 0; k < K; ++k) asm volatile("v_add_u32 %0, %0, %1" : "+v"(acc[k]) : "v"(a));
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime(); const uint64_t r1 = __builtin_amdgcn_s_memrealtime();
    uint32_t s = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) s += acc[k];
    if (threadIdx.x % 64 == 0) { out[threadIdx.x / 64] = t1 - t0; out[32 + threadIdx.x / 64] = r1 - r0; }
    if (s == 12345) out[63] = s;
}

// v_add_co / v_addc carry chain of one 64-bit add per step
template <int K>
__global__ void k_add64(uint64_t* out, uint32_t a0, uint32_t b0) {
    uint64_t acc[K];
    uint64_t a = a0 + threadIdx.x;
#pragma unroll
    for (int k = 0; k < K; ++k) acc[k] = k;
    const uint64_t t0 = __builtin_amdgcn_s_memtime(); const uint64_t r0 = __builtin_amdgcn_s_memrealtime();
#pragma unroll 1
    for (int r = 0; r < R; ++r) {
#pragma unroll
        for (int j = 0; j < 32 / K; ++j)
#pragma unroll
            for (int k = 0; k < K; ++k) asm volatile("v_lshl_add_u64 %0, %1, 0, %0" : "+v"(acc[k]) : "v"(a));
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime(); const uint64_t r1 = __builtin_amdgcn_s_memrealtime();
    uint64_t s = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) s += acc[k];
    if (threadIdx.x % 64 == 0) { out[threadIdx.x / 64] = t1 - t0; out[32 + threadIdx.x / 64] = r1 - r0; }
    if (s == 12345) out[63] = s;
}


template <int K>
__global__ void k_fma(uint64_t* out, uint32_t a0, uint32_t b0) {
    float acc[K];
    float a = 1.0001f + threadIdx.x, b = 0.999f;
#pragma unroll
    for (int k = 0; k < K; ++k) acc[k] = k;
    const uint64_t t0 = __builtin_amdgcn_s_memtime(); const uint64_t r0 = __builtin_amdgcn_s_memrealtime();
#pragma unroll 1
    for (int r = 0; r < R; ++r) {
#pragma unroll
        for (int j = 0; j < 32 / K; ++j)
#pragma unroll
            for (int k = 0; k < K; ++k) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(acc[k]) : "v"(a), "v"(b));
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime(); const uint64_t r1 = __builtin_amdgcn_s_memrealtime();
    float s = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) s += acc[k];
    if (threadIdx.x % 64 == 0) { out[threadIdx.x / 64] = t1 - t0; out[32 + threadIdx.x / 64] = r1 - r0; }
    if (s == 12345.f) out[63] = 1;
}

template <class F>
void run(const char* name, F kern, int waves, uint64_t* d) {
    uint64_t h[64] = {};
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(kern, dim3(1), dim3(64 * waves), 0, 0, d, 3u, 5u);
        hipDeviceSynchronize();
    }
    hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
    double mx = 0, rt = 0;
    for (int w = 0; w < waves; ++w) { mx = h[w] > mx ? h[w] : mx; rt = h[32 + w] > rt ? h[32 + w] : rt; }
    printf("%-12s waves %2d  ticks/instr/wave %.2f  ns/instr/wave %.3f  ticks per ns %.3f\n", name, waves,
           mx / (R * 32.0), rt * 10.0 / (R * 32.0), mx / (rt * 10.0));
}

int main() {
    uint64_t* d;
    hipMalloc(&d, 64 * 8);
    for (int i = 0; i < 200; ++i) hipLaunchKernelGGL(k_mad<8>, dim3(1024), dim3(256), 0, 0, d, 3u, 5u);  // warm the clock
    hipDeviceSynchronize();
    for (int w : {1, 4, 8, 12, 16}) {
        run("fma dep1", k_fma<1>, w, d);
        run("fma dep8", k_fma<8>, w, d);
        run("mad dep1", k_mad<1>, w, d);
        run("mad dep2", k_mad<2>, w, d);
        run("mad dep4", k_mad<4>, w, d);
        run("mad dep8", k_mad<8>, w, d);
        run("mad dep16", k_mad<16>, w, d);
        run("add dep1", k_add<1>, w, d);
        run("add dep8", k_add<8>, w, d);
        run("add64 dep1", k_add64<1>, w, d);
        run("add64 dep8", k_add64<8>, w, d);
    }
    return 0;
}
