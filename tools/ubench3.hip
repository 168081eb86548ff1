// ubench3.hip -- wave placement census and single-wave VALU issue/latency on gfx950.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <map>

#define CK(x)                                                                                      \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
            exit(1);                                                                               \
        }                                                                                          \
    } while (0)

// HW_REG_HW_ID (gfx9): wave_id[3:0] simd_id[5:4] pipe[7:6] cu_id[11:8] sh_id[12] se_id[15:13]
// HW_REG_XCC_ID: xcc_id[3:0]
__global__ void k_census(uint32_t* out, int spin) {
    uint32_t hw = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));   // HW_ID, offset 0, size 32
    uint32_t xcc = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (3 << 11));  // XCC_ID bits 0..3
    // keep waves resident long enough that all are co-resident
    uint64_t t0 = __builtin_amdgcn_s_memtime();
    while ((int64_t)(__builtin_amdgcn_s_memtime() - t0) < spin) {
    }
    if (threadIdx.x % 64 == 0) {
        const int w = (blockIdx.x * blockDim.x + threadIdx.x) / 64;
        out[2 * w] = hw;
        out[2 * w + 1] = xcc;
    }
}

// per-wave cycles for N dependent / independent instructions
template <int KIND>
__global__ void k_issue(uint64_t* out, int iters) {
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;
    uint64_t m0 = threadIdx.x, m1 = m0 + 1, m2 = m0 + 2, m3 = m0 + 3, cc;
    uint32_t x = threadIdx.x | 1;
    uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) {
        if (KIND == 0)  // 16 dependent VOP2 adds
            asm volatile(
                "v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n"
                "v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n"
                "v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n"
                "v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n"
                : "+v"(a0) : "v"(x));
        else if (KIND == 1)  // 16 independent VOP2 adds (4 chains)
            asm volatile(
                "v_add_u32 %0, %0, %4\n v_add_u32 %1, %1, %4\n v_add_u32 %2, %2, %4\n v_add_u32 %3, %3, %4\n"
                "v_add_u32 %0, %0, %4\n v_add_u32 %1, %1, %4\n v_add_u32 %2, %2, %4\n v_add_u32 %3, %3, %4\n"
                "v_add_u32 %0, %0, %4\n v_add_u32 %1, %1, %4\n v_add_u32 %2, %2, %4\n v_add_u32 %3, %3, %4\n"
                "v_add_u32 %0, %0, %4\n v_add_u32 %1, %1, %4\n v_add_u32 %2, %2, %4\n v_add_u32 %3, %3, %4\n"
                : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(x));
        else if (KIND == 2)  // 16 dependent v_mad_u64_u32
            asm volatile(
                "v_mad_u64_u32 %0, %1, %2, %2, %0\n v_mad_u64_u32 %0, %1, %2, %2, %0\n v_mad_u64_u32 %0, %1, %2, %2, %0\n v_mad_u64_u32 %0, %1, %2, %2, %0\n"
                "v_mad_u64_u32 %0, %1, %2, %2, %0\n v_mad_u64_u32 %0, %1, %2, %2, %0\n v_mad_u64_u32 %0, %1, %2, %2, %0\n v_mad_u64_u32 %0, %1, %2, %2, %0\n"
                "v_mad_u64_u32 %0, %1, %2, %2, %0\n v_mad_u64_u32 %0, %1, %2, %2, %0\n v_mad_u64_u32 %0, %1, %2, %2, %0\n v_mad_u64_u32 %0, %1, %2, %2, %0\n"
                "v_mad_u64_u32 %0, %1, %2, %2, %0\n v_mad_u64_u32 %0, %1, %2, %2, %0\n v_mad_u64_u32 %0, %1, %2, %2, %0\n v_mad_u64_u32 %0, %1, %2, %2, %0\n"
                : "+v"(m0), "=&s"(cc) : "v"(x));
        else  // 16 independent v_mad_u64_u32 (4 chains)
            asm volatile(
                "v_mad_u64_u32 %0, %4, %5, %5, %0\n v_mad_u64_u32 %1, %4, %5, %5, %1\n v_mad_u64_u32 %2, %4, %5, %5, %2\n v_mad_u64_u32 %3, %4, %5, %5, %3\n"
                "v_mad_u64_u32 %0, %4, %5, %5, %0\n v_mad_u64_u32 %1, %4, %5, %5, %1\n v_mad_u64_u32 %2, %4, %5, %5, %2\n v_mad_u64_u32 %3, %4, %5, %5, %3\n"
                "v_mad_u64_u32 %0, %4, %5, %5, %0\n v_mad_u64_u32 %1, %4, %5, %5, %1\n v_mad_u64_u32 %2, %4, %5, %5, %2\n v_mad_u64_u32 %3, %4, %5, %5, %3\n"
                "v_mad_u64_u32 %0, %4, %5, %5, %0\n v_mad_u64_u32 %1, %4, %5, %5, %1\n v_mad_u64_u32 %2, %4, %5, %5, %2\n v_mad_u64_u32 %3, %4, %5, %5, %3\n"
                : "+v"(m0), "+v"(m1), "+v"(m2), "+v"(m3), "=&s"(cc) : "v"(x));
    }
    uint64_t t1 = __builtin_amdgcn_s_memtime();
    const int w = (blockIdx.x * blockDim.x + threadIdx.x) / 64;
    if (threadIdx.x % 64 == 0) out[w] = t1 - t0;
    if ((a0 ^ a1 ^ a2 ^ a3 ^ (uint32_t)(m0 ^ m1 ^ m2 ^ m3)) == 0x12345) out[0] = 0;
}

static void census(const char* label, int blocks, int threads) {
    int waves = blocks * threads / 64;
    uint32_t* d;
    CK(hipMalloc(&d, waves * 8));
    k_census<<<blocks, threads>>>(d, 2000000);
    CK(hipDeviceSynchronize());
    uint32_t* h = (uint32_t*)malloc(waves * 8);
    CK(hipMemcpy(h, d, waves * 8, hipMemcpyDeviceToHost));
    std::map<uint64_t, int> per_simd, per_cu;
    for (int w = 0; w < waves; ++w) {
        uint32_t hw = h[2 * w], xcc = h[2 * w + 1] & 0xf;
        uint32_t simd = (hw >> 4) & 3, cu = (hw >> 8) & 0xf, sh = (hw >> 12) & 1, se = (hw >> 13) & 7;
        uint64_t cukey = ((uint64_t)xcc << 16) | (se << 8) | (sh << 4) | cu;
        per_cu[cukey]++;
        per_simd[(cukey << 4) | simd]++;
    }
    std::map<int, int> hist;
    for (auto& kv : per_simd) hist[kv.second]++;
    printf("{\"bench\": \"census\", \"launch\": \"%s\", \"waves\": %d, \"cus_used\": %zu, \"simds_used\": %zu, \"waves_per_simd_hist\": {",
           label, waves, per_cu.size(), per_simd.size());
    bool first = true;
    for (auto& kv : hist) {
        printf("%s\"%d\": %d", first ? "" : ", ", kv.first, kv.second);
        first = false;
    }
    printf("}}\n");
    free(h);
    CK(hipFree(d));
}

int main() {
    census("1024x64", 1024, 64);
    census("256x256", 256, 256);
    census("2048x64", 2048, 64);
    census("512x128", 512, 128);
    uint64_t* d;
    CK(hipMalloc(&d, 1 << 20));
    uint64_t h[4096];
    const char* names[4] = {"add_dep", "add_indep4", "mad_dep", "mad_indep4"};
    for (int k = 0; k < 4; ++k) {
        const int iters = 2048;
        // one block of 256 threads on one CU (4 waves, one per SIMD) -- no contention
        for (int cfg = 0; cfg < 2; ++cfg) {
            int blocks = cfg == 0 ? 1 : 256, threads = 256;
            if (k == 0) k_issue<0><<<blocks, threads>>>(d, iters);
            if (k == 1) k_issue<1><<<blocks, threads>>>(d, iters);
            if (k == 2) k_issue<2><<<blocks, threads>>>(d, iters);
            if (k == 3) k_issue<3><<<blocks, threads>>>(d, iters);
            CK(hipDeviceSynchronize());
            CK(hipMemcpy(h, d, 8 * 4, hipMemcpyDeviceToHost));
            printf("{\"bench\": \"issue\", \"kind\": \"%s\", \"blocks\": %d, \"cycles_per_instr_wave0\": %.2f}\n", names[k],
                   blocks, (double)h[0] / (iters * 16.0));
        }
    }
    return 0;
}
