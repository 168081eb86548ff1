// mul12_ubench.hip -- the Fq12 product of the final-exponentiation step machine
// with its second operand (a) loaded into registers from a lane-strided HBM
// slot, or (b) copied into LDS by buffer_load ... lds and streamed per Fq2
// (mul12_lds), at one wave per SIMD.  The slot stride is laundered per
// iteration so the loads are not hoisted out of the loop (as in the step
// machine, where every step names different slots).  Both variants must give
// the same values.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/mul12_ubench tools/mul12_ubench.hip
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#include "../paritytech-bn_amd/csrc/kernels.h"

#define CK(x)                                                                                      \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
            exit(1);                                                                               \
        }                                                                                          \
    } while (0)

namespace bn {
template <int V>
__global__ void __launch_bounds__(kBlock) k_mul(uint32_t* slots, size_t n, int reps) {
    const size_t i = lane_id();
    if (i >= n) return;
    __shared__ uint32_t yl[V == 1 ? kSlotWords * kBlock : 1];
    Fq12<kF> x = ld_fq12<kF>(slots, n, i);
#pragma unroll 1
    for (int r = 0; r < reps; ++r) {
        size_t nn = n;
        asm volatile("" : "+s"(nn));
        const uint32_t* yb = slots + kSlotWords * nn;
        if constexpr (V == 0) {
            x = mul12(x, ld_fq12<kF>(yb, nn, i));
        } else {
            lds_copy_fq12(yb + (size_t)blockIdx.x * kBlock, nn, yl);
            lds_copy_wait();
            mem_fence();
            x = mul12_lds(x, yl + threadIdx.x, false);
        }
    }
    st_fq12(slots + 2 * kSlotWords * n, n, i, x);
}
}  // namespace bn
using namespace bn;

int main(int argc, char** argv) {
    const size_t n = argc > 1 ? strtoull(argv[1], 0, 0) : 65536;
    const int reps = 40;
    uint32_t* slots;
    const size_t words = 3 * kSlotWords * n;
    CK(hipMalloc(&slots, words * 4));
    std::vector<uint32_t> h(words), r0(words), r1(words);
    uint64_t s = 0x1234567;
    for (size_t k = 0; k < words; ++k) {
        s = s * 6364136223846793005ull + 1442695040888963407ull;
        const size_t digit = (k / n) % 9;
        h[k] = (uint32_t)(s >> 35) & (digit == 8 ? 0x3fffffu : 0x1fffffffu);
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto run = [&](const char* name, void (*k)(uint32_t*, size_t, int), std::vector<uint32_t>& keep) {
        CK(hipMemcpy(slots, h.data(), words * 4, hipMemcpyHostToDevice));
        hipLaunchKernelGGL(k, dim3(grid_for(n)), dim3(kBlock), 0, 0, slots, n, 2);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(slots, h.data(), words * 4, hipMemcpyHostToDevice));
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(k, dim3(grid_for(n)), dim3(kBlock), 0, 0, slots, n, reps);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        CK(hipMemcpy(keep.data(), slots, words * 4, hipMemcpyDeviceToHost));
        printf("{\"case\": \"%s\", \"n\": %zu, \"ms\": %.4f, \"us_per_mul12\": %.3f}\n", name, n, ms, 1e3 * ms / reps);
    };
    run("mul12, operand in registers", k_mul<0>, r0);
    run("mul12_lds, operand in LDS", k_mul<1>, r1);
    size_t diff = 0;
    for (size_t k = 2 * kSlotWords * n; k < words; ++k) diff += r0[k] != r1[k];
    printf("{\"check\": \"register vs LDS operand\", \"differing_words\": %zu}\n", diff);
    return diff != 0;
}
