// fe_ubench.hip -- per-operation cost of the Fq12 step machine and of the
// register-resident Fq12 operations on MI355X (n lanes, one Fq12 per lane).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/fe_ubench tools/fe_ubench.hip
#include "../paritytech-bn_amd/csrc/kernels_fe.hip"

#include <stdio.h>
#include <stdlib.h>

#include <vector>

#define CK(x)                                                                                      \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
            exit(1);                                                                               \
        }                                                                                          \
    } while (0)

namespace bn {
template <int OP>
__global__ void __launch_bounds__(kBlock) k_reg(uint32_t* slots, size_t n, int reps) {
    const size_t i = lane_id();
    if (i >= n) return;
    __shared__ uint32_t yl[kSlotWords * kBlock];
    if constexpr (OP == 3) {
        lds_copy_fq12(slots + kSlotWords * n + (size_t)blockIdx.x * kBlock, n, yl);
        lds_copy_wait();
    }
    Fq12<kF> x = ld_fq12<kF>(slots, n, i);
    const Fq12<kF> y = ld_fq12<kF>(slots + kSlotWords * n, n, i);
#pragma unroll 1
    for (int r = 0; r < reps; ++r) {
        if constexpr (OP == 0) x = mul12(x, y);
        if constexpr (OP == 1) x = cyc_sqr(x);
        if constexpr (OP == 2) x = narrow12<kF>(fq12_sqr(x));
        if constexpr (OP == 3) x = mul12_lds(x, yl + threadIdx.x, false);
    }
    st_fq12(slots + 2 * kSlotWords * n, n, i, x);
}
// the same operations compiled for two resident waves per SIMD (<= 256 registers)
template <int OP>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(2, 2)))
k_reg2(uint32_t* slots, size_t n, int reps) {
    const size_t i = lane_id();
    if (i >= n) return;
    Fq12<kF> x = ld_fq12<kF>(slots, n, i);
    const Fq12<kF> y = ld_fq12<kF>(slots + kSlotWords * n, n, i);
#pragma unroll 1
    for (int r = 0; r < reps; ++r) {
        if constexpr (OP == 0) x = mul12(x, y);
        if constexpr (OP == 1) x = cyc_sqr(x);
        if constexpr (OP == 2) x = narrow12<kF>(fq12_sqr(x));
    }
    st_fq12(slots + 2 * kSlotWords * n, n, i, x);
}
}  // namespace bn
using namespace bn;

int main(int argc, char** argv) {
    const size_t n = argc > 1 ? strtoull(argv[1], 0, 0) : 65536;
    const int nslots = 8;
    uint32_t* slots;
    CK(hipMalloc(&slots, n * nslots * kSlotWords * 4));
    std::vector<uint32_t> h(n * nslots * kSlotWords);
    uint64_t s = 0x1234567;
    for (size_t k = 0; k < h.size(); ++k) {
        s = s * 6364136223846793005ull + 1442695040888963407ull;
        const size_t digit = (k / n) % 9;
        h[k] = (uint32_t)(s >> 35) & (digit == 8 ? 0x3fffffu : 0x1fffffffu);  // value < 2^254
    }
    CK(hipMemcpy(slots, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    uint32_t* dprog;
    CK(hipMalloc(&dprog, 4096 * 8));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto time_prog = [&](const char* name, std::vector<uint32_t> prog, double units) {
        CK(hipMemcpy(dprog, prog.data(), prog.size() * 4, hipMemcpyHostToDevice));
        const int steps = (int)prog.size() / 2;
        k_fq12_vm<<<grid_for(n), kBlock>>>(dprog, steps, slots, n);
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        k_fq12_vm<<<grid_for(n), kBlock>>>(dprog, steps, slots, n);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("{\"case\": \"%s\", \"n\": %zu, \"ms\": %.4f, \"us_per_unit\": %.3f}\n", name, n, ms,
               1e3 * ms / units);
    };
    auto step = [](std::vector<uint32_t>& p, uint32_t op, uint32_t d, uint32_t a, uint32_t b, uint32_t k,
                   uint32_t f) {
        uint32_t w[2];
        vm_step(w, op, d, a, b, k, f);
        p.push_back(w[0]);
        p.push_back(w[1]);
    };
    const int R = 40;
    {
        std::vector<uint32_t> p;
        for (int r = 0; r < R; ++r) step(p, OP_MUL, 2, r ? 2 : 0, 1, 0, 0);
        time_prog("vm MUL k=0 (2 loads + 1 store per product)", p, R);
    }
    {
        std::vector<uint32_t> p;
        for (int r = 0; r < R; ++r) step(p, OP_CYC, 2, r ? 2 : 0, 0, 1, 0);
        time_prog("vm CYC k=1 (1 load + 1 store per square)", p, R);
    }
    {
        std::vector<uint32_t> p;
        step(p, OP_CYC, 2, 0, 0, R, 0);
        time_prog("vm CYC k=40 (one step)", p, R);
    }
    {
        std::vector<uint32_t> p;
        for (int r = 0; r < R / 4; ++r) step(p, OP_MUL, 2, r ? 2 : 0, 1, 3, 0);
        time_prog("vm MUL k=3 (3 squares + product per step), per step", p, R / 4);
    }
    {
        std::vector<uint32_t> p;
        for (int r = 0; r < 4; ++r) step(p, OP_INV, 2, r ? 2 : 0, 0, 0, 0);
        time_prog("vm INV", p, 4);
    }
    auto time_reg = [&](const char* name, void (*kern)(uint32_t*, size_t, int)) {
        hipLaunchKernelGGL(kern, dim3(grid_for(n)), dim3(kBlock), 0, 0, slots, n, R);
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(kern, dim3(grid_for(n)), dim3(kBlock), 0, 0, slots, n, R);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("{\"case\": \"%s\", \"n\": %zu, \"ms\": %.4f, \"us_per_unit\": %.3f}\n", name, n, ms, 1e3 * ms / R);
    };
    time_reg("reg mul12", k_reg<0>);
    time_reg("reg cyc_sqr", k_reg<1>);
    time_reg("reg fq12_sqr", k_reg<2>);
    time_reg("reg mul12_lds (b from LDS)", k_reg<3>);
    time_reg("reg2 cyc_sqr (<=256 regs)", k_reg2<1>);
    time_reg("reg2 fq12_sqr (<=256 regs)", k_reg2<2>);
    time_reg("reg2 mul12 (<=256 regs)", k_reg2<0>);
    return 0;
}
