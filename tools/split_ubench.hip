// split_ubench.hip -- one lane vs two lanes per element (BN_SPLIT, fq2_split.h)
// on the final exponentiation's hot operations: chains of cyclotomic squarings
// and of Fq12 products over 2^16 elements (BASELINE config 2's batch), one
// launch per measurement, LDS fold table on as in the engine.  Built twice
// (-DBN_SPLIT=0 / 1); each build prints its own JSON lines, and a checksum of
// the canonical outputs so the two forms can be compared for equality.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -DBN_SPLIT=S -o tools/split_ubench_S tools/split_ubench.hip
#define BN_FOLD_LDS 1
#include <stdio.h>
#include <stdlib.h>

#include "../paritytech-bn_amd/csrc/kernels.h"

#define CK(x)                                                                                      \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
            exit(1);                                                                               \
        }                                                                                          \
    } while (0)

using namespace bn;
constexpr int kLanesPerElem = BN_SPLIT ? 2 : 1;

template <int OP>
#if BN_SPLIT
__attribute__((amdgpu_waves_per_eu(2, 2)))
#endif
__global__ void __launch_bounds__(256) k_chain(uint32_t* io, size_t nl, int reps, bn_gt* out) {
    fold_table_init();
    const size_t i = lane_id();
    if (i >= nl) return;
    Fq12<kF> x = ld_fq12<kF>(io, nl, i);
    Fq12<kF> y = ld_fq12<kF>(io + 108 * nl / kLanesPerElem, nl, i);
#pragma unroll 1
    for (int r = 0; r < reps; ++r) {
        if constexpr (OP == 0) x = cyc_sqr(x);
        if constexpr (OP == 1) x = mul12(x, y);
        if constexpr (OP == 2) x = narrow12<kF>(fq12_sqr(x));
    }
    st_gt(out[i / kLanesPerElem], x);
}

int main() {
    const size_t ne = 1 << 16, nl = ne * kLanesPerElem;
    uint32_t* io;
    bn_gt* out;
    CK(hipMalloc(&io, 2 * 108 * ne * 4));
    CK(hipMalloc(&out, ne * sizeof(bn_gt)));
    // deterministic digits < 2^29 (values < 2^261, i.e. bound <= 160... kept small:
    // top digit < 2^20 so every value is below 2p)
    uint32_t* h = (uint32_t*)malloc(2 * 108 * ne * 4);
    // element e, Fq k (0..11), digit l -> unsplit word (k*9+l)*ne + e;
    // split: Fq2 k/2 coordinate k%2 on lane 2e + k%2 -> word ((k/2)*9+l)*nl + 2e + k%2
    uint64_t st = 12345;
    for (int a = 0; a < 2; ++a)
        for (size_t e = 0; e < ne; ++e)
            for (int k = 0; k < 12; ++k)
                for (int l = 0; l < 9; ++l) {
                    st = st * 6364136223846793005ull + 1442695040888963407ull;
                    uint32_t v = (uint32_t)(st >> 35) & 0x1fffffffu;
                    if (l == 8) v &= 0xfffffu;
                    size_t w = BN_SPLIT ? ((size_t)((k / 2) * 9 + l) * nl + 2 * e + (k % 2))
                                        : ((size_t)(k * 9 + l) * ne + e);
                    h[(size_t)a * 108 * ne + w] = v;
                }
    CK(hipMemcpy(io, h, 2 * 108 * ne * 4, hipMemcpyHostToDevice));
    const char* names[] = {"cyc_sqr", "mul12", "fq12_sqr"};
    const int reps[] = {64, 16, 16};
    for (int op = 0; op < 3; ++op) {
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        auto launch = [&](int r) {
            const unsigned g = (unsigned)((nl + 255) / 256);
            if (op == 0) k_chain<0><<<g, 256>>>(io, nl, r, out);
            if (op == 1) k_chain<1><<<g, 256>>>(io, nl, r, out);
            if (op == 2) k_chain<2><<<g, 256>>>(io, nl, r, out);
        };
        launch(1);
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        launch(reps[op]);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        uint64_t* ho = (uint64_t*)malloc(ne * sizeof(bn_gt));
        CK(hipMemcpy(ho, out, ne * sizeof(bn_gt), hipMemcpyDeviceToHost));
        uint64_t cs = 0;
        for (size_t q = 0; q < ne * 48; ++q) cs = cs * 0x100000001b3ull ^ ho[q];
        free(ho);
        printf("{\"split\": %d, \"op\": \"%s\", \"elements\": %zu, \"reps\": %d, \"ms\": %.4f, \"us_per_op_per_2^16\": %.3f, "
               "\"checksum\": \"%016llx\"}\n",
               BN_SPLIT, names[op], ne, reps[op], ms, ms * 1e3 / reps[op], (unsigned long long)cs);
    }
    return 0;
}
