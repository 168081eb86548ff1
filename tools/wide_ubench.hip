// wide_ubench.hip -- latency of the 16-lane (fq12_wide.h) operations: one group
// (one element) runs a chain of `reps` products / cyclotomic squares /
// inversions / frobenius maps, or whole final exponentiations; one launch per
// measurement, timed with HIP events.  Also runs the same chains on `groups`
// groups at once to show the throughput side.  Prints JSON lines.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/wide_ubench tools/wide_ubench.hip
#define BN_FOLD_LDS 1
#include <stdio.h>
#include <stdlib.h>

#include "../paritytech-bn_amd/csrc/fq.h"
#define BN_SPLIT 1
#include "../paritytech-bn_amd/csrc/fq12_wide.h"

#define CK(x)                                                                                      \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
            exit(1);                                                                               \
        }                                                                                          \
    } while (0)

using namespace bn;

__global__ void __launch_bounds__(256) k_chain(int op, int reps, size_t groups, uint32_t* sink) {
    fold_table_init();
    const size_t e = lane_id() / kWLanes;
    if (e >= groups) return;
    const WL w = wl();
    // a fixed nonzero element: coordinate (e, c) = Montgomery one * (1 + 2e + c), folded
    Fq<2> x = widen<2>(fq_one());
#pragma unroll 1
    for (int k = 0; k < w.l; ++k) x = fq_fold(fq_add(x, fq_one()));
    Fq<2> y = x;
#pragma unroll 1
    for (int r = 0; r < reps; ++r) {
        switch (op) {
            case 0: x = w12_mul(x, y); break;
            case 1: x = w12_cyc(x); break;
            case 2: x = w12_inv(x); break;
            case 3: x = w12_frob<1>(x); break;
            case 4: x = w12_final_exp(x); break;
            default: x = w12_mul(x, x); break;
        }
    }
    uint32_t h = 0;
    for (int i = 0; i < 9; ++i) h ^= x.v[i];
    atomicXor(sink, h);
}

int main() {
    uint32_t* sink;
    CK(hipMalloc(&sink, 4));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const char* names[] = {"mul", "cyc", "inv", "frob1", "final_exp", "sqr_as_mul"};
    const int reps[] = {256, 256, 4, 64, 2, 256};
    for (size_t groups : {(size_t)1, (size_t)4096}) {
        for (int op = 0; op < 6; ++op) {
            const unsigned blocks = (unsigned)((groups * kWLanes + 255) / 256);
            k_chain<<<blocks, 256>>>(op, 1, groups, sink);  // warm
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(a));
            k_chain<<<blocks, 256>>>(op, reps[op], groups, sink);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, a, b));
            printf("{\"op\": \"%s\", \"groups\": %zu, \"reps\": %d, \"ms\": %.4f, \"us_per_op\": %.3f}\n", names[op],
                   groups, reps[op], ms, ms * 1e3 / reps[op]);
        }
    }
    return 0;
}
