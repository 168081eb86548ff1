// kernels_fe.hip -- final exponentiation (fq12.rs:62-124, 249-266) as a step
// program over lane-strided Fq12 slots (see kernels.h), plus the Gt output.
// Pairing-path layout (BN_PATH_SPLIT: two lanes per element, fq2_split.h);
// `n` counts elements, the grid has kPathLanes threads per element.
// fq_fold reads -q*p from an LDS table (fq.h; every kernel here calls
// fold_table_init first): 2-3 % faster on this path, measured
#ifndef BN_FOLD_LDS
#define BN_FOLD_LDS 1
#endif
#include "fq.h"
#define BN_SPLIT BN_PATH_SPLIT
#include "kernels.h"
#include "fe_vm.h"

namespace bn {

constexpr size_t kL = BN_SPLIT ? 2 : 1;  // lanes per element in this translation unit

// Launched with kPairBlock threads per block (kernels.h: two-wave issue balance;
// the program position is step * 256 + squarings done in the step).
__global__ void BN_PATH_ATTR __launch_bounds__(kPairBlock) k_fq12_vm(const uint32_t* __restrict__ prog, int nsteps,
                                                                    uint32_t* slots, size_t n) {
    fold_table_init();
    const Balance bal = balance_init();
    const size_t i = lane_id();
    if (i >= kL * n) return;
    (void)fq12_vm_run(prog, nsteps, slots, kL * n, i, bal, 0, true);
}

// out[e] = slot `out_slot`; slot 0 holds the Miller value: f == 0 means the
// reference returns None (fq12.rs:63-72) and pairing() panics -> zero Gt,
// ok[e] = 0, error bit.  flags[lane] (a zero input point) -> Fq12::one().
// Both lanes of an element hold the same flag and reach the same zero test
// (fq2_is_zero combines the two coordinates), so control flow is per element.
__global__ void BN_PATH_ATTR __launch_bounds__(kBlock) k_fe_out(const uint32_t* __restrict__ slots, size_t n, int out_slot,
                                                               const uint8_t* __restrict__ flags, bn_gt* __restrict__ out,
                                                               uint8_t* __restrict__ ok, int* __restrict__ err) {
    fold_table_init();
    const size_t i = lane_id(), e = i / kL;
    if (e >= n) return;
    const size_t nl = kL * n;
    const bool lead = (i % kL) == 0;
    const bool skip = flags && flags[i];
    const bool zero = !skip && fq12_is_zero(ld_fq12<kF>(slots, nl, i));
    if (ok && lead) ok[e] = zero ? 0 : 1;
    if (zero) {
        if (err && lead) err_or(err, BN_ERR_FE_ZERO);
        st_gt_zero(out[e]);
    } else if (skip) {
        st_gt(out[e], fq12_one());
    } else {
        st_gt(out[e], ld_fq12<kF>(slots + (size_t)out_slot * kSlotLaneWords * nl, nl, i));
    }
}

}  // namespace bn

BN_EXPORT_FOLD_CHECK(fe)
