// kernels_group.hip -- batched G1/G2 scalar multiplication (mod.rs:272-292), one lane per product.
// fq_fold reads -q*p from an LDS table (fq.h; every kernel here calls
// fold_table_init first)
#ifndef BN_FOLD_LDS
#define BN_FOLD_LDS 1
#endif
#include "kernels.h"

namespace bn {

// ---------------------------------------------------------------- scalar multiplication
// Launched with kPairBlock threads per block when the batch gives every CU a
// whole block (kG1MulPairBlockMin, capi.hip), else kBlock: the issue balance of
// kernels.h between the two waves each SIMD then holds.  (1024-thread blocks,
// four waves per SIMD, cap the kernel at 128 VGPRs: 428 B of spills.)
__global__ void __launch_bounds__(kPairBlock) k_g1_mul(const bn_g1* __restrict__ p, const bn_fr* __restrict__ k, size_t n,
                                                     bn_g1* __restrict__ out) {
    fold_table_init();
    const Balance bal = balance_init();
    const size_t i = lane_id();
    if (i >= n) return;
    uint32_t s[8];
    fr_to_canonical(k[i], s);
    G1J a = {widen<kPt>(ld_ref(p[i].x)), widen<kPt>(ld_ref(p[i].y)), widen<kPt>(ld_ref(p[i].z))};
    G1J r = jac_mul(a, s, [&](int t) { balance_step(bal, (uint32_t)t); });
    st_ref(out[i].x, r.x);
    st_ref(out[i].y, r.y);
    st_ref(out[i].z, r.z);
}
__global__ void __launch_bounds__(kBlock) k_g2_mul(const bn_g2* __restrict__ p, const bn_fr* __restrict__ k, size_t n,
                                                   bn_g2* __restrict__ out) {
    fold_table_init();
    const size_t i = lane_id();
    if (i >= n) return;
    uint32_t s[8];
    fr_to_canonical(k[i], s);
    G2J a = {widen<kPt>(ld_ref2(p[i].x)), widen<kPt>(ld_ref2(p[i].y)), widen<kPt>(ld_ref2(p[i].z))};
    G2J r = jac_mul(a, s);
    st_ref2(out[i].x, r.x);
    st_ref2(out[i].y, r.y);
    st_ref2(out[i].z, r.z);
}

}  // namespace bn

BN_EXPORT_FOLD_CHECK(group)
