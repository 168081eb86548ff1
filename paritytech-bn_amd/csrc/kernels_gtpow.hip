// kernels_gtpow.hip -- batched Gt::pow(Fr) (lib.rs:592-594 -> generic Fq12 pow,
// fields/mod.rs:35-46), one lane per power.
//
// The reference squares-and-multiplies over all 256 bits of U256::from(Fr)
// with the generic Fq12 square (the input need not lie in the cyclotomic
// subgroup: a Gt may hold a miller_loop_batch value), so this does too, with a
// fixed 4-bit window: a per-lane table x^0..x^15 in lane-strided HBM slots,
// 252 generic squarings and 63 products by a table entry.  x^e is unique, so
// the canonical output equals the reference's.
#include "kernels.h"

namespace bn {

__global__ void __launch_bounds__(kBlock) k_gt_pow(const bn_gt* __restrict__ a, const bn_fr* __restrict__ k, size_t n,
                                                   bn_gt* __restrict__ out, uint32_t* __restrict__ ws) {
    const size_t i = lane_id();
    if (i >= n) return;
    auto slot = [&](uint32_t t) { return ws + (size_t)t * kSlotWords * n; };
    const Fq12<kF> x = widen<kF>(ld_gt(a[i]));
    st_fq12(slot(0), n, i, widen<kF>(fq12_one()));
    st_fq12(slot(1), n, i, x);
    Fq12<kF> t = x;
#pragma unroll 1
    for (uint32_t j = 2; j < 16; ++j) {
        mem_fence();
        t = mul12(t, ld_fq12<kF>(slot(1), n, i));
        st_fq12(slot(j), n, i, t);
    }
    uint32_t e[8];
    fr_to_canonical(k[i], e);  // U256::from(Fr), fp.rs:13-20
    mem_fence();
    Fq12<kF> acc = ld_fq12<kF>(slot(e[7] >> 28), n, i);
#pragma unroll 1
    for (int w = 62; w >= 0; --w) {
#pragma unroll
        for (int s = 7; s > 0; --s) e[s] = (e[s] << 4) | (e[s - 1] >> 28);
        e[0] <<= 4;
#pragma unroll 1
        for (int s = 0; s < 4; ++s) acc = narrow12<kF>(fq12_sqr(acc));
        mem_fence();
        acc = mul12(acc, ld_fq12<kF>(slot(e[7] >> 28), n, i));
    }
    st_gt(out[i], acc);
}

}  // namespace bn
