// kernels_gtpow.hip -- batched Gt::pow(Fr) (lib.rs:592-594 -> generic Fq12 pow,
// fields/mod.rs:35-46), one lane per power.
//
// The reference squares-and-multiplies over all 256 bits of U256::from(Fr)
// with the generic Fq12 square (the input need not lie in the cyclotomic
// subgroup: a Gt may hold a miller_loop_batch value), so this does too, with a
// fixed 4-bit window: a per-lane table x^0..x^15 in lane-strided HBM slots,
// 252 generic squarings and 63 products by a table entry.  x^e is unique, so
// the canonical output equals the reference's.
//
// The table entry is selected per lane through the VGPR offset of a buffer
// descriptor built from the uniform workspace base (ld_fq12_buf_sel): the
// descriptor itself never depends on the lane (round 1 built it from a
// per-lane pointer, which the compiler lowers to readfirstlane waterfall loops,
// and that build faulted once the LDS fold table was enabled).
// fq_fold reads -q*p from the LDS table as in the other pairing-path kernels.
#ifndef BN_FOLD_LDS
#define BN_FOLD_LDS 1
#endif
#include "kernels.h"

namespace bn {

__global__ void __launch_bounds__(kBlock) k_gt_pow(const bn_gt* __restrict__ a, const bn_fr* __restrict__ k, size_t n,
                                                   bn_gt* __restrict__ out, uint32_t* __restrict__ ws) {
    fold_table_init();
    const size_t i = lane_id();
    if (i >= n) return;
    // slot access through a buffer descriptor with the stride laundered per use
    // (kernels.h, as in the step machine): no hoisted per-word offsets
    auto slot = [&](uint32_t t, size_t nn) { return ws + (size_t)t * kSlotWords * nn; };
    auto stride = [&]() {
        size_t nn = n;
        asm volatile("" : "+s"(nn));
        return nn;
    };
    // byte offset of lane i's copy of table entry t (t is per lane)
    auto sel = [&](uint32_t t, size_t nn) { return (uint32_t)(((size_t)t * kSlotWords * nn + i) * 4); };
    const Fq12<kF> x = widen<kF>(ld_gt(a[i]));
    {
        const size_t nn = stride();
        st_fq12_buf(slot(0, nn), nn, i, widen<kF>(fq12_one()));
        st_fq12_buf(slot(1, nn), nn, i, x);
    }
    Fq12<kF> t = x;
#pragma unroll 1
    for (uint32_t j = 2; j < 16; ++j) {
        const size_t nn = stride();
        t = mul12(t, ld_fq12_buf<kF>(slot(1, nn), nn, i));
        st_fq12_buf(slot(j, nn), nn, i, t);
    }
    uint32_t e[8];
    fr_to_canonical(k[i], e);  // U256::from(Fr), fp.rs:13-20
    Fq12<kF> acc;
    {
        const size_t nn = stride();
        acc = ld_fq12_buf_sel<kF>(ws, nn, sel(e[7] >> 28, nn));
    }
#pragma unroll 1
    for (int w = 62; w >= 0; --w) {
#pragma unroll
        for (int s = 7; s > 0; --s) e[s] = (e[s] << 4) | (e[s - 1] >> 28);
        e[0] <<= 4;
#pragma unroll 1
        for (int s = 0; s < 4; ++s) acc = narrow12<kF>(fq12_sqr(acc));
        const size_t nn = stride();
        acc = mul12(acc, ld_fq12_buf_sel<kF>(ws, nn, sel(e[7] >> 28, nn)));
    }
    st_gt(out[i], acc);
}

}  // namespace bn

BN_EXPORT_FOLD_CHECK(gtpow)
