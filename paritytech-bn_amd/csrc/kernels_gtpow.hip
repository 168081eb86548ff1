// kernels_gtpow.hip -- batched Gt::pow(Fr) (lib.rs:592-594 -> generic Fq12 pow,
// fields/mod.rs:35-46), on the pairing path's two-lane layout (BN_PATH_SPLIT,
// fq2_split.h: each lane holds one coordinate of every Fq2, so 2^16 powers are
// 2,048 waves, two per SIMD).
//
// The reference squares-and-multiplies over all 256 bits of U256::from(Fr)
// with the generic Fq12 square (the input need not lie in the cyclotomic
// subgroup: a Gt may hold a miller_loop_batch value), so this does too, with a
// fixed 4-bit window: a per-element table x^0..x^15 in lane-strided HBM slots,
// 252 squarings and 63 products by a table entry (the squarings cyclotomic when
// the whole wave holds cyclotomic-subgroup members, see below).  x^e is unique,
// so the canonical output equals the reference's.  Both lanes of an element
// hold the same scalar and select the same entry.
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
#include <type_traits>

#include "fq.h"
#define BN_SPLIT BN_PATH_SPLIT
#include "kernels.h"

namespace bn {

constexpr size_t kL = BN_SPLIT ? 2 : 1;  // lanes per element in this translation unit

// True when every element of the wave is a nonzero member of the cyclotomic
// subgroup (order p^4 - p^2 + 1, where every pairing output lies):
// x^(p^4) * x == x^(p^2).  There the Granger-Scott square (fq12.rs:198-247,
// tower.h fq12_cyclotomic_sqr) equals the generic square as a field element, at
// half its cost, so the power -- and its canonical image -- is unchanged.  The
// choice is wave-uniform: one non-member (a Miller value, say) sends its whole
// wave down the generic chain, and lanes never diverge.
__device__ __forceinline__ bool gt_pow_wave_cyclotomic(const Fq12<kF>& x) {
    const Fq12<kF> x2 = narrow12<kF>(fq12_frobenius_map<2>(x));
    const Fq12<kF> x4x = mul12(narrow12<kF>(fq12_frobenius_map<2>(x2)), x);
    const bool member = ((unsigned)fq12_is_zero(fq12_sub(x4x, x2)) & (unsigned)!fq12_is_zero(x)) != 0;
    return __all(member);
}

// Launched with kPairBlock threads per block (kernels.h: issue balance; program
// position = table entry, then 16 + 5 * window + squaring).
__global__ void BN_PATH_ATTR __launch_bounds__(kPairBlock) k_gt_pow(const bn_gt* __restrict__ a,
                                                                   const bn_fr* __restrict__ k, size_t n,
                                                                   bn_gt* __restrict__ out, uint32_t* __restrict__ ws) {
    fold_table_init();
    const Balance bal = balance_init();
    const size_t l = lane_id(), i = l / kL;
    if (i >= n) return;
    // slot access through a buffer descriptor with the lane stride laundered per
    // use (kernels.h, as in the step machine): no hoisted per-word offsets
    auto slot = [&](uint32_t t, size_t nn) { return ws + (size_t)t * kSlotLaneWords * nn; };
    auto stride = [&]() {
        size_t nn = kL * n;
        asm volatile("" : "+s"(nn));
        return nn;
    };
    // byte offset of lane l's copy of table entry t (t is per element)
    auto sel = [&](uint32_t t, size_t nn) { return (uint32_t)(((size_t)t * kSlotLaneWords * nn + l) * 4); };
    const Fq12<kF> x = widen<kF>(ld_gt(a[i]));
    {
        const size_t nn = stride();
        st_fq12_buf(slot(0, nn), nn, l, widen<kF>(fq12_one()));
        st_fq12_buf(slot(1, nn), nn, l, x);
    }
    Fq12<kF> t = x;
#pragma unroll 1
    for (uint32_t j = 2; j < 16; ++j) {
        balance_step(bal, j);
        const size_t nn = stride();
        t = mul12(t, ld_fq12_buf<kF>(slot(1, nn), nn, l));
        st_fq12_buf(slot(j, nn), nn, l, t);
    }
    uint32_t e0[8];
    fr_to_canonical(k[i], e0);  // U256::from(Fr), fp.rs:13-20
    // 63 windows of four squarings and one table product; Cyc selects the square
    auto chain = [&](auto cyc) {
        uint32_t e[8];
#pragma unroll
        for (int s = 0; s < 8; ++s) e[s] = e0[s];
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
            for (int s = 0; s < 4; ++s) {
                balance_step(bal, 16u + 5u * (uint32_t)(62 - w) + (uint32_t)s);
                if constexpr (decltype(cyc)::value) acc = cyc_sqr(acc);
                else acc = narrow12<kF>(fq12_sqr(acc));
            }
            const size_t nn = stride();
            acc = mul12(acc, ld_fq12_buf_sel<kF>(ws, nn, sel(e[7] >> 28, nn)));
        }
        return acc;
    };
    if (gt_pow_wave_cyclotomic(x)) st_gt(out[i], chain(std::true_type{}));
    else st_gt(out[i], chain(std::false_type{}));
}

}  // namespace bn

BN_EXPORT_FOLD_CHECK(gtpow)
