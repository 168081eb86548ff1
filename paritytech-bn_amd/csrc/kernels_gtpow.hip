// kernels_gtpow.hip -- batched Gt::pow(Fr) (lib.rs:592-594 -> generic Fq12 pow,
// fields/mod.rs:35-46), on the pairing path's two-lane layout (BN_PATH_SPLIT,
// fq2_split.h: each lane holds one coordinate of every Fq2, so 2^16 powers are
// 2,048 waves, two per SIMD).
//
// The reference squares-and-multiplies over all 256 bits of U256::from(Fr)
// with the generic Fq12 square (the input need not lie in the cyclotomic
// subgroup: a Gt may hold a miller_loop_batch value).  x^e is unique, so any
// chain gives the reference's canonical output; this one uses fixed windows, so
// the lanes of a wave never diverge, and a per-element table in lane-strided HBM
// slots.  Both lanes of an element hold the same scalar and select the same entry.
//  - A wave of cyclotomic-subgroup members (see below): signed 5-bit windows
//    (Booth recoding, digits -16..16 read straight off six scalar bits; a
//    negative digit multiplies by the conjugate, which is the inverse there):
//    table x^0..x^16 (kGtPowEntries, 15 products to build), 250 cyclotomic
//    squarings and 50 window products -- 65 products in all against the
//    unsigned 4-bit chain's 14 + 63 = 77.
//  - Otherwise: unsigned 4-bit windows, table x^0..x^15, 252 generic squarings
//    and 63 products.
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
    const bool cyc = gt_pow_wave_cyclotomic(x);  // wave-uniform
    {
        const size_t nn = stride();
        st_fq12_buf(slot(0, nn), nn, l, widen<kF>(fq12_one()));
        st_fq12_buf(slot(1, nn), nn, l, x);
    }
    Fq12<kF> t = x;
    const uint32_t entries = cyc ? (uint32_t)kGtPowEntries : 16u;
#pragma unroll 1
    for (uint32_t j = 2; j < entries; ++j) {
        balance_step(bal, j);
        const size_t nn = stride();
        t = mul12(t, ld_fq12_buf<kF>(slot(1, nn), nn, l));
        st_fq12_buf(slot(j, nn), nn, l, t);
    }
    uint32_t e0[8];
    fr_to_canonical(k[i], e0);  // U256::from(Fr), fp.rs:13-20
    if (cyc) {
        // e = 2k (k < r < 2^254): window i of the Booth recoding reads bits 5i - 1 ..
        // 5i + 4 of k, i.e. bits 5i .. 5i + 5 of e; window 50 sits at the top of e[7]
        // and each next one comes up by a left shift of 5
        uint32_t e[8];
#pragma unroll
        for (int s = 7; s > 0; --s) e[s] = (e0[s] << 1) | (e0[s - 1] >> 31);
        e[0] = e0[0] << 1;
        // digit = (f >> 1) + (f & 1) - 32 f5 of the 6-bit field f: its table entry,
        // conjugated when the digit is negative (x^-1 = conj(x) in the subgroup)
        auto entry = [&](uint32_t f) {
            const uint32_t v = (f >> 1) + (f & 1u);
            const bool neg = (f & 32u) != 0 && v != 32u;
            const uint32_t mag = (f & 32u) ? 32u - v : v;
            const size_t nn = stride();
            const Fq12<kF> y = ld_fq12_buf_sel<kF>(ws, nn, sel(mag, nn));
            const Fq12<kF> yc = fq12_conj(y);
            Fq12<kF> r;
            r.c0 = y.c0;
            r.c1.c0 = fq2_select(neg, yc.c1.c0, y.c1.c0);
            r.c1.c1 = fq2_select(neg, yc.c1.c1, y.c1.c1);
            r.c1.c2 = fq2_select(neg, yc.c1.c2, y.c1.c2);
            return r;
        };
        Fq12<kF> acc = entry(e[7] >> 26);
#pragma unroll 1
        for (int w = 49; w >= 0; --w) {
#pragma unroll
            for (int s = 7; s > 0; --s) e[s] = (e[s] << 5) | (e[s - 1] >> 27);
            e[0] <<= 5;
#pragma unroll 1
            for (int s = 0; s < 5; ++s) {
                balance_step(bal, 17u + 6u * (uint32_t)(49 - w) + (uint32_t)s);
                acc = cyc_sqr(acc);
            }
            acc = mul12(acc, entry(e[7] >> 26));
        }
        st_gt(out[i], acc);
        return;
    }
    // 63 windows of four generic squarings and one table product
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
            acc = narrow12<kF>(fq12_sqr(acc));
        }
        const size_t nn = stride();
        acc = mul12(acc, ld_fq12_buf_sel<kF>(ws, nn, sel(e[7] >> 28, nn)));
    }
    st_gt(out[i], acc);
}

}  // namespace bn

BN_EXPORT_FOLD_CHECK(gtpow)
