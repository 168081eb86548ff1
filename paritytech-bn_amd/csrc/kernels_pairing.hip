// kernels_pairing.hip -- to_affine + G2 line precomputation (mod.rs:199-216, 701-727) and the
// Miller loop (mod.rs:579-607).  Pairing-path layout (BN_PATH_SPLIT: two lanes
// per pairing, fq2_split.h; `n` counts pairings, the grid has kPathLanes
// threads per pairing).  G1 values (P, its affine form) are held by both lanes.
// fq_fold reads -q*p from an LDS table (fq.h; every kernel here calls
// fold_table_init first): 2-3 % faster on this path, measured
#ifndef BN_FOLD_LDS
#define BN_FOLD_LDS 1
#endif
#include "fq.h"
#define BN_SPLIT BN_PATH_SPLIT
#include "kernels.h"
#include "lines_wide.h"
#include "fe_vm.h"

namespace bn {

// to_affine + the 87 line coefficients (AffineG2::precompute) -> HBM.
// Launched with kPairBlock threads per block (kernels.h: issue balance).
__global__ void BN_PATH_ATTR __launch_bounds__(kPairBlock) k_prepare(const bn_g1* __restrict__ p,
                                                                    const bn_g2* __restrict__ q, size_t n,
                                                                    uint32_t* __restrict__ coeffs,
                                                                    uint32_t* __restrict__ paff,
                                                                    uint8_t* __restrict__ flags,
                                                                    int* __restrict__ err, int mode, int scale) {
    fold_table_init();
    const Balance bal = balance_init();
    const size_t l = lane_id(), i = l / kL, nl = kL * n;
    if (i >= n) return;
    const PairAffine a = pair_to_affine(p, q, i, l, flags, err, mode);
    st_fq(paff, nl, l, 0, a.px);
    st_fq(paff, nl, l, 1, a.py);
    const bool sc = BN_LINES_PRESCALED && scale;
    g2_precompute(a.qa, [&](int k, const Ell& e) {
        balance_step(bal, (uint32_t)k);
        st_fq2(coeffs, nl, l, k * 6 + 0, e.ell_0);
        if (sc) {  // wave-uniform
            st_fq2(coeffs, nl, l, k * 6 + 2, narrow<kLine>(fq2_scale(e.ell_vw, a.py)));
            st_fq2(coeffs, nl, l, k * 6 + 4, narrow<kLine>(fq2_scale(e.ell_vv, a.px)));
        } else {
            st_fq2(coeffs, nl, l, k * 6 + 2, e.ell_vw);
            st_fq2(coeffs, nl, l, k * 6 + 4, e.ell_vv);
        }
    });
}

#if BN_SPLIT
// Launched with kPairBlock threads per block (kernels.h: issue balance).
__global__ void BN_PATH_ATTR __launch_bounds__(kPairBlock) k_prepare_wide(const bn_g1* __restrict__ p,
                                                                         const bn_g2* __restrict__ q, size_t n,
                                                                         uint32_t* __restrict__ coeffs,
                                                                         uint32_t* __restrict__ paff,
                                                                         uint8_t* __restrict__ flags,
                                                                         int* __restrict__ err, int mode,
                                                                         int scale) {
    fold_table_init();
    const Balance bal = balance_init();
    const size_t l = lane_id(), i = l / kPW, nl = kL * n;
    if (i >= n) return;
    const size_t lt = i * kL + (l & 1);  // this lane's index in k_prepare's per-pair arrays
    const int k = pw_slot();
    const bool st = k == 0;
    const PairAffine a = pair_to_affine<true>(p, q, i, lt, flags, err, st ? mode : 0);
    if (st) {
        st_fq(paff, nl, lt, 0, a.px);
        st_fq(paff, nl, lt, 1, a.py);
    }
    // g2_precompute (pairing.h), AffineG2::precompute mod.rs:701-727
    const G2Aff<kPt>& qa = a.qa;
    G2Proj r = {qa.x, qa.y, widen<kPt>(fq2_one())};
    const auto qy_neg = fq2_neg(qa.y);
    int c = 0;
#if BN_LINES_PRESCALED
    // slot 0 stores ell_0; with `scale` slot 2 stores ell_vw * Py and slot 3 ell_vv * Px
    // (their own products, lines_wide.h PwEll), else slot 0 the unscaled pair
    const bool sc = scale != 0;
    // (one select and one store per lane, at a per-slot offset: with a store per slot
    // under its own branch the compiler staged the values through scratch)
    auto emit = [&](int cc, const PwEll& e) {
        if (sc) {
            const Fq2<kLine> x = fq2_select(k == 0, e.e.ell_0, fq2_select(k == 2, e.vw_py, e.vv_px));
            if (k != 1) st_fq2(coeffs, nl, lt, cc * 6 + (k == 0 ? 0 : k == 2 ? 2 : 4), x);
        } else if (st) {
            st_fq2(coeffs, nl, lt, cc * 6 + 0, e.e.ell_0);
            st_fq2(coeffs, nl, lt, cc * 6 + 2, e.e.ell_vw);
            st_fq2(coeffs, nl, lt, cc * 6 + 4, e.e.ell_vv);
        }
    };
    const Fq2<2> py_r = pw_real(a.py);
    const Fq2<2> px_r = pw_real(a.px);
    const auto px3_r = pw_real(fq_add(fq_add(a.px, a.px), a.px));
    const auto bxpy_q = fq2_scale(qa.x, a.py);  // base x * Py of Q (and -Q)
#pragma unroll 1
    for (int d = 0; d < BN_NAF_DIGITS; ++d) {
        balance_step(bal, (uint32_t)d);
        emit(c++, pw_doubling_step_p(r, k, py_r, px3_r));
        if ((kNafNonzero >> d) & 1u) {
            const bool minus = (kNafMinus >> d) & 1u;
            const G2Aff<kPt> base = {qa.x, fq2_select(minus, widen<kPt>(qy_neg), qa.y)};
            emit(c++, pw_mixed_addition_step_p(r, base, bxpy_q, k, py_r, px_r));
        }
    }
    G2Aff<kPt> q1 = mul_by_q(qa);
    G2Aff<kPt> q2 = mul_by_q(q1);
    q2.y = narrow<kPt>(fq2_neg(q2.y));
    emit(c++, pw_mixed_addition_step_p(r, q1, fq2_scale(q1.x, a.py), k, py_r, px_r));
    emit(c++, pw_mixed_addition_step_p(r, q2, fq2_scale(q2.x, a.py), k, py_r, px_r));
#else
    (void)scale;
    auto emit = [&](int cc, const Ell& e) {
        if (st) {
            st_fq2(coeffs, nl, lt, cc * 6 + 0, e.ell_0);
            st_fq2(coeffs, nl, lt, cc * 6 + 2, e.ell_vw);
            st_fq2(coeffs, nl, lt, cc * 6 + 4, e.ell_vv);
        }
    };
#pragma unroll 1
    for (int d = 0; d < BN_NAF_DIGITS; ++d) {
        balance_step(bal, (uint32_t)d);
        emit(c++, pw_doubling_step(r, k));
        if ((kNafNonzero >> d) & 1u) {
            const bool minus = (kNafMinus >> d) & 1u;
            const G2Aff<kPt> base = {qa.x, fq2_select(minus, widen<kPt>(qy_neg), qa.y)};
            emit(c++, pw_mixed_addition_step(r, base, k));
        }
    }
    G2Aff<kPt> q1 = mul_by_q(qa);
    G2Aff<kPt> q2 = mul_by_q(q1);
    q2.y = narrow<kPt>(fq2_neg(q2.y));
    emit(c++, pw_mixed_addition_step(r, q1, k));
    emit(c++, pw_mixed_addition_step(r, q2, k));
#endif
}
#endif

// The coefficients k_prepare wrote for pair i -> the reference images of its
// G2Precomp (mod.rs:566-577): 87 x {ell_0, ell_vw, ell_vv}, each a canonical Fq2
__global__ void BN_PATH_ATTR __launch_bounds__(kBlock) k_coeffs_store(const uint32_t* __restrict__ coeffs, size_t n,
                                                                     bn_fq2* __restrict__ out) {
    fold_table_init();
    const size_t l = lane_id(), i = l / kL, nl = kL * n;
    if (i >= n) return;
#pragma unroll 1
    for (int k = 0; k < BN_NUM_COEFFS; ++k)
#pragma unroll
        for (int j = 0; j < 3; ++j) st_ref2(out[(i * BN_NUM_COEFFS + k) * 3 + j], ld_fq2<kLine>(coeffs, nl, l, k * 6 + 2 * j));
}

// A/B form ("line coefficients"): to_affine, the line steps and the
// Miller loop fused in one kernel -- each coefficient is applied as soon as it is
// computed and never leaves registers (no 16.7 KB/pairing HBM round trip).  Same
// operations in the same order as k_prepare + k_miller, so the same Miller value.
// Launched with kPairBlock threads per block (kernels.h: two-wave issue balance).
__global__ void BN_PATH_ATTR __launch_bounds__(kPairBlock) k_pairing_fused(const bn_g1* __restrict__ p,
                                                                          const bn_g2* __restrict__ q, size_t n,
                                                                          uint8_t* __restrict__ flags,
                                                                          int* __restrict__ err, int mode,
                                                                          uint32_t* __restrict__ f_out) {
    fold_table_init();
    const Balance bal = balance_init();
    const size_t l = lane_id(), i = l / kL, nl = kL * n;
    if (i >= n) return;
    const PairAffine a = pair_to_affine(p, q, i, l, flags, err, mode);
    Fq12<kF> f = miller_fused(a.qa, a.px, a.py, [&](int d) { balance_step(bal, (uint32_t)d); });
    if (flags[l]) f = widen<kF>(fq12_one());
    st_fq12(f_out, nl, l, f);
}

// A/B form (miller_form 3): k_pairing_fused, k_fq12_vm and
// k_fe_out as one kernel.  The Miller value is stored to slot 0 (the step
// program reads it more than once) and the program runs right behind it on the
// same lanes; its last step's result (slot `out_slot`, checked by the host) is
// written straight to out[] as k_fe_out would.  Removes the two kernel tails
// between the phases (a wave waits for the slowest wave of the grid at each
// boundary).  Balance positions of the program are offset past the loop's.
__global__ void BN_PATH_ATTR __launch_bounds__(kPairBlock) k_pairing_full(const bn_g1* __restrict__ p,
                                                                         const bn_g2* __restrict__ q, size_t n,
                                                                         const uint32_t* __restrict__ prog, int nsteps,
                                                                         uint32_t* __restrict__ slots,
                                                                         bn_gt* __restrict__ out, int* __restrict__ err) {
    fold_table_init();
    const Balance bal = balance_init();
    const size_t l = lane_id(), i = l / kL, nl = kL * n;
    if (i >= n) return;
    const PairAffine a = pair_to_affine(p, q, i, l, nullptr, err, 0);
    Fq12<kF> f = miller_fused(a.qa, a.px, a.py, [&](int d) { balance_step(bal, (uint32_t)d); });
    if (a.skip) f = widen<kF>(fq12_one());
    // f == 0: the reference's final_exponentiation returns None and pairing()
    // panics (fq12.rs:63-72) -> zero Gt and the error bit, as k_fe_out
    const bool zero = !a.skip && fq12_is_zero(f);
    st_fq12(slots, nl, l, f);
    const Fq12<kF> r = fq12_vm_run(prog, nsteps, slots, nl, l, bal, 1u << 20, false);
    if (zero) {
        if ((l % kL) == 0) err_or(err, BN_ERR_FE_ZERO);
        st_gt_zero(out[i]);
    } else if (a.skip) {
        st_gt(out[i], fq12_one());
    } else {
        st_gt(out[i], r);
    }
}

__global__ void BN_PATH_ATTR __launch_bounds__(kBlock) k_miller(const uint32_t* __restrict__ coeffs,
                                                               const uint32_t* __restrict__ paff,
                                                               const uint8_t* __restrict__ flags, size_t n,
                                                               uint32_t* __restrict__ f_out) {
    fold_table_init();
    const size_t l = lane_id(), i = l / kL, nl = kL * n;
    if (i >= n) return;
    auto line = [&](int k) {
        return Ell{ld_fq2<kLine>(coeffs, nl, l, k * 6 + 0), ld_fq2<kLine>(coeffs, nl, l, k * 6 + 2),
                   ld_fq2<kLine>(coeffs, nl, l, k * 6 + 4)};
    };
#if BN_LINES_PRESCALED
    (void)paff;
    Fq12<kF> f = miller_loop_scaled(line);
#else
    const Fq<2> px = ld_fq<2>(paff, nl, l, 0);
    const Fq<2> py = ld_fq<2>(paff, nl, l, 1);
    Fq12<kF> f = miller_loop(px, py, line);
#endif
    if (flags[l]) f = widen<kF>(fq12_one());
    st_fq12(f_out, nl, l, f);
}

// Miller loop in segments (pairing_batch / miller_loop_batch, and small
// pairing_many batches): lane pair off[s] + g (segment s, group g) --
// segment-major, so a wave reads consecutive pairs' coefficients -- runs the
// segment's digits [lo, hi) of the loop from f = one for the K[s] pairs g, g + G,
// ..., g + (K[s]-1) G (G = G[s] = ceil(n / K[s])): per digit ONE squaring of the
// shared accumulator and the line of every pair (mod.rs:609-640's
// shared-squaring loop; squaring is a ring homomorphism and Fq12 is commutative,
// so the product over groups and the Horner recombination over segments give
// exactly miller_loop_batch's value).  The result goes to element off[s] + g of
// `out` (split layout, stride total); lane pairs past G[s] (a segment's padding
// to whole blocks) write nothing.
// A pair with a zero point (flags) or past n contributes the line one
// (ell_0 = 1, ell_vw = ell_vv = 0): the sparse product by it is f itself.
// Launched with kPairBlock threads per block (kernels.h: issue balance).
#ifndef BN_SEG_STAMPS
#define BN_SEG_STAMPS 0
#endif
#ifndef BN_SEG_LINE_BALANCE
#define BN_SEG_LINE_BALANCE 1
#endif
#if BN_SEG_STAMPS
// diagnostic build (tools/build_variant.sh segstamps -DBN_SEG_STAMPS=1, tools/seg_stamps.py):
// lane 0 of every wave of k_miller_seg records s_memrealtime (100 MHz) when the wave
// starts and ends, and its segment: where the kernel's wave lifetime goes
constexpr int kSegStampWaves = 4096;
__device__ uint64_t g_seg_stamps[kSegStampWaves][4];
#define SEG_STAMP(slot, v)                                                                  \
    do {                                                                                    \
        const size_t w_ = lane_id() / 64;                                                   \
        if ((threadIdx.x & 63u) == 0 && w_ < (size_t)kSegStampWaves) g_seg_stamps[w_][slot] = (v); \
    } while (0)
#else
#define SEG_STAMP(slot, v) ((void)0)
#endif
__global__ void BN_PATH_ATTR __launch_bounds__(kPairBlock) k_miller_seg(const uint32_t* __restrict__ coeffs,
                                                                       const uint32_t* __restrict__ paff,
                                                                       const uint8_t* __restrict__ flags, size_t n,
                                                                       SegPlan plan, uint32_t* __restrict__ out) {
    SEG_STAMP(0, __builtin_amdgcn_s_memrealtime());
    fold_table_init();
    const Balance bal = balance_init();
    const size_t l = lane_id(), lp = l / kL, nl = kL * n;
    if (lp >= (size_t)plan.total) return;
    int s = 0;
    while (s + 1 < plan.S && lp >= (size_t)plan.off[s + 1]) ++s;
    const size_t K = (size_t)plan.K[s], G = plan.G[s];
    const size_t g = lp - plan.off[s], c = l % kL;
    SEG_STAMP(2, (uint64_t)s);
    SEG_STAMP(3, (uint64_t)K);
    if (g >= G) return;
    const Ell one_line = {widen<kLine>(fq2_one()), widen<kLine>(fq2_zero()), widen<kLine>(fq2_zero())};
    // line k of pair t of this group, with the pair's affine P
    struct PairLine {
        Ell e;
        Fq<2> px, py;
    };
    auto pair_line = [&](size_t t, int k) {
        const size_t j = g + t * G;
        const bool live = j < n && !flags[j * kL + c];
        const size_t lt = (j < n ? j : 0) * kL + c;  // the pair's lane in the per-pair arrays
        PairLine r;
        mem_fence();  // load right before use: K pairs' lines are never held at once
        r.e = Ell{ld_fq2<kLine>(coeffs, nl, lt, k * 6 + 0), ld_fq2<kLine>(coeffs, nl, lt, k * 6 + 2),
                  ld_fq2<kLine>(coeffs, nl, lt, k * 6 + 4)};
#if !BN_LINES_PRESCALED  // (prescaled: the line as the loop multiplies by it, no P needed)
        r.px = ld_fq<2>(paff, nl, lt, 0);
        r.py = ld_fq<2>(paff, nl, lt, 1);
#endif
        if (!live) r.e = one_line;
        return r;
    };
    // Digits lo..hi-1, then (last segment) the two closing lines as pseudo-digits
    // 64 and 65 without a squaring; per digit one squaring (none at lo: f starts
    // at one, so the first line is f itself) and one or two passes over the K
    // pairs' lines.  One copy of the squaring and of the sparse product.
    const int lo = plan.lo[s], hi = plan.hi[s];
    const int end = hi == BN_NAF_DIGITS ? BN_NAF_DIGITS + 2 : hi;
    int idx = plan.idx[s];
    Fq12<kF> f = widen<kF>(fq12_one());
    // Issue balance (kernels.h) at every line, not only every digit: a segment is 3-8
    // digits of up to 16 K-pair lines each, and with one position per digit the
    // older wave of a SIMD ran up to a digit ahead of its partner and finished
    // ~150 us earlier, the younger one then running its last digit alone
    // (tools/seg_stamps.py: wave durations 370-520 us inside every segment, wave
    // life 0.72-0.84).  Positions: digit * 256, then 1 + pass * 64 + t per line (K <= 64).
#pragma unroll 1
    for (int i = lo; i < end; ++i) {
        const uint32_t dpos = (uint32_t)(i - lo) << 8;
        balance_step(bal, dpos);
        const bool closing = i >= BN_NAF_DIGITS;
        if (!closing && i > lo) f = narrow12<kF>(fq12_sqr(f));
        const int passes = closing ? 1 : 1 + (int)((kNafNonzero >> i) & 1u);
#pragma unroll 1
        for (int ps = 0; ps < passes; ++ps, ++idx) {
#pragma unroll 1
            for (size_t t = 0; t < K; ++t) {
                if (BN_SEG_LINE_BALANCE) balance_step(bal, dpos + 1u + ((uint32_t)ps << 6) + (uint32_t)t);
                const PairLine pl = pair_line(t, idx);
#if BN_LINES_PRESCALED
                if (i == lo && ps == 0 && t == 0)
                    f = line_from_one_scaled(pl.e);  // one * line (mod.rs:589 on f = one)
                else
                    f = apply_line_scaled(f, pl.e);
#else
                if (i == lo && ps == 0 && t == 0)
                    f = line_from_one(pl.e, pl.px, pl.py);  // one * line (mod.rs:589 on f = one)
                else
                    f = apply_line(f, pl.e, pl.px, pl.py);
#endif
            }
        }
    }
    st_fq12(out, kL * (size_t)plan.total, l, f);
    SEG_STAMP(1, __builtin_amdgcn_s_memrealtime());
}

// G2 * Fr (mod.rs:272-292) on the pairing path's two-lane layout: the chain of
// curve.h jac_mul with lane 2i + c holding coordinate c of element i, so a batch
// is twice the waves of a one-lane kernel (rounds 1-3) and each lane holds half the state.
// Both lanes of an element follow the same scalar, so the ballot schedule's
// decisions are the one-lane kernel's.  Launched with kPairBlock threads per
// block (kernels.h: issue balance).
__global__ void BN_PATH_ATTR __launch_bounds__(kPairBlock) k_g2_mul_split(const bn_g2* __restrict__ p,
                                                                         const bn_fr* __restrict__ k, size_t n,
                                                                         bn_g2* __restrict__ out) {
    fold_table_init();
    const Balance bal = balance_init();
    const size_t l = lane_id(), i = l / kL;
    if (i >= n) return;
    uint32_t s[8];
    fr_to_canonical(k[i], s);
    const G2J a = {widen<kPt>(ld_ref2(p[i].x)), widen<kPt>(ld_ref2(p[i].y)), widen<kPt>(ld_ref2(p[i].z))};
    const G2J r = jac_mul(a, s, [&](int t) { balance_step(bal, (uint32_t)t); });
    st_ref2(out[i].x, r.x);
    st_ref2(out[i].y, r.y);
    st_ref2(out[i].z, r.z);
}

}  // namespace bn

BN_EXPORT_FOLD_CHECK(pairing)

#if BN_SEG_STAMPS
extern "C" int bn_dbg_seg_stamps(uint64_t* out, int nwaves) {
    if (nwaves > bn::kSegStampWaves) nwaves = bn::kSegStampWaves;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(bn::g_seg_stamps), (size_t)nwaves * 4 * sizeof(uint64_t)) == hipSuccess
               ? nwaves : -1;
}
#endif
