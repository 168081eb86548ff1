// pairing.h -- optimal-ate pairing pieces, one lane per pairing.
//
// Replaces src/groups/mod.rs:579-727 (G2 precomputation, Miller loop) and
// src/fields/fq12.rs:62-124, 249-266 (final exponentiation, exp_by_neg_z).
#pragma once
#include "curve.h"

namespace bn {

// storage bound of the Miller accumulator and of the final-exponentiation temporaries
constexpr int kF = 2;
template <int S, int B>
BN_INLINE Fq12<S> narrow12(const Fq12<B>& a) {
    if constexpr (kv(B) <= S) {
        return widen<S>(fq12_norm(a));
    } else {
        return widen<S>(fq12_fold(a));
    }
}

// ---------------------------------------------------------------- G2 precomputation
// AffineG2::precompute, mod.rs:701-727.  `emit(k, ell)` receives line k (0..86).
template <int B, typename Emit>
BN_INLINE void g2_precompute(const G2Aff<B>& q, Emit&& emit) {
    G2Proj r = {widen<kPt>(q.x), widen<kPt>(q.y), widen<kPt>(fq2_one())};
    const G2Aff<B> q_neg = {q.x, fq2_neg(q.y)};
    int k = 0;
#pragma unroll 1
    for (int i = 0; i < BN_NAF_DIGITS; ++i) {
        emit(k++, doubling_step(r));
        if ((kNafNonzero >> i) & 1u) {  // uniform across the wave
            const bool minus = (kNafMinus >> i) & 1u;
            G2Aff<B> base = {q.x, fq2_select(minus, q_neg.y, q.y)};
            emit(k++, mixed_addition_step(r, base));
        }
    }
    G2Aff<kPt> q1 = mul_by_q(q);
    G2Aff<kPt> q2 = mul_by_q(q1);
    q2.y = fq2_neg(q2.y);
    emit(k++, mixed_addition_step(r, q1));
    emit(k++, mixed_addition_step(r, q2));
}

#if BN_SPLIT
// BN_DOT6_ASM: each output's six-product column sum as one v_mad_u64_u32 chain
// (dot2_asm.inc) instead of 17 64-bit column accumulators: k_miller_seg's loop
// spilled 27 dwords and reloaded 44 per line with the accumulators (scratch 320 ->
// 72 B per lane), config 5 1.84-1.90 -> 1.76-1.80 ms and its PMC traffic 1.62 ->
// 0.80 GB per product, k_pairing_full unchanged (profiles/r5w_ab_dot6.txt)
#ifndef BN_DOT6_ASM
#define BN_DOT6_ASM 1
#endif
// The same product f * (x0 + x4 w^3 + x2 w^4) on the two-lane layout, as six
// column sums reduced once each.  In the w-basis (f_m = coefficient of w^m:
// c0.c(m/2) for even m, c1.c((m-1)/2) for odd m; w^6 = xi)
//   out_m = f_m x0 + f_(m-3) x4 + f_(m-4) x2,  indices mod 6, times xi on a wrap,
// with xi moved onto the f side (xi f_2 .. xi f_5).  Each lane sums its
// coordinate of three Fq2 products -- six digit products, own(u) * v0 +
// partner(u) * (lane 0: K*p - v1, lane 1: v1) -- in one column accumulator and
// reduces once: 36 products + 6 reductions per lane instead of the 13-product
// formula's 26 + 13, and no combining adds, subtractions or folds.  The line
// side's operand forms are built once per coefficient.  The value is the
// reference's product (fq12.rs:130-196) -- the same residues.
struct LineOps {
    Fq<kLine> y;  // v0 on both lanes
    Fq<8> w;      // lane 0: K*p - v1, lane 1: v1 (normalized digits, value <= (kLine + 1) p)
};
template <int X>
BN_INLINE LineOps line_ops(const Fq2<X>& v_in) {
    const Fq<kv(X)> v = fq_norm(v_in.c);
    const bool odd = lane_odd();
#if defined(__HIP_DEVICE_COMPILE__)
    // w as fq2_mul_split forms it: the odd lane's own v1, the even lane the partner's K*p - v1
    Fq<kjoin(kv(X), kenc(kv(X) + 1, 2))> w;
    dpp_sel_own_partner(w.v, v.v, fq_neg_lazy(v).v);
    (void)odd;
    return {widen<kLine>(fq_bcast_c0(v)), widen<8>(fq_norm(w))};
#else
    const Fq<kv(X)> pv = fq_partner(v);
    return {widen<kLine>(fq_select(odd, pv, v)), widen<8>(fq_norm(fq_pick(odd, v, fq_neg_lazy(pv))))};
#endif
}
// t += u * v for this lane's coordinate (u: f side, normalized)
BN_INLINE void acc_mad2(Acc& t, const Fq<2>& u, const LineOps& v) {
    acc_mad(t, u, v.y);
    acc_mad(t, fq_partner(u), v.w);
}
template <int F, int X>
BN_INLINE Fq12<2> fq12_mul_by_024_lazy(const Fq12<F>& f_in, const Fq2<X>& x0_in, const Fq2<X>& x4_in,
                                       const Fq2<X>& x2_in) {
    static_assert(kl(F) == 1 && kv(F) <= 2, "fq12_mul_by_024_lazy: f normalized, bound 2");
    const LineOps x0 = line_ops(x0_in), x4 = line_ops(x4_in), x2 = line_ops(x2_in);
    const Fq<2> f0 = widen<2>(f_in.c0.c0.c), f1 = widen<2>(f_in.c1.c0.c), f2 = widen<2>(f_in.c0.c1.c);
    const Fq<2> f3 = widen<2>(f_in.c1.c1.c), f4 = widen<2>(f_in.c0.c2.c), f5 = widen<2>(f_in.c1.c2.c);
    auto xi = [](const Fq<2>& u) { return fq2_fold(fq2_mul_xi(Fq2<2>{u})).c; };
    // value per lane <= 3 * (2p * 4p + 2p * 5p) = 54 p^2: the reduction is below 1.4 p
    auto out = [&](const Fq<2>& a, const LineOps& va, const Fq<2>& b, const LineOps& vb, const Fq<2>& c,
                   const LineOps& vc) {
#if BN_DOT6_ASM && BN_DOT2_ASM && defined(__HIP_DEVICE_COMPILE__)
        // the same six-product column sum as one v_mad_u64_u32 chain (dot2_asm.inc
        // BN_ASM_DOT6): no 17-column accumulator held across the products
        const Fq<2> pa = fq_partner(a), pb = fq_partner(b), pc = fq_partner(c);
        Fq<2> r;
        asm(BN_ASM_DOT6 : BN_ASM_OUT9(r.v)
            : BN_ASM_IN9(a.v), BN_ASM_IN9(va.y.v), BN_ASM_IN9(pa.v), BN_ASM_IN9(va.w.v), BN_ASM_IN9(b.v),
              BN_ASM_IN9(vb.y.v), BN_ASM_IN9(pb.v), BN_ASM_IN9(vb.w.v), BN_ASM_IN9(c.v), BN_ASM_IN9(vc.y.v),
              BN_ASM_IN9(pc.v), BN_ASM_IN9(vc.w.v), BN_ASM_P
            : BN_ASM_CLOBBER);
        return Fq2<2>{r};
#else
        Acc t = {};
        acc_mad2(t, a, va);
        acc_mad2(t, b, vb);
        acc_mad2(t, c, vc);
        return Fq2<2>{acc_redc<2>(t)};
#endif
    };
    // outputs last-first, each xi*f_k made just before its first use: under the default
    // scheduler 0.7 % faster than first-first with the four xi*f_k up front
    // (k_pairing_fused 4.31 vs 4.34 ms, config 5 2.65 vs 2.70 ms, profiles/r2ax_ab_line_order.txt)
    const Fq2<2> o5 = out(f5, x0, f2, x4, f1, x2);
    const Fq2<2> o4 = out(f4, x0, f1, x4, f0, x2);
    const Fq<2> g5 = xi(f5);
    const Fq2<2> o3 = out(f3, x0, f0, x4, g5, x2);
    const Fq<2> g4 = xi(f4);
    const Fq2<2> o2 = out(f2, x0, g5, x4, g4, x2);
    const Fq<2> g3 = xi(f3);
    const Fq2<2> o1 = out(f1, x0, g4, x4, g3, x2);
    const Fq<2> g2 = xi(f2);
    const Fq2<2> o0 = out(f0, x0, g3, x4, g2, x2);
    return {{o0, o2, o4}, {o1, o3, o5}};
}
#endif

// f <- f * line(P): ell_vw.scale(Py), ell_vv.scale(Px)  (mod.rs:589)
template <int B, int PB>
BN_INLINE Fq12<kF> apply_line(const Fq12<B>& f, const Ell& c, const Fq<PB>& px, const Fq<PB>& py) {
#if BN_SPLIT
    return widen<kF>(fq12_mul_by_024_lazy(narrow12<2>(f), c.ell_0, narrow<kLine>(fq2_scale(c.ell_vw, py)),
                                          narrow<kLine>(fq2_scale(c.ell_vv, px))));
#else
    return narrow12<kF>(fq12_mul_by_024(f, c.ell_0, narrow<kLine>(fq2_scale(c.ell_vw, py)),
                                        narrow<kLine>(fq2_scale(c.ell_vv, px))));
#endif
}

// the same with the line already scaled by P (e.ell_vw = ell_vw * Py, e.ell_vv = ell_vv * Px:
// what the producers store with BN_LINES_PRESCALED, lines_wide.h PwEll)
template <int B>
BN_INLINE Fq12<kF> apply_line_scaled(const Fq12<B>& f, const Ell& e) {
#if BN_SPLIT
    return widen<kF>(fq12_mul_by_024_lazy(narrow12<2>(f), e.ell_0, e.ell_vw, e.ell_vv));
#else
    return narrow12<kF>(fq12_mul_by_024(f, e.ell_0, e.ell_vw, e.ell_vv));
#endif
}
BN_INLINE Fq12<kF> line_from_one_scaled(const Ell& e) {
    const Fq2<kF> z = widen<kF>(fq2_zero());
    return {{narrow<kF>(e.ell_0), z, narrow<kF>(e.ell_vv)}, {z, narrow<kF>(e.ell_vw), z}};
}

// The first step of a loop (or segment) that starts from f = one: one^2 * line
// is the line itself, x0 + x4 w^3 + x2 w^4 (w^3 = c1.c1, w^4 = c0.c2; the
// operands of apply_line), so the squaring and the sparse product are skipped
// (k_miller_seg at one pairing, 16 segments: 194 -> 177 us).  The same residues
// as fq12.rs mul_by_024 applied to Fq12::one().
template <int PB>
BN_INLINE Fq12<kF> line_from_one(const Ell& c, const Fq<PB>& px, const Fq<PB>& py) {
    const Fq2<kF> z = widen<kF>(fq2_zero());
    return {{narrow<kF>(c.ell_0), z, narrow<kF>(fq2_scale(c.ell_vv, px))},
            {z, narrow<kF>(fq2_scale(c.ell_vw, py)), z}};
}
// f^2 * line, or the line alone on the first step from f = one (wave-uniform `first`)
template <int PB>
BN_INLINE Fq12<kF> sqr_line(const Fq12<kF>& f, bool first, const Ell& c, const Fq<PB>& px, const Fq<PB>& py) {
    if (first) return line_from_one(c, px, py);
    return apply_line(narrow12<kF>(fq12_sqr(f)), c, px, py);
}

// G2Precomp::miller_loop, mod.rs:579-607.  `line(k)` returns coefficient k.
template <int PB, typename Line>
BN_INLINE Fq12<kF> miller_loop(const Fq<PB>& px, const Fq<PB>& py, Line&& line) {
    Fq12<kF> f = widen<kF>(fq12_one());
    int idx = 0;
#pragma unroll 1
    for (int i = 0; i < BN_NAF_DIGITS; ++i) {
        f = sqr_line(f, i == 0, line(idx++), px, py);
        if ((kNafNonzero >> i) & 1u) f = apply_line(f, line(idx++), px, py);
    }
    f = apply_line(f, line(idx++), px, py);
    f = apply_line(f, line(idx), px, py);
    return f;
}
// the same over lines already scaled by P (apply_line_scaled)
template <typename Line>
BN_INLINE Fq12<kF> miller_loop_scaled(Line&& line) {
    Fq12<kF> f = widen<kF>(fq12_one());
    int idx = 0;
#pragma unroll 1
    for (int i = 0; i < BN_NAF_DIGITS; ++i) {
        const Ell e = line(idx++);
        f = i == 0 ? line_from_one_scaled(e) : apply_line_scaled(narrow12<kF>(fq12_sqr(f)), e);
        if ((kNafNonzero >> i) & 1u) f = apply_line_scaled(f, line(idx++));
    }
    f = apply_line_scaled(f, line(idx++));
    f = apply_line_scaled(f, line(idx));
    return f;
}

// The Miller loop with the line steps inline (k_pairing_fused): the
// coefficients of g2_precompute applied as they are produced, in
// G2Precomp::miller_loop's order (mod.rs:579-607, 701-727)
// `step(i)` runs at the start of digit i (the kernels' issue balance, kernels.h)
struct NoStep {
    BN_INLINE void operator()(int) const {}
};
template <int B, int PB, typename Step = NoStep>
BN_INLINE Fq12<kF> miller_fused(const G2Aff<B>& q, const Fq<PB>& px, const Fq<PB>& py, Step&& step = Step{}) {
    G2Proj r = {widen<kPt>(q.x), widen<kPt>(q.y), widen<kPt>(fq2_one())};
    const G2Aff<B> q_neg = {q.x, fq2_neg(q.y)};
    Fq12<kF> f = widen<kF>(fq12_one());
#pragma unroll 1
    for (int i = 0; i < BN_NAF_DIGITS; ++i) {
        step(i);
        // (sqr_line's first-step shortcut here measured 5 % slower: 4.58 vs 4.35 ms,
        // a register-allocation change; it stays in the segment and coefficient loops)
        f = apply_line(narrow12<kF>(fq12_sqr(f)), doubling_step(r), px, py);
        if ((kNafNonzero >> i) & 1u) {
            const bool minus = (kNafMinus >> i) & 1u;
            G2Aff<B> base = {q.x, fq2_select(minus, q_neg.y, q.y)};
            f = apply_line(f, mixed_addition_step(r, base), px, py);
        }
    }
    G2Aff<kPt> q1 = mul_by_q(q);
    G2Aff<kPt> q2 = mul_by_q(q1);
    q2.y = fq2_neg(q2.y);
    f = apply_line(f, mixed_addition_step(r, q1), px, py);
    f = apply_line(f, mixed_addition_step(r, q2), px, py);
    return f;
}

// One segment of the Miller loop: digits [lo, hi) starting from f = one, with
// line coefficients from index `idx` on; the last segment (hi == 64) also
// applies the two lines after the loop.  Running the loop over digits
// [0, 64) in segments g_0 .. g_(S-1) gives f = (..((g_0)^(2^len_1) g_1)^(2^len_2)
// ..) g_(S-1): squaring is a ring homomorphism, so the Horner recombination
// (kernels_wide.hip k_horner_wide) reproduces mod.rs:579-640 exactly.
template <int PB, typename Line, typename Step = NoStep>
BN_INLINE Fq12<kF> miller_segment(const Fq<PB>& px, const Fq<PB>& py, int lo, int hi, int idx, Line&& line,
                                  Step&& step = Step{}) {
    Fq12<kF> f = widen<kF>(fq12_one());
#pragma unroll 1
    for (int i = lo; i < hi; ++i) {
        step(i - lo);
        f = sqr_line(f, i == lo, line(idx++), px, py);
        if ((kNafNonzero >> i) & 1u) f = apply_line(f, line(idx++), px, py);
    }
    if (hi == BN_NAF_DIGITS) {
        f = apply_line(f, line(idx++), px, py);
        f = apply_line(f, line(idx), px, py);
    }
    return f;
}

// ---------------------------------------------------------------- final exponentiation
BN_INLINE Fq12<kF> mul12(const Fq12<kF>& a, const Fq12<kF>& b) { return narrow12<kF>(fq12_mul(a, b)); }
BN_INLINE Fq12<kF> cyc_sqr(const Fq12<kF>& a) { return narrow12<kF>(fq12_cyclotomic_sqr(a)); }

// exp_by_neg_z, fq12.rs:121-124: cyclotomic_pow by u = 4965661367192848881 (fq12.rs:249-266),
// then conjugate.  The first set bit multiplies one by self, i.e. starts at self.
BN_INLINE Fq12<kF> exp_by_neg_z(const Fq12<kF>& a) {
    constexpr uint64_t u = 4965661367192848881ull;  // bit 62 is the top set bit
    Fq12<kF> res = a;
#pragma unroll 1
    for (int bit = 61; bit >= 0; --bit) {
        res = cyc_sqr(res);
        if ((u >> bit) & 1u) res = mul12(a, res);
    }
    return fq12_conj(res);
}

// fq12.rs:62-73 (first chunk, given f != 0)
BN_INLINE Fq12<kF> fe_first_chunk(const Fq12<kF>& f) {
    Fq12<kF> b = narrow12<kF>(fq12_inv(f));
    Fq12<kF> a = fq12_conj(f);
    Fq12<kF> c = mul12(a, b);
    Fq12<kF> d = narrow12<kF>(fq12_frobenius_map<2>(c));
    return mul12(d, c);
}
// fq12.rs:75-105 (last chunk)
BN_INLINE Fq12<kF> fe_last_chunk(const Fq12<kF>& self) {
    Fq12<kF> a = exp_by_neg_z(self);
    Fq12<kF> b = cyc_sqr(a);
    Fq12<kF> c = cyc_sqr(b);
    Fq12<kF> d = mul12(c, b);
    Fq12<kF> e = exp_by_neg_z(d);
    Fq12<kF> f = cyc_sqr(e);
    Fq12<kF> g = exp_by_neg_z(f);
    Fq12<kF> h = fq12_conj(d);
    Fq12<kF> i = fq12_conj(g);
    Fq12<kF> j = mul12(i, e);
    Fq12<kF> k = mul12(j, h);
    Fq12<kF> l = mul12(k, b);
    Fq12<kF> m = mul12(k, e);
    Fq12<kF> n = mul12(self, m);
    Fq12<kF> o = narrow12<kF>(fq12_frobenius_map<1>(l));
    Fq12<kF> p = mul12(o, n);
    Fq12<kF> q = narrow12<kF>(fq12_frobenius_map<2>(k));
    Fq12<kF> r = mul12(q, p);
    Fq12<kF> s = fq12_conj(self);
    Fq12<kF> t = mul12(s, l);
    Fq12<kF> u = narrow12<kF>(fq12_frobenius_map<3>(t));
    return mul12(u, r);
}

}  // namespace bn
