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

// f <- f * line(P): ell_vw.scale(Py), ell_vv.scale(Px)  (mod.rs:589)
template <int B, int PB>
BN_INLINE Fq12<kF> apply_line(const Fq12<B>& f, const Ell& c, const Fq<PB>& px, const Fq<PB>& py) {
    return narrow12<kF>(fq12_mul_by_024(f, c.ell_0, narrow<kLine>(fq2_scale(c.ell_vw, py)),
                                        narrow<kLine>(fq2_scale(c.ell_vv, px))));
}

// G2Precomp::miller_loop, mod.rs:579-607.  `line(k)` returns coefficient k.
template <int PB, typename Line>
BN_INLINE Fq12<kF> miller_loop(const Fq<PB>& px, const Fq<PB>& py, Line&& line) {
    Fq12<kF> f = widen<kF>(fq12_one());
    int idx = 0;
#pragma unroll 1
    for (int i = 0; i < BN_NAF_DIGITS; ++i) {
        f = apply_line(narrow12<kF>(fq12_sqr(f)), line(idx++), px, py);
        if ((kNafNonzero >> i) & 1u) f = apply_line(f, line(idx++), px, py);
    }
    f = apply_line(f, line(idx++), px, py);
    f = apply_line(f, line(idx), px, py);
    return f;
}

// The Miller loop with the line steps inline (k_pairing_fused): the
// coefficients of g2_precompute applied as they are produced, in
// G2Precomp::miller_loop's order (mod.rs:579-607, 701-727)
template <int B, int PB>
BN_INLINE Fq12<kF> miller_fused(const G2Aff<B>& q, const Fq<PB>& px, const Fq<PB>& py) {
    G2Proj r = {widen<kPt>(q.x), widen<kPt>(q.y), widen<kPt>(fq2_one())};
    const G2Aff<B> q_neg = {q.x, fq2_neg(q.y)};
    Fq12<kF> f = widen<kF>(fq12_one());
#pragma unroll 1
    for (int i = 0; i < BN_NAF_DIGITS; ++i) {
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
template <int PB, typename Line>
BN_INLINE Fq12<kF> miller_segment(const Fq<PB>& px, const Fq<PB>& py, int lo, int hi, int idx, Line&& line) {
    Fq12<kF> f = widen<kF>(fq12_one());
#pragma unroll 1
    for (int i = lo; i < hi; ++i) {
        f = apply_line(narrow12<kF>(fq12_sqr(f)), line(idx++), px, py);
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
