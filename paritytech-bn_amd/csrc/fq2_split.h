// fq2_split.h -- Fq2 = Fq[u]/(u^2+1) with TWO lanes per element (BN_SPLIT;
// included by tower.h inside namespace bn).
//
// Lanes 2j and 2j+1 of a wave hold coordinate c0 and c1 of element j.  Every
// Fq2 operation below computes this lane's coordinate of the result; the
// other coordinate, when needed, comes from the partner lane over DPP
// (quad_perm [1,0,3,2]: one v_mov_b32_dpp per 32-bit digit).  Additions,
// subtractions, halving, folds and scaling by an Fq are lane-local: each lane
// does half of the unsplit work.  A product is one column sum of two digit
// products per lane, reduced once -- lane 0: a0*b0 + a1*(K*p - b1), lane 1:
// a0*b1 + a1*b0 -- i.e. exactly one coordinate of fq2_mul_sb.
//
// Why: with one lane per element a batch of 2^16 pairings is 1024 waves, one
// per SIMD, and a lone wave issues one VALU instruction every ~6 cycles
// whatever the instruction; two waves per SIMD issue the digit-wise VOP2 work
// 2.5x faster and MADs ~15 % faster (profiles/r2d_valu_ubench.jsonl).  Split
// lanes give 2048 waves for the same batch, and each lane holds half the
// state (an Fq12 is 54 VGPRs), so two waves fit the register file.
//
// Bit-exactness: each lane computes the same residue as the corresponding
// coordinate of the one-lane formulas (the same ring identities), and values
// are canonicalized only at the boundary.

template <int B>
struct Fq2 {
    Fq<B> c;  // this lane's coordinate: c0 on even lanes, c1 on odd lanes
};

BN_INLINE bool lane_odd() {
#if defined(__HIP_DEVICE_COMPILE__)
    return (__builtin_amdgcn_workitem_id_x() & 1u) != 0;
#else
    return false;
#endif
}
// the partner lane's copy of a 32-bit value (lanes 2j <-> 2j+1)
BN_INLINE uint32_t swap_pair(uint32_t v) {
#if defined(__HIP_DEVICE_COMPILE__)
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);
#else
    return v;
#endif
}
template <int B>
BN_INLINE Fq<B> fq_partner(const Fq<B>& a) {
    Fq<B> r;
#pragma unroll
    for (int l = 0; l < 9; ++l) r.v[l] = swap_pair(a.v[l]);
    return r;
}
// coordinate c0 (CTRL 0xA0: quad_perm [0,0,2,2]) or c1 (0xF5: [1,1,3,3]) of the
// element on both lanes of the pair: one DPP move per digit, no select
template <int CTRL>
BN_INLINE uint32_t bcast_pair(uint32_t v) {
#if defined(__HIP_DEVICE_COMPILE__)
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, false);
#else
    return v;  // host builds run one lane per element: see the host forms below
#endif
}
template <int B>
BN_INLINE Fq<B> fq_bcast_c0(const Fq<B>& a) {
    Fq<B> r;
#pragma unroll
    for (int l = 0; l < 9; ++l) r.v[l] = bcast_pair<0xA0>(a.v[l]);
    return r;
}
template <int B>
BN_INLINE Fq<B> fq_bcast_c1(const Fq<B>& a) {
    Fq<B> r;
#pragma unroll
    for (int l = 0; l < 9; ++l) r.v[l] = bcast_pair<0xF5>(a.v[l]);
    return r;
}
template <int K>
BN_INLINE Fq2<K> wrap2(const Fq<K>& x) { return {x}; }

template <int B2, int B>
BN_INLINE Fq2<B2> widen(const Fq2<B>& a) { return {widen<B2>(a.c)}; }

BN_INLINE Fq2<1> fq2_const(const Limbs9& c0, const Limbs9& c1) {
    return {fq_select(lane_odd(), fq_from_limbs<1>(c1), fq_from_limbs<1>(c0))};
}
BN_INLINE Fq2<1> fq2_zero() { return {fq_zero()}; }
BN_INLINE Fq2<1> fq2_one() { return {fq_select(lane_odd(), fq_zero(), fq_one())}; }
template <int B>
BN_INLINE Fq2<B> fq2_select(bool c, const Fq2<B>& a, const Fq2<B>& b) { return {fq_select(c, a.c, b.c)}; }
template <int A, int B>
BN_INLINE auto fq2_add(const Fq2<A>& a, const Fq2<B>& b) { return wrap2(fq_add(a.c, b.c)); }
template <int A, int B>
BN_INLINE auto fq2_sub(const Fq2<A>& a, const Fq2<B>& b) { return wrap2(fq_sub(a.c, b.c)); }
template <int B>
BN_INLINE auto fq2_neg(const Fq2<B>& a) { return wrap2(fq_neg(a.c)); }
template <int B>
BN_INLINE auto fq2_dbl(const Fq2<B>& a) { return fq2_add(a, a); }
template <int B>
BN_INLINE Fq2<2> fq2_fold(const Fq2<B>& a) { return {fq_fold(a.c)}; }
template <int B>
BN_INLINE Fq2<kv(B)> fq2_norm(const Fq2<B>& a) { return {fq_norm(a.c)}; }
template <int B>
BN_INLINE auto fq2_half(const Fq2<B>& a) { return wrap2(fq_half(a.c)); }
// fq2.rs:48-53 (s must hold the same value on both lanes of the element)
template <int A, int B>
BN_INLINE auto fq2_scale(const Fq2<A>& a, const Fq<B>& s) { return wrap2(fq_mul(a.c, s)); }
template <int L, int B>
BN_INLINE auto pre(const Fq2<B>& a) {
    if constexpr (kv(B) <= L) return a; else return fq2_fold(a);
}
// both lanes agree: element zero iff both coordinates are
template <int B>
BN_INLINE bool fq2_is_zero(const Fq2<B>& a) {
    const uint32_t z = fq_is_zero(a.c) ? 1u : 0u;
    return (z & swap_pair(z)) != 0;
}
template <int A, int B>
BN_INLINE bool fq2_eq(const Fq2<A>& a, const Fq2<B>& b) {
    const uint32_t e = fq_eq(a.c, b.c) ? 1u : 0u;
    return (e & swap_pair(e)) != 0;
}
template <int B>
BN_INLINE void fq2_fence(Fq2<B>& a) {
    fq_fence(a.c);
}
// the fences around the two-lane products (below): 3 = inputs and results (rounds 2-4),
// 1 = results only, 0 = none (default).  They kept the compiler from interleaving the
// digit products of several Fq2 products; since every product is one asm statement
// (BN_DOT2_ASM) there is nothing to interleave, and the "+v" input fences only made
// the compiler copy every input it still needed (the fenced value counts as
// rewritten): k_pairing_full 6.3 % fewer instructions, scratch 716 -> 584 B/lane,
// 7.60-7.62 -> 7.47-7.49 ms (frac 0.491 -> 0.500), G2 * Fr 6.01-6.08 -> 5.82-5.86 ms
// (profiles/r5q_ab_fence.txt)
#ifndef BN_FQ2_FENCE
#define BN_FQ2_FENCE 0
#endif
template <int B>
BN_INLINE void fq2_fence_in(Fq2<B>& a) {
    if constexpr ((BN_FQ2_FENCE & 2) != 0) fq2_fence(a);
}
template <int B>
BN_INLINE void fq2_fence_out(Fq2<B>& a) {
    if constexpr ((BN_FQ2_FENCE & 1) != 0) fq2_fence(a);
}

// K*p - x without a carry pass (digits < (sub_spread(L)+2)*2^29, value <= (B+1)*p)
template <int K>
BN_INLINE Fq<kenc(kv(K) + 1, sub_spread(kl(K)) + 2)> fq_neg_lazy(const Fq<K>& x) {
    constexpr Limbs9 Q = kp_spread(kv(K) + 1, sub_spread(kl(K)));
    Fq<kenc(kv(K) + 1, sub_spread(kl(K)) + 2)> r;
#pragma unroll
    for (int i = 0; i < 9; ++i) r.v[i] = Q.v[i] - x.v[i];
    return r;
}
// fq2_mul_split takes its w operand (lane 0: K*p - b1, lane 1: b1) as one
// v_cndmask_b32_dpp per digit -- odd lanes keep their own b1, even lanes take the
// partner's K*p - b1 through the DPP swap -- instead of a broadcast, a negation
// and a select: 9 VALU fewer per product, k_pairing_full 7.79-7.81 -> 7.73-7.75 ms
// (profiles/r3r_ab_dppsel.txt)
#if defined(__HIP_DEVICE_COMPILE__)
#define BN_DPPSEL_VCC "s_mov_b32 vcc_lo, 0xaaaaaaaa\n\ts_mov_b32 vcc_hi, 0xaaaaaaaa\n\ts_nop 1\n\t"
#define BN_DPPSEL_OP(o, a, b) "v_cndmask_b32_dpp %" #o ", %" #a ", %" #b ", vcc quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
// w[i] = odd lane ? own[i] : the partner's neg[i].  The s_nop covers the two
// wait states a DPP read needs after the VALU write of its source (the hazard
// recognizer does not look inside inline asm).
BN_INLINE void dpp_sel_own_partner(uint32_t (&w)[9], const uint32_t (&own)[9], const uint32_t (&neg)[9]) {
    const uint32_t odd = __builtin_amdgcn_workitem_id_x() & 1u;
    asm(BN_DPPSEL_VCC BN_DPPSEL_OP(0, 9, 18) BN_DPPSEL_OP(1, 10, 19) BN_DPPSEL_OP(2, 11, 20) BN_DPPSEL_OP(3, 12, 21)
            BN_DPPSEL_OP(4, 13, 22) BN_DPPSEL_OP(5, 14, 23) BN_DPPSEL_OP(6, 15, 24) BN_DPPSEL_OP(7, 16, 25)
                BN_DPPSEL_OP(8, 17, 26)
        : "=&v"(w[0]), "=&v"(w[1]), "=&v"(w[2]), "=&v"(w[3]), "=&v"(w[4]), "=&v"(w[5]), "=&v"(w[6]), "=&v"(w[7]),
          "=&v"(w[8])
        : "v"(neg[0]), "v"(neg[1]), "v"(neg[2]), "v"(neg[3]), "v"(neg[4]), "v"(neg[5]), "v"(neg[6]), "v"(neg[7]),
          "v"(neg[8]), "v"(own[0]), "v"(own[1]), "v"(own[2]), "v"(own[3]), "v"(own[4]), "v"(own[5]), "v"(own[6]),
          "v"(own[7]), "v"(own[8]), "v"(odd)
        : "vcc");
}
#endif
// per-lane choice between two values of different static types (the join)
template <int A, int B>
BN_INLINE Fq<kjoin(A, B)> fq_pick(bool c, const Fq<A>& a, const Fq<B>& b) {
    Fq<kjoin(A, B)> r;
#pragma unroll
    for (int i = 0; i < 9; ++i) r.v[i] = c ? a.v[i] : b.v[i];
    return r;
}

// REDC(x*y + z*w): one Montgomery reduction of a two-product column sum (the
// fq_mul column scan with a second product per column).  Column sums stay
// below 2^64 when Lx*Ly + Lz*Lw <= 6.
template <int X, int Y, int Z, int W>
BN_INLINE auto fq_dot2(const Fq<X>& x, const Fq<Y>& y, const Fq<Z>& z, const Fq<W>& w) {
    static_assert(kl(X) * kl(Y) + kl(Z) * kl(W) <= 6, "fq_dot2: column sum could overflow 64 bits");
    constexpr int BO = 1 + (int)(((long long)kv(X) * kv(Y) + (long long)kv(Z) * kv(W)) * 5908 / 1000000 + 1);
    Fq<BO> r;
#if BN_DOT2_ASM && defined(__HIP_DEVICE_COMPILE__)
    if constexpr ((BN_DOT2_ASM & 1) != 0) {
        asm(BN_ASM_DOT2 : BN_ASM_OUT9(r.v) : BN_ASM_IN9(x.v), BN_ASM_IN9(y.v), BN_ASM_IN9(z.v), BN_ASM_IN9(w.v), BN_ASM_P
            : BN_ASM_CLOBBER);
        return r;
    }
#endif
    uint32_t m[9];
    uint64_t acc = 0;
#pragma unroll
    for (int k = 0; k < 17; ++k) {
        const int lo = k < 9 ? 0 : k - 8;
        const int hi = k < 9 ? k : 8;
#pragma unroll
        for (int i = lo; i <= hi; ++i) {
            acc += (uint64_t)x.v[i] * y.v[k - i];
            acc += (uint64_t)z.v[i] * w.v[k - i];
        }
#pragma unroll
        for (int i = lo; i <= hi; ++i)
            if (i < k) acc += (uint64_t)m[i] * kP29.v[k - i];
        if (k < 9) {
            m[k] = ((uint32_t)acc * BN_PINV29) & M29;
            acc += (uint64_t)m[k] * kP29.v[0];
        } else {
            r.v[k - 9] = (uint32_t)acc & M29;
        }
        acc >>= 29;
    }
    r.v[8] = (uint32_t)acc;
    return r;
}

// fq2.rs:136-148 (the same residues as fq2_mul_sb): lane 0 computes
// c0 = a0*b0 + a1*(K*p - b1), lane 1 computes c1 = a1*b0 + a0*b1, both as
// own_a * Y + partner_a * W with per-lane operand choice.
// the fq_dot2 column budget of fq2_mul_split(a, b) for digit bounds La, Lb: x = a,
// y = b or its partner (Lb), z = partner of a (La), w = b or K*p - partner (fq_neg_lazy)
constexpr int split_mul_cost(int La, int Lb) {
    return La * Lb + La * (Lb > sub_spread(Lb) + 2 ? Lb : sub_spread(Lb) + 2);
}
template <int A, int B>
BN_INLINE auto fq2_mul_split(const Fq2<A>& a, const Fq2<B>& b) {
    if constexpr (split_mul_cost(kl(A), kl(B)) > 6) {
        if constexpr (split_mul_cost(kl(B), kl(A)) <= 6) return fq2_mul_split(b, a);
        else if constexpr (kl(A) >= kl(B)) return fq2_mul_split(fq2_norm(a), b);
        else return fq2_mul_split(a, fq2_norm(b));
    } else {
        const bool odd = lane_odd();
        const Fq<A> pa = fq_partner(a.c);
#if defined(__HIP_DEVICE_COMPILE__)
        const Fq<B> y = fq_bcast_c0(b.c);
        const auto nb = fq_neg_lazy(b.c);  // the odd lane's is K*p - b1
        Fq<kjoin(B, kenc(kv(B) + 1, sub_spread(kl(B)) + 2))> w;
        dpp_sel_own_partner(w.v, b.c.v, nb.v);
        (void)odd;
#else
        const Fq<B> pb = fq_partner(b.c);
        const Fq<B> y = fq_select(odd, pb, b.c);
        const auto w = fq_pick(odd, b.c, fq_neg_lazy(pb));
#endif
        return wrap2(fq_dot2(a.c, y, pa, w));
    }
}
template <int A, int B>
BN_INLINE auto fq2_mul(const Fq2<A>& a_in, const Fq2<B>& b_in) {
    if constexpr (kv(A) > 40 || kv(B) > 40) return fq2_mul(pre<40>(a_in), pre<40>(b_in)); else {
    Fq2<A> a = a_in;
    Fq2<B> b = b_in;
    fq2_fence_in(a);
    fq2_fence_in(b);
    auto r = fq2_mul_split(a, b);
    fq2_fence_out(r);
    return r;
    }
}
template <class R, class S>
struct Fq2Pair {
    R a;
    S b;
};
template <int A, int B, int C, int D>
BN_INLINE auto fq2_mul2(const Fq2<A>& a_in, const Fq2<B>& b_in, const Fq2<C>& c_in, const Fq2<D>& d_in) {
    if constexpr (kv(A) > 40 || kv(B) > 40 || kv(C) > 40 || kv(D) > 40) {
        return fq2_mul2(pre<40>(a_in), pre<40>(b_in), pre<40>(c_in), pre<40>(d_in));
    } else {
        Fq2<A> a = a_in;
        Fq2<B> b = b_in;
        Fq2<C> c = c_in;
        Fq2<D> d = d_in;
        fq2_fence_in(a);
        fq2_fence_in(b);
        fq2_fence_in(c);
        fq2_fence_in(d);
        auto r = fq2_mul_split(a, b);
        auto q = fq2_mul_split(c, d);
        fq2_fence_out(r);
        fq2_fence_out(q);
        return Fq2Pair<decltype(r), decltype(q)>{r, q};
    }
}

// fq2.rs:105-117: c0 = (a0 - a1)(a0 + a1), c1 = 2*a0*a1 -- one product per lane:
// lane 0: (a0 + K*p - a1) * (a0 + a1), lane 1: a1 * (a0 + a0).  x keeps digits
// below 3*2^29 (no carry pass: fq_mul takes a 3 x 2 digit-bound product).
template <int A>
BN_INLINE auto fq2_sqr(const Fq2<A>& a_in) {
    if constexpr (kv(A) > 40) return fq2_sqr(fq2_fold(a_in)); else {
    Fq2<A> a = a_in;
    fq2_fence_in(a);
    const bool odd = lane_odd();
    const Fq<kv(A)> own = fq_norm(a.c);
    const Fq<kv(A)> par = fq_partner(own);
    const auto x = fq_pick(odd, own, fq_sub(own, par));
    const auto y = fq_add(par, fq_select(odd, par, own));
    auto r = wrap2(fq_mul(x, y));
    fq2_fence_out(r);
    return r;
    }
}
// x * xi, xi = 9 + u (fq2.rs:19-34, 55-57): lane 0: 9a0 - a1, lane 1: 9a1 + a0.
template <int A>
BN_INLINE auto fq2_mul_xi(const Fq2<A>& a) {
    if constexpr (kv(A) > 8) {
        return fq2_mul_xi(fq2_fold(a));
    } else {
        const Fq<kv(A)> own = fq_norm(a.c);
        const auto own9 = fq_add(fq_mul_small<8>(own), own);
        const Fq<kv(A)> par = fq_partner(own);
        return wrap2(fq_add(own9, fq_pick(lane_odd(), par, fq_neg_lazy(par))));
    }
}
// fq2.rs:59-68: odd powers conjugate: lane 1 negates (c1 * (p-1) == -c1)
template <int B>
BN_INLINE auto fq2_conj(const Fq2<B>& a) {
    const Fq<kv(B)> own = fq_norm(a.c);
    return wrap2(fq_select(lane_odd(), fq_neg(own), own));
}
// fq2.rs:119-130: t = (c0^2 + c1^2)^-1 on both lanes, then (c0 t, -c1 t); Quad: both
// lane pairs of every quad hold the same element (fq_inv_quad)
template <bool Quad = false, int B>
BN_INLINE auto fq2_inv(const Fq2<B>& a_in) {
    auto a = pre<40>(a_in);
    const auto sq = fq_sqr(a.c);
    const auto t = fq_inv<Quad>(fq_add(sq, fq_partner(sq)));  // the same norm on both lanes
    const auto r = fq_mul(a.c, t);
    return wrap2(fq_select(lane_odd(), fq_neg(r), r));
}
