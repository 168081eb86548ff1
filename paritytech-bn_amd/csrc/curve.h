// curve.h -- G1 / G2 Jacobian group law and the G2 line steps of the flipped
// Miller loop, one lane per point.
//
// Replaces src/groups/mod.rs:45-369 (generic G<P>), 371-472 (G1/G2 params),
// 515-564 (twist constants) and 693-776 (line steps).  The projective formulas
// are the reference's own -- they decide the Jacobian representation and the
// line coefficients, both of which are observable (G1*Fr output, pre-FE Miller
// values) -- so every coordinate is the same residue the reference computes.
#pragma once
#include "tower.h"

#if defined(__HIP_DEVICE_COMPILE__)
#define BN_ANY(p) (__any((int)(p)) != 0)
#define BN_ALL(p) (__all((int)(p)) != 0)
#else
#define BN_ANY(p) (p)
#define BN_ALL(p) (p)
#endif

namespace bn {

// ---------------------------------------------------------------- base-field dispatch
template <int A, int B>
BN_INLINE auto F_add(const Fq<A>& a, const Fq<B>& b) { return fq_add(a, b); }
template <int A, int B>
BN_INLINE auto F_add(const Fq2<A>& a, const Fq2<B>& b) { return fq2_add(a, b); }
template <int A, int B>
BN_INLINE auto F_sub(const Fq<A>& a, const Fq<B>& b) { return fq_sub(a, b); }
template <int A, int B>
BN_INLINE auto F_sub(const Fq2<A>& a, const Fq2<B>& b) { return fq2_sub(a, b); }
template <int A, int B>
BN_INLINE auto F_mul(const Fq<A>& a, const Fq<B>& b) { return fq_mul(a, b); }
template <int A, int B>
BN_INLINE auto F_mul(const Fq2<A>& a, const Fq2<B>& b) { return fq2_mul(a, b); }
template <int A>
BN_INLINE auto F_sqr(const Fq<A>& a) { return fq_sqr(a); }
template <int A>
BN_INLINE auto F_sqr(const Fq2<A>& a) { return fq2_sqr(a); }
template <int A>
BN_INLINE auto F_neg(const Fq<A>& a) { return fq_neg(a); }
template <int A>
BN_INLINE auto F_neg(const Fq2<A>& a) { return fq2_neg(a); }
template <int A>
BN_INLINE auto F_fold(const Fq<A>& a) { return fq_fold(a); }
template <int A>
BN_INLINE auto F_norm(const Fq<A>& a) { return fq_norm(a); }
template <int A>
BN_INLINE auto F_norm(const Fq2<A>& a) { return fq2_norm(a); }
template <int A>
BN_INLINE auto F_fold(const Fq2<A>& a) { return fq2_fold(a); }
template <int A>
BN_INLINE bool F_is_zero(const Fq<A>& a) { return fq_is_zero(a); }
template <int A>
BN_INLINE bool F_is_zero(const Fq2<A>& a) { return fq2_is_zero(a); }
template <int A>
BN_INLINE auto F_inv(const Fq<A>& a) { return fq_inv(a); }
template <int A>
BN_INLINE auto F_inv(const Fq2<A>& a) { return fq2_inv(a); }
template <int B2, int B>
BN_INLINE Fq<B2> F_widen(const Fq<B>& a) { return widen<B2>(a); }
template <int B2, int B>
BN_INLINE Fq2<B2> F_widen(const Fq2<B>& a) { return widen<B2>(a); }
template <int B>
BN_INLINE Fq<B> F_select(bool c, const Fq<B>& a, const Fq<B>& b) { return fq_select(c, a, b); }
template <int B>
BN_INLINE Fq2<B> F_select(bool c, const Fq2<B>& a, const Fq2<B>& b) { return fq2_select(c, a, b); }

// keep a value at storage bound S: widen when it already fits, else fold to 2
template <int S, template <int> class F, int B>
BN_INLINE F<S> narrow(const F<B>& a) {
    static_assert(S >= 2, "storage bound must admit a folded value");
    if constexpr (kv(B) <= S) {
        return F_widen<S>(F_norm(a));
    } else {
        return F_widen<S>(F_fold(a));
    }
}

// ---------------------------------------------------------------- Jacobian points
// storage bound of point coordinates between group operations
constexpr int kPt = 4;
template <template <int> class F>
struct Jac {
    F<kPt> x, y, z;
};
using G1J = Jac<Fq>;
using G2J = Jac<Fq2>;

template <template <int> class F>
BN_INLINE F<1> F_one();
template <>
BN_INLINE Fq<1> F_one<Fq>() { return fq_one(); }
template <>
BN_INLINE Fq2<1> F_one<Fq2>() { return fq2_one(); }
template <template <int> class F>
BN_INLINE F<1> F_zero();
template <>
BN_INLINE Fq<1> F_zero<Fq>() { return fq_zero(); }
template <>
BN_INLINE Fq2<1> F_zero<Fq2>() { return fq2_zero(); }

// zero = (0, 1, 0), mod.rs:230-236
template <template <int> class F>
BN_INLINE Jac<F> jac_zero() {
    return {F_widen<kPt>(F_zero<F>()), F_widen<kPt>(F_one<F>()), F_widen<kPt>(F_zero<F>())};
}
template <template <int> class F>
BN_INLINE bool jac_is_zero(const Jac<F>& p) { return F_is_zero(p.z); }  // mod.rs:246-248

// mod.rs:250-269 (d enters e * (d - x3) normalized, not folded: the product's operand
// fold covers it, 35 VALU fewer per doubling, G2 * Fr -0.4 %, profiles/r5ad_ab_double_dnorm.txt)
template <template <int> class F>
BN_INLINE Jac<F> jac_double(const Jac<F>& s) {
    auto a = F_sqr(s.x);
    auto b = F_sqr(s.y);
    auto c = F_sqr(b);
    auto d0 = F_sub(F_sub(F_sqr(F_add(s.x, b)), a), c);
    auto d = F_add(d0, d0);
    auto e = F_add(F_add(a, a), a);
    auto f = F_sqr(e);
    auto x3 = F_fold(F_sub(f, F_add(d, d)));
    auto c2 = F_add(c, c);
    auto c4 = F_add(c2, c2);
    auto eight_c = F_add(c4, c4);
    auto y1z1 = F_mul(s.y, s.z);
    return {narrow<kPt>(x3), narrow<kPt>(F_sub(F_mul(e, F_sub(F_norm(d), x3)), eight_c)), narrow<kPt>(F_add(y1z1, y1z1))};
}

// mod.rs:294-334, including both zero short-cuts and the doubling branch;
// o_zero = jac_is_zero(o), computed once by a caller that adds the same o often,
// and z2sq / z2cu = o.z^2, o.z^3 (the same residues whether computed here or
// once by such a caller: jac_mul's base is fixed, saving 2 of its 16 products)
template <template <int> class F, class Z2, class Z3>
BN_INLINE Jac<F> jac_add_pre(const Jac<F>& s, const Jac<F>& o, bool o_zero, const Z2& z2_squared,
                             const Z3& z2_cubed) {
    const bool s_zero = jac_is_zero(s);
    auto z1_squared = F_sqr(s.z);
    auto u1 = F_mul(s.x, z2_squared);
    auto u2 = F_mul(o.x, z1_squared);
    auto z1_cubed = F_mul(s.z, z1_squared);
    auto s1 = F_mul(s.y, z2_cubed);
    auto s2 = F_mul(o.y, z1_cubed);
    auto h = F_sub(u2, u1);
    auto s2_minus_s1 = F_sub(s2, s1);
    // u1 == u2 && s1 == s2  <=>  h == 0 && s2 - s1 == 0 (mod p); the second test only
    // when some lane of the wave has h == 0 (rare: wave-uniform guard)
    const bool h_zero = F_is_zero(h);
    bool same = false;
    if (BN_ANY(h_zero)) same = h_zero && F_is_zero(s2_minus_s1);
    auto i = F_sqr(F_add(h, h));
    auto j = F_mul(h, i);
    auto r = F_add(s2_minus_s1, s2_minus_s1);
    auto v = F_mul(u1, i);
    auto s1_j = F_mul(s1, j);
    auto x3 = F_fold(F_sub(F_sub(F_sqr(r), j), F_add(v, v)));
    auto y3 = F_sub(F_mul(r, F_sub(v, x3)), F_add(s1_j, s1_j));
    auto z3 = F_mul(F_sub(F_sub(F_sqr(F_add(s.z, o.z)), z1_squared), z2_squared), h);
    Jac<F> out = {narrow<kPt>(x3), narrow<kPt>(y3), narrow<kPt>(z3)};
    if (BN_ANY(same && !s_zero && !o_zero)) {  // rare: wave-uniform guard
        Jac<F> d = jac_double(s);
        const bool take = same && !s_zero && !o_zero;
        out = {F_select(take, d.x, out.x), F_select(take, d.y, out.y), F_select(take, d.z, out.z)};
    }
    if (BN_ANY(o_zero || s_zero)) {  // the zero shortcuts (mod.rs:298-304); rare in a chain: wave-uniform guard
        out = {F_select(o_zero, s.x, out.x), F_select(o_zero, s.y, out.y), F_select(o_zero, s.z, out.z)};
        out = {F_select(s_zero, o.x, out.x), F_select(s_zero, o.y, out.y), F_select(s_zero, o.z, out.z)};
    }
    return out;
}
template <template <int> class F>
BN_INLINE Jac<F> jac_add(const Jac<F>& s, const Jac<F>& o, bool o_zero) {
    const auto z2_squared = F_sqr(o.z);
    return jac_add_pre(s, o, o_zero, z2_squared, F_mul(o.z, z2_squared));
}

template <template <int> class F>
BN_INLINE Jac<F> jac_add(const Jac<F>& s, const Jac<F>& o) {
    return jac_add(s, o, jac_is_zero(o));
}

// mod.rs:336-350 (zero unchanged, else (x, -y, z)), at the storage bound
template <template <int> class F>
BN_INLINE Jac<F> jac_neg(const Jac<F>& a) {
    const bool z = jac_is_zero(a);
    return {a.x, F_select(z, a.y, narrow<kPt>(F_neg(a.y))), a.z};
}

// The per-lane bit state of one double-and-add chain (mod.rs:272-292): `w` holds
// the scalar shifted so that the next bit to consume is bit 31 of w[7]; `left` =
// bits still to consume after the top set bit; `need_add`: the chain's next step
// is the addition of the current bit.
struct MulBits {
    uint32_t w[8];
    int left;
    bool need_add;
    BN_INLINE void init(const uint32_t k[8]) {
#pragma unroll
        for (int i = 0; i < 8; ++i) w[i] = k[i];
        // top set bit: shift it out (its addition is pending), count the bits below it
        int top = -1;
#pragma unroll
        for (int i = 0; i < 8; ++i)
            if (w[i]) top = 32 * i + 31 - __builtin_clz(w[i]);
        need_add = top >= 0;  // zero + p: the reference's first addition (found_one)
        left = top;           // bits below the top one
        // left-align: shift by 255 - top + 1 so the bit below the top is bit 31 of w[7]
        const int sh = top >= 0 ? 256 - top : 0;  // 1..256
        const int ws = sh >> 5, bs = sh & 31;
        uint32_t t[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            uint32_t v = 0;
#pragma unroll
            for (int j = 0; j < 8; ++j) {  // t[i] = (w << sh) word i, from words i - ws and i - ws - 1
                const uint32_t hi = (i - j == ws) ? w[j] : 0u;
                const uint32_t lo = (i - j == ws + 1) ? w[j] : 0u;
                v |= (bs ? (hi << bs) | (lo >> (32 - bs)) : hi);
            }
            t[i] = v;
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) w[i] = t[i];
    }
    BN_INLINE bool wants_dbl() const { return !need_add && left > 0; }
    BN_INLINE bool done() const { return !need_add && left <= 0; }
    // the chain ran its pending addition
    BN_INLINE void added(bool ran) { need_add = ran ? false : need_add; }
    // the chain ran a doubling: it consumed the next bit, whose addition is pending when set
    BN_INLINE void doubled(bool ran) {
        const bool b = (w[7] >> 31) != 0;
        need_add = ran ? b : need_add;
        left -= ran ? 1 : 0;
#pragma unroll
        for (int i = 7; i > 0; --i) w[i] = ran ? (w[i] << 1) | (w[i - 1] >> 31) : w[i];
        w[0] = ran ? w[0] << 1 : w[0];
    }
};

// MSB-first double-and-add over the bits of the canonical scalar
// (mod.rs:272-292): for every bit below the top set one, a doubling, then an
// addition of p when the bit is set.  Every lane follows exactly the
// reference's chain, so the Jacobian output is bit-identical.
//
// The chains differ per lane, so a wave schedules them: each
// iteration runs ONE kind of step -- the addition for the lanes whose next step
// is an addition, or the doubling for those whose next step is a doubling --
// chosen by a ballot: the addition once at least 3/5 of the unfinished lanes
// wait for it (or no lane waits for a doubling).  A lane's own steps keep their
// order, so its result is unchanged; lanes simply drift apart within the wave.
// Lockstep execution (every bit runs the doubling and the masked addition on
// every lane, round 2) executes 253 x (7 + 16) Fq-mul per lane for
// random scalars; the scheduled chain ~8 % less (a simulation of 64 random
// 254-bit scalars: 5,302 against 5,819 Fq-mul-weighted steps).
// Diagnostic build (-DBN_MUL_STATS=1, tools/mul_stats.py): per iteration of the
// ballot loop, the first lane of the wave adds to g_mul_stats[0/1] the additions /
// doublings run, [2/3] the lanes they served and [4] the unfinished lanes -- the
// measured lane occupancy of the schedule.  The product build has none of it.
#if defined(BN_MUL_STATS) && BN_MUL_STATS && defined(__HIPCC__)
__device__ unsigned long long g_mul_stats[5];
#define BN_MUL_STATS_ON 1
#else
#define BN_MUL_STATS_ON 0
#endif
#if defined(BN_MUL_STATS) && BN_MUL_STATS && defined(__HIP_DEVICE_COMPILE__)
#define BN_MUL_STAT(is_add, served, live)                                                  \
    do {                                                                                   \
        if (__lane_id() == (unsigned)__ffsll(__ballot(1)) - 1) {                           \
            atomicAdd(&g_mul_stats[(is_add) ? 0 : 1], 1ull);                               \
            atomicAdd(&g_mul_stats[(is_add) ? 2 : 3], (unsigned long long)(served));       \
            atomicAdd(&g_mul_stats[4], (unsigned long long)(live));                        \
        }                                                                                  \
    } while (0)
#else
#define BN_MUL_STAT(is_add, served, live) ((void)0)
#endif
#if defined(__HIP_DEVICE_COMPILE__)
#define BN_BALLOT_COUNT(p) ((uint32_t)__popcll(__ballot((int)(p))))
#else
#define BN_BALLOT_COUNT(p) ((uint32_t)((p) ? 1 : 0))
#endif
// `step(t)` runs at the start of step t (the kernels' issue balance, kernels.h)
struct NoBitStep {
    BN_INLINE void operator()(int) const {}
};
template <template <int> class F, typename Step = NoBitStep>
BN_INLINE Jac<F> jac_mul(const Jac<F>& p, const uint32_t k[8], Step&& step = Step{}) {
    Jac<F> res = jac_zero<F>();
    const bool p_zero = jac_is_zero(p);
    // the base's z^2 and z^3, the same at every addition of the chain
    const auto pz2 = narrow<kPt>(F_sqr(p.z));
    const auto pz3 = narrow<kPt>(F_mul(p.z, pz2));
    MulBits mb;
    mb.init(k);
    int it = 0;
#pragma unroll 1
    for (;;) {
        const bool need_add = mb.need_add, need_dbl = mb.wants_dbl();
        const uint32_t n_add = BN_BALLOT_COUNT(need_add), n_dbl = BN_BALLOT_COUNT(need_dbl);
        if (n_add + n_dbl == 0) break;  // wave-uniform
        step(it++);
        const bool do_add = n_dbl == 0 || 5 * n_add >= 3 * (n_add + n_dbl);
        BN_MUL_STAT(do_add, do_add ? n_add : n_dbl, n_add + n_dbl);
        if (do_add) {
            Jac<F> a = jac_add_pre(res, p, p_zero, pz2, pz3);
            res = {F_select(need_add, a.x, res.x), F_select(need_add, a.y, res.y), F_select(need_add, a.z, res.z)};
            mb.added(need_add);
        } else {
            Jac<F> d = jac_double(res);
            res = {F_select(need_dbl, d.x, res.x), F_select(need_dbl, d.y, res.y), F_select(need_dbl, d.z, res.z)};
            mb.doubled(need_dbl);
        }
    }
    return res;
}

// Two chains per lane (p0*k0 and p1*k1): each iteration still runs ONE kind of step
// for the wave, but a lane serves it from whichever of its chains is ready for it
// (the one with more bits left when both are) -- the ballot sees twice the
// candidates, so fewer lanes idle in each step (measured on config 3's launch with
// the counter build: 1.289x the chains' own Fq-mul weight, against 1.407x for one
// chain per lane; the addition here weighs 16, its base's z^2, z^3 recomputed).
// Each chain's own steps keep their order: both outputs stay bit-exact.
// `base(c)` returns the base of chain c (0/1); the kernel keeps the two bases in
// LDS, so the loop holds two accumulators in registers, not four points.
// `bit(c, i)` returns bit i of chain c's canonical scalar and `top0`/`top1` are the
// scalars' top set bits (-1 for zero): the kernel keeps the scalars in LDS too, so
// a doubling reads the one bit it consumes instead of shifting 256-bit registers.
struct ChainPos {
    int left;       // bits below the current one still to consume
    bool need_add;  // the next step is the addition of the current bit
    BN_INLINE void init(int top) {
        need_add = top >= 0;  // zero + p: the reference's first addition (found_one)
        left = top;
    }
    BN_INLINE bool wants_dbl() const { return !need_add && left > 0; }
};
// the top set bit of a 256-bit scalar, -1 for zero
BN_INLINE int scalar_top_bit(const uint32_t k[8]) {
    int top = -1;
#pragma unroll
    for (int i = 0; i < 8; ++i)
        if (k[i]) top = 32 * i + 31 - __builtin_clz(k[i]);
    return top;
}
template <template <int> class F, typename Base, typename Bit, typename Step = NoBitStep>
BN_INLINE void jac_mul2(Base&& base, Bit&& bit, bool z0, bool z1, int top0, int top1, Jac<F>& out0, Jac<F>& out1,
                        Step&& step = Step{}) {
    Jac<F> r0 = jac_zero<F>(), r1 = jac_zero<F>();
    ChainPos m0, m1;
    m0.init(top0);
    m1.init(top1);
    int it = 0;
#pragma unroll 1
    for (;;) {
        const bool a0 = m0.need_add, a1 = m1.need_add, d0 = m0.wants_dbl(), d1 = m1.wants_dbl();
        const bool need_add = a0 || a1, need_dbl = d0 || d1;
        const uint32_t n_add = BN_BALLOT_COUNT(need_add), n_dbl = BN_BALLOT_COUNT(need_dbl);
        if (n_add + n_dbl == 0) break;  // wave-uniform
        step(it++);
        // half the lanes, not 3/5: with two candidates per lane the simulation's best
        // (1.29x against 1.30x at 3/5)
        const bool do_add = n_dbl == 0 || n_add >= n_dbl;
        const uint32_t n_live = BN_MUL_STATS_ON ? BN_BALLOT_COUNT(need_add || need_dbl) : 0u;
        BN_MUL_STAT(do_add, do_add ? n_add : n_dbl, n_live);
        (void)n_live;
        // the chain that runs: chain 0 when it can, unless chain 1 can too and has more bits left
        const bool c0 = do_add ? a0 : d0, c1 = do_add ? a1 : d1;
        const bool use0 = c0 && (!c1 || m0.left >= m1.left);
        const bool w0 = (c0 || c1) && use0, w1 = (c0 || c1) && !use0;
        const Jac<F> r = {F_select(use0, r0.x, r1.x), F_select(use0, r0.y, r1.y), F_select(use0, r0.z, r1.z)};
        Jac<F> t;
        if (do_add)
            t = jac_add(r, base(use0 ? 0 : 1), use0 ? z0 : z1);
        else
            t = jac_double(r);
        r0 = {F_select(w0, t.x, r0.x), F_select(w0, t.y, r0.y), F_select(w0, t.z, r0.z)};
        r1 = {F_select(w1, t.x, r1.x), F_select(w1, t.y, r1.y), F_select(w1, t.z, r1.z)};
        if (do_add) {
            m0.need_add = w0 ? false : m0.need_add;
            m1.need_add = w1 ? false : m1.need_add;
        } else {
            // the doubling consumed bit left - 1 of the chain that ran: its addition is
            // pending when the bit is set
            const int pos = (use0 ? m0.left : m1.left) - 1;
            const bool b = bit(use0 ? 0 : 1, pos < 0 ? 0 : pos);
            m0.need_add = w0 ? b : m0.need_add;
            m1.need_add = w1 ? b : m1.need_add;
            m0.left -= w0 ? 1 : 0;
            m1.left -= w1 ? 1 : 0;
        }
    }
    out0 = r0;
    out1 = r1;
}

// ---------------------------------------------------------------- curve constants
BN_INLINE Fq2<1> xi_const() { return fq2_const(Limbs9{BN_XI_C0}, Limbs9{BN_XI_C1}); }
BN_INLINE Fq2<1> g2_coeff_b() { return fq2_const(Limbs9{BN_G2B_C0}, Limbs9{BN_G2B_C1}); }  // mod.rs:452-467
BN_INLINE Fq<1> two_inv() { return fq_from_limbs<1>(Limbs9{BN_TWO_INV}); }                  // mod.rs:521-528
BN_INLINE Fq2<1> twist_mul_by_q_x() { return fq2_const(Limbs9{BN_TWIST_Q_X_C0}, Limbs9{BN_TWIST_Q_X_C1}); }
BN_INLINE Fq2<1> twist_mul_by_q_y() { return fq2_const(Limbs9{BN_TWIST_Q_Y_C0}, Limbs9{BN_TWIST_Q_Y_C1}); }

// ---------------------------------------------------------------- flipped Miller loop steps
template <int B>
struct G2Aff {
    Fq2<B> x, y;
};
constexpr int kLine = 4;  // storage bound of line coefficients
struct Ell {
    Fq2<kLine> ell_0, ell_vw, ell_vv;
};
// homogeneous-projective R on the twist between steps
struct G2Proj {
    Fq2<kPt> x, y, z;
};

// mod.rs:754-776 -- the twist() * i product is xi * i (ring identity)
BN_INLINE Ell doubling_step(G2Proj& s) {
    // x * two_inv is the halving x / 2 mod p: the same residue, no product
    auto a = fq2_half(fq2_mul(s.x, s.y));
    auto b = fq2_sqr(s.y);
    auto c = fq2_sqr(s.z);
    auto d = fq2_add(fq2_add(c, c), c);
    auto e = fq2_mul(g2_coeff_b(), d);
    auto f = fq2_add(fq2_add(e, e), e);
    auto g = fq2_half(fq2_add(b, f));
    auto h = fq2_sub(fq2_sqr(fq2_add(s.y, s.z)), fq2_add(b, c));
    auto i = fq2_sub(e, b);
    auto j = fq2_sqr(s.x);
    auto e_sq = fq2_sqr(e);
    s.x = narrow<kPt>(fq2_mul(a, fq2_sub(b, f)));
    s.y = narrow<kPt>(fq2_sub(fq2_sqr(g), fq2_add(fq2_add(e_sq, e_sq), e_sq)));
    s.z = narrow<kPt>(fq2_mul(b, h));
    return {narrow<kLine>(fq2_mul_xi(i)), narrow<kLine>(fq2_neg(h)), narrow<kLine>(fq2_add(fq2_add(j, j), j))};
}
// mod.rs:731-752
template <int BB>
BN_INLINE Ell mixed_addition_step(G2Proj& s, const G2Aff<BB>& base) {
    auto d = fq2_sub(s.x, fq2_mul(s.z, base.x));
    auto e = fq2_sub(s.y, fq2_mul(s.z, base.y));
    auto f = fq2_sqr(d);
    auto g = fq2_sqr(e);
    auto h = fq2_mul(d, f);
    auto i = fq2_mul(s.x, f);
    auto j = fq2_sub(fq2_add(fq2_mul(s.z, g), h), fq2_add(i, i));
    auto nx = fq2_mul(d, j);
    auto ny = fq2_sub(fq2_mul(e, fq2_sub(i, j)), fq2_mul(h, s.y));
    auto nz = fq2_mul(s.z, h);
    s.x = narrow<kPt>(nx);
    s.y = narrow<kPt>(ny);
    s.z = narrow<kPt>(nz);
    auto l0 = fq2_mul_xi(fq2_sub(fq2_mul(e, base.x), fq2_mul(d, base.y)));
    return {narrow<kLine>(l0), narrow<kLine>(d), narrow<kLine>(fq2_neg(e))};
}
// mod.rs:694-699
template <int B>
BN_INLINE G2Aff<kPt> mul_by_q(const G2Aff<B>& q) {
    return {narrow<kPt>(fq2_mul(twist_mul_by_q_x(), fq2_conj(q.x))), narrow<kPt>(fq2_mul(twist_mul_by_q_y(), fq2_conj(q.y)))};
}

// ATE_LOOP_COUNT_NAF, mod.rs:14 (3 == -1): 64 digits, 21 nonzero -> 87 lines.
// Bit i of kNafNonzero / kNafMinus is digit i of the reference array.
#define BN_NAF_DIGITS 64
#define BN_NUM_COEFFS 87
constexpr uint64_t naf_mask(int want) {
    const uint8_t naf[64] = {1, 0, 1, 0, 0, 0, 3, 0, 3, 0, 0, 0, 3, 0, 1, 0, 3, 0, 0, 3, 0, 0, 0, 0, 0, 1, 0, 0, 3, 0, 1, 0,
                             0, 3, 0, 0, 0, 0, 3, 0, 1, 0, 0, 0, 3, 0, 3, 0, 0, 1, 0, 0, 0, 3, 0, 0, 3, 0, 1, 0, 1, 0, 0, 0};
    uint64_t m = 0;
    for (int i = 0; i < 64; ++i)
        if ((want == 0 && naf[i] != 0) || (want == 3 && naf[i] == 3)) m |= 1ull << i;
    return m;
}
constexpr uint64_t kNafNonzero = naf_mask(0);
constexpr uint64_t kNafMinus = naf_mask(3);

}  // namespace bn
