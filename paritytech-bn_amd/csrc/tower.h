// tower.h -- Fq2 / Fq6 / Fq12 tower of BN254 on CDNA4, one lane per element.
//
// Replaces src/fields/fq2.rs, fq6.rs, fq12.rs.  Each function returns the same
// residue (mod p, per coefficient) as the reference function it cites; where
// the formula differs it differs only by a ring identity (x * (p-1) is a
// negation, x * xi with xi = 9+u is a digit-wise add chain, binary GCD instead
// of binary-Euclid inversion), never in the value.  Formulas that are NOT ring
// identities -- Granger-Scott cyclotomic squaring, the sparse line product --
// follow the reference's own expressions.
//
// Bounds: FqN<B> means every coefficient is an Fq<B> (value <= B*p).  Return
// types are deduced, so the compiler proves every intermediate stays below
// 2^261; fq*_fold() brings a value back to bound 2 where a formula would
// otherwise overflow (the static_asserts in fq.h say where).
#pragma once
#include "fq.h"


namespace bn {

constexpr int cmax(int a, int b) { return a > b ? a : b; }

// ---------------------------------------------------------------- binary-GCD inversion
// Pornin's optimized binary GCD ("Optimized Binary GCD for Modular Inversion",
// 2020, Algorithm 2) with 29-bit steps to match the digit size: each outer
// round runs 29 binary-GCD steps on 60-bit approximations of (a, b) -- their
// low 29 bits exact, the top 31 bits of max(len(a), len(b), 60) -- collecting
// the update factors (f0, g0, f1, g1), |f| + |g| <= 2^29, then applies them to
// the full (a, b) (exact division by 2^29, sign fixes) and to (u, v) with a
// Montgomery division by 2^29 (add k*p, drop the low digit), which keeps
// a == y*u and b == y*v (mod p).  ceil((2*254 - 1)/29) = 18 rounds reach b = 1,
// so v = y^-1; one spare round (a no-op once a = 0).  No data-dependent branch:
// every lane runs the same instructions.  About a third of the instructions of
// the Fermat chain (253 squarings).  y^-1 is unique, so the value equals the
// reference's binary extended Euclid (arith.rs:324-370) bit for bit.
constexpr int kInvRounds = 19;  // ceil((2 * 254 - 1) / 29) = 18, plus one spare
constexpr Limbs9 kR3 = {{0x0e2312b2u, 0x16c05ca2u, 0x0bc84389u, 0x1cdf310bu, 0x11adafddu, 0x032e568eu, 0x1d6ae48cu,
                         0x10d4cd1fu, 0x0026c2d2u}};  // 2^783 mod p: REDC(v * R^3) = v * R^2
// (x*f0 + y*g0) / 2^29 for the exact (a, b) update: the low digit cancels; the
// result comes back with the sign removed (m: all ones when it was negative)
BN_INLINE uint32_t bgcd_lin_exact(const uint32_t (&x)[9], const uint32_t (&y)[9], int32_t f, int32_t g,
                                  uint32_t (&r)[9]) {
    int64_t c = 0;
#pragma unroll
    for (int i = 0; i < 9; ++i) {
        const int64_t t = (int64_t)(int32_t)x[i] * f + (int64_t)(int32_t)y[i] * g + c;
        if (i) r[i - 1] = (uint32_t)t & M29;
        c = t >> 29;
    }
    r[8] = (uint32_t)c;  // signed top digit
    const uint32_t m = (uint32_t)((int32_t)r[8] >> 31);
    // conditional negation, carried: -X = sum (-d_i) 2^(29 i)
    int64_t cn = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int64_t t = (int64_t)(int32_t)((r[i] ^ m) - m) + cn;
        r[i] = (uint32_t)t & M29;
        cn = t >> 29;
    }
    r[8] = (uint32_t)((int64_t)(int32_t)((r[8] ^ m) - m) + cn);
    return m;
}
// (x*f + y*g) / 2^29 mod p for the (u, v) update: + k*p clears the low digit,
// + 3p (|x f + y g| / 2^29 < 2p for x, y < 2p, and k*p / 2^29 < p) keeps every
// digit non-negative; the result is < 6p, normalized
BN_INLINE Fq<6> bgcd_lin_mont(const Fq<2>& x, const Fq<2>& y, int32_t f, int32_t g) {
    constexpr Limbs9 P3 = kp_plain(3);
    int64_t t[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) t[i] = (int64_t)(int32_t)x.v[i] * f + (int64_t)(int32_t)y.v[i] * g;
    const uint32_t k = ((uint32_t)t[0] * BN_PINV29) & M29;
#pragma unroll
    for (int i = 0; i < 9; ++i) t[i] += (int64_t)((uint64_t)k * kP29.v[i]);
    Fq<6> r;
    int64_t c = t[0] >> 29;
#pragma unroll
    for (int i = 1; i < 9; ++i) {
        const int64_t s = t[i] + c + P3.v[i - 1];
        r.v[i - 1] = (uint32_t)s & M29;
        c = s >> 29;
    }
    r.v[8] = (uint32_t)(c + P3.v[8]);
    return r;
}
template <int B>
BN_INLINE Fq<2> fq_inv_bgcd(const Fq<B>& x) {
    const Fq<1> y = fq_canonical(x);  // the plain integer x*R mod p
    uint32_t a[9], b[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) {
        a[i] = y.v[i];
        b[i] = kP29.v[i];
    }
    Fq<2> u = fq_from_limbs<2>(Limbs9{{1, 0, 0, 0, 0, 0, 0, 0, 0}}), v = widen<2>(fq_zero());
#pragma unroll 1
    for (int round = 0; round < kInvRounds; ++round) {
        // n = max(len(a), len(b), 60): the bit length of a | b
        uint32_t n = 60;
#pragma unroll
        for (int d = 0; d < 9; ++d) {
            const uint32_t o = a[d] | b[d];
            const uint32_t len = 29u * d + 32u - (uint32_t)__builtin_clz(o | 1u);
            n = (o != 0 && len > n) ? len : n;
        }
        const uint32_t s = n - 31, dd = s / 29, off = s - 29 * dd;
        uint32_t a0 = 0, a1 = 0, a2 = 0, b0 = 0, b1 = 0, b2 = 0;
#pragma unroll
        for (int d = 1; d < 9; ++d) {
            const bool h = dd == (uint32_t)d;
            a0 = h ? a[d] : a0;
            b0 = h ? b[d] : b0;
            a1 = h ? (d + 1 < 9 ? a[d + 1 < 9 ? d + 1 : 8] : 0u) : a1;
            b1 = h ? (d + 1 < 9 ? b[d + 1 < 9 ? d + 1 : 8] : 0u) : b1;
            a2 = h ? (d + 2 < 9 ? a[d + 2 < 9 ? d + 2 : 8] : 0u) : a2;
            b2 = h ? (d + 2 < 9 ? b[d + 2 < 9 ? d + 2 : 8] : 0u) : b2;
        }
        const uint64_t wa = (uint64_t)a0 | ((uint64_t)a1 << 29) | ((uint64_t)a2 << 58);
        const uint64_t wb = (uint64_t)b0 | ((uint64_t)b1 << 29) | ((uint64_t)b2 << 58);
        uint64_t ab = (uint64_t)a[0] | (((wa >> off) & 0x7fffffffu) << 29);
        uint64_t bb = (uint64_t)b[0] | (((wb >> off) & 0x7fffffffu) << 29);
        // update factors packed as f + g*2^32 in one 64-bit word (the steps are
        // linear, so the pack stays exact; |f|, |g| <= 2^29)
        uint64_t pa = 1, pb = (uint64_t)1 << 32;  // (f0, g0) = (1, 0), (f1, g1) = (0, 1)
#pragma unroll
        for (int j = 0; j < 29; ++j) {
            const bool odd = (ab & 1u) != 0;
            const bool sw = odd & (ab < bb);
            const uint64_t ta = sw ? bb : ab, tb = sw ? ab : bb, tp = sw ? pb : pa, tq = sw ? pa : pb;
            ab = (ta - (odd ? tb : 0)) >> 1;
            pa = tp - (odd ? tq : 0);
            bb = tb;
            pb = tq << 1;
        }
        int32_t f0 = (int32_t)(uint32_t)pa, f1 = (int32_t)(uint32_t)pb;
        int32_t g0 = (int32_t)((int64_t)(pa - (uint64_t)(int64_t)f0) >> 32);
        int32_t g1 = (int32_t)((int64_t)(pb - (uint64_t)(int64_t)f1) >> 32);
        uint32_t na[9], nb[9];
        const uint32_t ma = bgcd_lin_exact(a, b, f0, g0, na);
        const uint32_t mb = bgcd_lin_exact(a, b, f1, g1, nb);
        f0 = (int32_t)(((uint32_t)f0 ^ ma) - ma);
        g0 = (int32_t)(((uint32_t)g0 ^ ma) - ma);
        f1 = (int32_t)(((uint32_t)f1 ^ mb) - mb);
        g1 = (int32_t)(((uint32_t)g1 ^ mb) - mb);
#pragma unroll
        for (int i = 0; i < 9; ++i) {
            a[i] = na[i];
            b[i] = nb[i];
        }
        const Fq<2> nu = fq_fold(bgcd_lin_mont(u, v, f0, g0));
        v = fq_fold(bgcd_lin_mont(u, v, f1, g1));
        u = nu;
    }
#if defined(BN_HOST_CHECKS) && !defined(__HIP_DEVICE_COMPILE__)
    // y != 0 must end with b == gcd == 1 (y == 0 keeps a = 0, b = p, v = 0 and
    // returns 0, as the Fermat chain does)
    uint32_t not_one = b[0] ^ 1u, nz = 0;
    for (int i = 1; i < 9; ++i) not_one |= b[i];
    for (int i = 0; i < 9; ++i) nz |= y.v[i];
    if (nz && not_one) {
        fprintf(stderr, "fq_inv_bgcd: %d rounds did not reach b == 1\n", kInvRounds);
        abort();
    }
#endif
    return fq_mul(v, fq_from_limbs<1>(kR3));
}
// ---------------------------------------------------------------- the same inversion on a quad of lanes
// Where the four lanes 4q .. 4q+3 hold the same x (the eight lanes of a pair in
// k_prepare_wide and the latency kernel's producer, the lane pairs of a wide group)
// they split each round's four linear updates instead of each running all four:
// lane 4q + r keeps a (r = 0), b (1), u (2) or v (3) and updates it from its own
// value and its partner's (quad_perm [1,0,3,2]: a <-> b, u <-> v); the 29 steps on
// the approximations run on every lane alike, the approximations taken from lanes
// 0 and 1 of the quad.  One code path for the four updates: (x c + y d + K p) / 2^29
// with K = 0 on the exact lanes and K = k + 3 * 2^29 on the Montgomery lanes (k
// clears the low digit; 3 * 2^29 p adds the 3p that keeps the digits non-negative,
// as bgcd_lin_mont).  The exact update's sign fix (a negative result is negated,
// and fq_inv_bgcd negates f, g for the (u, v) update with it) reaches the
// Montgomery lanes as 6p - r, a negation mod p of their result: the same residue.
// About 0.7x fq_inv_bgcd's instructions per lane; the inverse is unique, so the
// value is fq_inv_bgcd's (host builds run fq_inv_bgcd itself).
template <int CTRL>
BN_INLINE uint32_t quad_perm(uint32_t v) {
#if defined(__HIP_DEVICE_COMPILE__)
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, false);
#else
    return v;
#endif
}
template <int B>
BN_INLINE Fq<2> fq_inv_quad(const Fq<B>& x) {
#if !defined(__HIP_DEVICE_COMPILE__)
    return fq_inv_bgcd(x);
#else
    const uint32_t role = __builtin_amdgcn_workitem_id_x() & 3u;  // 0 a, 1 b, 2 u, 3 v
    const bool odd = (role & 1u) != 0;
    const uint32_t mont = role >= 2 ? ~0u : 0u;
    constexpr Limbs9 P6 = kp_plain(6);
    const Fq<1> y = fq_canonical(x);
    uint32_t own[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) own[i] = role == 0 ? y.v[i] : role == 1 ? kP29.v[i] : (role == 2 && i == 0) ? 1u : 0u;
#pragma unroll 1
    for (int round = 0; round < kInvRounds; ++round) {
        // n = max(len(a), len(b), 60) on lanes 0 and 1 (the other lanes' n is unused)
        uint32_t len = 0;
#pragma unroll
        for (int d = 0; d < 9; ++d) len = own[d] != 0 ? 29u * d + 32u - (uint32_t)__builtin_clz(own[d] | 1u) : len;
        // (the partner's length read once, outside any select: a DPP read placed in a
        // divergent arm would see the masked-off lanes' stale registers)
        const uint32_t len_p = quad_perm<0xB1>(len);
        len = len > len_p ? len : len_p;
        const uint32_t n = len > 60u ? len : 60u;
        const uint32_t s = n - 31, dd = s / 29, off = s - 29 * dd;
        uint32_t w0 = 0, w1 = 0, w2 = 0;
#pragma unroll
        for (int d = 1; d < 9; ++d) {
            const bool h = dd == (uint32_t)d;
            w0 = h ? own[d] : w0;
            w1 = h ? (d + 1 < 9 ? own[d + 1 < 9 ? d + 1 : 8] : 0u) : w1;
            w2 = h ? (d + 2 < 9 ? own[d + 2 < 9 ? d + 2 : 8] : 0u) : w2;
        }
        const uint64_t wv = (uint64_t)w0 | ((uint64_t)w1 << 29) | ((uint64_t)w2 << 58);
        const uint64_t ap = (uint64_t)own[0] | (((wv >> off) & 0x7fffffffu) << 29);
        const uint32_t ap_lo = (uint32_t)ap, ap_hi = (uint32_t)(ap >> 32);
        uint64_t ab = (uint64_t)quad_perm<0x00>(ap_lo) | ((uint64_t)quad_perm<0x00>(ap_hi) << 32);  // lane 0's a
        uint64_t bb = (uint64_t)quad_perm<0x55>(ap_lo) | ((uint64_t)quad_perm<0x55>(ap_hi) << 32);  // lane 1's b
        uint64_t pa = 1, pb = (uint64_t)1 << 32;
#pragma unroll
        for (int j = 0; j < 29; ++j) {
            const bool odd_a = (ab & 1u) != 0;
            const bool sw = odd_a & (ab < bb);
            const uint64_t ta = sw ? bb : ab, tb = sw ? ab : bb, tp = sw ? pb : pa, tq = sw ? pa : pb;
            ab = (ta - (odd_a ? tb : 0)) >> 1;
            pa = tp - (odd_a ? tq : 0);
            bb = tb;
            pb = tq << 1;
        }
        const int32_t f0 = (int32_t)(uint32_t)pa, f1 = (int32_t)(uint32_t)pb;
        const int32_t g0 = (int32_t)((int64_t)(pa - (uint64_t)(int64_t)f0) >> 32);
        const int32_t g1 = (int32_t)((int64_t)(pb - (uint64_t)(int64_t)f1) >> 32);
        // a' = a f0 + b g0, b' = a f1 + b g1 (u', v' alike): own * c + partner * e
        const int32_t c = odd ? g1 : f0, e = odd ? f1 : g0;
        int64_t t[9];
#pragma unroll
        for (int i = 0; i < 9; ++i)
            t[i] = (int64_t)(int32_t)own[i] * c + (int64_t)(int32_t)quad_perm<0xB1>(own[i]) * e;
        const uint32_t K = ((((uint32_t)t[0] * BN_PINV29) & M29) + (3u << 29)) & mont;
#pragma unroll
        for (int i = 0; i < 9; ++i) t[i] += (int64_t)((uint64_t)K * kP29.v[i]);
        uint32_t r[9];
        int64_t cr = t[0] >> 29;
#pragma unroll
        for (int i = 1; i < 9; ++i) {
            const int64_t sm = t[i] + cr;
            r[i - 1] = (uint32_t)sm & M29;
            cr = sm >> 29;
        }
        r[8] = (uint32_t)cr;  // signed top digit on the exact lanes
        // the exact lanes' sign (lanes 0, 1), also on the Montgomery lanes (quad_perm [0,1,0,1])
        const uint32_t m = quad_perm<0x44>((uint32_t)((int32_t)r[8] >> 31));
        Fq<6> z;
        int64_t cn = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int64_t v = (int64_t)(int32_t)((r[i] ^ m) - m) + (int64_t)(P6.v[i] & m & mont) + cn;
            z.v[i] = (uint32_t)v & M29;
            cn = v >> 29;
        }
        z.v[8] = (uint32_t)((int64_t)(int32_t)((r[8] ^ m) - m) + (int64_t)(P6.v[8] & m & mont) + cn);
        // the Montgomery lanes' value (< 6p) back below 2p; a, b <= p stay as they are (q = 0)
        const Fq<2> zf = fq_fold(z);
#pragma unroll
        for (int i = 0; i < 9; ++i) own[i] = zf.v[i];
    }
    Fq<2> v;  // lane 3's v
#pragma unroll
    for (int i = 0; i < 9; ++i) v.v[i] = quad_perm<0xFF>(own[i]);
    return fq_mul(v, fq_from_limbs<1>(kR3));
#endif
}
// the inverse is unique, so this equals the reference's binary extended Euclid
// (arith.rs:324-370 + fp.rs:108-117) bit for bit; Quad: the four lanes of every
// quad hold the same a (fq_inv_quad)
template <bool Quad = false, int B>
BN_INLINE Fq<2> fq_inv(const Fq<B>& a) {
    if constexpr (Quad) return fq_inv_quad(a); else return fq_inv_bgcd(a);
}
// x unchanged when its bound is <= L, else folded to 2 (decided at compile time)
template <int L, int B>
BN_INLINE auto pre(const Fq<B>& a) {
    if constexpr (kv(B) <= L) return a; else return fq_fold(a);
}

// Fq2: one lane per element (below), or with BN_SPLIT two lanes per element,
// one coordinate each (fq2_split.h)
#ifndef BN_SPLIT
#define BN_SPLIT 0
#endif
#if BN_SPLIT
#include "fq2_split.h"
#else

template <int B>
struct Fq2 {
    Fq<B> c0, c1;
};

// ================================================================ Fq2 = Fq[u]/(u^2+1)
template <int A, int B>
BN_INLINE Fq2<kjoin(A, B)> mk2(const Fq<A>& x, const Fq<B>& y) {
    return {widen<kjoin(A, B)>(x), widen<kjoin(A, B)>(y)};
}
template <int B2, int B>
BN_INLINE Fq2<B2> widen(const Fq2<B>& a) { return {widen<B2>(a.c0), widen<B2>(a.c1)}; }

BN_INLINE Fq2<1> fq2_zero() { return {fq_zero(), fq_zero()}; }
BN_INLINE Fq2<1> fq2_one() { return {fq_one(), fq_zero()}; }
template <int B>
BN_INLINE Fq2<B> fq2_select(bool c, const Fq2<B>& a, const Fq2<B>& b) {
    return {fq_select(c, a.c0, b.c0), fq_select(c, a.c1, b.c1)};
}
template <int A, int B>
BN_INLINE auto fq2_add(const Fq2<A>& a, const Fq2<B>& b) { return mk2(fq_add(a.c0, b.c0), fq_add(a.c1, b.c1)); }
template <int A, int B>
BN_INLINE auto fq2_sub(const Fq2<A>& a, const Fq2<B>& b) { return mk2(fq_sub(a.c0, b.c0), fq_sub(a.c1, b.c1)); }
template <int B>
BN_INLINE auto fq2_neg(const Fq2<B>& a) { return mk2(fq_neg(a.c0), fq_neg(a.c1)); }
template <int B>
BN_INLINE auto fq2_dbl(const Fq2<B>& a) { return fq2_add(a, a); }
template <int B>
BN_INLINE Fq2<2> fq2_fold(const Fq2<B>& a) {
#if BN_FOLD_LDS && defined(__HIP_DEVICE_COMPILE__)
    if constexpr (kl(B) <= 6) {
        const FoldEnt e0 = fold_fetch(a.c0), e1 = fold_fetch(a.c1);
        return {fold_apply(a.c0, e0), fold_apply(a.c1, e1)};
    }
#endif
    return {fq_fold(a.c0), fq_fold(a.c1)};
}
template <int B>
BN_INLINE bool fq2_is_zero(const Fq2<B>& a) {
    const bool z0 = fq_is_zero(a.c0), z1 = fq_is_zero(a.c1);
    return z0 && z1;
}
template <int L, int B>
BN_INLINE auto pre(const Fq2<B>& a) {
    if constexpr (kv(B) <= L) return a; else return fq2_fold(a);
}
template <int A, int B>
BN_INLINE bool fq2_eq(const Fq2<A>& a, const Fq2<B>& b) {
    const bool e0 = fq_eq(a.c0, b.c0), e1 = fq_eq(a.c1, b.c1);
    return e0 && e1;
}

template <int B>
BN_INLINE Fq2<kv(B)> fq2_norm(const Fq2<B>& a) { return {fq_norm(a.c0), fq_norm(a.c1)}; }
// the fences serialize independent Fq2 products in program order (fewer live
// registers than letting the compiler interleave them)
template <int B>
BN_INLINE void fq2_fence(Fq2<B>& a) {
    fq_fence(a.c0);
    fq_fence(a.c1);
}

template <int B>
BN_INLINE auto fq2_half(const Fq2<B>& a) { return mk2(fq_half(a.c0), fq_half(a.c1)); }
// fq2.rs:48-53
template <int A, int B>
BN_INLINE auto fq2_scale(const Fq2<A>& a, const Fq<B>& s) { return mk2(fq_mul(a.c0, s), fq_mul(a.c1, s)); }

// Fq2 product with one Montgomery reduction per output coordinate (lazy
// reduction): per column k of the schoolbook products P = a0*b0, Q = a1*b1 and
// T = (a0+a1)*(b0+b1) are summed unreduced, and the two coordinates
//   c0 = REDC(P - Q)          (signed 64-bit columns)
//   c1 = REDC(T - P - Q)      (= a0*b1 + a1*b0 >= 0, unsigned columns)
// are reduced in the same column loop: 3*81 + 2*81 multiply-adds instead of
// 3*162.  Column bounds: |P - Q| + m*p < 27*2^58 < 2^63 and the c1 column
// < 45*2^58 < 2^64 when La*Lb <= 2 (T may wrap mod 2^64 mid-sum; the final
// column value is exact).  c0 may come out negative (> -A*B*p^2/R): a multiple
// of p is added back.
// K0 with K0*p > A*B*p^2/R by at least p/2 (so the top digit of c0 + K0*p is >= 0)
constexpr int fq2_neg_margin(int A, int B) { return 2 + (int)(((long long)A * B * 5908) / 1000000); }
template <int A, int B>
BN_INLINE auto fq2_mul_lazy(const Fq2<A>& a, const Fq2<B>& b) {
    if constexpr (kl(A) * kl(B) > 2) {
        if constexpr (kl(A) >= kl(B)) return fq2_mul_lazy(fq2_norm(a), b); else return fq2_mul_lazy(a, fq2_norm(b));
    } else {
    static_assert(kv(A) <= 40 && kv(B) <= 40, "fq2_mul_lazy bound");
    constexpr int K0 = fq2_neg_margin(kv(A), kv(B));
    constexpr int B0 = mul_bound(kv(A), kv(B)) + K0;
    constexpr int B1 = 1 + (int)(((long long)2 * kv(A) * kv(B) * 5908 + 999999) / 1000000);
    const auto s = fq_add(a.c0, a.c1);
    const auto t = fq_add(b.c0, b.c1);
    uint32_t m0[9], m1[9];
    Fq<kenc(B0, 2)> c0;
    Fq<B1> c1;
    int64_t acc0 = 0;
    uint64_t acc1 = 0;
#pragma unroll
    for (int k = 0; k < 17; ++k) {
        const int lo = k < 9 ? 0 : k - 8;
        const int hi = k < 9 ? k : 8;
        uint64_t P = 0, Q = 0;
#pragma unroll
        for (int i = lo; i <= hi; ++i) {
            P += (uint64_t)a.c0.v[i] * b.c0.v[k - i];
            Q += (uint64_t)a.c1.v[i] * b.c1.v[k - i];
            acc1 += (uint64_t)s.v[i] * t.v[k - i];
        }
        acc0 += (int64_t)(P - Q);
        acc1 -= P + Q;
#pragma unroll
        for (int i = lo; i <= hi; ++i) {
            if (i < k) {
                acc0 += (int64_t)((uint64_t)m0[i] * kP29.v[k - i]);
                acc1 += (uint64_t)m1[i] * kP29.v[k - i];
            }
        }
        if (k < 9) {
            m0[k] = ((uint32_t)acc0 * BN_PINV29) & M29;
            m1[k] = ((uint32_t)acc1 * BN_PINV29) & M29;
            acc0 += (int64_t)((uint64_t)m0[k] * kP29.v[0]);
            acc1 += (uint64_t)m1[k] * kP29.v[0];
        } else {
            c0.v[k - 9] = (uint32_t)acc0 & M29;
            c1.v[k - 9] = (uint32_t)acc1 & M29;
        }
        acc0 >>= 29;  // arithmetic
        acc1 >>= 29;
    }
    // c0 + K0*p: digits 0..7 < 2^30, the (signed) top digit becomes >= 0
    constexpr Limbs9 KP = kp_plain(K0);
#pragma unroll
    for (int i = 0; i < 8; ++i) c0.v[i] += KP.v[i];
    c0.v[8] = (uint32_t)acc0 + KP.v[8];
    c1.v[8] = (uint32_t)acc1;
    return mk2(c0, c1);
    }
}

// Fq2 product by schoolbook with one Montgomery reduction per output
// coordinate and no subtraction: c0 = a0*b0 - a1*b1 is accumulated as
// a0*b0 + a1*(K*p - b1), where K*p - b1 (kp_spread, K = B + 1) has non-negative
// digits below (Lb+2)*2^29, so both coordinates are plain unsigned column sums
// of 2 x 81 products plus their 81-product reduction: 486 multiply-adds and no
// 64-bit adds or subtracts (on gfx950 a carry op costs as much as a
// multiply-add).  Column sums: c0 < 9*(La*Lb + La*(Lb+2) + 1)*2^58 + 2^35 and
// c1 < 9*(2*La*Lb + 1)*2^58 + 2^35, both below 2^64 when La*(2*Lb+2) <= 6;
// the operands are swapped (the product commutes) or normalized otherwise.
template <int A, int B>
BN_INLINE auto fq2_mul_sb(const Fq2<A>& a, const Fq2<B>& b) {
    if constexpr (kl(A) * (2 * kl(B) + 2) > 6) {
        if constexpr (kl(B) * (2 * kl(A) + 2) <= 6) return fq2_mul_sb(b, a);
        else if constexpr (kl(A) >= kl(B)) return fq2_mul_sb(fq2_norm(a), b);
        else return fq2_mul_sb(a, fq2_norm(b));
    } else {
    static_assert(kv(A) <= 40 && kv(B) <= 40, "fq2_mul_sb bound");
    constexpr Limbs9 NQ = kp_spread(kv(B) + 1, kl(B));
    constexpr int B0 = 1 + (int)(((long long)kv(A) * (2 * kv(B) + 1) * 5908 + 999999) / 1000000);
    constexpr int B1 = 1 + (int)(((long long)2 * kv(A) * kv(B) * 5908 + 999999) / 1000000);
    uint32_t nb[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) nb[i] = NQ.v[i] - b.c1.v[i];
    uint32_t m0[9], m1[9];
    Fq<B0> c0;
    Fq<B1> c1;
    uint64_t acc0 = 0, acc1 = 0;
#pragma unroll
    for (int k = 0; k < 17; ++k) {
        const int lo = k < 9 ? 0 : k - 8;
        const int hi = k < 9 ? k : 8;
#pragma unroll
        for (int i = lo; i <= hi; ++i) {
            acc0 += (uint64_t)a.c0.v[i] * b.c0.v[k - i];
            acc1 += (uint64_t)a.c0.v[i] * b.c1.v[k - i];
            acc0 += (uint64_t)a.c1.v[i] * nb[k - i];
            acc1 += (uint64_t)a.c1.v[i] * b.c0.v[k - i];
        }
#pragma unroll
        for (int i = lo; i <= hi; ++i) {
            if (i < k) {
                acc0 += (uint64_t)m0[i] * kP29.v[k - i];
                acc1 += (uint64_t)m1[i] * kP29.v[k - i];
            }
        }
        if (k < 9) {
            m0[k] = ((uint32_t)acc0 * BN_PINV29) & M29;
            m1[k] = ((uint32_t)acc1 * BN_PINV29) & M29;
            acc0 += (uint64_t)m0[k] * kP29.v[0];
            acc1 += (uint64_t)m1[k] * kP29.v[0];
        } else {
            c0.v[k - 9] = (uint32_t)acc0 & M29;
            c1.v[k - 9] = (uint32_t)acc1 & M29;
        }
        acc0 >>= 29;
        acc1 >>= 29;
    }
    c0.v[8] = (uint32_t)acc0;
    c1.v[8] = (uint32_t)acc1;
    return mk2(c0, c1);
    }
}

// fq2.rs:136-148: the same product (Karatsuba, bb * (p-1) + aa == aa - bb)
template <int A, int B>
BN_INLINE auto fq2_mul(const Fq2<A>& a_in, const Fq2<B>& b_in) {
    if constexpr (kv(A) > 40 || kv(B) > 40) return fq2_mul(pre<40>(a_in), pre<40>(b_in)); else {
    Fq2<A> a = a_in;
    Fq2<B> b = b_in;
    fq2_fence(a);
    fq2_fence(b);
    auto r = fq2_mul_sb(a, b);  // schoolbook, lazy reduction: 17 % faster than Karatsuba (r1k_fq2_ubench)
    fq2_fence(r);
    return r;
    }
}
// Two independent Fq2 products computed together: the fences bracket the
// pair, so the two column sums interleave (twice the independent multiply-add
// chains for one wave) while no more than two products are in flight.
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
        fq2_fence(a);
        fq2_fence(b);
        fq2_fence(c);
        fq2_fence(d);
        auto r = fq2_mul_sb(a, b);
        auto q = fq2_mul_sb(c, d);
        fq2_fence(r);
        fq2_fence(q);
        return Fq2Pair<decltype(r), decltype(q)>{r, q};
    }
}

// fq2.rs:105-117: (c1*(p-1) + c0)(c0 + c1) - ab - ab*(p-1) == (c0 - c1)(c0 + c1); c1 = 2ab
template <int A>
BN_INLINE auto fq2_sqr(const Fq2<A>& a_in) {
    if constexpr (kv(A) > 40) return fq2_sqr(fq2_fold(a_in)); else {
    Fq2<A> a = a_in;
    fq2_fence(a);
    auto ab = fq_mul(a.c0, a.c1);
    auto c0 = fq_mul(fq_sub(a.c0, a.c1), fq_add(a.c0, a.c1));
    auto r = mk2(c0, fq_dbl(ab));
    fq2_fence(r);
    return r;
    }
}
// x * xi, xi = 9 + u (fq2.rs:19-34, 55-57): (9a0 - a1) + (a0 + 9a1) u.
// Inputs above bound 8 are folded first so the result stays <= 82.
template <int A>
BN_INLINE auto fq2_mul_xi(const Fq2<A>& a) {
    if constexpr (kv(A) > 8) {
        return fq2_mul_xi(fq2_fold(a));
    } else {
        auto n0 = fq_add(fq_mul_small<8>(a.c0), a.c0);
        auto n1 = fq_add(fq_mul_small<8>(a.c1), a.c1);
        return mk2(fq_sub(n0, a.c1), fq_add(a.c0, n1));
    }
}
// fq2.rs:59-68: odd powers conjugate (c1 * (p-1) == -c1)
template <int B>
BN_INLINE auto fq2_conj(const Fq2<B>& a) { return mk2(a.c0, fq_neg(a.c1)); }

// fq2.rs:119-130
template <int B>
BN_INLINE auto fq2_inv(const Fq2<B>& a_in) {
    auto a = pre<40>(a_in);
    auto t = fq_inv(fq_add(fq_sqr(a.c0), fq_sqr(a.c1)));  // c0^2 - (p-1) c1^2
    return mk2(fq_mul(a.c0, t), fq_neg(fq_mul(a.c1, t)));
}

BN_INLINE Fq2<1> fq2_const(const Limbs9& c0, const Limbs9& c1) { return {fq_from_limbs<1>(c0), fq_from_limbs<1>(c1)}; }

#endif  // BN_SPLIT

template <int B>
struct Fq6 {
    Fq2<B> c0, c1, c2;
};
template <int B>
struct Fq12 {
    Fq6<B> c0, c1;
};

// ================================================================ Fq6 = Fq2[v]/(v^3 - xi)
template <int A, int B, int C>
BN_INLINE Fq6<kjoin(A, kjoin(B, C))> mk6(const Fq2<A>& x, const Fq2<B>& y, const Fq2<C>& z) {
    constexpr int M = kjoin(A, kjoin(B, C));
    return {widen<M>(x), widen<M>(y), widen<M>(z)};
}
template <int B2, int B>
BN_INLINE Fq6<B2> widen(const Fq6<B>& a) { return {widen<B2>(a.c0), widen<B2>(a.c1), widen<B2>(a.c2)}; }
BN_INLINE Fq6<1> fq6_zero() { return {fq2_zero(), fq2_zero(), fq2_zero()}; }
BN_INLINE Fq6<1> fq6_one() { return {fq2_one(), fq2_zero(), fq2_zero()}; }
template <int A, int B>
BN_INLINE auto fq6_add(const Fq6<A>& a, const Fq6<B>& b) {
    return mk6(fq2_add(a.c0, b.c0), fq2_add(a.c1, b.c1), fq2_add(a.c2, b.c2));
}
template <int A, int B>
BN_INLINE auto fq6_sub(const Fq6<A>& a, const Fq6<B>& b) {
    return mk6(fq2_sub(a.c0, b.c0), fq2_sub(a.c1, b.c1), fq2_sub(a.c2, b.c2));
}
template <int B>
BN_INLINE auto fq6_neg(const Fq6<B>& a) { return mk6(fq2_neg(a.c0), fq2_neg(a.c1), fq2_neg(a.c2)); }
template <int B>
BN_INLINE Fq6<2> fq6_fold(const Fq6<B>& a) {
#if BN_FOLD_LDS && defined(__HIP_DEVICE_COMPILE__) && !BN_SPLIT
    if constexpr (kl(B) <= 6) {
        const FoldEnt e0 = fold_fetch(a.c0.c0), e1 = fold_fetch(a.c0.c1), e2 = fold_fetch(a.c1.c0),
                      e3 = fold_fetch(a.c1.c1), e4 = fold_fetch(a.c2.c0), e5 = fold_fetch(a.c2.c1);
        return {{fold_apply(a.c0.c0, e0), fold_apply(a.c0.c1, e1)}, {fold_apply(a.c1.c0, e2), fold_apply(a.c1.c1, e3)},
                {fold_apply(a.c2.c0, e4), fold_apply(a.c2.c1, e5)}};
    }
#endif
    return {fq2_fold(a.c0), fq2_fold(a.c1), fq2_fold(a.c2)};
}
template <int B>
BN_INLINE Fq6<kv(B)> fq6_norm(const Fq6<B>& a) { return {fq2_norm(a.c0), fq2_norm(a.c1), fq2_norm(a.c2)}; }
template <int B>
BN_INLINE bool fq6_is_zero(const Fq6<B>& a) {
    return ((unsigned)fq2_is_zero(a.c0) & (unsigned)fq2_is_zero(a.c1) & (unsigned)fq2_is_zero(a.c2)) != 0;  // no branches
}
template <int L, int B>
BN_INLINE auto pre(const Fq6<B>& a) {
    if constexpr (kv(B) <= L) return a; else return fq6_fold(a);
}
// fq6.rs:109-115
template <int B>
BN_INLINE auto fq6_mul_by_nonresidue(const Fq6<B>& a) { return mk6(fq2_mul_xi(a.c2), a.c0, a.c1); }

// fq6.rs:197-207
template <int A, int B>
BN_INLINE auto fq6_mul(const Fq6<A>& a, const Fq6<B>& b) {
    if constexpr (kv(A) > 20 || kv(B) > 20) return fq6_mul(pre<20>(a), pre<20>(b)); else {
    // the six Fq2 products in three independent pairs (one at a time: within noise,
    // profiles/r3z_ab_fq6_pairs.txt)
    const auto p1 = fq2_mul2(a.c0, b.c0, a.c1, b.c1);
    const auto& a_a = p1.a;
    const auto& b_b = p1.b;
    const auto p2 = fq2_mul2(a.c2, b.c2, fq2_add(a.c1, a.c2), fq2_add(b.c1, b.c2));
    const auto& c_c = p2.a;
    auto t0 = fq2_sub(fq2_sub(p2.b, b_b), c_c);
    const auto p3 = fq2_mul2(fq2_add(a.c0, a.c1), fq2_add(b.c0, b.c1), fq2_add(a.c0, a.c2), fq2_add(b.c0, b.c2));
    auto t1 = fq2_sub(fq2_sub(p3.a, a_a), b_b);
    auto t2 = fq2_sub(p3.b, a_a);
    return mk6(fq2_add(fq2_mul_xi(t0), a_a), fq2_add(t1, fq2_mul_xi(c_c)), fq2_sub(fq2_add(t2, b_b), c_c));
    }
}
// fq6.rs:163-177
template <int A>
BN_INLINE auto fq6_sqr(const Fq6<A>& a) {
    if constexpr (kv(A) > 20) return fq6_sqr(fq6_fold(a)); else {
    auto s0 = fq2_sqr(a.c0);
    auto s1 = fq2_dbl(fq2_mul(a.c0, a.c1));
    auto s2 = fq2_sqr(fq2_add(fq2_sub(a.c0, a.c1), a.c2));
    auto s3 = fq2_dbl(fq2_mul(a.c1, a.c2));
    auto s4 = fq2_sqr(a.c2);
    return mk6(fq2_add(s0, fq2_mul_xi(s3)), fq2_add(s1, fq2_mul_xi(s4)),
               fq2_sub(fq2_sub(fq2_add(fq2_add(s1, s2), s3), s0), s4));
    }
}
// fq6.rs:179-191
template <int B>
BN_INLINE auto fq6_inv(const Fq6<B>& a_in) {
    auto a = fq6_fold(a_in);
    auto c0 = fq2_fold(fq2_sub(fq2_sqr(a.c0), fq2_mul(a.c1, fq2_mul_xi(a.c2))));
    auto c1 = fq2_fold(fq2_sub(fq2_mul_xi(fq2_sqr(a.c2)), fq2_mul(a.c0, a.c1)));
    auto c2 = fq2_fold(fq2_sub(fq2_sqr(a.c1), fq2_mul(a.c0, a.c2)));
    auto t = fq2_inv(fq2_fold(fq2_add(fq2_mul_xi(fq2_add(fq2_mul(a.c2, c1), fq2_mul(a.c1, c2))), fq2_mul(a.c0, c0))));
    return mk6(fq2_mul(t, c0), fq2_mul(t, c1), fq2_mul(t, c2));
}

// Frobenius coefficients (internal form, generated from fq6.rs:5-90 / fq12.rs:6-48)
BN_INLINE Fq2<1> fq6_frob_c1(int n) {
    if (n == 1) return fq2_const(Limbs9{BN_FQ6_C1_1_C0}, Limbs9{BN_FQ6_C1_1_C1});
    if (n == 2) return fq2_const(Limbs9{BN_FQ6_C1_2_C0}, Limbs9{BN_FQ6_C1_2_C1});
    return fq2_const(Limbs9{BN_FQ6_C1_3_C0}, Limbs9{BN_FQ6_C1_3_C1});
}
BN_INLINE Fq2<1> fq6_frob_c2(int n) {
    if (n == 1) return fq2_const(Limbs9{BN_FQ6_C2_1_C0}, Limbs9{BN_FQ6_C2_1_C1});
    if (n == 2) return fq2_const(Limbs9{BN_FQ6_C2_2_C0}, Limbs9{BN_FQ6_C2_2_C1});
    return fq2_const(Limbs9{BN_FQ6_C2_3_C0}, Limbs9{BN_FQ6_C2_3_C1});
}
BN_INLINE Fq2<1> fq12_frob_c1(int n) {
    if (n == 1) return fq2_const(Limbs9{BN_FQ12_C1_1_C0}, Limbs9{BN_FQ12_C1_1_C1});
    if (n == 2) return fq2_const(Limbs9{BN_FQ12_C1_2_C0}, Limbs9{BN_FQ12_C1_2_C1});
    return fq2_const(Limbs9{BN_FQ12_C1_3_C0}, Limbs9{BN_FQ12_C1_3_C1});
}
// fq6.rs:125-131 for power 1..3; power 2 coefficients are real (c1 == 0): two Fq products
template <int POWER, int B>
BN_INLINE auto fq6_frobenius_map(const Fq6<B>& a) {
    if constexpr (POWER == 2) {
        return mk6(a.c0, fq2_scale(a.c1, fq_from_limbs<1>(Limbs9{BN_FQ6_C1_2_C0})), fq2_scale(a.c2, fq_from_limbs<1>(Limbs9{BN_FQ6_C2_2_C0})));
    } else {
        return mk6(fq2_conj(a.c0), fq2_mul(fq2_conj(a.c1), fq6_frob_c1(POWER)), fq2_mul(fq2_conj(a.c2), fq6_frob_c2(POWER)));
    }
}

// ================================================================ Fq12 = Fq6[w]/(w^2 - v)
template <int A, int B>
BN_INLINE Fq12<kjoin(A, B)> mk12(const Fq6<A>& x, const Fq6<B>& y) {
    return {widen<kjoin(A, B)>(x), widen<kjoin(A, B)>(y)};
}
template <int B2, int B>
BN_INLINE Fq12<B2> widen(const Fq12<B>& a) { return {widen<B2>(a.c0), widen<B2>(a.c1)}; }
BN_INLINE Fq12<1> fq12_one() { return {fq6_one(), fq6_zero()}; }
template <int B>
BN_INLINE Fq12<2> fq12_fold(const Fq12<B>& a) { return {fq6_fold(a.c0), fq6_fold(a.c1)}; }
template <int B>
BN_INLINE Fq12<kv(B)> fq12_norm(const Fq12<B>& a) { return {fq6_norm(a.c0), fq6_norm(a.c1)}; }
template <int B>
BN_INLINE bool fq12_is_zero(const Fq12<B>& a) { return ((unsigned)fq6_is_zero(a.c0) & (unsigned)fq6_is_zero(a.c1)) != 0; }
template <int L, int B>
BN_INLINE auto pre(const Fq12<B>& a) {
    if constexpr (kv(B) <= L) return a; else return fq12_fold(a);
}
template <int B>
BN_INLINE auto fq12_conj(const Fq12<B>& a) { return mk12(a.c0, fq6_neg(a.c1)); }  // unitary_inverse, fq12.rs:126-128
template <int A, int B>
BN_INLINE auto fq12_add(const Fq12<A>& a, const Fq12<B>& b) { return mk12(fq6_add(a.c0, b.c0), fq6_add(a.c1, b.c1)); }
template <int A, int B>
BN_INLINE auto fq12_sub(const Fq12<A>& a, const Fq12<B>& b) { return mk12(fq6_sub(a.c0, b.c0), fq6_sub(a.c1, b.c1)); }
template <int B>
BN_INLINE auto fq12_neg(const Fq12<B>& a) { return mk12(fq6_neg(a.c0), fq6_neg(a.c1)); }

// fq12.rs:319-327
template <int A, int B>
BN_INLINE auto fq12_mul(const Fq12<A>& a, const Fq12<B>& b) {
    if constexpr (kv(A) > 10 || kv(B) > 10) return fq12_mul(pre<10>(a), pre<10>(b)); else {
    auto aa = fq6_fold(fq6_mul(a.c0, b.c0));
    auto bb = fq6_fold(fq6_mul(a.c1, b.c1));
    auto t = fq6_mul(fq6_add(a.c0, a.c1), fq6_add(b.c0, b.c1));
    return mk12(fq6_add(fq6_mul_by_nonresidue(bb), aa), fq6_sub(fq6_sub(t, aa), bb));
    }
}
// fq12.rs:295-303
template <int A>
BN_INLINE auto fq12_sqr(const Fq12<A>& a) {
    if constexpr (kv(A) > 2) return fq12_sqr(fq12_fold(a)); else {
    auto ab = fq6_fold(fq6_mul(a.c0, a.c1));
    auto t = fq6_mul(fq6_add(fq6_mul_by_nonresidue(a.c1), a.c0), fq6_add(a.c0, a.c1));
    return mk12(fq6_sub(fq6_sub(t, ab), fq6_mul_by_nonresidue(ab)), fq6_add(ab, ab));
    }
}
// fq12.rs:305-313
template <int B>
BN_INLINE auto fq12_inv(const Fq12<B>& a_in) {
    auto a = fq12_fold(a_in);
    auto t = fq6_inv(fq6_sub(fq6_fold(fq6_sqr(a.c0)), fq6_mul_by_nonresidue(fq6_fold(fq6_sqr(a.c1)))));
    return mk12(fq6_mul(a.c0, t), fq6_neg(fq6_mul(a.c1, t)));
}
// fq12.rs:112-119
template <int POWER, int B>
BN_INLINE auto fq12_frobenius_map(const Fq12<B>& a) {
    auto c1 = fq6_frobenius_map<POWER>(a.c1);
    if constexpr (POWER == 2) {
        const Fq<1> k = fq_from_limbs<1>(Limbs9{BN_FQ12_C1_2_C0});  // real: fq12.rs:6-48 power 2 has c1 == 0
        return mk12(fq6_frobenius_map<POWER>(a.c0), mk6(fq2_scale(c1.c0, k), fq2_scale(c1.c1, k), fq2_scale(c1.c2, k)));
    } else {
        Fq2<1> k = fq12_frob_c1(POWER);
        return mk12(fq6_frobenius_map<POWER>(a.c0), mk6(fq2_mul(c1.c0, k), fq2_mul(c1.c1, k), fq2_mul(c1.c2, k)));
    }
}

// fq12.rs:130-196 -- sparse product with a line (slots 0, 2, 4 nonzero)
template <int F, int X>
BN_INLINE auto fq12_mul_by_024(const Fq12<F>& f, const Fq2<X>& ell_0, const Fq2<X>& ell_vw, const Fq2<X>& ell_vv) {
    const auto& z0 = f.c0.c0;
    const auto& z1 = f.c0.c1;
    const auto& z2 = f.c0.c2;
    const auto& z3 = f.c1.c0;
    const auto& z4 = f.c1.c1;
    const auto& z5 = f.c1.c2;
    const auto& x0 = ell_0;
    const auto& x2 = ell_vv;
    const auto& x4 = ell_vw;

    auto d0 = fq2_mul(z0, x0);
    auto d2 = fq2_mul(z2, x2);
    auto d4 = fq2_mul(z4, x4);
    auto t2 = fq2_add(z0, z4);
    auto t1 = fq2_add(z0, z2);
    auto s0 = fq2_add(fq2_add(z1, z3), z5);

    auto s1a = fq2_mul(z1, x2);
    auto n0 = fq2_add(fq2_mul_xi(fq2_add(s1a, d4)), d0);

    auto t3a = fq2_mul(z5, x4);
    auto s1b = fq2_add(s1a, t3a);
    auto t4a = fq2_mul_xi(fq2_add(t3a, d2));
    auto t3b = fq2_mul(z1, x0);
    auto s1c = fq2_add(s1b, t3b);
    auto n1 = fq2_add(t4a, t3b);

    auto t3c = fq2_sub(fq2_sub(fq2_mul(t1, fq2_add(x0, x2)), d0), d2);
    auto t4b = fq2_mul(z3, x4);
    auto s1d = fq2_add(s1c, t4b);
    auto n2 = fq2_add(t3c, t4b);

    auto t3d = fq2_sub(fq2_sub(fq2_mul(fq2_add(z2, z4), fq2_add(x2, x4)), d2), d4);
    auto t4c = fq2_mul_xi(t3d);
    auto t3e = fq2_mul(z3, x0);
    auto s1e = fq2_fold(fq2_add(s1d, t3e));
    auto n3 = fq2_add(t4c, t3e);

    auto t3f = fq2_mul(z5, x2);
    auto s1f = fq2_add(s1e, t3f);
    auto t4d = fq2_mul_xi(t3f);
    auto t3g = fq2_sub(fq2_sub(fq2_mul(t2, fq2_add(x0, x4)), d0), d4);
    auto n4 = fq2_add(t4d, t3g);

    auto n5 = fq2_sub(fq2_mul(s0, fq2_add(fq2_add(x0, x2), x4)), s1f);
    return mk12(mk6(n0, n1, n2), mk6(n3, n4, n5));
}

// fq12.rs:198-247 -- Granger-Scott cyclotomic squaring (the reference's formula)
// BN_CYC_LAZY: t0, t2, t4 and xi*t5 leave with a carry pass instead of a fold (their
// digits normalized, the value bound carried on to the outputs' folds): 65 VALU fewer
// per square with the asm column sums, k_pairing_full 7.47-7.48 -> 7.37-7.38 ms,
// Gt::pow -1.2 % (profiles/r5u_ab_cyc_lazy.txt).  Every fold stays under the bound
// check (fq.h fold_fetch; tools/fold_check.py).
#ifndef BN_CYC_LAZY
#define BN_CYC_LAZY 1
#endif
#if BN_CYC_LAZY
#define BN_CYC_T(x) fq2_norm(x)
#else
#define BN_CYC_T(x) fq2_fold(x)
#endif
template <int A>
BN_INLINE auto fq12_cyclotomic_sqr(const Fq12<A>& a) {
    const auto& z0 = a.c0.c0;
    const auto& z4 = a.c0.c1;
    const auto& z3 = a.c0.c2;
    const auto& z2 = a.c1.c0;
    const auto& z1 = a.c1.c1;
    const auto& z5 = a.c1.c2;
    auto tmp01 = fq2_mul(z0, z1);
    auto t0 = BN_CYC_T(fq2_sub(fq2_sub(fq2_mul(fq2_add(z0, z1), fq2_add(fq2_mul_xi(z1), z0)), tmp01), fq2_mul_xi(tmp01)));
    auto t1 = fq2_dbl(tmp01);
    auto tmp23 = fq2_mul(z2, z3);
    auto t2 = BN_CYC_T(fq2_sub(fq2_sub(fq2_mul(fq2_add(z2, z3), fq2_add(fq2_mul_xi(z3), z2)), tmp23), fq2_mul_xi(tmp23)));
    auto t3 = fq2_dbl(tmp23);
    auto tmp45 = fq2_mul(z4, z5);
    auto xi45 = fq2_mul_xi(tmp45);  // also gives xi * t5 = 2 * xi * tmp45 below
    auto t4 = BN_CYC_T(fq2_sub(fq2_sub(fq2_mul(fq2_add(z4, z5), fq2_add(fq2_mul_xi(z5), z4)), tmp45), xi45));

    auto n0 = fq2_add(fq2_dbl(fq2_sub(t0, z0)), t0);
    auto n1 = fq2_add(fq2_dbl(fq2_add(t1, z1)), t1);
    auto x5 = BN_CYC_T(fq2_dbl(xi45));  // xi * t5
    auto n2 = fq2_add(fq2_dbl(fq2_add(x5, z2)), x5);
    auto n3 = fq2_add(fq2_dbl(fq2_sub(t4, z3)), t4);
    auto n4 = fq2_add(fq2_dbl(fq2_sub(t2, z4)), t2);
    auto n5 = fq2_add(fq2_dbl(fq2_add(t3, z5)), t3);
    return mk12(mk6(n0, n4, n3), mk6(n2, n1, n5));
}

}  // namespace bn
