// codec.h -- encodings, square roots, point validation and decompression,
// one lane per element.
//
// Replaces, per element:
//   Fq::from_slice / to_big_endian        lib.rs:154-170, fp.rs:46-54
//   Fq2::from_slice (U512 divrem by p)    lib.rs:260-267, arith.rs:82-96, 116-138
//   Fr::from_slice / to_big_endian        lib.rs:45-55 (new_mul_factor; the raw image out)
//   Fq::sqrt, Fq2::sqrt                   fp.rs:245-260, fq2.rs:208-224
//   AffineG::new (curve + order check)    groups/mod.rs:95-113
//   G1/G2::from_compressed                lib.rs:359-375, 506-526
//
// Values, not formulas, are what must match here: every output is either a
// canonical image (unique) or a status, so square-and-multiply chains may be
// any chain for the same exponent, the order check may be any evaluation of
// [r]P == 0, and the field work reuses the engine's Fq (fq.h).  The byte-level
// integer work (comparisons against p and p^2, exact division by p, Fr
// Montgomery by 32-bit CIOS) is written on little-endian 32-bit words.
#pragma once
#include "curve.h"

namespace bn {

// per-element status: the values of bn_elem_status (include/bn254mi.h)
enum : uint8_t {
    ST_OK = 0,
    ST_FIELD_NOT_MEMBER = 3,      // FieldError::NotMember
    ST_CURVE_INVALID_ENCODING = 4,  // CurveError::InvalidEncoding
    ST_CURVE_NOT_MEMBER = 5,      // CurveError::NotMember
    ST_GROUP_NOT_ON_CURVE = 6,    // groups::Error::NotOnCurve
    ST_GROUP_NOT_IN_SUBGROUP = 7  // groups::Error::NotInSubgroup
};

// ---------------------------------------------------------------- 32-bit word integers
// a < b for n-word little-endian integers (borrow of a - b)
template <int N>
BN_INLINE bool wlt(const uint32_t* a, const uint32_t* b) {
    int64_t br = 0;
#pragma unroll
    for (int i = 0; i < N; ++i) br = ((int64_t)a[i] - (int64_t)b[i] + br) >> 32;
    return br < 0;
}
// big-endian bytes -> little-endian words (bytes [0] is the most significant)
template <int N>
BN_INLINE void words_from_be(const uint8_t* s, uint32_t* w) {
#pragma unroll
    for (int i = 0; i < N; ++i) {
        const uint8_t* b = s + 4 * (N - 1 - i);
        w[i] = (uint32_t)b[0] << 24 | (uint32_t)b[1] << 16 | (uint32_t)b[2] << 8 | b[3];
    }
}
template <int N>
BN_INLINE void be_from_words(const uint32_t* w, uint8_t* s) {
#pragma unroll
    for (int i = 0; i < N; ++i) {
        uint8_t* b = s + 4 * (N - 1 - i);
        b[0] = (uint8_t)(w[i] >> 24);
        b[1] = (uint8_t)(w[i] >> 16);
        b[2] = (uint8_t)(w[i] >> 8);
        b[3] = (uint8_t)w[i];
    }
}

// internal value -> canonical plain integer words (U256::from(Fq), fp.rs:13-20)
template <int B>
BN_INLINE void fq_plain_words(const Fq<B>& a, uint32_t w[8]) {
    fq_words_from_digits(fq_cond_sub_p(widen<2>(fq_mul(a, fq_from_limbs<1>(Limbs9{BN_TO_CANON})))), w);
}
// plain integer words (any value < 2^256) -> internal; the digits of a 256-bit
// integer are normalized and its value is below 6p
BN_INLINE Fq<2> fq_from_plain_words(const uint32_t w[8]) {
    return fq_mul(widen<6>(fq_digits_from_words(w)), fq_from_limbs<1>(Limbs9{BN_FROM_CANON}));
}

// Fp::new (fp.rs:46-54): the value if it is below p
BN_INLINE bool fq_new_plain(const uint32_t w[8], Fq<2>& out) {
    constexpr uint32_t PW[8] = BN_P_W32;
    out = fq_from_plain_words(w);
    return wlt<8>(w, PW);
}

// Fq2::from_slice (lib.rs:260-267): v = 512-bit big-endian; c0 = v mod p,
// c1 = v div p, NotMember when the quotient is not below p (U512::divrem,
// arith.rs:116-138), i.e. when v >= p^2.
BN_INLINE bool fq2_from_u512(const uint32_t v[16], Fq2<2>& out) {
    constexpr uint32_t P2[16] = BN_P2_W32;
    constexpr uint32_t PINV[8] = BN_PINV_W32;
    const bool ok = wlt<16>(v, P2);
    // r = v mod p: internal(lo) + internal(hi * 2^256), back to a plain canonical integer
    const Fq<2> lo = fq_from_plain_words(v);
    const Fq<2> hi = fq_mul(widen<6>(fq_digits_from_words(v + 8)), fq_from_limbs<1>(Limbs9{BN_FROM_CANON_HI}));
    const auto x = fq_add(lo, hi);
    uint32_t r[8];
    fq_plain_words(x, r);
    // q = (v - r) / p, exact: the low 256 bits of (v - r) times p^-1 mod 2^256
    uint32_t d[8], q[8];
    int64_t br = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int64_t t = (int64_t)v[i] - (int64_t)r[i] + br;
        d[i] = (uint32_t)t;
        br = t >> 32;
        q[i] = 0;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        uint64_t c = 0;
#pragma unroll
        for (int j = 0; i + j < 8; ++j) {
            const uint64_t t = (uint64_t)d[i] * PINV[j] + q[i + j] + c;
            q[i + j] = (uint32_t)t;
            c = t >> 32;
        }
    }
    out = {fq_from_plain_words(r), fq_from_plain_words(q)};
    return ok;
}

// Fr::new_mul_factor (fp.rs:57-60): a * R^2 * R^-1 mod r for any 256-bit a,
// HAC 14.32 with 32-bit digits and one conditional subtraction; a < 2^256 and
// R^2 mod r < r keep the pre-subtraction value below 2r, so the result is the
// canonical Montgomery image the reference computes.
BN_INLINE void fr_from_plain_words(const uint32_t a[8], uint32_t out[8]) {
    constexpr uint32_t RW[8] = BN_R_W32;
    constexpr uint32_t R2[8] = BN_R2_R_W32;
    uint32_t t[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        uint64_t c = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const uint64_t s = (uint64_t)a[i] * R2[j] + t[j] + c;
            t[j] = (uint32_t)s;
            c = s >> 32;
        }
        uint64_t s = (uint64_t)t[8] + c;
        t[8] = (uint32_t)s;
        t[9] = (uint32_t)(s >> 32);
        const uint32_t m = t[0] * 0xefffffffu;  // -r^-1 mod 2^32
        c = ((uint64_t)m * RW[0] + t[0]) >> 32;
#pragma unroll
        for (int j = 1; j < 8; ++j) {
            s = (uint64_t)m * RW[j] + t[j] + c;
            t[j - 1] = (uint32_t)s;
            c = s >> 32;
        }
        s = (uint64_t)t[8] + c;
        t[7] = (uint32_t)s;
        t[8] = t[9] + (uint32_t)(s >> 32);
    }
    uint32_t d[8];
    int64_t br = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int64_t s = (int64_t)t[j] - RW[j] + br;
        d[j] = (uint32_t)s;
        br = s >> 32;
    }
    const bool ge = (t[8] != 0) || (br == 0);
#pragma unroll
    for (int j = 0; j < 8; ++j) out[j] = ge ? d[j] : t[j];
}

// ---------------------------------------------------------------- square roots
// bit `bit` of a constant 256-bit exponent (wave-uniform: scalar branch)
BN_INLINE bool ebit(const uint64_t (&e)[4], int bit) { return (e[bit >> 6] >> (bit & 63)) & 1u; }
constexpr uint64_t kPm3d4[4] = BN_PM3D4;  // (p-3)/4, 252 bits
constexpr uint64_t kPm1d2[4] = BN_PM1D2;  // (p-1)/2, 253 bits

// x^e for a constant e with top bit `top` (fields/mod.rs:35-46 gives the same value)
template <int B>
BN_INLINE Fq<2> fq_pow_const(const Fq<B>& a, const uint64_t (&e)[4], int top) {
    const Fq<2> x = widen<2>(fq_reduce(a));
    Fq<2> r = x;
#pragma unroll 1
    for (int bit = top - 1; bit >= 0; --bit) {
        r = fq_sqr(r);
        if (ebit(e, bit)) r = fq_mul(r, x);
    }
    return r;
}
template <int B>
BN_INLINE Fq2<kPt> fq2_pow_const(const Fq2<B>& a, const uint64_t (&e)[4], int top) {
    const Fq2<kPt> x = narrow<kPt>(a);
    Fq2<kPt> r = x;
#pragma unroll 1
    for (int bit = top - 1; bit >= 0; --bit) {
        r = narrow<kPt>(fq2_sqr(r));
        if (ebit(e, bit)) r = narrow<kPt>(fq2_mul(r, x));
    }
    return r;
}
constexpr int kTopPm3d4 = 251;  // (p-3)/4 < 2^252, bit 251 set
constexpr int kTopPm1d2 = 252;

// Fq::sqrt, fp.rs:245-260: Some(a^((p+1)/4)) unless a^((p-1)/2) == -1
template <int B>
BN_INLINE bool fq_sqrt(const Fq<B>& a, Fq<2>& out) {
    const Fq<2> a1 = fq_pow_const(a, kPm3d4, kTopPm3d4);
    const auto a1a = fq_mul(a1, a);
    const auto a0 = fq_mul(a1, a1a);
    out = widen<2>(a1a);
    return !fq_eq(a0, fq_neg(fq_one()));
}
// Fq2::sqrt, fq2.rs:208-224 (alpha^p is the conjugate of alpha: Frobenius)
template <int B>
BN_INLINE bool fq2_sqrt(const Fq2<B>& a_in, Fq2<kPt>& out) {
    const Fq2<kPt> a = narrow<kPt>(a_in);
    const Fq2<kPt> a1 = fq2_pow_const(a, kPm3d4, kTopPm3d4);
    const Fq2<kPt> a1a = narrow<kPt>(fq2_mul(a1, a));
    const Fq2<kPt> alpha = narrow<kPt>(fq2_mul(a1, a1a));
    const auto a0 = fq2_mul(fq2_conj(alpha), alpha);
    const auto minus_one = fq2_neg(fq2_one());
    const bool none = fq2_eq(a0, minus_one);
    const bool alpha_m1 = fq2_eq(alpha, minus_one);
    // alpha == -1: i * a1a = (-a1a.c1, a1a.c0); else (alpha + 1)^((p-1)/2) * a1a
    const Fq2<kPt> b = fq2_pow_const(fq2_add(alpha, fq2_one()), kPm1d2, kTopPm1d2);
    const Fq2<kPt> gen = narrow<kPt>(fq2_mul(b, a1a));
    const Fq2<kPt> ia = narrow<kPt>(mk2(fq_neg(a1a.c1), a1a.c0));
    out = fq2_select(alpha_m1, ia, gen);
    return !none;
}

// ---------------------------------------------------------------- points
// y^2 == x^3 + b (mod.rs:96)
template <int X, int Y>
BN_INLINE bool g1_on_curve(const Fq<X>& x, const Fq<Y>& y) {
    return fq_eq(fq_sqr(y), fq_add(fq_mul(fq_sqr(x), x), fq_from_limbs<1>(Limbs9{BN_G1B})));
}
template <int X, int Y>
BN_INLINE bool g2_on_curve(const Fq2<X>& x, const Fq2<Y>& y) {
    return fq2_eq(fq2_sqr(y), fq2_add(fq2_mul(fq2_sqr(x), x), g2_coeff_b()));
}

// Projective equality with the reference's zero handling (mod.rs:169-195)
template <template <int> class F>
BN_INLINE bool jac_eq(const Jac<F>& a, const Jac<F>& b) {
    const bool az = jac_is_zero(a), bz = jac_is_zero(b);
    const auto z1s = F_sqr(a.z), z2s = F_sqr(b.z);
    const bool ex = F_is_zero(F_sub(F_mul(a.x, z2s), F_mul(b.x, z1s)));
    const bool ey = F_is_zero(F_sub(F_mul(a.y, F_mul(b.z, z2s)), F_mul(b.y, F_mul(a.z, z1s))));
    return az ? bz : (!bz && ex && ey);
}

// NAF of the trace t = 6u^2 + 1 (constants.inc)
constexpr uint64_t kTNafNz[4] = BN_TNAF_NZ;
constexpr uint64_t kTNafNeg[4] = BN_TNAF_NEG;

// The order check of AffineG<G2Params>::new (mod.rs:99-108): the reference
// tests p * (-1) + p == 0, i.e. [r]P == 0.  On the twist the Frobenius map
// psi (the reference's mul_by_q, mod.rs:694-699) satisfies psi^2 - t psi + p = 0
// on every point, and r = p + 1 - t, so
//     [r]P = [t](psi(P) - P) - (psi^2(P) - P)
// exactly, and [r]P == 0 <=> [t](psi(P) - P) == psi^2(P) - P: the same boolean
// from a 127-bit chain instead of a 254-bit one.  (tools/psi_check.py checks
// the identity and both outcomes with plain integers.)  The group law is the
// reference's complete Jacobian one (mod.rs:250-334).
template <int B>
BN_INLINE bool g2_in_subgroup(const Fq2<B>& x, const Fq2<B>& y) {
    const G2Aff<kPt> p0 = {narrow<kPt>(x), narrow<kPt>(y)};
    const G2Aff<kPt> p1 = mul_by_q(p0);  // psi(P)
    const G2Aff<kPt> p2 = mul_by_q(p1);  // psi^2(P)
    const Fq2<kPt> one = widen<kPt>(fq2_one());
    const G2J pn = {p0.x, narrow<kPt>(fq2_neg(p0.y)), one};
    const G2J q = jac_add(G2J{p1.x, p1.y, one}, pn);  // psi(P) - P
    const G2J s = jac_add(G2J{p2.x, p2.y, one}, pn);  // psi^2(P) - P
    const G2J qn = jac_neg(q);
    G2J acc = q;  // top digit (+1)
#pragma unroll 1
    for (int bit = BN_TNAF_TOP - 1; bit >= 0; --bit) {
        acc = jac_double(acc);
        if (ebit(kTNafNz, bit)) acc = jac_add(acc, ebit(kTNafNeg, bit) ? qn : q);
    }
    return jac_eq(acc, s);
}

// canonical y > canonical(-y) as Fq2::to_u512 values c1 * p + c0 (lib.rs:517, fq2.rs:226-231):
// lexicographic on (c1, c0) because c0 < p
template <int A, int B>
BN_INLINE bool fq2_u512_gt(const Fq2<A>& a, const Fq2<B>& b) {
    uint32_t a0[8], a1[8], b0[8], b1[8];
    fq_plain_words(a.c0, a0);
    fq_plain_words(a.c1, a1);
    fq_plain_words(b.c0, b0);
    fq_plain_words(b.c1, b1);
    uint32_t A16[16], B16[16];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        A16[i] = a0[i];
        A16[i + 8] = a1[i];
        B16[i] = b0[i];
        B16[i + 8] = b1[i];
    }
    return wlt<16>(B16, A16);
}

// G1::from_compressed (lib.rs:359-375) of 33 bytes; x, y internal on success
BN_INLINE uint8_t g1_decompress(const uint8_t b[33], Fq<2>& x, Fq<2>& y) {
    const uint8_t sign = b[0];
    uint32_t w[8];
    words_from_be<8>(b + 1, w);
    const bool member = fq_new_plain(w, x);
    const auto y2 = fq_add(fq_mul(fq_sqr(x), x), fq_from_limbs<1>(Limbs9{BN_G1B}));
    const bool has_root = fq_sqrt(y2, y);
    uint32_t yw[8];
    fq_plain_words(y, yw);
    const bool odd = yw[0] & 1u;
    const bool flip = (sign == 2 && odd) || (sign == 3 && !odd);
    y = fq_select(flip, widen<2>(fq_neg(y)), y);
    if (!member) return ST_FIELD_NOT_MEMBER;  // CurveError::Field(FieldError::NotMember)
    if (!has_root) return ST_CURVE_NOT_MEMBER;
    if (sign != 2 && sign != 3) return ST_CURVE_INVALID_ENCODING;
    if (!g1_on_curve(x, y)) return ST_CURVE_NOT_MEMBER;  // AffineG1::new (G1: no order check)
    return ST_OK;
}

// G2::from_compressed (lib.rs:506-526) of 65 bytes
BN_INLINE uint8_t g2_decompress(const uint8_t b[65], Fq2<kPt>& x, Fq2<kPt>& y) {
    const uint8_t sign = b[0];
    uint32_t v[16];
    words_from_be<16>(b + 1, v);
    Fq2<2> xr;
    const bool member = fq2_from_u512(v, xr);
    x = widen<kPt>(xr);
    const auto y2 = fq2_add(fq2_mul(fq2_sqr(x), x), g2_coeff_b());
    Fq2<kPt> r;
    const bool has_root = fq2_sqrt(y2, r);
    const Fq2<kPt> rn = widen<kPt>(fq2_neg(r));
    const bool y_gt = fq2_u512_gt(r, rn);
    // sign 10: the smaller of y, -y; sign 11: the larger
    y = fq2_select(sign == 10 ? y_gt : !y_gt, rn, r);
    const bool in_group = g2_in_subgroup(x, y);
    if (!member) return ST_FIELD_NOT_MEMBER;
    if (!has_root) return ST_CURVE_NOT_MEMBER;
    if (sign != 10 && sign != 11) return ST_CURVE_INVALID_ENCODING;
    if (!g2_on_curve(x, y) || !in_group) return ST_CURVE_NOT_MEMBER;  // AffineG2::new -> NotMember
    return ST_OK;
}

}  // namespace bn
