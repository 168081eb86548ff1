// fq.h -- BN254 base field Fq on CDNA4 (gfx950), one lane per element.
//
// Replaces src/arith.rs:281-316 + 473-545 and src/fields/fp.rs:7-164 of the
// reference (U256 Montgomery arithmetic with 2 x u128 digits).
//
// Internal representation (chosen from measurements on MI355X):
//   x is held as X = x * 2^261 mod p (Montgomery, R = 2^261) in NINE 29-bit
//   digits, one per 32-bit VGPR.  29-bit digits let a column of the Montgomery
//   product accumulate all 18 digit products in one 64-bit register with
//   v_mad_u64_u32 and NO per-product carry instruction (on gfx950 a carry op
//   costs as much as the multiply itself), and let additions/subtractions run
//   digit-wise with full-rate VOP2 instructions.
//
//   Values are kept "weakly reduced": digits normalized (< 2^29) but the value
//   may exceed p.  Fq<B> carries a compile-time bound: value <= B*p.  Every
//   operation derives its output bound, and static_asserts keep every value
//   below 2^261 and every column sum below 2^64 -- so no overflow is possible
//   on any input.  Values become canonical (the reference's memory image) only
//   at the boundary (fq_store_ref / fq_canonical).
//
// Bit-exactness: each function computes the same residue mod p as the
// reference function it replaces, and the boundary emits the unique canonical
// Montgomery image the reference stores.
#pragma once
#include <stdint.h>
#if defined(BN_HOST_CHECKS)
#include <stdio.h>
#include <stdlib.h>
#endif

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define BN_HD __host__ __device__
#define BN_INLINE __host__ __device__ __forceinline__
#else
#define BN_HD
#define BN_INLINE inline __attribute__((always_inline))
#endif

// Layout of the pairing-path kernels: 1 = two lanes per element (fq2_split.h),
// 0 = one lane per element.  A pairing-path translation unit sets
// BN_SPLIT = BN_PATH_SPLIT before including kernels.h; every other unit
// (host side, group and codec kernels) keeps BN_SPLIT = 0.
#ifndef BN_PATH_SPLIT
#define BN_PATH_SPLIT 1
#endif

namespace bn {

#include "constants.inc"

constexpr uint32_t M29 = 0x1fffffffu;
struct Limbs9 {
    uint32_t v[9];
};
constexpr Limbs9 kP29 = {BN_P29};

// bound bookkeeping ------------------------------------------------------
// An Fq carries a compile-time bound code K = B + 256*(L-1):
//   B = value bound: value <= B*p (B <= 160, so value < 2^261);
//   L = digit bound: every digit < L*2^29 (L == 1: normalized).
// Additions, subtractions and small multiples leave digits unnormalized
// ("lazy", one VOP2 per digit) while L stays <= kMaxLimb; a Montgomery product
// accepts La*Lb <= 6 (its column sums stay below 2^64) and normalizes an
// operand first otherwise.  Normalized values have K == B, so plain bounds read
// as before.
// p / 2^261 < 0.005908 ; output of a Montgomery product of values <= A*p, <= B*p
// is <= (1 + A*B*p/R) * p.
constexpr int mul_bound(int A, int B) { return 1 + (int)(((long long)A * B * 5908 + 999999) / 1000000); }
constexpr int kMaxBound = 160;  // 160 * p < 2^261
constexpr int kMaxLimb = 7;     // digits < 7*2^29: a carry pass cannot overflow 32 bits
constexpr int kv(int K) { return K & 255; }
constexpr int kl(int K) { return (K >> 8) + 1; }
constexpr int kenc(int B, int L) { return B + 256 * (L - 1); }
constexpr int kjoin(int A, int B) {
    return kenc(kv(A) > kv(B) ? kv(A) : kv(B), kl(A) > kl(B) ? kl(A) : kl(B));
}

template <int K>
struct Fq {
    static_assert(kv(K) >= 1 && kv(K) <= kMaxBound, "Fq value bound out of range");
    static_assert(kl(K) >= 1 && kl(K) <= kMaxLimb, "Fq digit bound out of range");
    static constexpr int kK = K;  // the bound code, for static checks on deduced types
    uint32_t v[9];
};

// widen the static bound (free)
template <int K2, int K>
BN_INLINE Fq<K2> widen(const Fq<K>& a) {
    static_assert(kv(K) <= kv(K2) && kl(K) <= kl(K2), "widen: narrowing");
    Fq<K2> r;
#pragma unroll
    for (int i = 0; i < 9; ++i) r.v[i] = a.v[i];
    return r;
}

// Register fence: the digits pass through an empty volatile asm.  Work that
// consumes a fenced value cannot start before the fence and volatile asms keep
// program order, so fencing a product's inputs and its result serializes the
// products in program order.  This bounds the compiler's interleaving of
// independent products (which otherwise keeps dozens of partial products live
// and spills); it emits no instruction.
template <int B>
BN_INLINE void fq_fence(Fq<B>& a) {
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile("" : "+v"(a.v[0]), "+v"(a.v[1]), "+v"(a.v[2]), "+v"(a.v[3]), "+v"(a.v[4]), "+v"(a.v[5]),
                 "+v"(a.v[6]), "+v"(a.v[7]), "+v"(a.v[8]));
#else
    (void)a;
#endif
}

template <int B = 1>
BN_INLINE Fq<B> fq_from_limbs(const Limbs9& l) {
    Fq<B> r;
#pragma unroll
    for (int i = 0; i < 9; ++i) r.v[i] = l.v[i];
    return r;
}
BN_INLINE Fq<1> fq_zero() { return fq_from_limbs<1>(Limbs9{{0, 0, 0, 0, 0, 0, 0, 0, 0}}); }
BN_INLINE Fq<1> fq_one() { return fq_from_limbs<1>(Limbs9{BN_ONE}); }

// carry-propagate digits 0..7 into 8 (full-rate VOP2: lshr, and, add); the
// top digit stays < 2^29 because the value is < 2^261
template <int K>
BN_INLINE Fq<kv(K)> fq_norm(const Fq<K>& a) {
    Fq<kv(K)> r;
#pragma unroll
    for (int i = 0; i < 9; ++i) r.v[i] = a.v[i];
    if constexpr (kl(K) > 1) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            r.v[i + 1] += r.v[i] >> 29;
            r.v[i] &= M29;
        }
    }
    return r;
}

// a + b, lazy (arith.rs:281-287 computes the same residue)
template <int A, int B>
BN_INLINE auto fq_add(const Fq<A>& a, const Fq<B>& b) {
    if constexpr (kl(A) + kl(B) > kMaxLimb) {
        if constexpr (kl(A) >= kl(B)) return fq_add(fq_norm(a), b); else return fq_add(a, fq_norm(b));
    } else {
        Fq<kenc(kv(A) + kv(B), kl(A) + kl(B))> r;
#pragma unroll
        for (int i = 0; i < 9; ++i) r.v[i] = a.v[i] + b.v[i];
        return r;
    }
}
template <int B>
BN_INLINE auto fq_dbl(const Fq<B>& a) { return fq_add(a, a); }

// K*p with digits raised so that subtracting any value with digit bound L
// (digits < L*2^29) and value <= (K-1)*p leaves every digit non-negative:
// digit i gets +(L+1)*2^29 and digit i+1 pays -(L+1) (net zero), and the top
// digit keeps a margin of p/2^232 > 2^21 over the subtrahend's top digit.
// Digits of the result are < (L+2)*2^29.
constexpr Limbs9 kp_spread(int K, int L) {
    Limbs9 r = {{0, 0, 0, 0, 0, 0, 0, 0, 0}};
    unsigned long long c = 0;
    for (int i = 0; i < 9; ++i) {
        unsigned long long t = (unsigned long long)K * kP29.v[i] + c;
        r.v[i] = (uint32_t)(t & M29);
        c = t >> 29;
    }
    for (int i = 0; i < 8; ++i) {
        r.v[i] += (uint32_t)(L + 1) << 29;
        r.v[i + 1] -= (uint32_t)(L + 1);
    }
    return r;
}

// the normalized digits of K*p
constexpr Limbs9 kp_plain(int K) { return kp_spread(K, -1); }

// digit headroom kp_spread needs to subtract a value of digit bound L: one
// 2^29 per digit covers a normalized subtrahend (digits <= 2^29 - 1), else L
constexpr int sub_spread(int L) { return L == 1 ? 0 : L; }

// a - b + (B+1)*p, lazy (arith.rs:290-296 computes the same residue); digits
// < (La + sub_spread(Lb) + 2) * 2^29
template <int A, int B>
BN_INLINE auto fq_sub(const Fq<A>& a, const Fq<B>& b) {
    if constexpr (kl(A) + sub_spread(kl(B)) + 2 > kMaxLimb) {
        if constexpr (kl(A) >= kl(B)) return fq_sub(fq_norm(a), b); else return fq_sub(a, fq_norm(b));
    } else {
        constexpr Limbs9 Q = kp_spread(kv(B) + 1, sub_spread(kl(B)));
        Fq<kenc(kv(A) + kv(B) + 1, kl(A) + sub_spread(kl(B)) + 2)> r;
#pragma unroll
        for (int i = 0; i < 9; ++i) r.v[i] = (a.v[i] + Q.v[i]) - b.v[i];
        return r;
    }
}
// B*p - a, normalized, same bound (arith.rs:309-316: -0 stays 0, and B*p == 0 mod p)
template <int K>
BN_INLINE Fq<kv(K)> fq_neg(const Fq<K>& a_in) {
    const Fq<kv(K)> a = fq_norm(a_in);
    constexpr int B = kv(K);
    // K*p with digits 0..7 raised into [2^29-1, 2^30); the top digit is taken
    // modulo 2^32 and is right after the carry pass because the total is >= 0
    constexpr Limbs9 Q = kp_spread(B, 0);
    Fq<B> r;
#pragma unroll
    for (int i = 0; i < 9; ++i) r.v[i] = Q.v[i] - a.v[i];
    return fq_norm(Fq<kenc(B, 2)>{{r.v[0], r.v[1], r.v[2], r.v[3], r.v[4], r.v[5], r.v[6], r.v[7], r.v[8]}});
}

// Sticky device error bits (bn_status codes as bit numbers) of a call: the word
// is global memory (the context's d_err), so the OR goes through a global-space
// pointer -- a generic-pointer atomicOr gets an aperture test from the backend,
// which in kernels_pairing.hip it emitted as an illegal VOPC ("Operand has
// incorrect register class", V_CMP_NE_U32_e32 0, src_shared_base) as soon as the
// unit's code changed (the fold-check build in rounds 3-4, the column-sum asm).
#if defined(__HIPCC__)
__device__ __forceinline__ void err_or(int* err, int bit) {
    __hip_atomic_fetch_or((__attribute__((address_space(1))) int*)err, 1 << bit, __ATOMIC_RELAXED,
                          __HIP_MEMORY_SCOPE_AGENT);
}
#endif

// ---------------------------------------------------------------- single-chain column sums
// BN_DOT2_ASM (device code, on by default): fq_mul, fq_sqr and fq2_split.h
// fq_dot2 run the hand-scheduled product scan of dot2_asm.inc
// (tools/gen_dot2_asm.py): one v_mad_u64_u32 chain per product, each column
// started from the previous column's carry, so no carry-merge instruction per
// column (the compiler's schedule starts each column as its own chain and adds
// the carry with a v_lshl_add_u64: 16 per product, 3,748 in k_pairing_full).  A
// dependent v_mad_u64_u32 issues as fast as an independent one on gfx950
// (profiles/r3j_mad_issue.txt).  The same column sums in another association
// order: identical digits.  Measured (profiles/r5b_ab_dot2_asm.txt, two
// interleaved rounds): k_pairing_full 7.75 -> 7.60 ms, config 5 2.17 -> 2.08-2.12
// ms, G2 * Fr 6.19 -> 5.92 ms, config 3 8.11 -> 7.64 ms.  BN_DOT2_ASM=0 builds
// the compiler's form (host builds always use it).
// Bits: 1 = fq_dot2, 2 = fq_mul, 4 = fq_sqr.
#ifndef BN_DOT2_ASM
#define BN_DOT2_ASM 7
#endif
#if BN_DOT2_ASM && defined(__HIP_DEVICE_COMPILE__)
#include "dot2_asm.inc"
#define BN_ASM_OUT9(a) "=&v"(a[0]), "=&v"(a[1]), "=&v"(a[2]), "=&v"(a[3]), "=&v"(a[4]), "=&v"(a[5]), \
                       "=&v"(a[6]), "=&v"(a[7]), "=&v"(a[8])
#define BN_ASM_IN9(a) "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]), "v"(a[5]), "v"(a[6]), "v"(a[7]), "v"(a[8])
#define BN_ASM_P                                                                                              \
    "s"(kP29.v[0]), "s"(kP29.v[1]), "s"(kP29.v[2]), "s"(kP29.v[3]), "s"(kP29.v[4]), "s"(kP29.v[5]),        \
        "s"(kP29.v[6]), "s"(kP29.v[7]), "s"(kP29.v[8]), "s"((uint32_t)BN_PINV29)
#define BN_ASM_CLOBBER "vcc", "v2", "v3"
#endif

// ---------------------------------------------------------------- column accumulator
// The digit products of several Fq products summed by columns in 17 64-bit
// accumulators and reduced once (fq12_wide.h's twelve-product sums).  Measured
// (profiles/r2n_wide_ubench_latency_forms.jsonl): for a SINGLE product this form is not
// faster than the product-scanning fq_mul even on a lone wave (0.67 vs 0.62 us
// per product in an inversion chain), so fq_mul keeps product scanning.
struct Acc {
    uint64_t c[17];
};
// t += x * y by columns: every column gains at most nine products < 2^58
template <int A, int B>
BN_INLINE void acc_mad(Acc& t, const Fq<A>& x, const Fq<B>& y) {
    static_assert(kl(A) == 1 && kl(B) == 1, "acc_mad: normalized operands");
#pragma unroll
    for (int i = 0; i < 9; ++i)
#pragma unroll
        for (int j = 0; j < 9; ++j) t.c[i + j] += (uint64_t)x.v[i] * y.v[j];
}
// one carry step on every column at once (independent, not a ripple): columns
// end below 2^29 + 2^35, room for 54 more products before a reduction
BN_INLINE void acc_carry_par(Acc& t) {
    uint64_t h[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        h[k] = t.c[k] >> 29;
        t.c[k] &= M29;
    }
#pragma unroll
    for (int k = 0; k < 16; ++k) t.c[k + 1] += h[k];
}
// Montgomery reduction (R = 2^261) of the columns; each column plus the nine
// m*p products it receives and a carry < 2^36 must stay below 2^64 (at most 54
// products < 2^58 since the last acc_carry_par, or 54 in all).  BO: the
// caller's output bound.
template <int BO>
BN_INLINE Fq<BO> acc_redc(Acc& t) {
    Fq<BO> r;
#pragma unroll
    for (int k = 0; k < 9; ++k) {
        if (k) t.c[k] += t.c[k - 1] >> 29;
        const uint32_t m = ((uint32_t)t.c[k] * BN_PINV29) & M29;
#pragma unroll
        for (int j = 0; j < 9; ++j) t.c[k + j] += (uint64_t)m * kP29.v[j];
    }
    t.c[9] += t.c[8] >> 29;
#pragma unroll
    for (int k = 9; k < 16; ++k) {
        r.v[k - 9] = (uint32_t)t.c[k] & M29;
        t.c[k + 1] += t.c[k] >> 29;
    }
    r.v[7] = (uint32_t)t.c[16] & M29;
    r.v[8] = (uint32_t)(t.c[16] >> 29);
    return r;
}
// a * b * 2^-261 mod p: Montgomery product by finely integrated product
// scanning.  Column k accumulates every a_i*b_j and m_i*p_j with i+j == k in a
// 64-bit accumulator (9 products < La*Lb*2^58, 9 < 2^58 and the carry-in stay
// below 2^64 when La*Lb <= 6), derives m_k = acc * (-p^-1) mod 2^29 for k < 9
// so the low digit cancels, then shifts by 29.  hipcc emits one v_mad_u64_u32
// per product.  The result is normalized.
template <int A, int B>
BN_INLINE auto fq_mul(const Fq<A>& a_in, const Fq<B>& b_in) {
    if constexpr (kl(A) * kl(B) > 6) {
        if constexpr (kl(A) >= kl(B)) return fq_mul(fq_norm(a_in), b_in); else return fq_mul(a_in, fq_norm(b_in));
    } else {
    static_assert((long long)kv(A) * kv(B) <= 160 * 160, "product bound");
    const Fq<A>& a = a_in;
    const Fq<B>& b = b_in;
    Fq<mul_bound(kv(A), kv(B))> r;
#if BN_DOT2_ASM && defined(__HIP_DEVICE_COMPILE__)
    if constexpr ((BN_DOT2_ASM & 2) != 0) {
        asm(BN_ASM_MUL : BN_ASM_OUT9(r.v) : BN_ASM_IN9(a.v), BN_ASM_IN9(b.v), BN_ASM_P : BN_ASM_CLOBBER);
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
            acc += (uint64_t)a.v[i] * b.v[k - i];
            if (i < k) acc += (uint64_t)m[i] * kP29.v[k - i];
        }
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
}
// a^2 * 2^-261 mod p: fq_mul's column scan with each cross product a_i*a_j
// (i < j) taken once against the doubled digit 2*a_j, so a column holds at most
// four cross products (< 2L^2 * 2^58 each), one square and nine m*p terms:
// 45 + 81 digit products instead of 81 + 81.  The same residue as fq_mul(a, a).
template <int B>
BN_INLINE auto fq_sqr(const Fq<B>& a_in) {
    if constexpr (kl(B) > 2) {
        return fq_sqr(fq_norm(a_in));
    } else {
    static_assert((long long)kv(B) * kv(B) <= 160 * 160, "product bound");
    static_assert(kl(B) * kl(B) * 9 + 9 + 1 < 64, "fq_sqr: column sum could overflow 64 bits");
    const Fq<B>& a = a_in;
    uint32_t d[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) d[i] = a.v[i] << 1;
    Fq<mul_bound(kv(B), kv(B))> r;
#if BN_DOT2_ASM && defined(__HIP_DEVICE_COMPILE__)
    if constexpr ((BN_DOT2_ASM & 4) != 0) {
        asm(BN_ASM_SQR : BN_ASM_OUT9(r.v) : BN_ASM_IN9(a.v), BN_ASM_IN9(d), BN_ASM_P : BN_ASM_CLOBBER);
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
            const int j = k - i;
            if (i < j) acc += (uint64_t)a.v[i] * d[j];
            else if (i == j) acc += (uint64_t)a.v[i] * a.v[i];
            if (i < k) acc += (uint64_t)m[i] * kP29.v[k - i];
        }
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
}

// bring any value back to bound 2 (a Montgomery product with one)
template <int B>
BN_INLINE auto fq_reduce(const Fq<B>& a) { return fq_mul(a, fq_one()); }

// x * c for a small constant c, lazy while the digits stay < 7*2^29; c == 8
// on a normalized value (digits < 2^32) is carried at once
template <int C, int B>
BN_INLINE auto fq_mul_small(const Fq<B>& a) {
    static_assert(C >= 1 && C <= 8, "digit * C must fit 32 bits");
    if constexpr (kl(B) > 1 && C * kl(B) > kMaxLimb) {
        return fq_mul_small<C>(fq_norm(a));
    } else if constexpr (C * kl(B) > kMaxLimb) {  // C == 8, normalized input
        Fq<C * kv(B)> o;
#pragma unroll
        for (int i = 0; i < 9; ++i) o.v[i] = a.v[i] * C;  // <= 8*(2^29-1): the carries fit
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            o.v[i + 1] += o.v[i] >> 29;
            o.v[i] &= M29;
        }
        return o;
    } else {
        Fq<kenc(C * kv(B), C * kl(B))> r;
#pragma unroll
        for (int i = 0; i < 9; ++i) r.v[i] = a.v[i] * C;
        return r;
    }
}

// x / 2 mod p, the residue of x * two_inv (groups/mod.rs:521-528) without a
// product: add p when x is odd (after normalizing), carry, then shift every
// digit right by one bit, taking the low bit of the next digit.  A value
// <= B*p becomes <= (B+1)/2 * p.
template <int K>
BN_INLINE auto fq_half(const Fq<K>& a_in) {
    constexpr int B = kv(K);
    static_assert(B + 1 <= 161, "fq_half: x + p must stay below 2^261");
    const Fq<B> a = fq_norm(a_in);
    const uint32_t mask = 0u - (a.v[0] & 1u);
    uint32_t t[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) t[i] = a.v[i] + (kP29.v[i] & mask);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        t[i + 1] += t[i] >> 29;
        t[i] &= M29;
    }
    Fq<(B + 2) / 2> r;
#pragma unroll
    for (int i = 0; i < 8; ++i) r.v[i] = (t[i] >> 1) | ((t[i + 1] & 1u) << 28);
    r.v[8] = t[8] >> 1;
    return r;
}

// Partial reduction to bound 2 without a multiplication: estimate
// q <= floor(x/p) from the top digit (x8 * 2^232 / p, computed in f32 with a
// constant rounded 2^-18 low so the estimate never overshoots), then x - q*p.
// About a fifth of a Montgomery product; used where bounds would otherwise grow.
//
// With BN_FOLD_LDS (device code of a translation unit that defines it, and
// whose kernels call fold_table_init() first), -q*p comes from a 161-entry
// table in LDS as eight 29-bit digits plus a signed top digit, so the fold is
// one add3/shift/and carry pass: ~32 instructions instead of ~58.
#ifndef BN_FOLD_LDS
#define BN_FOLD_LDS 0
#endif
// Diagnostic build (-DBN_DEVICE_CHECKS=1, `make -C paritytech-bn_amd dbg`):
// every device fold counts the lanes whose quotient estimate exceeds the
// static bound of its input (q <= kv(B) <= kMaxBound is what makes the LDS
// table index and the subtraction safe); kernels.h exports the per-TU counter
// as bn_dbg_fold_bad_<tu>(), read by tools/fold_check.py.
#ifndef BN_DEVICE_CHECKS
#define BN_DEVICE_CHECKS 0
#endif
#if BN_DEVICE_CHECKS && defined(__HIPCC__)
static __device__ unsigned g_fold_bad;
// The counter is bumped in a function of its own: with the atomic inlined into
// every fold, the backend emitted an illegal VOPC for kernels_pairing.hip
// ("Operand has incorrect register class", V_CMP_NE_U32_e32 0, src_shared_base),
// which kept that unit out of the checked build in rounds 3-4.
static __device__ __noinline__ void fold_bad_hit() {
    __hip_atomic_fetch_add((__attribute__((address_space(1))) unsigned*)&g_fold_bad, 1u, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}
#define BN_FOLD_CHECK(q, B)                                \
    do {                                                   \
        if ((q) > (uint32_t)kv(B)) fold_bad_hit();         \
    } while (0)
#else
#define BN_FOLD_CHECK(q, B) ((void)0)
#endif
#if BN_FOLD_LDS
constexpr int kFoldQ = kMaxBound + 1;  // q <= x8 * 2^232/p < 161
constexpr int kFoldStride = 12;        // words per entry: 16-byte aligned rows
alignas(16) __shared__ uint32_t g_fold_tab[kFoldQ * kFoldStride];
// every thread of the block must call this before the first fold
__device__ __forceinline__ void fold_table_init() {
    for (int q = threadIdx.x; q < kFoldQ; q += blockDim.x) {
        int64_t carry = 0;
        for (int i = 0; i < 8; ++i) {
            const int64_t t = carry - (int64_t)q * kP29.v[i];
            g_fold_tab[q * kFoldStride + i] = (uint32_t)t & M29;
            carry = t >> 29;
        }
        g_fold_tab[q * kFoldStride + 8] = (uint32_t)(carry - (int64_t)q * kP29.v[8]);  // signed top digit
    }
    __syncthreads();
}
// two phases, so that a caller folding several values issues every table read
// before the first use (one wave per SIMD cannot hide an LDS round trip)
struct FoldEnt {
    uint4 a, b;
    uint32_t c;
};
template <int B>
__device__ __forceinline__ FoldEnt fold_fetch(const Fq<B>& x) {
    static_assert(kl(B) <= 6, "fold_fetch: normalize first");
    const uint32_t q = (uint32_t)((float)x.v[8] * 3.1531629e-07f);  // as fq_fold
#if defined(__HIP_DEVICE_COMPILE__)
    BN_FOLD_CHECK(q, B);
#endif
    const uint32_t* e = g_fold_tab + q * kFoldStride;
    return FoldEnt{*(const uint4*)e, *(const uint4*)(e + 4), e[8]};
}
template <int B>
__device__ __forceinline__ Fq<2> fold_apply(const Fq<B>& x, const FoldEnt& f) {
    const uint32_t t[9] = {f.a.x, f.a.y, f.a.z, f.a.w, f.b.x, f.b.y, f.b.z, f.b.w, f.c};
    Fq<2> r;
    uint32_t carry = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const uint32_t s = x.v[i] + t[i] + carry;
        r.v[i] = s & M29;
        carry = s >> 29;
    }
    r.v[8] = x.v[8] + t[8] + carry;  // x - q*p >= 0: exact modulo 2^32
    return r;
}
#else
BN_INLINE void fold_table_init() {}
#endif

template <int B>
BN_INLINE Fq<2> fq_fold(const Fq<B>& x) {
    const float c = 3.1531629e-07f;  // < 2^232/p * (1 - 2^-18)
#if BN_FOLD_LDS && defined(__HIP_DEVICE_COMPILE__)
    if constexpr (kl(B) > 6) {
        return fq_fold(fq_norm(x));  // x_i + t_i + carry must stay below 2^32
    } else {
        return fold_apply(x, fold_fetch(x));
    }
#endif
    const uint32_t q = (uint32_t)((float)x.v[8] * c);
#if defined(BN_HOST_CHECKS) && !defined(__HIP_DEVICE_COMPILE__)
    if (q > (uint32_t)kv(B)) {  // the value exceeds its static bound B*p
        fprintf(stderr, "fq_fold: q = %u > bound %d\n", q, kv(B));
        abort();
    }
#endif
#if defined(__HIP_DEVICE_COMPILE__)
    BN_FOLD_CHECK(q, B);
#endif
    Fq<2> r;
    int64_t carry = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        int64_t t = (int64_t)x.v[i] - (int64_t)((uint64_t)q * kP29.v[i]) + carry;
        r.v[i] = (uint32_t)t & M29;
        carry = t >> 29;
    }
    r.v[8] = (uint32_t)((int64_t)x.v[8] - (int64_t)((uint64_t)q * kP29.v[8]) + carry);
    return r;
}

// select (per lane)
template <int B>
BN_INLINE Fq<B> fq_select(bool c, const Fq<B>& a, const Fq<B>& b) {
    Fq<B> r;
#pragma unroll
    for (int i = 0; i < 9; ++i) r.v[i] = c ? a.v[i] : b.v[i];
    return r;
}

// ---------------------------------------------------------------- canonical forms
// subtract p once if value >= p (input value < 2p)
BN_INLINE Fq<1> fq_cond_sub_p(const Fq<2>& x) {
    uint32_t d[9];
    int32_t borrow = 0;
#pragma unroll
    for (int i = 0; i < 9; ++i) {
        int32_t t = (int32_t)x.v[i] - (int32_t)kP29.v[i] + borrow;
        borrow = t >> 29;  // arithmetic: -1 on borrow
        d[i] = (uint32_t)t & M29;
    }
    const bool ge = borrow == 0;  // x - p >= 0
    Fq<1> r;
#pragma unroll
    for (int i = 0; i < 9; ++i) r.v[i] = ge ? d[i] : x.v[i];
    return r;
}
// the unique representative in [0, p) of the same internal value (X mod p)
template <int B>
BN_INLINE Fq<1> fq_canonical(const Fq<B>& a) {
    return fq_cond_sub_p(widen<2>(fq_reduce(a)));
}
// a == 0 (mod p) without a product: the fold leaves a normalized value
// x <= 2p with the same residue, and x == 0 (mod p) iff x is 0, p or 2p (three
// digit-wise compares; about half the instructions of fq_canonical's REDC)
template <int B>
BN_INLINE bool fq_is_zero(const Fq<B>& a) {
    const Fq<2> x = fq_fold(a);
    constexpr Limbs9 P1 = kp_plain(1), P2 = kp_plain(2);
    uint32_t o0 = 0, o1 = 0, o2 = 0;
#pragma unroll
    for (int i = 0; i < 9; ++i) {
        o0 |= x.v[i];
        o1 |= x.v[i] ^ P1.v[i];
        o2 |= x.v[i] ^ P2.v[i];
    }
    return (o0 == 0) | (o1 == 0) | (o2 == 0);
}
template <int A, int B>
BN_INLINE bool fq_eq(const Fq<A>& a, const Fq<B>& b) {
    return fq_is_zero(fq_sub(a, b));
}

// ---------------------------------------------------------------- boundary
// The reference memory image of an Fq: x*2^256 mod p, canonical, as eight
// little-endian 32-bit words (== four u64 limbs == U256([u128;2])).
BN_INLINE Fq<1> fq_digits_from_words(const uint32_t w[8]) {
    Fq<1> r;  // plain repacking of a 256-bit integer into 29-bit digits
#pragma unroll
    for (int i = 0; i < 9; ++i) {
        const int bit = 29 * i, j = bit >> 5, s = bit & 31;
        uint64_t lo = w[j];
        uint64_t hi = (j + 1 < 8) ? w[j + 1] : 0;
        r.v[i] = (uint32_t)(((hi << 32 | lo) >> s) & M29);
    }
    return r;
}
BN_INLINE void fq_words_from_digits(const Fq<1>& a, uint32_t w[8]) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int bit = 32 * j, i = bit / 29, s = bit % 29;
        uint64_t v = (uint64_t)a.v[i] >> s;
        if (i + 1 < 9) v |= (uint64_t)a.v[i + 1] << (29 - s);
        if (i + 2 < 9 && 58 - s < 32) v |= (uint64_t)a.v[i + 2] << (58 - s);
        w[j] = (uint32_t)v;
    }
}
// reference image (canonical x*2^256 mod p) -> internal
BN_INLINE Fq<2> fq_load_ref(const uint32_t w[8]) {
    return fq_mul(fq_digits_from_words(w), fq_from_limbs<1>(Limbs9{BN_TO_INTERNAL}));
}
// internal -> reference image, canonical
template <int B>
BN_INLINE void fq_store_ref(const Fq<B>& a, uint32_t w[8]) {
    Fq<1> c = fq_cond_sub_p(widen<2>(fq_mul(a, fq_from_limbs<1>(Limbs9{BN_TO_REF}))));
    fq_words_from_digits(c, w);
}
// canonical plain integer -> internal
BN_INLINE Fq<2> fq_from_canonical_words(const uint32_t w[8]) {
    return fq_mul(fq_digits_from_words(w), fq_from_limbs<1>(Limbs9{BN_FROM_CANON}));
}

}  // namespace bn
