/*
 * bn_oracle.c -- CPU restatement of substrate-bn 0.6.0 (risc0/paritytech-bn)
 * for the BN254 pairing hot path.  TEST INFRASTRUCTURE ONLY (see bn_oracle.h).
 *
 * Faithful to the reference algorithms, function by function:
 *   - 256-bit integers held as two u128 digits, Montgomery multiplication by
 *     HAC 14.32 with u128 digits (src/arith.rs:473-545), one conditional
 *     subtraction (src/arith.rs:300-306);
 *   - binary extended-Euclid inversion (src/arith.rs:324-370) then x R^3
 *     (src/fields/fp.rs:108-117);
 *   - the Fq2/Fq6/Fq12 formulas as written, including the multiplications by
 *     the non-residues (src/fields/fq2.rs, fq6.rs, fq12.rs);
 *   - Jacobian group law, double-and-add scalar multiplication, the flipped
 *     Miller-loop line precomputation, the Miller loop and the final
 *     exponentiation (src/groups/mod.rs).
 * Being the same algorithm, it is also the "port" CPU baseline bench.py times.
 */
#include "bn_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

typedef unsigned __int128 u128;
typedef struct { u128 d[2]; } u256;                 /* src/arith.rs:9-11 */

#define M64 ((u128)0xFFFFFFFFFFFFFFFFull)
static inline u256 U(uint64_t a, uint64_t b, uint64_t c, uint64_t d) { /* arith.rs:13-20 */
    u256 r;
    r.d[0] = ((u128)b << 64) | a;
    r.d[1] = ((u128)d << 64) | c;
    return r;
}

/* ------------------------------------------------------------------ */
/* field parameters: field_impl! instantiations, src/fields/fp.rs:166-222 */
typedef struct { u256 m, r2, r3, one; u128 inv; } fparams;
static fparams FQP, FRP;
static pthread_once_t params_once = PTHREAD_ONCE_INIT;
static void init_params(void) {
    FQP.m = U(0x3c208c16d87cfd47ull, 0x97816a916871ca8dull, 0xb85045b68181585dull, 0x30644e72e131a029ull);
    FQP.r2 = U(0xf32cfc5b538afa89ull, 0xb5e71911d44501fbull, 0x47ab1eff0a417ff6ull, 0x06d89f71cab8351full);
    FQP.r3 = U(0xb1cd6dafda1530dfull, 0x62f210e6a7283db6ull, 0xef7f0b0c0ada0afbull, 0x20fd6e902d592544ull);
    FQP.one = U(0xd35d438dc58f0d9dull, 0x0a78eb28f5c70b3dull, 0x666ea36f7879462cull, 0x0e0a77c19a07df2full);
    FQP.inv = ((u128)0x9ede7d651eca6ac9ull << 64) | 0x87d20782e4866389ull;
    FRP.m = U(0x43e1f593f0000001ull, 0x2833e84879b97091ull, 0xb85045b68181585dull, 0x30644e72e131a029ull);
    FRP.r2 = U(0x1bb8e645ae216da7ull, 0x53fe3ab1e35c59e3ull, 0x8c49833d53bb8085ull, 0x0216d0b17f4e44a5ull);
    FRP.r3 = U(0x5e94d8e1b4bf0040ull, 0x2a489cbe1cfbb6b8ull, 0x893cc664a19fcfedull, 0x0cf8594b7fcc657cull);
    FRP.one = U(0xac96341c4ffffffbull, 0x36fc76959f60cd29ull, 0x666ea36f7879462eull, 0x0e0a77c19a07df2full);
    FRP.inv = ((u128)0x6586864b4c6911b3ull << 64) | 0xc2e1f593efffffffull;
}
static inline const fparams* FP(int field) {
    pthread_once(&params_once, init_params);
    return field ? &FRP : &FQP;
}
#define FQ (&FQP)

/* ------------------------------------------------------------------ */
/* U256 helpers: src/arith.rs:172-192, 248-250, 398-469 */
static inline int u256_cmp(const u256* a, const u256* b) {
    for (int i = 1; i >= 0; --i) {
        if (a->d[i] < b->d[i]) return -1;
        if (a->d[i] > b->d[i]) return 1;
    }
    return 0;
}
static inline int u256_is_zero(const u256* a) { return a->d[0] == 0 && a->d[1] == 0; }
static inline int u256_eq(const u256* a, const u256* b) { return a->d[0] == b->d[0] && a->d[1] == b->d[1]; }

static inline u128 adc(u128 a, u128 b, u128* carry) {          /* arith.rs:427-435 */
    u128 lo = (a & M64) + (b & M64) + *carry;
    u128 hi = (a >> 64) + (b >> 64) + (lo >> 64);
    *carry = hi >> 64;
    return (hi << 64) | (lo & M64);
}
static inline void add_nocarry(u128 a[2], const u128 b[2]) {   /* arith.rs:437-446 */
    u128 carry = 0;
    for (int i = 0; i < 2; ++i) a[i] = adc(a[i], b[i], &carry);
}
static inline u128 sbb(u128 a, u128 b, u128* borrow) {         /* arith.rs:450-460 */
    u128 one64 = (u128)1 << 64;
    u128 t0 = one64 + (a & M64) - (b & M64) - *borrow;
    u128 b0 = t0 >> 64, r0 = t0 & M64;
    u128 t1 = one64 + (a >> 64) - (b >> 64) - (b0 == 0);
    u128 b1 = t1 >> 64, r1 = t1 & M64;
    *borrow = (b1 == 0);
    return (r1 << 64) | r0;
}
static inline void sub_noborrow(u128 a[2], const u128 b[2]) {  /* arith.rs:448-469 */
    u128 borrow = 0;
    for (int i = 0; i < 2; ++i) a[i] = sbb(a[i], b[i], &borrow);
}
static inline void div2(u128 a[2]) {                           /* arith.rs:399-405 */
    u128 tmp = a[1] << 127;
    a[1] >>= 1;
    a[0] >>= 1;
    a[0] |= tmp;
}

/* mac_with_carry / mac_digit: arith.rs:473-522 */
static inline u128 mac_with_carry(u128 a, u128 b, u128 c, u128* carry) {
    u128 b_hi = b >> 64, b_lo = b & M64, c_hi = c >> 64, c_lo = c & M64;
    u128 a_hi = a >> 64, a_lo = a & M64;
    u128 carry_hi = *carry >> 64, carry_lo = *carry & M64;
    u128 x = b_lo * c_lo + a_lo + carry_lo;
    u128 x_hi = x >> 64, x_lo = x & M64;
    u128 y = b_lo * c_hi;
    u128 y_hi = y >> 64, y_lo = y & M64;
    u128 z = b_hi * c_lo;
    u128 z_hi = z >> 64, z_lo = z & M64;
    u128 r = (x_hi + y_lo) + (z_lo + a_hi) + carry_hi;
    u128 r_hi = r >> 64, r_lo = r & M64;
    *carry = (b_hi * c_hi) + r_hi + y_hi + z_hi;
    return (r_lo << 64) | x_lo;
}
static inline void mac_digit(int from_index, u128 acc[4], const u128 b[2], u128 c) {
    if (c == 0) return;
    u128 carry = 0;
    for (int i = 0; i < 2; ++i) {
        int ai = i + from_index;
        acc[ai] = mac_with_carry(acc[ai], b[i], c, &carry);
    }
    for (int i = 0; i < 2; ++i) {
        int ai = i + from_index + 2;
        if (ai < 4) {
            u128 a_hi = acc[ai] >> 64, a_lo = acc[ai] & M64;
            u128 carry_hi = carry >> 64, carry_lo = carry & M64;
            u128 x = a_lo + carry_lo;
            u128 r = (x >> 64) + a_hi + carry_hi;
            carry = r >> 64;
            acc[ai] = ((r & M64) << 64) | (x & M64);
        }
    }
}
static inline void mul_reduce(u128 this_[2], const u128 by[2], const u128 modulus[2], u128 inv) {
    /* HAC 14.32, arith.rs:525-545 */
    u128 res[4] = {0, 0, 0, 0};
    for (int i = 0; i < 2; ++i) mac_digit(i, res, by, this_[i]);
    for (int i = 0; i < 2; ++i) {
        u128 k = inv * res[i];
        mac_digit(i, res, modulus, k);
    }
    this_[0] = res[2];
    this_[1] = res[3];
}

/* modular U256 ops: arith.rs:280-316 */
static inline void u256_add(u256* a, const u256* b, const u256* m) {
    add_nocarry(a->d, b->d);
    if (u256_cmp(a, m) >= 0) sub_noborrow(a->d, m->d);
}
static inline void u256_sub(u256* a, const u256* b, const u256* m) {
    if (u256_cmp(a, b) < 0) add_nocarry(a->d, m->d);
    sub_noborrow(a->d, b->d);
}
static inline void u256_mul(u256* a, const u256* b, const u256* m, u128 inv) {
    mul_reduce(a->d, b->d, m->d, inv);
    if (u256_cmp(a, m) >= 0) sub_noborrow(a->d, m->d);
}
static inline void u256_neg(u256* a, const u256* m) {
    if (!u256_is_zero(a)) {
        u256 tmp = *m;
        sub_noborrow(tmp.d, a->d);
        *a = tmp;
    }
}
static void u256_invert(u256* self, const u256* modulo) {      /* arith.rs:324-370 */
    u256 u = *self, v = *modulo, b = U(1, 0, 0, 0), c = U(0, 0, 0, 0);
    const u256 one = U(1, 0, 0, 0);
    while (!u256_eq(&u, &one) && !u256_eq(&v, &one)) {
        while ((u.d[0] & 1) == 0) {
            div2(u.d);
            if ((b.d[0] & 1) == 0) {
                div2(b.d);
            } else {
                add_nocarry(b.d, modulo->d);
                div2(b.d);
            }
        }
        while ((v.d[0] & 1) == 0) {
            div2(v.d);
            if ((c.d[0] & 1) == 0) {
                div2(c.d);
            } else {
                add_nocarry(c.d, modulo->d);
                div2(c.d);
            }
        }
        if (u256_cmp(&u, &v) >= 0) {
            sub_noborrow(u.d, v.d);
            u256_sub(&b, &c, modulo);
        } else {
            sub_noborrow(v.d, u.d);
            u256_sub(&c, &b, modulo);
        }
    }
    *self = u256_eq(&u, &one) ? b : c;
}

/* ------------------------------------------------------------------ */
/* Fp (field_impl!): src/fields/fp.rs:7-164 */
typedef u256 fe;
static inline fe fe_add(fe a, fe b, const fparams* P) { u256_add(&a, &b, &P->m); return a; }
static inline fe fe_sub(fe a, fe b, const fparams* P) { u256_sub(&a, &b, &P->m); return a; }
static inline fe fe_mul(fe a, fe b, const fparams* P) { u256_mul(&a, &b, &P->m, P->inv); return a; }
static inline fe fe_neg(fe a, const fparams* P) { u256_neg(&a, &P->m); return a; }
static inline int fe_is_zero(fe a) { return u256_is_zero(&a); }
static inline int fe_eq(fe a, fe b) { return u256_eq(&a, &b); }
static inline fe fe_zero(void) { return U(0, 0, 0, 0); }
static inline fe fe_one(const fparams* P) { return P->one; }
static int fe_inverse(fe* a, const fparams* P) {               /* fp.rs:108-117 */
    if (fe_is_zero(*a)) return 1;
    u256_invert(a, &P->m);
    u256_mul(a, &P->r3, &P->m, P->inv);
    return 0;
}
static inline fe fe_squared(fe a, const fparams* P) { return fe_mul(a, a, P); } /* fields/mod.rs:31 */

static inline fe K(uint64_t a, uint64_t b, uint64_t c, uint64_t d) { return U(a, b, c, d); } /* const_fq */

/* ------------------------------------------------------------------ */
/* Fq2 = Fq[u]/(u^2 + 1): src/fields/fq2.rs */
typedef struct { fe c0, c1; } fq2;
static inline fe fq_non_residue(void) {                        /* fq2.rs:7-16 */
    return K(0x68c3488912edefaaull, 0x8d087f6872aabf4full, 0x51e1a24709081231ull, 0x2259d6b14729c0faull);
}
static inline fq2 F2(fe a, fe b) { fq2 r = {a, b}; return r; }
static inline fq2 fq2_nonresidue(void) {                       /* fq2.rs:19-34 */
    return F2(K(0xf60647ce410d7ff7ull, 0x2f3d6f4dd31bd011ull, 0x2943337e3940c6d1ull, 0x1d9598e8a7e39857ull),
              K(0xd35d438dc58f0d9dull, 0x0a78eb28f5c70b3dull, 0x666ea36f7879462cull, 0x0e0a77c19a07df2full));
}
static inline fq2 fq2_zero(void) { return F2(fe_zero(), fe_zero()); }
static inline fq2 fq2_one(void) { return F2(FQ->one, fe_zero()); }
static inline int fq2_is_zero(fq2 a) { return fe_is_zero(a.c0) && fe_is_zero(a.c1); }
static inline int fq2_eq(fq2 a, fq2 b) { return fe_eq(a.c0, b.c0) && fe_eq(a.c1, b.c1); }
static inline fq2 fq2_add(fq2 a, fq2 b) { return F2(fe_add(a.c0, b.c0, FQ), fe_add(a.c1, b.c1, FQ)); }
static inline fq2 fq2_sub(fq2 a, fq2 b) { return F2(fe_sub(a.c0, b.c0, FQ), fe_sub(a.c1, b.c1, FQ)); }
static inline fq2 fq2_neg(fq2 a) { return F2(fe_neg(a.c0, FQ), fe_neg(a.c1, FQ)); }
static inline fq2 fq2_scale(fq2 a, fe by) { return F2(fe_mul(a.c0, by, FQ), fe_mul(a.c1, by, FQ)); }
static inline fq2 fq2_mul(fq2 a, fq2 b) {                      /* fq2.rs:136-148 */
    fe aa = fe_mul(a.c0, b.c0, FQ);
    fe bb = fe_mul(a.c1, b.c1, FQ);
    return F2(fe_add(fe_mul(bb, fq_non_residue(), FQ), aa, FQ),
              fe_sub(fe_sub(fe_mul(fe_add(a.c0, a.c1, FQ), fe_add(b.c0, b.c1, FQ), FQ), aa, FQ), bb, FQ));
}
static inline fq2 fq2_squared(fq2 a) {                         /* fq2.rs:105-117 */
    fe ab = fe_mul(a.c0, a.c1, FQ);
    fe t = fe_mul(fe_add(fe_mul(a.c1, fq_non_residue(), FQ), a.c0, FQ), fe_add(a.c0, a.c1, FQ), FQ);
    return F2(fe_sub(fe_sub(t, ab, FQ), fe_mul(ab, fq_non_residue(), FQ), FQ), fe_add(ab, ab, FQ));
}
static inline fq2 fq2_mul_by_nonresidue(fq2 a) { return fq2_mul(a, fq2_nonresidue()); } /* fq2.rs:55-57 */
static inline fq2 fq2_frobenius_map(fq2 a, int power) {        /* fq2.rs:59-68 */
    if (power % 2 == 0) return a;
    return F2(a.c0, fe_mul(a.c1, fq_non_residue(), FQ));
}
static int fq2_inverse(fq2 a, fq2* out) {                      /* fq2.rs:119-130 */
    fe t = fe_sub(fe_squared(a.c0, FQ), fe_mul(fe_squared(a.c1, FQ), fq_non_residue(), FQ), FQ);
    if (fe_inverse(&t, FQ)) return 1;
    *out = F2(fe_mul(a.c0, t, FQ), fe_neg(fe_mul(a.c1, t, FQ), FQ));
    return 0;
}

/* ------------------------------------------------------------------ */
/* Fq6 = Fq2[v]/(v^3 - xi): src/fields/fq6.rs */
typedef struct { fq2 c0, c1, c2; } fq6;
static inline fq6 F6(fq2 a, fq2 b, fq2 c) { fq6 r = {a, b, c}; return r; }
static fq2 fq6_frob_c1(int n) {                                /* fq6.rs:5-47 */
    switch (n % 6) {
    case 0: return fq2_one();
    case 1: return F2(K(13075984984163199792ull, 3782902503040509012ull, 8791150885551868305ull, 1825854335138010348ull),
                      K(7963664994991228759ull, 12257807996192067905ull, 13179524609921305146ull, 2767831111890561987ull));
    case 2: return F2(K(3697675806616062876ull, 9065277094688085689ull, 6918009208039626314ull, 2775033306905974752ull), fe_zero());
    case 3: return F2(K(14532872967180610477ull, 12903226530429559474ull, 1868623743233345524ull, 2316889217940299650ull),
                      K(12447993766991532972ull, 4121872836076202828ull, 7630813605053367399ull, 740282956577754197ull));
    default: abort();
    }
}
static fq2 fq6_frob_c2(int n) {                                /* fq6.rs:48-90 */
    switch (n % 6) {
    case 0: return fq2_one();
    case 1: return F2(K(8314163329781907090ull, 11942187022798819835ull, 11282677263046157209ull, 1576150870752482284ull),
                      K(6763840483288992073ull, 7118829427391486816ull, 4016233444936635065ull, 2630958277570195709ull));
    case 2: return F2(K(8183898218631979349ull, 12014359695528440611ull, 12263358156045030468ull, 3187210487005268291ull), fe_zero());
    case 3: return F2(K(4938922280314430175ull, 13823286637238282975ull, 15589480384090068090ull, 481952561930628184ull),
                      K(3105754162722846417ull, 11647802298615474591ull, 13057042392041828081ull, 1660844386505564338ull));
    default: abort();
    }
}
static inline fq6 fq6_zero(void) { return F6(fq2_zero(), fq2_zero(), fq2_zero()); }
static inline fq6 fq6_one(void) { return F6(fq2_one(), fq2_zero(), fq2_zero()); }
static inline int fq6_is_zero(fq6 a) { return fq2_is_zero(a.c0) && fq2_is_zero(a.c1) && fq2_is_zero(a.c2); }
static inline fq6 fq6_add(fq6 a, fq6 b) { return F6(fq2_add(a.c0, b.c0), fq2_add(a.c1, b.c1), fq2_add(a.c2, b.c2)); }
static inline fq6 fq6_sub(fq6 a, fq6 b) { return F6(fq2_sub(a.c0, b.c0), fq2_sub(a.c1, b.c1), fq2_sub(a.c2, b.c2)); }
static inline fq6 fq6_neg(fq6 a) { return F6(fq2_neg(a.c0), fq2_neg(a.c1), fq2_neg(a.c2)); }
static inline fq6 fq6_mul_by_nonresidue(fq6 a) { return F6(fq2_mul_by_nonresidue(a.c2), a.c0, a.c1); } /* fq6.rs:109-115 */
static inline fq6 fq6_scale(fq6 a, fq2 by) { return F6(fq2_mul(a.c0, by), fq2_mul(a.c1, by), fq2_mul(a.c2, by)); }
static inline fq6 fq6_frobenius_map(fq6 a, int power) {        /* fq6.rs:125-131 */
    return F6(fq2_frobenius_map(a.c0, power),
              fq2_mul(fq2_frobenius_map(a.c1, power), fq6_frob_c1(power)),
              fq2_mul(fq2_frobenius_map(a.c2, power), fq6_frob_c2(power)));
}
static fq6 fq6_squared(fq6 a) {                                /* fq6.rs:163-177 */
    fq2 s0 = fq2_squared(a.c0);
    fq2 ab = fq2_mul(a.c0, a.c1);
    fq2 s1 = fq2_add(ab, ab);
    fq2 s2 = fq2_squared(fq2_add(fq2_sub(a.c0, a.c1), a.c2));
    fq2 bc = fq2_mul(a.c1, a.c2);
    fq2 s3 = fq2_add(bc, bc);
    fq2 s4 = fq2_squared(a.c2);
    return F6(fq2_add(s0, fq2_mul_by_nonresidue(s3)),
              fq2_add(s1, fq2_mul_by_nonresidue(s4)),
              fq2_sub(fq2_sub(fq2_add(fq2_add(s1, s2), s3), s0), s4));
}
static int fq6_inverse(fq6 a, fq6* out) {                      /* fq6.rs:179-191 */
    fq2 c0 = fq2_sub(fq2_squared(a.c0), fq2_mul(a.c1, fq2_mul_by_nonresidue(a.c2)));
    fq2 c1 = fq2_sub(fq2_mul_by_nonresidue(fq2_squared(a.c2)), fq2_mul(a.c0, a.c1));
    fq2 c2 = fq2_sub(fq2_squared(a.c1), fq2_mul(a.c0, a.c2));
    fq2 t;
    if (fq2_inverse(fq2_add(fq2_mul_by_nonresidue(fq2_add(fq2_mul(a.c2, c1), fq2_mul(a.c1, c2))),
                            fq2_mul(a.c0, c0)), &t))
        return 1;
    *out = F6(fq2_mul(t, c0), fq2_mul(t, c1), fq2_mul(t, c2));
    return 0;
}
static fq6 fq6_mul(fq6 a, fq6 b) {                             /* fq6.rs:197-207 */
    fq2 a_a = fq2_mul(a.c0, b.c0);
    fq2 b_b = fq2_mul(a.c1, b.c1);
    fq2 c_c = fq2_mul(a.c2, b.c2);
    fq2 r0 = fq2_add(fq2_mul_by_nonresidue(fq2_sub(fq2_sub(fq2_mul(fq2_add(a.c1, a.c2), fq2_add(b.c1, b.c2)), b_b), c_c)), a_a);
    fq2 r1 = fq2_add(fq2_sub(fq2_sub(fq2_mul(fq2_add(a.c0, a.c1), fq2_add(b.c0, b.c1)), a_a), b_b), fq2_mul_by_nonresidue(c_c));
    fq2 r2 = fq2_sub(fq2_add(fq2_sub(fq2_mul(fq2_add(a.c0, a.c2), fq2_add(b.c0, b.c2)), a_a), b_b), c_c);
    return F6(r0, r1, r2);
}

/* ------------------------------------------------------------------ */
/* Fq12 = Fq6[w]/(w^2 - v): src/fields/fq12.rs */
typedef struct { fq6 c0, c1; } fq12;
static inline fq12 F12(fq6 a, fq6 b) { fq12 r = {a, b}; return r; }
static fq2 fq12_frob_c1(int power) {                           /* fq12.rs:6-48 */
    switch (power % 12) {
    case 0: return fq2_one();
    case 1: return F2(K(12653890742059813127ull, 14585784200204367754ull, 1278438861261381767ull, 212598772761311868ull),
                      K(11683091849979440498ull, 14992204589386555739ull, 15866167890766973222ull, 1200023580730561873ull));
    case 2: return F2(K(14595462726357228530ull, 17349508522658994025ull, 1017833795229664280ull, 299787779797702374ull), fe_zero());
    case 3: return F2(K(3914496794763385213ull, 790120733010914719ull, 7322192392869644725ull, 581366264293887267ull),
                      K(12817045492518885689ull, 4440270538777280383ull, 11178533038884588256ull, 2767537931541304486ull));
    default: abort();
    }
}
static inline fq12 fq12_one(void) { return F12(fq6_one(), fq6_zero()); }
static inline int fq12_is_zero(fq12 a) { return fq6_is_zero(a.c0) && fq6_is_zero(a.c1); }
static inline fq12 fq12_add(fq12 a, fq12 b) { return F12(fq6_add(a.c0, b.c0), fq6_add(a.c1, b.c1)); }
static inline fq12 fq12_sub(fq12 a, fq12 b) { return F12(fq6_sub(a.c0, b.c0), fq6_sub(a.c1, b.c1)); }
static inline fq12 fq12_neg(fq12 a) { return F12(fq6_neg(a.c0), fq6_neg(a.c1)); }
static fq12 fq12_mul(fq12 a, fq12 b) {                         /* fq12.rs:319-327 */
    fq6 aa = fq6_mul(a.c0, b.c0);
    fq6 bb = fq6_mul(a.c1, b.c1);
    return F12(fq6_add(fq6_mul_by_nonresidue(bb), aa),
               fq6_sub(fq6_sub(fq6_mul(fq6_add(a.c0, a.c1), fq6_add(b.c0, b.c1)), aa), bb));
}
static fq12 fq12_squared(fq12 a) {                             /* fq12.rs:295-303 */
    fq6 ab = fq6_mul(a.c0, a.c1);
    fq6 t = fq6_mul(fq6_add(fq6_mul_by_nonresidue(a.c1), a.c0), fq6_add(a.c0, a.c1));
    return F12(fq6_sub(fq6_sub(t, ab), fq6_mul_by_nonresidue(ab)), fq6_add(ab, ab));
}
static int fq12_inverse(fq12 a, fq12* out) {                   /* fq12.rs:305-313 */
    fq6 t;
    if (fq6_inverse(fq6_sub(fq6_squared(a.c0), fq6_mul_by_nonresidue(fq6_squared(a.c1))), &t)) return 1;
    *out = F12(fq6_mul(a.c0, t), fq6_neg(fq6_mul(a.c1, t)));
    return 0;
}
static inline fq12 fq12_unitary_inverse(fq12 a) { return F12(a.c0, fq6_neg(a.c1)); } /* fq12.rs:126-128 */
static fq12 fq12_frobenius_map(fq12 a, int power) {            /* fq12.rs:112-119 */
    return F12(fq6_frobenius_map(a.c0, power),
               fq6_scale(fq6_frobenius_map(a.c1, power), fq12_frob_c1(power)));
}
static fq12 fq12_mul_by_024(fq12 f, fq2 ell_0, fq2 ell_vw, fq2 ell_vv) { /* fq12.rs:130-196 */
    fq2 z0 = f.c0.c0, z1 = f.c0.c1, z2 = f.c0.c2, z3 = f.c1.c0, z4 = f.c1.c1, z5 = f.c1.c2;
    fq2 x0 = ell_0, x2 = ell_vv, x4 = ell_vw;
    fq2 d0 = fq2_mul(z0, x0), d2 = fq2_mul(z2, x2), d4 = fq2_mul(z4, x4);
    fq2 t2 = fq2_add(z0, z4), t1 = fq2_add(z0, z2), s0 = fq2_add(fq2_add(z1, z3), z5);
    fq2 s1 = fq2_mul(z1, x2);
    fq2 t3 = fq2_add(s1, d4);
    fq2 t4 = fq2_add(fq2_mul_by_nonresidue(t3), d0);
    fq2 n0 = t4;
    t3 = fq2_mul(z5, x4);
    s1 = fq2_add(s1, t3);
    t3 = fq2_add(t3, d2);
    t4 = fq2_mul_by_nonresidue(t3);
    t3 = fq2_mul(z1, x0);
    s1 = fq2_add(s1, t3);
    t4 = fq2_add(t4, t3);
    fq2 n1 = t4;
    fq2 t0 = fq2_add(x0, x2);
    t3 = fq2_sub(fq2_sub(fq2_mul(t1, t0), d0), d2);
    t4 = fq2_mul(z3, x4);
    s1 = fq2_add(s1, t4);
    t3 = fq2_add(t3, t4);
    t0 = fq2_add(z2, z4);
    fq2 n2 = t3;
    t1 = fq2_add(x2, x4);
    t3 = fq2_sub(fq2_sub(fq2_mul(t0, t1), d2), d4);
    t4 = fq2_mul_by_nonresidue(t3);
    t3 = fq2_mul(z3, x0);
    s1 = fq2_add(s1, t3);
    t4 = fq2_add(t4, t3);
    fq2 n3 = t4;
    t3 = fq2_mul(z5, x2);
    s1 = fq2_add(s1, t3);
    t4 = fq2_mul_by_nonresidue(t3);
    t0 = fq2_add(x0, x4);
    t3 = fq2_sub(fq2_sub(fq2_mul(t2, t0), d0), d4);
    t4 = fq2_add(t4, t3);
    fq2 n4 = t4;
    t0 = fq2_add(fq2_add(x0, x2), x4);
    t3 = fq2_sub(fq2_mul(s0, t0), s1);
    fq2 n5 = t3;
    return F12(F6(n0, n1, n2), F6(n3, n4, n5));
}
static fq12 fq12_cyclotomic_squared(fq12 a) {                  /* fq12.rs:198-247 */
    fq2 z0 = a.c0.c0, z4 = a.c0.c1, z3 = a.c0.c2, z2 = a.c1.c0, z1 = a.c1.c1, z5 = a.c1.c2;
    fq2 tmp = fq2_mul(z0, z1);
    fq2 t0 = fq2_sub(fq2_sub(fq2_mul(fq2_add(z0, z1), fq2_add(fq2_mul_by_nonresidue(z1), z0)), tmp),
                     fq2_mul_by_nonresidue(tmp));
    fq2 t1 = fq2_add(tmp, tmp);
    tmp = fq2_mul(z2, z3);
    fq2 t2 = fq2_sub(fq2_sub(fq2_mul(fq2_add(z2, z3), fq2_add(fq2_mul_by_nonresidue(z3), z2)), tmp),
                     fq2_mul_by_nonresidue(tmp));
    fq2 t3 = fq2_add(tmp, tmp);
    tmp = fq2_mul(z4, z5);
    fq2 t4 = fq2_sub(fq2_sub(fq2_mul(fq2_add(z4, z5), fq2_add(fq2_mul_by_nonresidue(z5), z4)), tmp),
                     fq2_mul_by_nonresidue(tmp));
    fq2 t5 = fq2_add(tmp, tmp);
    z0 = fq2_sub(t0, z0); z0 = fq2_add(z0, z0); z0 = fq2_add(z0, t0);
    z1 = fq2_add(t1, z1); z1 = fq2_add(z1, z1); z1 = fq2_add(z1, t1);
    tmp = fq2_mul_by_nonresidue(t5);
    z2 = fq2_add(tmp, z2); z2 = fq2_add(z2, z2); z2 = fq2_add(z2, tmp);
    z3 = fq2_sub(t4, z3); z3 = fq2_add(z3, z3); z3 = fq2_add(z3, t4);
    z4 = fq2_sub(t2, z4); z4 = fq2_add(z4, z4); z4 = fq2_add(z4, t2);
    z5 = fq2_add(t3, z5); z5 = fq2_add(z5, z5); z5 = fq2_add(z5, t3);
    return F12(F6(z0, z4, z3), F6(z2, z1, z5));
}
static fq12 fq12_cyclotomic_pow(fq12 a, u256 by) {             /* fq12.rs:249-266 */
    fq12 res = fq12_one();
    int found_one = 0;
    for (int n = 255; n >= 0; --n) {
        int bit = (int)((by.d[n / 128] >> (n % 128)) & 1);
        if (found_one) res = fq12_cyclotomic_squared(res);
        if (bit) {
            found_one = 1;
            res = fq12_mul(a, res);
        }
    }
    return res;
}
static fq12 fq12_exp_by_neg_z(fq12 a) {                        /* fq12.rs:121-124 */
    return fq12_unitary_inverse(fq12_cyclotomic_pow(a, U(4965661367192848881ull, 0, 0, 0)));
}
static int fe_first_chunk(fq12 self, fq12* out) {              /* fq12.rs:62-73 */
    fq12 b;
    if (fq12_inverse(self, &b)) return 1;
    fq12 a = fq12_unitary_inverse(self);
    fq12 c = fq12_mul(a, b);
    fq12 d = fq12_frobenius_map(c, 2);
    *out = fq12_mul(d, c);
    return 0;
}
static fq12 fe_last_chunk(fq12 self) {                         /* fq12.rs:75-105 */
    fq12 a = fq12_exp_by_neg_z(self);
    fq12 b = fq12_cyclotomic_squared(a);
    fq12 c = fq12_cyclotomic_squared(b);
    fq12 d = fq12_mul(c, b);
    fq12 e = fq12_exp_by_neg_z(d);
    fq12 f = fq12_cyclotomic_squared(e);
    fq12 g = fq12_exp_by_neg_z(f);
    fq12 h = fq12_unitary_inverse(d);
    fq12 i = fq12_unitary_inverse(g);
    fq12 j = fq12_mul(i, e);
    fq12 k = fq12_mul(j, h);
    fq12 l = fq12_mul(k, b);
    fq12 m = fq12_mul(k, e);
    fq12 n = fq12_mul(self, m);
    fq12 o = fq12_frobenius_map(l, 1);
    fq12 p = fq12_mul(o, n);
    fq12 q = fq12_frobenius_map(k, 2);
    fq12 r = fq12_mul(q, p);
    fq12 s = fq12_unitary_inverse(self);
    fq12 t = fq12_mul(s, l);
    fq12 u = fq12_frobenius_map(t, 3);
    return fq12_mul(u, r);
}
static int fq12_final_exponentiation(fq12 f, fq12* out) {      /* fq12.rs:107-110 */
    fq12 a;
    if (fe_first_chunk(f, &a)) return 1;
    *out = fe_last_chunk(a);
    return 0;
}
static fq12 fq12_pow(fq12 a, u256 by) {                        /* fields/mod.rs:35-46 */
    fq12 res = fq12_one();
    for (int n = 255; n >= 0; --n) {
        res = fq12_squared(res);
        if ((by.d[n / 128] >> (n % 128)) & 1) res = fq12_mul(a, res);
    }
    return res;
}

/* ------------------------------------------------------------------ */
/* Jacobian group G<P>: src/groups/mod.rs:45-369 (generic over the base field) */
#define DEFINE_GROUP(G, F, F_zero, F_one, F_is_zero, F_eq, F_add, F_sub, F_mul, F_neg, F_sq, F_inv)   \
    typedef struct { F x, y, z; } G;                                                                 \
    static inline G G##_zero(void) { G r = {F_zero(), F_one(), F_zero()}; return r; }                \
    static inline int G##_is_zero(const G* a) { return F_is_zero(a->z); }                            \
    static G G##_double(const G* s) {               /* mod.rs:250-269 */                             \
        F a = F_sq(s->x), b = F_sq(s->y), c = F_sq(b);                                               \
        F d = F_sub(F_sub(F_sq(F_add(s->x, b)), a), c);                                              \
        d = F_add(d, d);                                                                             \
        F e = F_add(F_add(a, a), a);                                                                 \
        F f = F_sq(e);                                                                               \
        F x3 = F_sub(f, F_add(d, d));                                                                \
        F eight_c = F_add(c, c);                                                                     \
        eight_c = F_add(eight_c, eight_c);                                                           \
        eight_c = F_add(eight_c, eight_c);                                                           \
        F y1z1 = F_mul(s->y, s->z);                                                                  \
        G r = {x3, F_sub(F_mul(e, F_sub(d, x3)), eight_c), F_add(y1z1, y1z1)};                       \
        return r;                                                                                    \
    }                                                                                                \
    static G G##_add(const G* s, const G* o) {      /* mod.rs:294-334 */                             \
        if (G##_is_zero(s)) return *o;                                                               \
        if (G##_is_zero(o)) return *s;                                                               \
        F z1_squared = F_sq(s->z), z2_squared = F_sq(o->z);                                          \
        F u1 = F_mul(s->x, z2_squared), u2 = F_mul(o->x, z1_squared);                                \
        F z1_cubed = F_mul(s->z, z1_squared), z2_cubed = F_mul(o->z, z2_squared);                    \
        F s1 = F_mul(s->y, z2_cubed), s2 = F_mul(o->y, z1_cubed);                                    \
        if (F_eq(u1, u2) && F_eq(s1, s2)) return G##_double(s);                                      \
        F h = F_sub(u2, u1);                                                                         \
        F s2_minus_s1 = F_sub(s2, s1);                                                               \
        F i = F_sq(F_add(h, h));                                                                     \
        F j = F_mul(h, i);                                                                           \
        F r = F_add(s2_minus_s1, s2_minus_s1);                                                       \
        F v = F_mul(u1, i);                                                                          \
        F s1_j = F_mul(s1, j);                                                                       \
        F x3 = F_sub(F_sub(F_sq(r), j), F_add(v, v));                                                \
        G out = {x3, F_sub(F_mul(r, F_sub(v, x3)), F_add(s1_j, s1_j)),                               \
                 F_mul(F_sub(F_sub(F_sq(F_add(s->z, o->z)), z1_squared), z2_squared), h)};           \
        return out;                                                                                  \
    }                                                                                                \
    static G G##_neg(const G* a) {                  /* mod.rs:336-350 */                             \
        if (G##_is_zero(a)) return *a;                                                               \
        G r = {a->x, F_neg(a->y), a->z};                                                             \
        return r;                                                                                    \
    }                                                                                                \
    static G G##_mul_u256(const G* p, u256 k) {     /* mod.rs:272-292 */                             \
        G res = G##_zero();                                                                          \
        int found_one = 0;                                                                           \
        for (int n = 255; n >= 0; --n) {                                                             \
            int bit = (int)((k.d[n / 128] >> (n % 128)) & 1);                                        \
            if (found_one) res = G##_double(&res);                                                   \
            if (bit) {                                                                               \
                found_one = 1;                                                                       \
                res = G##_add(&res, p);                                                              \
            }                                                                                        \
        }                                                                                            \
        return res;                                                                                  \
    }                                                                                                \
    static int G##_eq(const G* a, const G* b) {     /* mod.rs:169-195 */                             \
        if (G##_is_zero(a)) return G##_is_zero(b);                                                   \
        if (G##_is_zero(b)) return 0;                                                                \
        F z1_squared = F_sq(a->z), z2_squared = F_sq(b->z);                                          \
        if (!F_eq(F_mul(a->x, z2_squared), F_mul(b->x, z1_squared))) return 0;                       \
        F z1_cubed = F_mul(a->z, z1_squared), z2_cubed = F_mul(b->z, z2_squared);                    \
        if (!F_eq(F_mul(a->y, z2_cubed), F_mul(b->y, z1_cubed))) return 0;                           \
        return 1;                                                                                    \
    }                                                                                                \
    static int G##_to_affine(const G* p, F* x, F* y) {  /* mod.rs:199-216 */                         \
        if (F_is_zero(p->z)) return 1;                                                               \
        if (F_eq(p->z, F_one())) { *x = p->x; *y = p->y; return 0; }                                 \
        F zinv;                                                                                      \
        F_inv(p->z, &zinv);                                                                          \
        F zinv_squared = F_sq(zinv);                                                                 \
        *x = F_mul(p->x, zinv_squared);                                                              \
        *y = F_mul(p->y, F_mul(zinv_squared, zinv));                                                 \
        return 0;                                                                                    \
    }

static inline fe fq_zero(void) { return fe_zero(); }
static inline fe fq_one(void) { return FQ->one; }
static inline int fq_is_zero(fe a) { return fe_is_zero(a); }
static inline int fq_eq(fe a, fe b) { return fe_eq(a, b); }
static inline fe fq_add(fe a, fe b) { return fe_add(a, b, FQ); }
static inline fe fq_sub(fe a, fe b) { return fe_sub(a, b, FQ); }
static inline fe fq_mul(fe a, fe b) { return fe_mul(a, b, FQ); }
static inline fe fq_neg(fe a) { return fe_neg(a, FQ); }
static inline fe fq_sq(fe a) { return fe_squared(a, FQ); }
static inline int fq_inv(fe a, fe* out) { *out = a; return fe_inverse(out, FQ); }
static inline int fq2_inv(fq2 a, fq2* out) { return fq2_inverse(a, out); }

DEFINE_GROUP(g1, fe, fq_zero, fq_one, fq_is_zero, fq_eq, fq_add, fq_sub, fq_mul, fq_neg, fq_sq, fq_inv)
DEFINE_GROUP(g2, fq2, fq2_zero, fq2_one, fq2_is_zero, fq2_eq, fq2_add, fq2_sub, fq2_mul, fq2_neg, fq2_squared, fq2_inv)

static g1 g1_one_pt(void) {                                     /* mod.rs:381-392 */
    g1 r = {fq_one(), K(0xa6ba871b8b1e1b3aull, 0x14f1d651eb8e167bull, 0xccdd46def0f28c58ull, 0x1c14ef83340fbe5eull), fq_one()};
    return r;
}
static fe g1_coeff_b(void) {                                   /* mod.rs:394-401 */
    return K(0x7a17caa950ad28d7ull, 0x1f6ac17ae15521b9ull, 0x334bea4e696bd284ull, 0x2a1f6744ce179d8eull);
}
static g2 g2_one_pt(void) {                                     /* mod.rs:418-450 */
    g2 r = {F2(K(0x8e83b5d102bc2026ull, 0xdceb1935497b0172ull, 0xfbb8264797811adfull, 0x19573841af96503bull),
               K(0xafb4737da84c6140ull, 0x6043dd5a5802d8c4ull, 0x09e950fc52a02f86ull, 0x14fef0833aea7b6bull)),
            F2(K(0x619dfa9d886be9f6ull, 0xfe7fd297f59e9b78ull, 0xff9e1a62231b7dfeull, 0x28fd7eebae9e4206ull),
               K(0x64095b56c71856eeull, 0xdc57f922327d3cbbull, 0x55f935be33351076ull, 0x0da4a0e693fd6482ull)),
            fq2_one()};
    return r;
}
static fq2 g2_coeff_b(void) {                                  /* mod.rs:452-467 */
    return F2(K(0x3bf938e377b802a8ull, 0x020b1b273633535dull, 0x26b7edf049755260ull, 0x2514c6324384a86dull),
              K(0x38e7ecccd1dcff67ull, 0x65f0b37d93ce0d3eull, 0xd749d0dd22ac00aaull, 0x0141b9ce4a688d4dull));
}

/* ------------------------------------------------------------------ */
/* G2 line precomputation + Miller loop: src/groups/mod.rs:9-14, 515-776 */
static const uint8_t ATE_LOOP_COUNT_NAF[64] = {                /* mod.rs:14 */
    1, 0, 1, 0, 0, 0, 3, 0, 3, 0, 0, 0, 3, 0, 1, 0, 3, 0, 0, 3, 0, 0, 0, 0, 0, 1, 0, 0, 3, 0, 1, 0,
    0, 3, 0, 0, 0, 0, 3, 0, 1, 0, 0, 0, 3, 0, 3, 0, 0, 1, 0, 0, 0, 3, 0, 0, 3, 0, 1, 0, 1, 0, 0, 0};

static inline fq2 twist(void) { return fq2_nonresidue(); }     /* mod.rs:516-518 */
static inline fe two_inv(void) {                               /* mod.rs:521-528 */
    return K(9781510331150239090ull, 15059239858463337189ull, 10331104244869713732ull, 2249375503248834476ull);
}
static inline fq2 twist_mul_by_q_x(void) {                     /* mod.rs:531-546 */
    return F2(K(13075984984163199792ull, 3782902503040509012ull, 8791150885551868305ull, 1825854335138010348ull),
              K(7963664994991228759ull, 12257807996192067905ull, 13179524609921305146ull, 2767831111890561987ull));
}
static inline fq2 twist_mul_by_q_y(void) {                     /* mod.rs:549-564 */
    return F2(K(16482010305593259561ull, 13488546290961988299ull, 3578621962720924518ull, 2681173117283399901ull),
              K(11661927080404088775ull, 553939530661941723ull, 7860678177968807019ull, 3208568454732775116ull));
}
typedef struct { fq2 x, y; } g2aff;
typedef struct { fq2 ell_0, ell_vw, ell_vv; } ell;

static ell mixed_addition_step(g2* s, const g2aff* base) {     /* mod.rs:731-752 */
    fq2 d = fq2_sub(s->x, fq2_mul(s->z, base->x));
    fq2 e = fq2_sub(s->y, fq2_mul(s->z, base->y));
    fq2 f = fq2_squared(d);
    fq2 g = fq2_squared(e);
    fq2 h = fq2_mul(d, f);
    fq2 i = fq2_mul(s->x, f);
    fq2 j = fq2_sub(fq2_add(fq2_mul(s->z, g), h), fq2_add(i, i));
    s->x = fq2_mul(d, j);
    s->y = fq2_sub(fq2_mul(e, fq2_sub(i, j)), fq2_mul(h, s->y));
    s->z = fq2_mul(s->z, h);
    ell c = {fq2_mul(twist(), fq2_sub(fq2_mul(e, base->x), fq2_mul(d, base->y))), d, fq2_neg(e)};
    return c;
}
static ell doubling_step(g2* s) {                              /* mod.rs:754-776 */
    fq2 a = fq2_scale(fq2_mul(s->x, s->y), two_inv());
    fq2 b = fq2_squared(s->y);
    fq2 c = fq2_squared(s->z);
    fq2 d = fq2_add(fq2_add(c, c), c);
    fq2 e = fq2_mul(g2_coeff_b(), d);
    fq2 f = fq2_add(fq2_add(e, e), e);
    fq2 g = fq2_scale(fq2_add(b, f), two_inv());
    fq2 h = fq2_sub(fq2_squared(fq2_add(s->y, s->z)), fq2_add(b, c));
    fq2 i = fq2_sub(e, b);
    fq2 j = fq2_squared(s->x);
    fq2 e_sq = fq2_squared(e);
    s->x = fq2_mul(a, fq2_sub(b, f));
    s->y = fq2_sub(fq2_squared(g), fq2_add(fq2_add(e_sq, e_sq), e_sq));
    s->z = fq2_mul(b, h);
    ell out = {fq2_mul(twist(), i), fq2_neg(h), fq2_add(fq2_add(j, j), j)};
    return out;
}
static g2aff mul_by_q(const g2aff* q) {                        /* mod.rs:694-699 */
    g2aff r = {fq2_mul(twist_mul_by_q_x(), fq2_frobenius_map(q->x, 1)),
               fq2_mul(twist_mul_by_q_y(), fq2_frobenius_map(q->y, 1))};
    return r;
}
static void precompute(const g2aff* q, ell coeffs[ORC_NUM_COEFFS]) { /* mod.rs:701-727 */
    g2 r = {q->x, q->y, fq2_one()};
    int k = 0;
    g2aff q_neg = {q->x, fq2_neg(q->y)};
    for (int i = 0; i < 64; ++i) {
        coeffs[k++] = doubling_step(&r);
        if (ATE_LOOP_COUNT_NAF[i] == 1) coeffs[k++] = mixed_addition_step(&r, q);
        if (ATE_LOOP_COUNT_NAF[i] == 3) coeffs[k++] = mixed_addition_step(&r, &q_neg);
    }
    g2aff q1 = mul_by_q(q);
    g2aff q2 = mul_by_q(&q1);
    q2.y = fq2_neg(q2.y);
    coeffs[k++] = mixed_addition_step(&r, &q1);
    coeffs[k++] = mixed_addition_step(&r, &q2);
    if (k != ORC_NUM_COEFFS) abort();
}
static inline fq12 line(fq12 f, const ell* c, fe px, fe py) {
    return fq12_mul_by_024(f, c->ell_0, fq2_scale(c->ell_vw, py), fq2_scale(c->ell_vv, px));
}
static fq12 miller_loop(const ell coeffs[ORC_NUM_COEFFS], fe px, fe py) { /* mod.rs:579-607 */
    fq12 f = fq12_one();
    int idx = 0;
    for (int i = 0; i < 64; ++i) {
        f = line(fq12_squared(f), &coeffs[idx++], px, py);
        if (ATE_LOOP_COUNT_NAF[i] != 0) f = line(f, &coeffs[idx++], px, py);
    }
    f = line(f, &coeffs[idx++], px, py);
    f = line(f, &coeffs[idx], px, py);
    return f;
}
static fq12 miller_loop_multi(ell (*coeffs)[ORC_NUM_COEFFS], const fe* px, const fe* py, size_t n) {
    /* miller_loop_batch, mod.rs:609-640 */
    fq12 f = fq12_one();
    int idx = 0;
    for (int i = 0; i < 64; ++i) {
        f = fq12_squared(f);
        for (size_t t = 0; t < n; ++t) f = line(f, &coeffs[t][idx], px[t], py[t]);
        idx++;
        if (ATE_LOOP_COUNT_NAF[i] != 0) {
            for (size_t t = 0; t < n; ++t) f = line(f, &coeffs[t][idx], px[t], py[t]);
            idx++;
        }
    }
    for (size_t t = 0; t < n; ++t) f = line(f, &coeffs[t][idx], px[t], py[t]);
    idx++;
    for (size_t t = 0; t < n; ++t) f = line(f, &coeffs[t][idx], px[t], py[t]);
    return f;
}
static fq12 pairing_one(const g1* p, const g2* q) {            /* mod.rs:894-902 */
    fe px, py;
    g2aff qa;
    if (g1_to_affine(p, &px, &py) || g2_to_affine(q, &qa.x, &qa.y)) return fq12_one();
    ell coeffs[ORC_NUM_COEFFS];
    precompute(&qa, coeffs);
    fq12 out;
    if (fq12_final_exponentiation(miller_loop(coeffs, px, py), &out)) abort(); /* "miller loop cannot produce zero" */
    return out;
}

/* ------------------------------------------------------------------ */
/* exported C API (memory images are byte-identical to the internal types) */
_Static_assert(sizeof(fe) == sizeof(orc_fe), "fe image");
_Static_assert(sizeof(fq12) == sizeof(orc_fq12), "fq12 image");
_Static_assert(sizeof(g1) == sizeof(orc_g1), "g1 image");
_Static_assert(sizeof(g2) == sizeof(orc_g2), "g2 image");
_Static_assert(sizeof(ell) == sizeof(orc_ell_coeffs), "ell image");

#define LD(T, p) (*(const T*)(const void*)(p))
#define ST(T, p, v) (*(T*)(void*)(p) = (v))

void orc_fe_from_canonical(int field, const orc_fe* a, orc_fe* out) { /* fp.rs:46-54 */
    const fparams* P = FP(field);
    fe x = LD(fe, a);
    u256_mul(&x, &P->r2, &P->m, P->inv);
    ST(fe, out, x);
}
void orc_fe_to_canonical(int field, const orc_fe* a, orc_fe* out) {   /* fp.rs:13-20 */
    const fparams* P = FP(field);
    fe x = LD(fe, a), one = U(1, 0, 0, 0);
    u256_mul(&x, &one, &P->m, P->inv);
    ST(fe, out, x);
}
void orc_fe_add(int f, const orc_fe* a, const orc_fe* b, orc_fe* o) { ST(fe, o, fe_add(LD(fe, a), LD(fe, b), FP(f))); }
void orc_fe_sub(int f, const orc_fe* a, const orc_fe* b, orc_fe* o) { ST(fe, o, fe_sub(LD(fe, a), LD(fe, b), FP(f))); }
void orc_fe_mul(int f, const orc_fe* a, const orc_fe* b, orc_fe* o) { ST(fe, o, fe_mul(LD(fe, a), LD(fe, b), FP(f))); }
void orc_fe_neg(int f, const orc_fe* a, orc_fe* o) { ST(fe, o, fe_neg(LD(fe, a), FP(f))); }
int orc_fe_inverse(int f, const orc_fe* a, orc_fe* o) {
    fe x = LD(fe, a);
    int r = fe_inverse(&x, FP(f));
    ST(fe, o, x);
    return r;
}
void orc_fq2_mul(const orc_fq2* a, const orc_fq2* b, orc_fq2* o) { FP(0); ST(fq2, o, fq2_mul(LD(fq2, a), LD(fq2, b))); }
void orc_fq2_squared(const orc_fq2* a, orc_fq2* o) { FP(0); ST(fq2, o, fq2_squared(LD(fq2, a))); }
int orc_fq2_inverse(const orc_fq2* a, orc_fq2* o) { FP(0); return fq2_inverse(LD(fq2, a), (fq2*)(void*)o); }
void orc_fq6_mul(const orc_fq6* a, const orc_fq6* b, orc_fq6* o) { FP(0); ST(fq6, o, fq6_mul(LD(fq6, a), LD(fq6, b))); }
void orc_fq6_squared(const orc_fq6* a, orc_fq6* o) { FP(0); ST(fq6, o, fq6_squared(LD(fq6, a))); }
int orc_fq6_inverse(const orc_fq6* a, orc_fq6* o) { FP(0); return fq6_inverse(LD(fq6, a), (fq6*)(void*)o); }
void orc_fq12_mul(const orc_fq12* a, const orc_fq12* b, orc_fq12* o) { FP(0); ST(fq12, o, fq12_mul(LD(fq12, a), LD(fq12, b))); }
void orc_fq12_squared(const orc_fq12* a, orc_fq12* o) { FP(0); ST(fq12, o, fq12_squared(LD(fq12, a))); }
void orc_fq12_add(const orc_fq12* a, const orc_fq12* b, orc_fq12* o) { FP(0); ST(fq12, o, fq12_add(LD(fq12, a), LD(fq12, b))); }
void orc_fq12_sub(const orc_fq12* a, const orc_fq12* b, orc_fq12* o) { FP(0); ST(fq12, o, fq12_sub(LD(fq12, a), LD(fq12, b))); }
void orc_fq12_neg(const orc_fq12* a, orc_fq12* o) { FP(0); ST(fq12, o, fq12_neg(LD(fq12, a))); }
int orc_fq12_inverse(const orc_fq12* a, orc_fq12* o) { FP(0); return fq12_inverse(LD(fq12, a), (fq12*)(void*)o); }
void orc_fq12_frobenius_map(const orc_fq12* a, int power, orc_fq12* o) { FP(0); ST(fq12, o, fq12_frobenius_map(LD(fq12, a), power)); }
void orc_fq12_cyclotomic_squared(const orc_fq12* a, orc_fq12* o) { FP(0); ST(fq12, o, fq12_cyclotomic_squared(LD(fq12, a))); }
void orc_fq12_exp_by_neg_z(const orc_fq12* a, orc_fq12* o) { FP(0); ST(fq12, o, fq12_exp_by_neg_z(LD(fq12, a))); }
void orc_fq12_mul_by_024(const orc_fq12* f, const orc_fq2* e0, const orc_fq2* evw, const orc_fq2* evv, orc_fq12* o) {
    FP(0);
    ST(fq12, o, fq12_mul_by_024(LD(fq12, f), LD(fq2, e0), LD(fq2, evw), LD(fq2, evv)));
}
void orc_fq12_pow(const orc_fq12* a, const orc_fe* e, orc_fq12* o) { FP(0); ST(fq12, o, fq12_pow(LD(fq12, a), LD(u256, e))); }
int orc_final_exponentiation(const orc_fq12* f, orc_fq12* o) { FP(0); return fq12_final_exponentiation(LD(fq12, f), (fq12*)(void*)o); }

void orc_g1_one(orc_g1* o) { FP(0); ST(g1, o, g1_one_pt()); }
void orc_g2_one(orc_g2* o) { FP(0); ST(g2, o, g2_one_pt()); }
void orc_g1_add(const orc_g1* a, const orc_g1* b, orc_g1* o) { FP(0); ST(g1, o, g1_add((const g1*)(const void*)a, (const g1*)(const void*)b)); }
void orc_g1_double(const orc_g1* a, orc_g1* o) { FP(0); ST(g1, o, g1_double((const g1*)(const void*)a)); }
void orc_g1_neg(const orc_g1* a, orc_g1* o) { FP(0); ST(g1, o, g1_neg((const g1*)(const void*)a)); }
int orc_g1_eq(const orc_g1* a, const orc_g1* b) { FP(0); return g1_eq((const g1*)(const void*)a, (const g1*)(const void*)b); }
void orc_g1_mul(const orc_g1* p, const orc_fe* k, orc_g1* o) {
    orc_fe kc;
    orc_fe_to_canonical(1, k, &kc);                             /* U256::from(Fr), fp.rs:13-20 */
    ST(g1, o, g1_mul_u256((const g1*)(const void*)p, LD(u256, &kc)));
}
int orc_g1_to_affine(const orc_g1* p, orc_fe* x, orc_fe* y) { FP(0); return g1_to_affine((const g1*)(const void*)p, (fe*)(void*)x, (fe*)(void*)y); }
void orc_g2_add(const orc_g2* a, const orc_g2* b, orc_g2* o) { FP(0); ST(g2, o, g2_add((const g2*)(const void*)a, (const g2*)(const void*)b)); }
void orc_g2_double(const orc_g2* a, orc_g2* o) { FP(0); ST(g2, o, g2_double((const g2*)(const void*)a)); }
void orc_g2_neg(const orc_g2* a, orc_g2* o) { FP(0); ST(g2, o, g2_neg((const g2*)(const void*)a)); }
int orc_g2_eq(const orc_g2* a, const orc_g2* b) { FP(0); return g2_eq((const g2*)(const void*)a, (const g2*)(const void*)b); }
void orc_g2_mul(const orc_g2* p, const orc_fe* k, orc_g2* o) {
    orc_fe kc;
    orc_fe_to_canonical(1, k, &kc);
    ST(g2, o, g2_mul_u256((const g2*)(const void*)p, LD(u256, &kc)));
}
int orc_g2_to_affine(const orc_g2* p, orc_g2_affine* o) {
    FP(0);
    return g2_to_affine((const g2*)(const void*)p, (fq2*)(void*)&o->x, (fq2*)(void*)&o->y);
}
int orc_g1_on_curve_affine(const orc_fe* x, const orc_fe* y) {  /* mod.rs:96 (curve equation only) */
    FP(0);
    fe X = LD(fe, x), Y = LD(fe, y);
    return fq_eq(fq_sq(Y), fq_add(fq_mul(fq_sq(X), X), g1_coeff_b()));
}

void orc_g2_precompute(const orc_g2_affine* q, orc_ell_coeffs out[ORC_NUM_COEFFS]) {
    FP(0);
    precompute((const g2aff*)(const void*)q, (ell*)(void*)out);
}
void orc_miller_loop(const orc_ell_coeffs c[ORC_NUM_COEFFS], const orc_fe* px, const orc_fe* py, orc_fq12* o) {
    FP(0);
    ST(fq12, o, miller_loop((const ell*)(const void*)c, LD(fe, px), LD(fe, py)));
}
void orc_pairing(const orc_g1* p, const orc_g2* q, orc_fq12* o) {
    FP(0);
    ST(fq12, o, pairing_one((const g1*)(const void*)p, (const g2*)(const void*)q));
}
void orc_pairing_batch(const orc_g1* p, const orc_g2* q, size_t n, orc_fq12* o) { /* mod.rs:904-926 */
    FP(0);
    ell (*coeffs)[ORC_NUM_COEFFS] = malloc((n ? n : 1) * sizeof(*coeffs));
    fe* px = malloc((n ? n : 1) * sizeof(fe));
    fe* py = malloc((n ? n : 1) * sizeof(fe));
    size_t m = 0;
    for (size_t t = 0; t < n; ++t) {
        fe x, y;
        g2aff qa;
        if (g1_to_affine((const g1*)(const void*)&p[t], &x, &y)) continue;
        if (g2_to_affine((const g2*)(const void*)&q[t], &qa.x, &qa.y)) continue;
        px[m] = x;
        py[m] = y;
        precompute(&qa, coeffs[m]);
        m++;
    }
    fq12 r = fq12_one();
    if (m) {
        if (fq12_final_exponentiation(miller_loop_multi(coeffs, px, py, m), &r)) abort();
    }
    ST(fq12, o, r);
    free(coeffs);
    free(px);
    free(py);
}
int orc_miller_loop_batch(const orc_g2* q, const orc_g1* p, size_t n, orc_fq12* o) { /* lib.rs:625-633 */
    FP(0);
    ell (*coeffs)[ORC_NUM_COEFFS] = malloc((n ? n : 1) * sizeof(*coeffs));
    fe* px = malloc((n ? n : 1) * sizeof(fe));
    fe* py = malloc((n ? n : 1) * sizeof(fe));
    int rc = 0;
    for (size_t t = 0; t < n && !rc; ++t) {
        g2aff qa;
        if (g2_to_affine((const g2*)(const void*)&q[t], &qa.x, &qa.y)) { rc = 1; break; }
        precompute(&qa, coeffs[t]);
        if (g1_to_affine((const g1*)(const void*)&p[t], &px[t], &py[t])) { rc = 1; break; }
    }
    if (!rc) ST(fq12, o, miller_loop_multi(coeffs, px, py, n));
    free(coeffs);
    free(px);
    free(py);
    return rc;
}

/* ---- threaded batch helpers ---- */
typedef struct {
    int kind;
    const void *a, *b;
    void* out;
    size_t lo, hi;
} job;
static void* run_job(void* arg) {
    job* j = (job*)arg;
    for (size_t i = j->lo; i < j->hi; ++i) {
        if (j->kind == 0)
            orc_pairing((const orc_g1*)j->a + i, (const orc_g2*)j->b + i, (orc_fq12*)j->out + i);
        else if (j->kind == 1)
            orc_g1_mul((const orc_g1*)j->a + i, (const orc_fe*)j->b + i, (orc_g1*)j->out + i);
        else
            orc_g2_mul((const orc_g2*)j->a + i, (const orc_fe*)j->b + i, (orc_g2*)j->out + i);
    }
    return NULL;
}
static void run_many(int kind, const void* a, const void* b, size_t n, void* out, int nthreads) {
    FP(0);
    if (nthreads < 1) nthreads = 1;
    if ((size_t)nthreads > n) nthreads = n ? (int)n : 1;
    pthread_t th[256];
    job jobs[256];
    if (nthreads > 256) nthreads = 256;
    for (int t = 0; t < nthreads; ++t) {
        jobs[t].kind = kind;
        jobs[t].a = a;
        jobs[t].b = b;
        jobs[t].out = out;
        jobs[t].lo = n * t / nthreads;
        jobs[t].hi = n * (t + 1) / nthreads;
        pthread_create(&th[t], NULL, run_job, &jobs[t]);
    }
    for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
}
void orc_pairing_many(const orc_g1* p, const orc_g2* q, size_t n, orc_fq12* out, int nthreads) { run_many(0, p, q, n, out, nthreads); }

/* pairing_batch (mod.rs:904-926) on several threads: thread t runs the shared
 * loop (miller_loop_multi) over its contiguous slice of the non-zero pairs, and
 * the partial values are multiplied in slice order before the one final
 * exponentiation.  Squaring is a ring homomorphism and Fq12 is commutative, so
 * the product of the slices' loop values IS the single shared loop value:
 * the result equals orc_pairing_batch's bit for bit (tests/test_oracle.py). */
typedef struct {
    const orc_g1* p;
    const orc_g2* q;
    size_t lo, hi;
    fq12 f;
    size_t live;
} bjob;
static void* run_bjob(void* arg) {
    bjob* j = (bjob*)arg;
    size_t n = j->hi - j->lo;
    ell (*coeffs)[ORC_NUM_COEFFS] = malloc((n ? n : 1) * sizeof(*coeffs));
    fe* px = malloc((n ? n : 1) * sizeof(fe));
    fe* py = malloc((n ? n : 1) * sizeof(fe));
    size_t m = 0;
    for (size_t t = j->lo; t < j->hi; ++t) {
        fe x, y;
        g2aff qa;
        if (g1_to_affine((const g1*)(const void*)&j->p[t], &x, &y)) continue;
        if (g2_to_affine((const g2*)(const void*)&j->q[t], &qa.x, &qa.y)) continue;
        px[m] = x;
        py[m] = y;
        precompute(&qa, coeffs[m]);
        m++;
    }
    j->f = m ? miller_loop_multi(coeffs, px, py, m) : fq12_one();
    j->live = m;
    free(coeffs);
    free(px);
    free(py);
    return NULL;
}
void orc_pairing_batch_mt(const orc_g1* p, const orc_g2* q, size_t n, orc_fq12* o, int nthreads) {
    FP(0);
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    if ((size_t)nthreads > n) nthreads = n ? (int)n : 1;
    pthread_t th[256];
    bjob jobs[256];
    for (int t = 0; t < nthreads; ++t) {
        jobs[t].p = p;
        jobs[t].q = q;
        jobs[t].lo = n * t / nthreads;
        jobs[t].hi = n * (t + 1) / nthreads;
        pthread_create(&th[t], NULL, run_bjob, &jobs[t]);
    }
    fq12 f = fq12_one();
    size_t live = 0;
    for (int t = 0; t < nthreads; ++t) {
        pthread_join(th[t], NULL);
        f = fq12_mul(f, jobs[t].f);
        live += jobs[t].live;
    }
    fq12 r = fq12_one();
    if (live && fq12_final_exponentiation(f, &r)) abort();
    ST(fq12, o, r);
}
void orc_g1_mul_many(const orc_g1* p, const orc_fe* k, size_t n, orc_g1* out, int nthreads) { run_many(1, p, k, n, out, nthreads); }
void orc_g2_mul_many(const orc_g2* p, const orc_fe* k, size_t n, orc_g2* out, int nthreads) { run_many(2, p, k, n, out, nthreads); }

/* ------------------------------------------------------------------ */
/* Encodings, validation, square roots, decompression, Gt::pow        */
/*                                          */

/* U256::from_slice, arith.rs:202-216 (32 bytes big endian; the length check is the caller's) */
static u256 u256_from_be(const uint8_t* s) {
    u256 r;
    for (int l = 1, i = 0; l >= 0; --l, i += 16) {
        u128 v = 0;
        for (int k = 0; k < 16; ++k) v = (v << 8) | s[i + k];           /* BigEndian::read_u128 */
        r.d[l] = v;
    }
    return r;
}
/* U256::to_big_endian, arith.rs:218-231 */
static void u256_to_be(u256 a, uint8_t* s) {
    for (int l = 1, i = 0; l >= 0; --l, i += 16)
        for (int k = 0; k < 16; ++k) s[i + k] = (uint8_t)(a.d[l] >> (8 * (15 - k)));
}
typedef struct { u128 d[4]; } u512;                                  /* arith.rs:23 */
static u512 u512_from_be(const uint8_t* s) {                        /* arith.rs:82-96 */
    u512 r;
    for (int l = 3, i = 0; l >= 0; --l, i += 16) {
        u128 v = 0;
        for (int k = 0; k < 16; ++k) v = (v << 8) | s[i + k];
        r.d[l] = v;
    }
    return r;
}
static int u256_set_bit(u256* a, int n, int to) {                  /* arith.rs:252-267 */
    if (n >= 256) return 0;
    const int part = n / 128, bit = n - 128 * part;
    if (to) a->d[part] |= (u128)1 << bit; else a->d[part] &= ~((u128)1 << bit);
    return 1;
}
/* U512::divrem, arith.rs:116-138: remainder, and the quotient if it is below the modulus */
static int u512_divrem(const u512* a, const u256* m, u256* q_out, u256* r_out) {
    int q_some = 1;
    u256 q = U(0, 0, 0, 0), r = U(0, 0, 0, 0);
    for (int i = 511; i >= 0; --i) {
        const u128 top = r.d[0] >> 127;                              /* mul2, arith.rs:409-414 */
        r.d[0] <<= 1;
        r.d[1] = (r.d[1] << 1) | top;
        u256_set_bit(&r, 0, (int)((a->d[i / 128] >> (i % 128)) & 1));
        if (u256_cmp(&r, m) >= 0) {
            sub_noborrow(r.d, m->d);
            if (q_some && !u256_set_bit(&q, i, 1)) q_some = 0;
        }
    }
    if (q_some && u256_cmp(&q, m) >= 0) q_some = 0;
    *q_out = q;
    *r_out = r;
    return q_some;
}
/* U512::new(c1, c0, modulo) = c1 * modulo + c0, arith.rs:47-80 (used by Fq2::to_u512) */
static u512 u512_new(const u256* c1, const u256* c0, const u256* m) {
    u128 res[4] = {0, 0, 0, 0};
    for (int i = 0; i < 2; ++i) mac_digit(i, res, m->d, c1->d[i]);
    u128 carry = 0;
    for (int i = 0; i < 2; ++i) res[i] = adc(res[i], c0->d[i], &carry);
    for (int i = 0; i < 2; ++i) {
        const u128 a1 = res[i + 2] >> 64, a0 = res[i + 2] & M64;
        u128 s0 = a0 + carry, c = s0 >> 64, r0 = s0 & M64;
        u128 s1 = a1 + c, r1 = s1 & M64;
        carry = s1 >> 64;
        res[i + 2] = (r1 << 64) | r0;
    }
    u512 o = {{res[0], res[1], res[2], res[3]}};
    return o;
}
static int u512_cmp(const u512* a, const u512* b) {                 /* arith.rs:147-160 */
    for (int i = 3; i >= 0; --i) {
        if (a->d[i] < b->d[i]) return -1;
        if (a->d[i] > b->d[i]) return 1;
    }
    return 0;
}

/* Fp::new (fp.rs:46-54): below the modulus -> Montgomery, else None */
static int fe_new(u256 a, const fparams* P, fe* out) {
    if (u256_cmp(&a, &P->m) >= 0) return 1;
    u256_mul(&a, &P->r2, &P->m, P->inv);
    *out = a;
    return 0;
}
static u256 fe_into_u256(fe a, const fparams* P) {                 /* fp.rs:13-20 */
    u256 one = U(1, 0, 0, 0);
    u256_mul(&a, &one, &P->m, P->inv);
    return a;
}
/* generic FieldElement::pow, fields/mod.rs:35-46 (256 bits, MSB first) */
static fe fe_pow(fe a, u256 by, const fparams* P) {
    fe res = P->one;
    for (int n = 255; n >= 0; --n) {
        res = fe_squared(res, P);
        if ((by.d[n / 128] >> (n % 128)) & 1) res = fe_mul(a, res, P);
    }
    return res;
}
static fq2 fq2_pow(fq2 a, u256 by) {
    fq2 res = fq2_one();
    for (int n = 255; n >= 0; --n) {
        res = fq2_squared(res);
        if ((by.d[n / 128] >> (n % 128)) & 1) res = fq2_mul(a, res);
    }
    return res;
}
/* lazy_static FQ_MINUS3_DIV4 / FQ_MINUS1_DIV2 (fp.rs:235-243, fq2.rs:192-200), as U256 (canonical) */
static u256 fq_minus3_div4(void) {
    fe three, four, inv4;
    fe_new(U(3, 0, 0, 0), FQ, &three);
    fe_new(U(4, 0, 0, 0), FQ, &four);
    inv4 = four;
    fe_inverse(&inv4, FQ);
    return fe_into_u256(fe_mul(fe_neg(three, FQ), inv4, FQ), FQ);
}
static u256 fq_minus1_div2(void) {
    fe one, two, inv2;
    fe_new(U(1, 0, 0, 0), FQ, &one);
    fe_new(U(2, 0, 0, 0), FQ, &two);
    inv2 = two;
    fe_inverse(&inv2, FQ);
    return fe_into_u256(fe_mul(fe_neg(one, FQ), inv2, FQ), FQ);
}
/* Fq::sqrt, fp.rs:245-260 */
static int fq_sqrt(fe a, fe* out) {
    fe a1 = fe_pow(a, fq_minus3_div4(), FQ);
    fe a1a = fq_mul(a1, a);
    fe a0 = fq_mul(a1, a1a);
    u256 am1 = FQ->m;
    u256 one = U(1, 0, 0, 0);
    u256_sub(&am1, &one, &FQ->m);
    fe m1;
    fe_new(am1, FQ, &m1);
    if (fq_eq(a0, m1)) return 1;
    *out = a1a;
    return 0;
}
static fq2 fq2_i(void) { return F2(fq_zero(), fq_one()); }       /* fq2.rs:203-205 */
/* Fq2::sqrt, fq2.rs:208-224 */
static int fq2_sqrt(fq2 a, fq2* out) {
    fq2 a1 = fq2_pow(a, fq_minus3_div4());
    fq2 a1a = fq2_mul(a1, a);
    fq2 alpha = fq2_mul(a1, a1a);
    fq2 a0 = fq2_mul(fq2_pow(alpha, FQ->m), alpha);
    const fq2 neg_one = fq2_neg(fq2_one());
    if (fq2_eq(a0, neg_one)) return 1;
    if (fq2_eq(alpha, neg_one)) {
        *out = fq2_mul(fq2_i(), a1a);
    } else {
        fq2 b = fq2_pow(fq2_add(alpha, fq2_one()), fq_minus1_div2());
        *out = fq2_mul(b, a1a);
    }
    return 0;
}
static u512 fq2_to_u512(fq2 a) {                                   /* fq2.rs:226-231 */
    u256 c0 = fe_into_u256(a.c0, FQ), c1 = fe_into_u256(a.c1, FQ);
    return u512_new(&c1, &c0, &FQ->m);
}

/* AffineG::new, mod.rs:95-113 (G1: check_order false; G2: true) */
static int g1_affine_new(fe x, fe y) {
    if (!fq_eq(fq_sq(y), fq_add(fq_mul(fq_sq(x), x), g1_coeff_b()))) return ORC_GROUP_NOT_ON_CURVE;
    return ORC_OK;
}
static int g2_affine_new(fq2 x, fq2 y) {
    if (!fq2_eq(fq2_squared(y), fq2_add(fq2_mul(fq2_squared(x), x), g2_coeff_b()))) return ORC_GROUP_NOT_ON_CURVE;
    g2 p = {x, y, fq2_one()};
    /* p * (-Fr::one()) + p != G::zero(); U256::from(-Fr::one()) = r - 1 */
    u256 rm1 = FRP.m;
    rm1.d[0] -= 1;                                                   /* r is odd: no borrow */
    g2 t = g2_mul_u256(&p, rm1);
    t = g2_add(&t, &p);
    g2 z = g2_zero();
    if (!g2_eq(&t, &z)) return ORC_GROUP_NOT_IN_SUBGROUP;
    return ORC_OK;
}

/* ---- exported ---- */
int orc_fq_from_slice(const uint8_t* s, orc_fe* out) {             /* lib.rs:154-159 */
    FP(0);
    fe x;
    if (fe_new(u256_from_be(s), FQ, &x)) return ORC_FIELD_NOT_MEMBER;
    ST(fe, out, x);
    return ORC_OK;
}
void orc_fq_to_big_endian(const orc_fe* a, uint8_t* s) {            /* lib.rs:160-170 */
    FP(0);
    u256 x = fe_into_u256(LD(fe, a), FQ);
    u256_mul(&x, &FQ->one, &FQ->m, FQ->inv);
    u256_to_be(x, s);
}
int orc_fq2_from_slice(const uint8_t* s, orc_fq2* out) {           /* lib.rs:260-267 */
    FP(0);
    u512 v = u512_from_be(s);
    u256 q, r;
    int q_some = u512_divrem(&v, &FQ->m, &q, &r);
    fe c0, c1;
    if (fe_new(r, FQ, &c0)) return ORC_FIELD_NOT_MEMBER;
    if (!q_some) return ORC_FIELD_NOT_MEMBER;
    if (fe_new(q, FQ, &c1)) return ORC_FIELD_NOT_MEMBER;
    fq2 o = F2(c0, c1);
    ST(fq2, out, o);
    return ORC_OK;
}
void orc_fr_from_slice(const uint8_t* s, orc_fe* out) {             /* lib.rs:45-49, fp.rs:57-60 */
    u256 a = u256_from_be(s);
    const fparams* P = FP(1);
    u256_mul(&a, &P->r2, &P->m, P->inv);                             /* new_mul_factor */
    ST(fe, out, a);
}
void orc_fr_to_big_endian(const orc_fe* a, uint8_t* s) {            /* lib.rs:50-55: raw Montgomery */
    u256_to_be(LD(u256, a), s);
}
int orc_u512_divrem(const uint8_t* be64, orc_fe* q, orc_fe* r) {    /* arith.rs:116-138; 1 = quotient Some */
    FP(0);
    u512 v = u512_from_be(be64);
    return u512_divrem(&v, &FQ->m, (u256*)(void*)q, (u256*)(void*)r);
}
int orc_fq_sqrt(const orc_fe* a, orc_fe* out) { FP(0); return fq_sqrt(LD(fe, a), (fe*)(void*)out); }
int orc_fq2_sqrt(const orc_fq2* a, orc_fq2* out) { FP(0); return fq2_sqrt(LD(fq2, a), (fq2*)(void*)out); }
int orc_g1_affine_new(const orc_fe* x, const orc_fe* y, orc_g1* out) {
    FP(0);
    int st = g1_affine_new(LD(fe, x), LD(fe, y));
    if (st == ORC_OK) { g1 p = {LD(fe, x), LD(fe, y), fq_one()}; ST(g1, out, p); }  /* to_jacobian, mod.rs:220-226 */
    return st;
}
int orc_g2_affine_new(const orc_fq2* x, const orc_fq2* y, orc_g2* out) {
    FP(0);
    int st = g2_affine_new(LD(fq2, x), LD(fq2, y));
    if (st == ORC_OK) { g2 p = {LD(fq2, x), LD(fq2, y), fq2_one()}; ST(g2, out, p); }
    return st;
}
/* G1::from_compressed, lib.rs:359-375 */
int orc_g1_from_compressed(const uint8_t* bytes, size_t len, orc_g1* out) {
    FP(0);
    if (len != 33) return ORC_CURVE_INVALID_ENCODING;
    const uint8_t sign = bytes[0];
    fe x;
    if (fe_new(u256_from_be(bytes + 1), FQ, &x)) return ORC_FIELD_NOT_MEMBER;  /* CurveError::Field(NotMember) */
    fe y_squared = fq_add(fq_mul(fq_mul(x, x), x), g1_coeff_b());
    fe y;
    if (fq_sqrt(y_squared, &y)) return ORC_CURVE_NOT_MEMBER;
    const int odd = (int)(fe_into_u256(y, FQ).d[0] & 1);
    if (sign == 2 && odd) y = fq_neg(y);
    else if (sign == 3 && !odd) y = fq_neg(y);
    else if (sign != 3 && sign != 2) return ORC_CURVE_INVALID_ENCODING;
    if (g1_affine_new(x, y) != ORC_OK) return ORC_CURVE_NOT_MEMBER;
    g1 p = {x, y, fq_one()};
    ST(g1, out, p);
    return ORC_OK;
}
/* G2::from_compressed, lib.rs:506-526 */
int orc_g2_from_compressed(const uint8_t* bytes, size_t len, orc_g2* out) {
    FP(0);
    if (len != 65) return ORC_CURVE_INVALID_ENCODING;
    const uint8_t sign = bytes[0];
    fq2 x;
    int st = orc_fq2_from_slice(bytes + 1, (orc_fq2*)(void*)&x);
    if (st != ORC_OK) return st;                                     /* CurveError::Field(..) */
    fq2 y_squared = fq2_add(fq2_mul(fq2_mul(x, x), x), g2_coeff_b());
    fq2 y;
    if (fq2_sqrt(y_squared, &y)) return ORC_CURVE_NOT_MEMBER;
    fq2 y_neg = fq2_neg(y);
    u512 a = fq2_to_u512(y), b = fq2_to_u512(y_neg);
    const int y_gt = u512_cmp(&a, &b) > 0;
    fq2 e_y;
    if (sign == 10) e_y = y_gt ? y_neg : y;
    else if (sign == 11) e_y = y_gt ? y : y_neg;
    else return ORC_CURVE_INVALID_ENCODING;
    if (g2_affine_new(x, e_y) != ORC_OK) return ORC_CURVE_NOT_MEMBER;
    g2 p = {x, e_y, fq2_one()};
    ST(g2, out, p);
    return ORC_OK;
}
/* Gt::pow, lib.rs:592-594 -> Fq12 pow (fields/mod.rs:35-46) by U256::from(Fr) */
void orc_gt_pow(const orc_fq12* a, const orc_fe* fr_mont, orc_fq12* out) {
    FP(0);
    u256 e = fe_into_u256(LD(fe, fr_mont), FP(1));
    ST(fq12, out, fq12_pow(LD(fq12, a), e));
}

/* threaded forms for the large-sample parity tests */
typedef struct { int kind; const uint8_t* in; void* out; uint8_t* st; size_t lo, hi; } cjob;
static void* run_cjob(void* arg) {
    cjob* j = (cjob*)arg;
    for (size_t i = j->lo; i < j->hi; ++i) {
        if (j->kind == 0) j->st[i] = (uint8_t)orc_g1_from_compressed(j->in + 33 * i, 33, (orc_g1*)j->out + i);
        else if (j->kind == 1) j->st[i] = (uint8_t)orc_g2_from_compressed(j->in + 65 * i, 65, (orc_g2*)j->out + i);
        else {
            const orc_fq2* xy = (const orc_fq2*)(const void*)j->in + 2 * i;
            j->st[i] = (uint8_t)orc_g2_affine_new(&xy[0], &xy[1], (orc_g2*)j->out + i);
        }
    }
    return NULL;
}
void orc_decode_many(int kind, const uint8_t* in, size_t n, void* out, uint8_t* status, int nthreads) {
    FP(0);
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    if ((size_t)nthreads > n) nthreads = n ? (int)n : 1;
    pthread_t th[256];
    cjob jobs[256];
    for (int t = 0; t < nthreads; ++t) {
        cjob j = {kind, in, out, status, n * t / nthreads, n * (t + 1) / nthreads};
        jobs[t] = j;
        pthread_create(&th[t], NULL, run_cjob, &jobs[t]);
    }
    for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
}
