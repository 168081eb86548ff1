// fq12_wide.h -- one Fq12 spread over twelve lanes ("wide" layout), for the
// latency-bound end of the pairing path: the final exponentiation of a handful
// of values (pairing_batch, small batches) and the product reduction of
// pairing_batch / miller_loop_batch (mod.rs:609-640, 904-926).
//
// Why: the batch layout (fq2_split.h) runs one Fq12 on two lanes, so a single
// final exponentiation is one lane pair doing ~17k dependent Fq products --
// 2.9 ms on an otherwise idle GPU (profiles/r2f_kernel_stats_product.csv).
// Here a group of 16 lanes holds one element: lane 2e + c holds coordinate c
// of the Fq2 coefficient of w^e (Fq12 = Fq2[w]/(w^6 - xi); w^e is c0.c(e/2)
// for even e and c1.c((e-1)/2) for odd e, fq12.rs:52-55).  Lanes 12..15 mirror
// lanes 10..11 (e = 5) and are never read.  A product is a schoolbook sum over
// the six coefficients of each operand, so every lane accumulates twelve digit
// products into one set of column sums and reduces ONCE: out_e = sum_i a'_i *
// b_(e-i mod 6) with a'_i = xi*a_i when i > e (w^6 = xi).  Operands are
// exchanged through a per-group LDS area (each lane writes its coordinate,
// then reads the ones it needs; a wave runs its LDS operations in order, so
// the exchange needs no barrier).  Within a lane pair the two-lane Fq2
// operations of fq2_split.h apply unchanged (partner over DPP).
//
// Bit-exactness: every operation computes the field value of the reference
// operation it replaces (schoolbook vs Karatsuba is a ring identity; the
// cyclotomic squaring is the reference's Granger-Scott formula, fq12.rs:198-247),
// and images are canonicalized at the boundary as everywhere else.
#pragma once
#include "kernels.h"

namespace bn {
static_assert(BN_SPLIT, "fq12_wide.h builds on the two-lane Fq2 of fq2_split.h");

constexpr int kWLanes = 16;                         // lanes per element (12 hold coordinates)
constexpr int kWSlot = 12;                          // words per LDS slot: one Fq, 48 B aligned
constexpr int kWArr = kWLanes * kWSlot;             // words of one operand array of a group
// operand arrays per group: 5 for w12_sqr; 4 (w12_mul only) in the two-wave
// latency build, whose LDS must fit two blocks per CU (kernels_latency_w2.hip)
#ifndef BN_WIDE_ARRS
#define BN_WIDE_ARRS 5
#endif
constexpr int kWArrs = BN_WIDE_ARRS;
constexpr int kWGroupWords = kWArrs * kWArr;        // 3.75 KB per group
// threads of the blocks of the including translation unit's wide kernels (256:
// 16 groups)
#ifndef BN_WIDE_THREADS
#define BN_WIDE_THREADS kBlock
#endif
constexpr int kWGroups = BN_WIDE_THREADS / kWLanes;  // 16 groups per 256-thread block
__shared__ uint32_t g_wide[kWGroups * kWGroupWords];  // 60 KB

// this lane's place in its group
struct WL {
    uint32_t* gb;  // the group's LDS operand area
    int l;         // lane in group, 0..15 (LDS slot)
    int e;         // w exponent of the coefficient (lanes 12..15 mirror e = 5)
    int c;         // coordinate: 0 = c0, 1 = c1 of the Fq2 coefficient
};
__device__ __forceinline__ WL wl() {
    const int t = (int)threadIdx.x;
    WL w;
    w.l = t & (kWLanes - 1);
    w.e = (w.l >> 1) < 5 ? (w.l >> 1) : 5;
    w.c = t & 1;
    w.gb = g_wide + (t / kWLanes) * kWGroupWords;
    return w;
}
// Gt image index of this lane's coordinate (c_i.c_j.c_k at 6i + 2j + k)
__device__ __forceinline__ int w_gt_index(const WL& w) { return 6 * (w.e & 1) + 2 * (w.e >> 1) + w.c; }
// tower index of the lane's Fq2 (c_i.c_j at 3i + j): the slot j of the
// lane-strided split layout (kernels.h st_fq12/ld_fq12)
__device__ __forceinline__ int w_tower_index(const WL& w) { return 3 * (w.e & 1) + (w.e >> 1); }

template <int K>
__device__ __forceinline__ void w_put(uint32_t* arr, int slot, const Fq<K>& x) {
    static_assert(kl(K) == 1, "w_put: normalized digits");
    uint32_t* p = arr + slot * kWSlot;
    *(uint4*)p = make_uint4(x.v[0], x.v[1], x.v[2], x.v[3]);
    *(uint4*)(p + 4) = make_uint4(x.v[4], x.v[5], x.v[6], x.v[7]);
    p[8] = x.v[8];
}
template <int K>
__device__ __forceinline__ Fq<K> w_get(const uint32_t* arr, int slot) {
    const uint32_t* p = arr + slot * kWSlot;
    const uint4 a = *(const uint4*)p, b = *(const uint4*)(p + 4);
    return Fq<K>{{a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w, p[8]}};
}
// this lane's coordinate of element e of a lane-strided split Fq12 array
// (stride = elements in the array)
__device__ __forceinline__ Fq<2> w_ld_split(const uint32_t* f, size_t stride, size_t e, const WL& w) {
    return ld_fq<2>(f, 2 * stride, 2 * e + w.c, w_tower_index(w));
}
__device__ __forceinline__ void w_st_split(uint32_t* f, size_t stride, size_t e, const WL& w, const Fq<2>& x) {
    if (w.l < 12) st_fq(f, 2 * stride, 2 * e + w.c, w_tower_index(w), x);
}

// the writes above are complete before any lane reads (and the compiler keeps order)
__device__ __forceinline__ void w_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// normalized, value <= 2p
template <int K>
__device__ __forceinline__ Fq<2> w_narrow(const Fq<K>& a) {
    if constexpr (kv(K) <= 2) return widen<2>(fq_norm(a)); else return fq_fold(a);
}

// The twelve-product sums use the column accumulator of fq.h (Acc, acc_mad,
// acc_carry_par, acc_redc).

// ---------------------------------------------------------------- operations
// this lane's coordinate of xi * (the lane pair's Fq2), xi = 9 + u (fq2.rs:19-34)
template <int K>
__device__ __forceinline__ Fq<2> w_xi(const Fq<K>& a) { return fq2_fold(fq2_mul_xi(Fq2<K>{a})).c; }

// a * b (fq12.rs:319-327), schoolbook over the w-basis, one reduction per lane
__device__ __noinline__ Fq<2> w12_mul(Fq<2> a, Fq<2> b) {
    const WL w = wl();
    uint32_t* A_ = w.gb;
    uint32_t* X_ = w.gb + kWArr;
    uint32_t* B_ = w.gb + 2 * kWArr;
    uint32_t* N_ = w.gb + 3 * kWArr;
    w_put(A_, w.l, a);
    w_put(X_, w.l, w_xi(a));
    w_put(B_, w.l, b);
    w_put(N_, w.l, fq_neg(b));
    w_sync();
    Acc t = {};
#pragma unroll
    for (int i = 0; i < 6; ++i) {
        const bool wrap = i > w.e;                  // a_i * b_(e-i+6) * w^6, w^6 = xi
        const int j = wrap ? w.e - i + 6 : w.e - i;
        const uint32_t* src = wrap ? X_ : A_;
        const Fq<2> x0 = w_get<2>(src, 2 * i), x1 = w_get<2>(src, 2 * i + 1);
        // c0: x0*b0 - x1*b1, c1: x0*b1 + x1*b0
        const Fq<2> yo = w_get<2>(B_, 2 * j + w.c);
        const Fq<2> yx = w_get<2>(w.c ? B_ : N_, 2 * j + 1 - w.c);
        acc_mad(t, x0, yo);
        acc_mad(t, x1, yx);
        if (i == 2) acc_carry_par(t);  // six normalized products per batch keep columns < 2^64
    }
    // value <= 12 * (2p)^2: the result is below (48 p / 2^261 + 1) p < 2p
    return acc_redc<2>(t);
}

// a^2 (fq12.rs:319-327 with b = a), the schoolbook sum folded by symmetry: out_e
// = sum over i + j = e (mod 6) of a'_i a_j pairs each unordered {i, j}, i != j,
// twice, so out_e = 2 * (sum over the cross pairs of xi^w a_i a_j + sum over
// the squares of xi^w a_i (a_i / 2)), w = [i + j >= 6] (w^6 = xi).  Every lane
// has at most four such terms (two cross + two squares for even e, three cross
// for odd e): eight digit products instead of twelve, one doubling of the
// columns, one reduction.  The same residues as w12_mul(a, a).
// Per lane e, term t: operand source of x (0 = a, 1 = xi a, 2 = a/2, 3 = xi a / 2)
// and the indices i (of x) and j (of y = a); source 3 with i = 6 reads the zero
// slots 12, 13 of the xi a / 2 array (an absent fourth term).
constexpr uint64_t w_sqr_code(int src, int i, int j) { return (uint64_t)(src | (i << 2) | (j << 5)); }
constexpr uint64_t w_sqr_term(uint64_t e0, uint64_t e1, uint64_t e2, uint64_t e3, uint64_t e4, uint64_t e5) {
    return e0 | (e1 << 8) | (e2 << 16) | (e3 << 24) | (e4 << 32) | (e5 << 40);
}
constexpr uint64_t kWSqrTerm[4] = {
    w_sqr_term(w_sqr_code(1, 1, 5), w_sqr_code(0, 0, 1), w_sqr_code(0, 0, 2), w_sqr_code(0, 0, 3), w_sqr_code(0, 0, 4), w_sqr_code(0, 0, 5)),
    w_sqr_term(w_sqr_code(1, 2, 4), w_sqr_code(1, 2, 5), w_sqr_code(1, 3, 5), w_sqr_code(0, 1, 2), w_sqr_code(0, 1, 3), w_sqr_code(0, 1, 4)),
    w_sqr_term(w_sqr_code(2, 0, 0), w_sqr_code(1, 3, 4), w_sqr_code(2, 1, 1), w_sqr_code(1, 4, 5), w_sqr_code(2, 2, 2), w_sqr_code(0, 2, 3)),
    w_sqr_term(w_sqr_code(3, 3, 3), w_sqr_code(3, 6, 0), w_sqr_code(3, 4, 4), w_sqr_code(3, 6, 0), w_sqr_code(3, 5, 5), w_sqr_code(3, 6, 0)),
};
// (squarings as w12_mul(a, a) instead: within 1 %, profiles/r3y_ab_wide_sqr.txt)
#if BN_WIDE_ARRS >= 5
__device__ __noinline__ Fq<2> w12_sqr(Fq<2> a) {
    const WL w = wl();
    uint32_t* A_ = w.gb;
    uint32_t* X_ = w.gb + kWArr;
    uint32_t* N_ = w.gb + 2 * kWArr;
    uint32_t* H_ = w.gb + 3 * kWArr;
    uint32_t* XH_ = w.gb + 4 * kWArr;
    const Fq<2> xa = w_xi(a);
    w_put(A_, w.l, a);
    w_put(X_, w.l, xa);
    w_put(N_, w.l, fq_neg(a));
    w_put(H_, w.l, fq_half(a));
    w_put(XH_, w.l, w.l < 12 ? fq_half(xa) : widen<2>(fq_zero()));  // slots 12..15: the zero operand
    w_sync();
    Acc t = {};
#pragma unroll 1
    for (int q = 0; q < 4; ++q) {
        const uint64_t tq = q == 0 ? kWSqrTerm[0] : q == 1 ? kWSqrTerm[1] : q == 2 ? kWSqrTerm[2] : kWSqrTerm[3];
        const uint32_t code = (uint32_t)(tq >> (8 * w.e)) & 0xffu;
        const uint32_t src = code & 3u, i = (code >> 2) & 7u, j = code >> 5;
        const uint32_t* xs = src == 0 ? A_ : src == 1 ? X_ : src == 2 ? H_ : XH_;
        const Fq<2> x0 = w_get<2>(xs, (int)(2 * i)), x1 = w_get<2>(xs, (int)(2 * i + 1));
        // c0: x0*y0 + x1*(-y1), c1: x0*y1 + x1*y0
        const Fq<2> yo = w_get<2>(A_, (int)(2 * j) + w.c);
        const Fq<2> yx = w_get<2>(w.c ? A_ : N_, (int)(2 * j) + 1 - w.c);
        acc_mad(t, x0, yo);
        acc_mad(t, x1, yx);
        if (q == 2) acc_carry_par(t);  // six normalized products per batch keep columns < 2^64
    }
    // columns < 2^36 + 18 * 2^58, doubled < 2^37 + 36 * 2^58: with the reduction's
    // nine m*p products and its carries they stay below 2^64
#pragma unroll
    for (int k = 0; k < 17; ++k) t.c[k] <<= 1;
    // value <= 2 * 8 * (2p)^2: the result is below (64 p / 2^261 + 1) p < 2p
    return acc_redc<2>(t);
}
__device__ __forceinline__ Fq<2> w12_square(const Fq<2>& a) { return w12_sqr(a); }
#else
__device__ __forceinline__ Fq<2> w12_square(const Fq<2>& a) { return w12_mul(a, a); }
#endif

// Line ring of k_pairing_latency (kernels_wide.hip): per pair kLatRing lines of
// x0, x4, x2, each stored as the three operand forms of the split product --
// c0, c1 and -c1 (slots 3q, 3q + 1, 3q + 2; kWSlot words each) -- so a consumer
// lane reads its two operands with no select or negation
#ifndef BN_LAT_RING
#define BN_LAT_RING 16
#endif
constexpr int kLatRing = BN_LAT_RING;      // lines in flight per pair
constexpr int kLatLineWords = 9 * kWSlot;  // words per line
__shared__ uint32_t g_lat_ring[kLatPairs * kLatRing * kLatLineWords];  // 54 KB

// a * line (fq12.rs:130-196, mul_by_024 on the w-basis): the line is
// x0 + x4 w^3 + x2 w^4, its three Fq2 coefficients read from the ring at word
// ln_off (an offset, so the compiler addresses LDS, not flat memory).  out_e = sum over the
// three nonzero line coefficients b_m of a'_(e-m) * b_m with a'_i = xi * a_i
// when the index wraps (w^6 = xi): six digit products per lane, one reduction.
// The same residues as the reference's sparse product.
// BN_W12_LINE_DOT6: the six digit products of w12_mul_line as one asm chain (as the
// two-lane line product, pairing.h BN_DOT6_ASM) instead of 17 column accumulators:
// the two-wave latency kernel at 4,096 pairs 1.58 -> 1.56-1.57 ms, the rest within
// noise (profiles/r5aa_ab_w12_line_dot6.txt)
#ifndef BN_W12_LINE_DOT6
#define BN_W12_LINE_DOT6 1
#endif
__device__ __noinline__ Fq<2> w12_mul_line(Fq<2> a, uint32_t ln_off) {
    const WL w = wl();
    const uint32_t* ln = g_lat_ring + ln_off;
    uint32_t* A_ = w.gb;
    uint32_t* X_ = w.gb + kWArr;
    w_put(A_, w.l, a);
    w_put(X_, w.l, w_xi(a));
    w_sync();
    constexpr int kM[3] = {0, 3, 4};  // w-exponents of x0, x4, x2
#if BN_W12_LINE_DOT6 && BN_DOT2_ASM && defined(__HIP_DEVICE_COMPILE__)
    // the six digit products as one v_mad_u64_u32 chain (dot2_asm.inc BN_ASM_DOT6)
    Fq<2> xs[6];
    Fq<kLine> ys[6];
#pragma unroll
    for (int q = 0; q < 3; ++q) {
        const int m = kM[q];
        const bool wrap = m > w.e;
        const int i = wrap ? w.e - m + 6 : w.e - m;
        const uint32_t* src = wrap ? X_ : A_;
        xs[2 * q] = w_get<2>(src, 2 * i);
        xs[2 * q + 1] = w_get<2>(src, 2 * i + 1);
        ys[2 * q] = w_get<kLine>(ln, 3 * q + w.c);
        ys[2 * q + 1] = w_get<kLine>(ln, 3 * q + (w.c ? 0 : 2));
    }
    Fq<2> r;
    asm(BN_ASM_DOT6 : BN_ASM_OUT9(r.v)
        : BN_ASM_IN9(xs[0].v), BN_ASM_IN9(ys[0].v), BN_ASM_IN9(xs[1].v), BN_ASM_IN9(ys[1].v), BN_ASM_IN9(xs[2].v),
          BN_ASM_IN9(ys[2].v), BN_ASM_IN9(xs[3].v), BN_ASM_IN9(ys[3].v), BN_ASM_IN9(xs[4].v), BN_ASM_IN9(ys[4].v),
          BN_ASM_IN9(xs[5].v), BN_ASM_IN9(ys[5].v), BN_ASM_P
        : BN_ASM_CLOBBER);
    return r;
#else
    Acc t = {};
#pragma unroll
    for (int q = 0; q < 3; ++q) {
        const int m = kM[q];
        const bool wrap = m > w.e;
        const int i = wrap ? w.e - m + 6 : w.e - m;
        const uint32_t* src = wrap ? X_ : A_;
        const Fq<2> x0 = w_get<2>(src, 2 * i), x1 = w_get<2>(src, 2 * i + 1);
        // line coordinates: normalized, value <= kLine p (the producer narrows them)
        // c0: x0*b0 + x1*(-b1), c1: x0*b1 + x1*b0
        const Fq<kLine> yo = w_get<kLine>(ln, 3 * q + w.c);
        const Fq<kLine> yx = w_get<kLine>(ln, 3 * q + (w.c ? 0 : 2));
        acc_mad(t, x0, yo);
        acc_mad(t, x1, yx);
    }
    // value <= 6 * 2p * 4p: the reduction is below (48 p / 2^261 + 1) p < 2p
    return acc_redc<2>(t);
#endif
}
// the line x0 + x4 w^3 + x2 w^4 itself as an element (one * line, the first
// step of the loop from f = one)
__device__ __forceinline__ Fq<2> w12_from_line(uint32_t ln_off) {
    const WL w = wl();
    const uint32_t* ln = g_lat_ring + ln_off;
    const int q = w.e == 0 ? 0 : w.e == 3 ? 1 : 2;
    const Fq<kLine> v = w_get<kLine>(ln, 3 * q + w.c);
    return w_narrow(fq_select(w.e == 0 || w.e == 3 || w.e == 4, v, widen<kLine>(fq_zero())));
}

// Granger-Scott cyclotomic squaring (fq12.rs:198-247).  Pairs (z0,z1), (z2,z3),
// (z4,z5) are the coefficient pairs (w^k, w^(k+3)), k = 0, 1, 2.  Lane pair e < 3
// computes tmp_e = x*y for pair k = e; lane pair e >= 3 computes
// (x + y)(xi*y + x) for pair k = e - 3; then every lane forms its output
// coordinate from them: t0 = P3 - P0 - xi*P0 etc. as in the reference.
// Operands are chosen by LDS address rather than by per-digit selects: slots
// 12..15 of A_ (the mirror lanes') hold zero, the "absent" term of the lo lanes,
// and each lane reads its own and its partner coordinate of V directly; xi * a
// stays unfolded (bound 21p: the product's column budget and bound allow it)
// and the product is stored at its own bound 3p.  787 -> 7xx VALU per squaring
// (profiles/r5e_*).
__device__ __forceinline__ Fq<21> w_xi_loose(const Fq<2>& a) { return fq_norm(fq2_mul_xi(Fq2<2>{a}).c); }
__device__ __noinline__ Fq<2> w12_cyc(Fq<2> a) {
    const WL w = wl();
    uint32_t* A_ = w.gb;
    uint32_t* X_ = w.gb + kWArr;
    uint32_t* P_ = w.gb + 2 * kWArr;
    uint32_t* Q_ = w.gb + 3 * kWArr;
    constexpr int kZ = 12;  // a zero slot of A_
    w_put(A_, w.l, fq_select(w.l >= 12, widen<2>(fq_zero()), a));
    w_put(X_, w.l, w_xi_loose(a));
    w_sync();
    const bool hi = w.e >= 3;
    const int k = hi ? w.e - 3 : w.e, c = w.c;
    // U = hi ? x + y : x;  V = hi ? xi*y + x : y: this lane's coordinate of V and
    // its partner's, each as (xi*y or y) + (x or zero)
    const uint32_t* VS = hi ? X_ : A_;
    const Fq<4> u0 = fq_norm(fq_add(w_get<2>(A_, 2 * k), w_get<2>(A_, hi ? 2 * k + 6 : kZ)));
    const Fq<4> u1 = fq_norm(fq_add(w_get<2>(A_, 2 * k + 1), w_get<2>(A_, hi ? 2 * k + 7 : kZ)));
    const auto vo = fq_add(w_get<21>(VS, 2 * k + 6 + c), w_get<2>(A_, hi ? 2 * k + c : kZ));
    const auto vp = fq_add(w_get<21>(VS, 2 * k + 7 - c), w_get<2>(A_, hi ? 2 * k + 1 - c : kZ));
    // lane c of U*V: c0 = u0 v0 - u1 v1 (vx = -v1), c1 = u0 v1 + u1 v0 (vx = v0)
    const auto vx = fq_pick(c != 0, vp, fq_neg_lazy(vp));
    const auto p = fq_dot2(u0, vo, u1, vx);
    static_assert(kl(decltype(fq_dot2(u0, vo, u1, vx))::kK) == 1 && kv(decltype(fq_dot2(u0, vo, u1, vx))::kK) <= 3,
                  "w12_cyc: the product is stored as a normalized value <= 3p");
    const Fq<3> pn = widen<3>(p);
    w_put(P_, w.l, pn);
    w_put(Q_, w.l, w_xi(pn));
    w_sync();
    // even e (z0, z4, z3 = w^0, w^2, w^4): 3*(P_(k+3) - P_k - xi*P_k) - 2*a with k = e/2
    // odd e: z1 = w^3: 6*P_0 + 2a;  z5 = w^5: 6*P_1 + 2a;  z2 = w^1: 6*xi*P_2 + 2a
    const int ka = w.e >> 1;
    const Fq<3> pu = w_get<3>(P_, 2 * (ka + 3) + c), pv = w_get<3>(P_, 2 * ka + c);
    const Fq<2> pw = w_get<2>(Q_, 2 * ka + c);
    const Fq<3> px = w.e == 1 ? widen<3>(w_get<2>(Q_, 4 + c)) : w_get<3>(P_, (w.e >= 3 ? w.e - 3 : 0) + c);
    // one stream for both parities: 3*T + (-2a | 2a), T = ta (even e) or 2*px (odd e)
    const bool even = (w.e & 1) == 0;
    const auto ta = fq_norm(fq_sub(fq_sub(pu, pv), pw));
    const auto t = fq_pick(even, ta, fq_dbl(px));
    const auto a2 = fq_dbl(a);
    const auto s = fq_pick(even, fq_neg_lazy(a2), a2);
    return fq_fold(fq_add(fq_add(t, fq_add(t, t)), s));
}

// The same squaring on a PAIR of groups of one wave (lanes 32j..32j+15: the main
// group, 32j+16..32j+31: the helper), both holding the element: kernels_tail.hip's
// squarer.  The helper's lo lanes compute xi * P_k = (xi x_k) * y_k (xi * x_k is in
// its X_ array already) while the main group computes P_k, so the xi * P values
// the output needs come with the products instead of a w_xi pass after them (~95
// VALU and one LDS round trip fewer per squaring on the chain); both groups then
// form every output coordinate from the main group's P_ and the helper's.  The
// values are the reference's: xi * (x y) and (xi x) y are the same field element.
__device__ __noinline__ Fq<2> w12_cyc32(Fq<2> a) {
    const WL w = wl();
    const bool helper = (((int)threadIdx.x / kWLanes) & 1) != 0;
    uint32_t* A_ = w.gb;
    uint32_t* X_ = w.gb + kWArr;
    uint32_t* P_ = w.gb + 2 * kWArr;
    const uint32_t* PM = (helper ? w.gb - kWGroupWords : w.gb) + 2 * kWArr;  // the main group's products
    const uint32_t* PH = (helper ? w.gb : w.gb + kWGroupWords) + 2 * kWArr;  // the helper's
    constexpr int kZ = 12;  // a zero slot of A_
    w_put(A_, w.l, fq_select(w.l >= 12, widen<2>(fq_zero()), a));
    w_put(X_, w.l, w_xi_loose(a));
    w_sync();
    const bool hi = w.e >= 3;
    const int k = hi ? w.e - 3 : w.e, c = w.c;
    // U = hi ? x + y : (helper ? xi*x : x);  V = hi ? xi*y + x : y
    const uint32_t* US = (helper && !hi) ? X_ : A_;
    const uint32_t* VS = hi ? X_ : A_;
    const Fq<23> u0 = fq_norm(fq_add(w_get<21>(US, 2 * k), w_get<2>(A_, hi ? 2 * k + 6 : kZ)));
    const Fq<23> u1 = fq_norm(fq_add(w_get<21>(US, 2 * k + 1), w_get<2>(A_, hi ? 2 * k + 7 : kZ)));
    const auto vo = fq_add(w_get<21>(VS, 2 * k + 6 + c), w_get<2>(A_, hi ? 2 * k + c : kZ));
    const auto vp = fq_add(w_get<21>(VS, 2 * k + 7 - c), w_get<2>(A_, hi ? 2 * k + 1 - c : kZ));
    const auto vx = fq_pick(c != 0, vp, fq_neg_lazy(vp));
    const auto p = fq_dot2(u0, vo, u1, vx);
    static_assert(kl(decltype(fq_dot2(u0, vo, u1, vx))::kK) == 1 && kv(decltype(fq_dot2(u0, vo, u1, vx))::kK) <= 8,
                  "w12_cyc32: the products are stored as normalized values <= 8p");
    w_put(P_, w.l, widen<8>(p));
    w_sync();
    // even e: 3*(P_(k+3) - P_k - xi*P_k) - 2*a with k = e/2; odd e: z1 = w^3: 6*P_0 + 2a;
    // z5 = w^5: 6*P_1 + 2a;  z2 = w^1: 6*xi*P_2 + 2a  (w12_cyc)
    const int ka = w.e >> 1;
    const Fq<8> pu = w_get<8>(PM, 2 * (ka + 3) + c), pv = w_get<8>(PM, 2 * ka + c);
    const Fq<8> pw = w_get<8>(PH, 2 * ka + c);
    const Fq<8> px = w_get<8>(w.e == 1 ? PH : PM, w.e == 1 ? 4 + c : (w.e >= 3 ? w.e - 3 : 0) + c);
    const bool even = (w.e & 1) == 0;
    const auto ta = fq_norm(fq_sub(fq_sub(pu, pv), pw));
    const auto t = fq_pick(even, ta, fq_dbl(px));
    const auto a2 = fq_dbl(a);
    const auto s = fq_pick(even, fq_neg_lazy(a2), a2);
    return fq_fold(fq_add(fq_add(t, fq_add(t, t)), s));
}
// the squaring on the final exponentiation's squarer chain (w12_exp_sq,
// w12_fe_last_s): kernels_tail.hip runs it on a pair of groups
#ifndef BN_S_CYC
#define BN_S_CYC w12_cyc
#endif

// unitary inverse (fq12.rs:126-128): the w^odd coefficients negate
__device__ __forceinline__ Fq<2> w12_conj(const Fq<2>& a) {
    const WL w = wl();
    return fq_select((w.e & 1) != 0, fq_neg(a), a);
}

// frobenius_map(K) (fq12.rs:112-119, fq6.rs:125-131): coefficient c_i.c_j maps
// to conj^K(x) * fq6_frob_c_j(K) [* fq12_frob_c1(K) for i = 1]
template <int K>
__device__ __noinline__ Fq<2> w12_frob(Fq<2> a) {
    const WL w = wl();
    const int j = w.e >> 1, i = w.e & 1;
    Fq2<2> x = {a};
    if constexpr (K & 1) x = widen<2>(fq2_conj(x));
    const Fq2<1> c6 = fq2_select(j == 1, fq6_frob_c1(K), fq2_select(j == 2, fq6_frob_c2(K), fq2_one()));
    const Fq2<1> c12 = fq2_select(i == 1, fq12_frob_c1(K), fq2_one());
    const auto y = fq2_mul(x, c6);
    return w_narrow(fq2_mul(y, c12).c);
}

// inverse (fq12.rs:305-313): every lane pair gathers the element into the
// two-lane layout, inverts it there (one Fermat inversion of an Fq), and keeps
// its own coefficient
__device__ __noinline__ Fq<2> w12_inv(Fq<2> a) {
    const WL w = wl();
    uint32_t* A_ = w.gb;
    w_put(A_, w.l, a);
    w_sync();
    auto g = [&](int e) { return Fq2<2>{w_get<2>(A_, 2 * e + w.c)}; };
    const Fq12<2> f = {{g(0), g(2), g(4)}, {g(1), g(3), g(5)}};
    const Fq12<2> r = fq12_fold(fq12_inv(f));
    Fq<2> o = r.c0.c0.c;
    o = fq_select(w.e == 1, r.c1.c0.c, o);
    o = fq_select(w.e == 2, r.c0.c1.c, o);
    o = fq_select(w.e == 3, r.c1.c1.c, o);
    o = fq_select(w.e == 4, r.c0.c2.c, o);
    o = fq_select(w.e == 5, r.c1.c2.c, o);
    return o;
}

// every coordinate of the group's element is zero
__device__ __forceinline__ bool w12_is_zero(const Fq<2>& a) {
    const uint64_t m = __ballot(fq_is_zero(a));
    const int sh = (int)(threadIdx.x & 63u) & ~(kWLanes - 1);
    return ((m >> sh) & 0xfffull) == 0xfffull;
}

// ---------------------------------------------------------------- final exponentiation
// exp_by_neg_z (fq12.rs:121-124): conj(x^u), u = 4965661367192848881, by signed
// width-4 windows (x^-d = conj(x^d) in the cyclotomic subgroup, where the final
// exponentiation applies it); the digit table is planned at compile time.
struct ZWin {
    int n = 0;
    int8_t d[32] = {};
    uint8_t run[32] = {};  // squarings before digit t (run[0]: unused)
    uint8_t tail = 0;      // squarings after the last digit
};
constexpr ZWin z_windows() {
    ZWin w;
    uint64_t u = 4965661367192848881ull;
    int dd[32] = {}, pp[32] = {}, n = 0;
    for (int pos = 0; u; ++pos, u >>= 1) {
        if (!(u & 1)) continue;
        int z = (int)(u & 15);
        if (z >= 8) z -= 16;
        dd[n] = z;
        pp[n] = pos;
        ++n;
        u -= (uint64_t)(int64_t)z;
    }
    w.n = n;
    for (int t = 0; t < n; ++t) {  // top digit first
        w.d[t] = (int8_t)dd[n - 1 - t];
        w.run[t] = (uint8_t)(t ? pp[n - t] - pp[n - 1 - t] : 0);
    }
    w.tail = (uint8_t)pp[0];
    return w;
}
constexpr ZWin kZWin = z_windows();

__device__ __noinline__ Fq<2> w12_exp_by_neg_z(Fq<2> x) {
    const Fq<2> x2 = w12_cyc(x);
    const Fq<2> x3 = w12_mul(x, x2);
    const Fq<2> x5 = w12_mul(x3, x2);
    const Fq<2> x7 = w12_mul(x5, x2);
    auto pick = [&](int d) {
        const int m = d < 0 ? -d : d;
        Fq<2> y = m == 1 ? x : m == 3 ? x3 : m == 5 ? x5 : x7;
        return d < 0 ? w12_conj(y) : y;
    };
    Fq<2> r = pick(kZWin.d[0]);
#pragma unroll 1
    for (int t = 1; t < kZWin.n; ++t) {
#pragma unroll 1
        for (int s = 0; s < kZWin.run[t]; ++s) r = w12_cyc(r);
        r = w12_mul(r, pick(kZWin.d[t]));
    }
#pragma unroll 1
    for (int s = 0; s < kZWin.tail; ++s) r = w12_cyc(r);
    return w12_conj(r);
}

// the first chunk of the final exponentiation (fq12.rs:62-73) of a nonzero f:
// f^((p^6 - 1)(p^2 + 1)), an element of the cyclotomic subgroup
__device__ __noinline__ Fq<2> w12_fe_first(Fq<2> f) {
    const Fq<2> b0 = w12_inv(f);
    const Fq<2> c0 = w12_mul(w12_conj(f), b0);
    const Fq<2> d0 = w12_frob<2>(c0);
    return w12_mul(d0, c0);
}
// its last chunk (fq12.rs:75-105) of s = w12_fe_first(f)
__device__ __noinline__ Fq<2> w12_fe_last(Fq<2> s) {
    const Fq<2> a = w12_exp_by_neg_z(s);
    const Fq<2> b = w12_cyc(a);
    const Fq<2> c = w12_cyc(b);
    const Fq<2> d = w12_mul(c, b);
    const Fq<2> e = w12_exp_by_neg_z(d);
    const Fq<2> f1 = w12_cyc(e);
    const Fq<2> g = w12_exp_by_neg_z(f1);
    const Fq<2> j = w12_mul(w12_conj(g), e);
    const Fq<2> k = w12_mul(j, w12_conj(d));
    const Fq<2> l = w12_mul(k, b);
    const Fq<2> m = w12_mul(k, e);
    const Fq<2> n = w12_mul(s, m);
    const Fq<2> o = w12_frob<1>(l);
    const Fq<2> p = w12_mul(o, n);
    const Fq<2> q = w12_frob<2>(k);
    const Fq<2> r = w12_mul(q, p);
    const Fq<2> t = w12_mul(w12_conj(s), l);
    const Fq<2> u = w12_frob<3>(t);
    return w12_mul(u, r);
}
// final_exponentiation (fq12.rs:107-110) of a nonzero f: first chunk and last
// chunk in the reference's order
__device__ __forceinline__ Fq<2> w12_final_exp(const Fq<2>& f) { return w12_fe_last(w12_fe_first(f)); }


// ---------------------------------------------------------------- two-group final exponentiation
// The same final exponentiation on TWO 16-lane groups of one element, in
// different waves: a squarer S runs the chain of dependent squarings and a
// multiplier M folds the products in beside it, so most products leave the
// critical path (a lone wave issues one v_mad_u64_u32 per ~9.5 cycles whatever
// the dependences, profiles/r3j_mad_issue.txt: the two groups' streams run in
// parallel on their SIMDs).  exp_by_neg_z right to left over the NAF of u:
// x^u = prod over the nonzero digits d_k of (x^(2^k))^(d_k), x^-1 = conj(x) in
// the cyclotomic subgroup.  S squares x 62 times and hands over x^(2^k) at each
// of the 24 nonzero digits; M multiplies them into its accumulator (at least two
// squarings apart, so M keeps up) and returns conj(acc).  The values are the
// reference's (fq12.rs:75-110): the same group elements, another addition chain.
// Channel (LDS, per element): a ring of kDuoRing S -> M items and two M -> S
// result slots; counters cnt[0] = items published by S, cnt[1] = items taken by
// M, cnt[2] = results published by M.  A writer waits for its LDS writes
// (lgkmcnt(0)) before bumping a counter; a reader spins on the counter
// (s_sleep) and then reads -- a wave runs its LDS operations in order.
struct ZNaf {
    uint64_t nz = 0, minus = 0;  // digit positions, negative digits
    int top = 0, n = 0;
};
constexpr ZNaf z_naf() {
    ZNaf r;
    uint64_t u = 4965661367192848881ull;
    for (int pos = 0; u; ++pos, u >>= 1) {
        if (!(u & 1)) continue;
        const bool neg = (u & 3) == 3;  // digit -1 when u = 3 mod 4
        r.nz |= 1ull << pos;
        if (neg) r.minus |= 1ull << pos;
        r.top = pos;
        ++r.n;
        u = neg ? u + 1 : u - 1;
    }
    return r;
}
constexpr ZNaf kZNaf = z_naf();
static_assert(kZNaf.top == 62 && kZNaf.n == 24, "NAF of u");

#ifndef BN_DUO_RING
#define BN_DUO_RING 4
#endif
constexpr int kDuoRing = BN_DUO_RING;             // S -> M items in flight
constexpr int kDuoWords = (kDuoRing + 2) * kWArr;  // channel words per element
// The cap of every capped LDS hand-off wait (here and latency_kernel.h): ~4 s of
// s_sleep 1, never reached while both sides run.  A build parameter so that the
// failure-path library (`make -C paritytech-bn_amd cap0`, BN_SPIN_CAP=0) trips
// the waits deterministically and tests/test_gpu_failure.py can check that the
// call then fails with BN_ERR_INTERNAL instead of returning a value.
#ifndef BN_SPIN_CAP
#define BN_SPIN_CAP (1u << 26)
#endif
constexpr uint32_t kSpinCap = BN_SPIN_CAP;
constexpr uint32_t kDuoSpinCap = kSpinCap;

// A wait that runs out of its cap would go on to read a slot that was never
// published: it sets the BN_ERR_INTERNAL bit of *err, so the call fails
// (check_err, bn_dev_status) instead of returning a wrong Gt.  The outcome is
// decided on the counter itself (a counter that arrived during the last sleep
// is a success), and `dead` makes it sticky for the wave: after one wait has run
// out, the later ones do not spin again (the call has failed already).
__device__ __forceinline__ void duo_wait(const volatile uint32_t* c, uint32_t v, int* err, bool& dead) {
    uint32_t spins = 0;
    if (!dead)
        for (; *c < v && spins < kDuoSpinCap; ++spins) __builtin_amdgcn_s_sleep(1);
    if (*c < v) {
        dead = true;
        if (err) err_or(err, BN_ERR_INTERNAL);
    }
    asm volatile("" ::: "memory");
}
__device__ __forceinline__ void duo_signal(volatile uint32_t* c, uint32_t v) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the data (or the reads) are done first
    if ((threadIdx.x & (kWLanes - 1)) == 0) *c = v;
}
struct WDuo {
    uint32_t* ch;           // kDuoWords words of LDS
    volatile uint32_t* cnt;  // three counters, zero at the start
    uint32_t items, results;
    int* err;  // device error word: BN_ERR_INTERNAL when a wait runs out of its cap
    bool dead = false;  // a wait of this wave has run out of its cap (duo_wait)
    __device__ void put(const Fq<2>& x) {  // S
        if (items >= (uint32_t)kDuoRing) duo_wait(cnt + 1, items + 1 - kDuoRing, err, dead);
        w_put(ch + (items % kDuoRing) * kWArr, (int)(threadIdx.x & (kWLanes - 1)), x);
        duo_signal(cnt, ++items);
    }
    __device__ Fq<2> take() {  // M
        duo_wait(cnt, items + 1, err, dead);
        const Fq<2> x = w_get<2>(ch + (items % kDuoRing) * kWArr, (int)(threadIdx.x & (kWLanes - 1)));
        duo_signal(cnt + 1, ++items);
        return x;
    }
    __device__ void put_result(const Fq<2>& x) {  // M
        w_put(ch + (kDuoRing + results % 2) * kWArr, (int)(threadIdx.x & (kWLanes - 1)), x);
        duo_signal(cnt + 2, ++results);
    }
    __device__ Fq<2> get_result() {  // S
        duo_wait(cnt + 2, results + 1, err, dead);
        const Fq<2> x = w_get<2>(ch + (kDuoRing + results % 2) * kWArr, (int)(threadIdx.x & (kWLanes - 1)));
        ++results;
        return x;
    }
};
// S's side of exp_by_neg_z
__device__ __noinline__ Fq<2> w12_exp_sq(Fq<2> x, WDuo& d) {
#pragma unroll 1
    for (int k = 0;; ++k) {
        if ((kZNaf.nz >> k) & 1u) d.put(x);
        if (k == kZNaf.top) break;
        x = BN_S_CYC(x);
    }
    return d.get_result();
}
// M's side: the product of the handed-over powers; returns the first (x itself)
__device__ __noinline__ Fq<2> w12_exp_mul(WDuo& d) {
    const Fq<2> x = d.take();  // digit 0 is nonzero (u is odd)
    Fq<2> acc = (kZNaf.minus & 1u) ? w12_conj(x) : x;
#pragma unroll 1
    for (int k = 1; k <= kZNaf.top; ++k) {
        if (!((kZNaf.nz >> k) & 1u)) continue;
        const Fq<2> y = d.take();
        acc = w12_mul(acc, ((kZNaf.minus >> k) & 1u) ? w12_conj(y) : y);
    }
    d.put_result(w12_conj(acc));
    return x;
}
// The last chunk of the final exponentiation (fq12.rs:75-105) of s =
// w12_fe_first(f) on S; returns the result on S.
// The hand-overs: [24 powers of s], b, [24 powers of d], [24 powers of f1], k.
// M returns a, e, g and then o = frob(k*b), u = frob^3(conj(s)*k*b) while S
// forms m, n and q (the reference's names, fq12.rs:75-105).
__device__ __noinline__ Fq<2> w12_fe_last_s(Fq<2> s, WDuo& d) {
    const Fq<2> a = w12_exp_sq(s, d);
    const Fq<2> b = BN_S_CYC(a);
    d.put(b);
    const Fq<2> c = BN_S_CYC(b);
    const Fq<2> dd = w12_mul(c, b);
    const Fq<2> e = w12_exp_sq(dd, d);
    const Fq<2> f1 = BN_S_CYC(e);
    const Fq<2> g = w12_exp_sq(f1, d);
    const Fq<2> j = w12_mul(w12_conj(g), e);
    const Fq<2> k = w12_mul(j, w12_conj(dd));
    d.put(k);
    const Fq<2> m = w12_mul(k, e);
    const Fq<2> n = w12_mul(s, m);
    const Fq<2> q = w12_frob<2>(k);
    const Fq<2> o = d.get_result();
    const Fq<2> pp = w12_mul(o, n);
    const Fq<2> r = w12_mul(q, pp);
    const Fq<2> u = d.get_result();
    return w12_mul(u, r);
}
// final_exponentiation (fq12.rs:107-110) of f on S (first chunk, then the last on S and M)
__device__ __forceinline__ Fq<2> w12_final_exp_s(const Fq<2>& f, WDuo& d) { return w12_fe_last_s(w12_fe_first(f), d); }
// M's part of the same final exponentiation
__device__ __noinline__ void w12_final_exp_m(WDuo& d) {
    const Fq<2> s = w12_exp_mul(d);  // a
    const Fq<2> b = d.take();
    (void)w12_exp_mul(d);            // e
    (void)w12_exp_mul(d);            // g
    const Fq<2> k = d.take();
    const Fq<2> l = w12_mul(k, b);
    d.put_result(w12_frob<1>(l));    // o
    const Fq<2> t = w12_mul(w12_conj(s), l);
    d.put_result(w12_frob<3>(t));    // u
}

}  // namespace bn
