// kernels_tail.hip -- k_horner_tree2: the recombination and final exponentiation
// of ONE product (pairing_batch / miller_loop_batch, mod.rs:609-640, 904-926;
// fq12.rs:62-110), the tail of config 5: k_horner_tree (kernels_wide.hip)'s
// recombination on the 16-lane groups, then the final exponentiation's last chunk
// on the whole block in the digit-sliced layout (BN_TAIL_DS, fq12_ds.h: one digit
// per lane, ~1.7x shorter squarings and ~1.5x shorter products than the 16-lane
// ones on the chain, tools/ds_check).  BN_TAIL_DS=0 builds the round-5 form: the
// squarer S on a PAIR of 16-lane groups of one wave (w12_cyc32: the helper
// computes the xi * P products beside the main group's P), channel ch < 4: S =
// groups 2ch, 2ch + 1 (waves 0-1), M = group 8 + ch (wave 2).  Values are
// k_horner_tree's.
#ifndef BN_TAIL_DS
#define BN_TAIL_DS 1
#endif
// k_seg_fe1's first chunk with the Fq12 inversion's products spread over a group's
// lane pairs (w12_fe_first_par); 0: w12_fe_first on one group (A/B)
#ifndef BN_FE1_PAR
#define BN_FE1_PAR 1
#endif
#ifndef BN_TAIL_LATE_M
#define BN_TAIL_LATE_M 0
#endif
#define BN_FOLD_LDS 1
#define BN_WIDE_ARRS 4
#define BN_S_CYC w12_cyc32
#include "fq.h"
#define BN_SPLIT 1
#include "fq12_wide.h"
#if BN_TAIL_DS
#include "fq12_ds.h"
#endif
#ifndef TAIL_STAMP  // (fq12_ds.h defines the diagnostic stamps; BN_TAIL_DS=0 builds have none)
#define BN_TAIL_STAMPS 0
#define TAIL_STAMP(i) ((void)0)
#endif

namespace bn {

constexpr int kTailThreads = BN_WIDE_THREADS;
static_assert(kTailThreads == kTailBlock, "the launch (kernels.h kTailBlock) and the LDS layout agree");
static_assert(kWGroups == 16, "four waves of four groups");
constexpr int kTailDuo = 4;  // final-exponentiation channels: S pairs in waves 0-1, M in wave 2
#if BN_TAIL_DS
static_assert(kDsThreads == kTailThreads, "the digit-sliced element takes the whole block");
#else
__shared__ uint32_t g_tail_ch[kTailDuo * kDuoWords];
#endif
__shared__ uint32_t g_tail_cnt[kTailDuo * 4];
__shared__ uint32_t g_tail_zero;

#if BN_TAIL_DS
// ---------------------------------------------------------------- the first chunk, in parallel
// fq12.rs:62-73 of a nonzero f: c = conj(f) * f^-1 = conj(f)^2 * N^-1 with N = f conj(f)
// = c0^2 - v c1^2 in Fq6 (fq12.rs:305-313: f^-1 = conj(f) N^-1), then frob^2(c) * c.
// w12_fe_first runs the Fq12 inversion on one lane pair (its ~46 Fq2 products in a
// row); here the products of each stage of N and of N's inversion (fq6.rs:141-166)
// are spread over the 8 lane pairs of group 0 (round r: lane pair P takes product
// P + 8r, operands and results through LDS, one wave: no barrier), while group 4
// (another wave) squares conj(f).  Inverses are unique, so the value is
// w12_fe_first's.  Fq2 ids in g_inv (two slots each): 0..5 the coefficients z_e of
// w^e (c0 = (z0, z2, z4), c1 = (z1, z3, z5)), then the stage results.
constexpr int kInvIds = 48;
__shared__ uint32_t g_inv[2 * kInvIds * kWSlot];
__device__ __forceinline__ Fq2<2> inv_get(int id) {
    return {w_get<2>(g_inv, 2 * id + (int)(threadIdx.x & 1u))};
}
__device__ __forceinline__ void inv_put(int id, const Fq2<2>& v) { w_put(g_inv, 2 * id + (int)(threadIdx.x & 1u), v.c); }
// one round: lane pair P computes id dst[P] = op1[P] * op2[P] (P < n; a square when op1 == op2)
struct InvRound {
    int n;
    int8_t a[8], b[8], d[8];
};
__device__ __forceinline__ void inv_round(const InvRound& r) {
    const int P = (int)(threadIdx.x >> 1) & 7;
    const int a = r.a[P < r.n ? P : 0], b = r.b[P < r.n ? P : 0], d = r.d[P < r.n ? P : 0];
    const Fq2<2> x = inv_get(a), y = inv_get(b);
    const Fq2<2> z = fq2_fold(fq2_mul(x, y));
    w_sync();  // every lane pair has read its operands
    if (P < r.n) inv_put(d, z);
    w_sync();
}
// ids: a0 0, b0 1, a1 2, b1 3, a2 4, b2 5 (z_e = id e)
enum : int8_t {
    kA00 = 8, kA11, kA22, kA01, kA02, kA12, kB00, kB11, kB22, kB01, kB02, kB12,  // stage A products
    kN0 = 20, kN1, kN2,                                                           // N = c0^2 - v c1^2
    kM00 = 23, kM11, kM22, kM01, kM02, kM12,                                      // stage B products
    kC0 = 29, kC1, kC2,                                                           // fq6_inv's c0, c1, c2
    kU0 = 32, kU1, kU2,                                                           // n2 C1, n1 C2, n0 C0
    kT = 35, kTi,                                                                 // t, t^-1
    kT0 = 37, kT1, kT2                                                            // N^-1
};
__device__ __noinline__ Fq2<2> inv_xi(const Fq2<2>& x) { return fq2_fold(fq2_mul_xi(x)); }
// group 0 computes N^-1 (ids kT0..kT2) from the element in ids 0..5
__device__ __noinline__ void inv_fq6_par() {
    const int P = (int)(threadIdx.x >> 1) & 7;
    constexpr InvRound A1 = {8, {0, 2, 4, 0, 0, 2, 1, 3}, {0, 2, 4, 2, 4, 4, 1, 3}, {kA00, kA11, kA22, kA01, kA02, kA12, kB00, kB11}};
    constexpr InvRound A2 = {4, {5, 1, 1, 3}, {5, 3, 5, 5}, {kB22, kB01, kB02, kB12}};
    inv_round(A1);
    inv_round(A2);
    {  // N0 = a0^2 + xi (2 a1a2) - xi (b1^2 + 2 b0b2); N1 = 2 a0a1 + xi a2^2 - b0^2 - xi (2 b1b2);
       // N2 = a1^2 + 2 a0a2 - 2 b0b1 - xi b2^2  (lane pairs 0, 1, 2; each computes its own)
        const int i = P < 3 ? P : 0;
        const Fq2<2> g0 = inv_get(i == 0 ? kA00 : i == 1 ? kA01 : kA11);
        const Fq2<2> g1 = inv_get(i == 0 ? kA12 : i == 1 ? kA22 : kA02);
        const Fq2<2> h0 = inv_get(i == 0 ? kB11 : i == 1 ? kB00 : kB01);
        const Fq2<2> h1 = inv_get(i == 0 ? kB02 : i == 1 ? kB12 : kB22);
        // N0 = g0 + xi (2 g1 - h0 - 2 h1); N1 = 2 g0 + xi g1 - h0 - xi 2 h1; N2 = g0 + 2 g1 - 2 h0 - xi h1
        Fq2<2> nv;
        if (i == 0) {
            nv = fq2_fold(fq2_add(g0, inv_xi(fq2_fold(fq2_sub(fq2_dbl(g1), fq2_add(h0, fq2_dbl(h1)))))));
        } else if (i == 1) {
            nv = fq2_fold(fq2_sub(fq2_add(fq2_dbl(g0), inv_xi(fq2_fold(fq2_sub(g1, fq2_dbl(h1))))), h0));
        } else {
            nv = fq2_fold(fq2_sub(fq2_add(g0, fq2_dbl(g1)), fq2_add(fq2_dbl(h0), inv_xi(h1))));
        }
        w_sync();
        if (P < 3) inv_put(kN0 + i, nv);
        w_sync();
    }
    // fq6_inv (fq6.rs:141-166) of N = (n0, n1, n2)
    constexpr InvRound B = {6, {kN0, kN1, kN2, kN0, kN0, kN1, 0, 0}, {kN0, kN1, kN2, kN1, kN2, kN2, 0, 0},
                            {kM00, kM11, kM22, kM01, kM02, kM12, 0, 0}};
    inv_round(B);
    {  // C0 = n0^2 - xi n1n2, C1 = xi n2^2 - n0n1, C2 = n1^2 - n0n2
        const int i = P < 3 ? P : 0;
        const Fq2<2> u = inv_get(i == 0 ? kM00 : i == 1 ? kM22 : kM11);
        const Fq2<2> v = inv_get(i == 0 ? kM12 : i == 1 ? kM01 : kM02);
        const Fq2<2> cv = i == 0 ? fq2_fold(fq2_sub(u, inv_xi(v))) : i == 1 ? fq2_fold(fq2_sub(inv_xi(u), v))
                                                                     : fq2_fold(fq2_sub(u, v));
        w_sync();
        if (P < 3) inv_put(kC0 + i, cv);
        w_sync();
    }
    constexpr InvRound Cr = {3, {kN2, kN1, kN0, 0, 0, 0, 0, 0}, {kC1, kC2, kC0, 0, 0, 0, 0, 0}, {kU0, kU1, kU2, 0, 0, 0, 0, 0}};
    inv_round(Cr);
    {  // t = n0 C0 + xi (n2 C1 + n1 C2), t^-1 (every lane pair: the same value)
        const Fq2<2> t = fq2_fold(fq2_add(inv_get(kU2), inv_xi(fq2_fold(fq2_add(inv_get(kU0), inv_get(kU1))))));
        const Fq2<2> ti = fq2_fold(fq2_inv<true>(t));  // group 0's four quads hold the same t
        w_sync();
        if (P == 0) inv_put(kTi, ti);
        w_sync();
    }
    constexpr InvRound E = {3, {kC0, kC1, kC2, 0, 0, 0, 0, 0}, {kTi, kTi, kTi, 0, 0, 0, 0, 0}, {kT0, kT1, kT2, 0, 0, 0, 0, 0}};
    inv_round(E);
}
// w12_fe_first of f (group 0 holds f; every thread of the block calls, threads < 256);
// returns the first chunk on group 0
__device__ __noinline__ Fq<2> w12_fe_first_par(Fq<2> f) {
    const WL w = wl();
    const int grp = (int)threadIdx.x / kWLanes;
    if (grp == 0 && w.l < 12) w_put(g_inv, w.l, f);  // ids 0..5: lane l = 2e + c is slot l
    __syncthreads();
    Fq<2> sq = f;
    if (grp == 0) {
        inv_fq6_par();
    } else if (grp == 4) {  // another wave: conj(f)^2 beside the inversion
        const int l = w.l < 12 ? w.l : 10 + (w.l & 1);
        sq = w12_square(w12_conj(w_get<2>(g_inv, l)));
    }
    __syncthreads();
    if (grp == 4 && w.l < 12) w_put(g_inv, 2 * 40 + w.l, sq);  // ids 40..45: conj(f)^2
    __syncthreads();
    Fq<2> r = f;
    if (grp == 0) {
        const Fq<2> s2 = w_get<2>(g_inv, 2 * 40 + (w.l < 12 ? w.l : 10 + (w.l & 1)));
        // N^-1 as an Fq12 with c1 = 0: coefficient w^(2j) = T_j, odd w-exponents zero
        const Fq<2> tv = w_get<2>(g_inv, 2 * (kT0 + (w.e >> 1)) + w.c);
        const Fq<2> t12 = fq_select((w.e & 1) != 0, widen<2>(fq_zero()), tv);
        const Fq<2> c = w12_mul(s2, t12);  // conj(f) * f^-1
        r = w12_mul(w12_frob<2>(c), c);
    }
    return r;
}
#endif

#if BN_TAIL_DS
// pairing_batch with several segments: block s takes segment s's value g_s (element
// s of the split-layout array g, stride S), runs the final exponentiation's first
// chunk on it (w12_fe_first, fq12.rs:62-73: a power map, so E1(prod g_s^(2^e_s)) =
// prod E1(g_s)^(2^e_s)) and then its e_s = len_(s+1) + ... + len_(S-1)
// squarings in the cyclotomic subgroup on the whole block (ds_cyc), and writes the
// result back in place; zf[s] = 1 when g_s is zero (the product is zero: the
// reference's final_exponentiation returns None, fq12.rs:63-72).  The segments'
// squarings run side by side on S CUs instead of on the 16-lane groups of one block.
constexpr int kDsChanOff = 1024;  // the S <-> M channel (8-byte aligned), after the zero flags (kernels.h kTailChanWords)
static_assert(kDsChanOff + kDsChanWords <= kTailChanWords, "tail channel size");
// k_horner_tree2's role word (after the S <= kMaxSeg zero flags): its two blocks hand
// values over by polling global memory, which needs both resident at once -- HIP
// does not promise that (another stream's kernels may hold every CU when block 1
// would start).  So the roles are claimed, not assumed: the multiplier block swaps
// 0 -> kRoleM when it starts, the squarer block swaps 0 -> kRoleSolo when it reaches
// the final exponentiation.  Whichever comes first decides: M present -> the
// two-block chain; M not started yet -> the squarer runs the last chunk alone
// (ds_fe_last, the same value) and a late M finds kRoleSolo and returns.  Neither
// side ever waits on a block that is not running.
constexpr int kRoleWord = 1000;
constexpr uint32_t kRoleM = 1, kRoleSolo = 2;
static_assert(kRoleWord >= kMaxSeg && kRoleWord < kDsChanOff, "role word between the zero flags and the channel");
__device__ __forceinline__ uint32_t tail_claim(uint32_t* zf, uint32_t role) {  // thread 0; returns the word's old value
    uint32_t expect = 0;
    __hip_atomic_compare_exchange_strong((__attribute__((address_space(1))) uint32_t*)(zf + kRoleWord), &expect, role,
                                         __ATOMIC_RELAXED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return expect;
}
__shared__ uint32_t g_tail_role;
__global__ void __launch_bounds__(kTailThreads) k_seg_fe1(uint32_t* __restrict__ g, SegPlan plan,
                                                          uint32_t* __restrict__ zf) {
    fold_table_init();
    const WL w = wl();
    const int s = (int)blockIdx.x;
    {  // k_horner_tree2's channel: every stamp cleared (the blocks share the words), the role word too
        uint64_t* ch = (uint64_t*)(zf + kDsChanOff);
        for (int i = s * kTailThreads + (int)threadIdx.x; i < kDsChanWords / 2; i += plan.S * kTailThreads)
            __hip_atomic_store(ch + i, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (s == 0 && threadIdx.x == 0)
            __hip_atomic_store((__attribute__((address_space(1))) uint32_t*)(zf + kRoleWord), 0u, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    }
    int e = 0;
    for (int t = s + 1; t < plan.S; ++t) e += plan.hi[t] - plan.lo[t];
    Fq<2> x = widen<2>(fq_zero());
    if (threadIdx.x < (unsigned)kWLanes) {  // group 0
        x = w_ld_split(g, (size_t)plan.S, (size_t)s, w);
        const bool zero = w12_is_zero(x);
        if (threadIdx.x == 0) zf[s] = zero ? 1u : 0u;
    }
    if (BN_TAIL_STAMPS && s == 0) TAIL_STAMP(16);
#if BN_FE1_PAR
    x = w12_fe_first_par(x);  // group 0 gets the first chunk
#else
    if (threadIdx.x < (unsigned)kWLanes) x = w12_fe_first(x);
#endif
    if (BN_TAIL_STAMPS && s == 0) TAIL_STAMP(17);
    ds_init();
    uint32_t d = ds_from_w12(x);
#pragma unroll 1
    for (int k = 0; k < e; ++k) d = ds_cyc_body(d);
    x = ds_to_w12(d);
    if (threadIdx.x < 12) w_st_split(g, (size_t)plan.S, (size_t)s, w, x);
    if (BN_TAIL_STAMPS && s == 0) TAIL_STAMP(18);
}

// ---------------------------------------------------------------- the whole tail in one launch
// pairing_batch's tail as ONE launch of max(S, 3) blocks, without k_horner_tree2's
// launch and its 16-lane product tree (four levels of w12_mul, ~21 us): block s < S
// runs segment s's first chunk and squarings as k_seg_fe1 does, then the segment
// values meet in a chain of nodes.  Node k joins d_k (block k, side 0) with
// P_(k+1) = d_(k+1) ... d_(S-1) (side 1: its carrier; block S - 1 carries d_(S-1) to
// node S - 2): both sides store their value (stamped words) and swap the node's word
// to the epoch; the one that finds the epoch there is second, reads the other side's
// value, multiplies, and carries P_k on to node k - 1; the first one is done.
// e_s falls with s, so the blocks arrive in the order S - 1, ..., 0 and P_1 is
// (mostly) ready when block 0 gets there: the product costs one digit-sliced product
// behind the longest segment.  No block waits for one that may not have started: the
// second arriver reads a value whose writer has already arrived.  A block that leaves
// a node first (and the spare blocks of a plan with S < 3) offers itself as one of
// the last chunk's two multipliers (fq12_ds.h ds_fe_last_m2); the carrier of P_0
// runs the last chunk as the squarer, with both multipliers if two have claimed the
// role by then, else alone.  Roles are claimed on an epoch-tagged word, never
// assumed (as k_horner_tree2's): bit 0 / 1 = M_0 / M_1 claimed, bit 2 = the squarer
// has decided; a multiplier waits for that decision and leaves unless it is two.  A zero segment value makes the product zero, and
// the final exponentiation of zero is zero: the carrier tests its result (the
// reference's None, fq12.rs:63-72).  Values are the same as k_seg_fe1 + k_horner_tree2
// (Fq12 products commute).
constexpr int kLinkNodeOff = kRoleWord + 1;     // node k's word
constexpr int kLinkOff = kDsChanOff + kDsChanWords;  // node k side j: 128 stamped words at slot 2k + j
static_assert(kLinkNodeOff + kMaxSeg <= kDsChanOff && kLinkOff + 2 * kMaxSeg * 256 <= kTailWsWords, "tail words");
// the role word: epoch * 8 + bits (bit 0: M_0 claimed, bit 1: M_1, bit 2: the squarer decided)
constexpr uint32_t kTailM0 = 1, kTailM1 = 2, kTailDecided = 4;
typedef __attribute__((address_space(1))) uint32_t tail_word;
__device__ __forceinline__ uint32_t tail_bits(uint32_t cur, uint32_t epoch) { return (cur >> 3) == epoch ? cur & 7u : 0u; }
// thread 0 of a multiplier candidate: 1 + par when it got M_par, 0 when none is left
__device__ uint32_t tail_claim_m(uint32_t* rw, uint32_t epoch) {
    tail_word* p = (tail_word*)rw;
    uint32_t cur = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (;;) {
        const uint32_t b = tail_bits(cur, epoch);
        if (b & kTailDecided) return 0;
        const uint32_t add = !(b & kTailM0) ? kTailM0 : !(b & kTailM1) ? kTailM1 : 0u;
        if (!add) return 0;
        if (__hip_atomic_compare_exchange_strong(p, &cur, epoch * 8u + (b | add), __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT))
            return add == kTailM0 ? 1u : 2u;
    }
}
// thread 0 of the squarer: sets the decided bit; returns the multiplier bits at that moment
__device__ uint32_t tail_decide(uint32_t* rw, uint32_t epoch) {
    tail_word* p = (tail_word*)rw;
    uint32_t cur = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (;;) {
        const uint32_t b = tail_bits(cur, epoch);
        if (__hip_atomic_compare_exchange_strong(p, &cur, epoch * 8u + (b | kTailDecided), __ATOMIC_RELAXED,
                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
            return b & (kTailM0 | kTailM1);
    }
}
// thread 0 of a multiplier: the squarer's decision (its multiplier bits), or 0 when the
// wait runs out of its cap (the call fails: BN_ERR_INTERNAL)
__device__ uint32_t tail_await_decision(uint32_t* rw, uint32_t epoch, int* err) {
    tail_word* p = (tail_word*)rw;
    for (uint32_t spins = 0; spins < kSpinCap; ++spins) {
        const uint32_t b = tail_bits(__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT), epoch);
        if (b & kTailDecided) return b & (kTailM0 | kTailM1);
        __builtin_amdgcn_s_sleep(1);
    }
    if (err) err_or(err, BN_ERR_INTERNAL);
    return 0;
}
// a multiplier candidate of the last chunk: claims M_0 or M_1 on the role word rw, waits
// for the squarer's decision, runs its share if the squarer takes both multipliers
__device__ __forceinline__ void tail_multiplier(uint32_t* rw, DsChan& ch, uint32_t epoch, int* err) {
#if BN_TAIL_LATE_M
    for (int t = 0; t < 40000; ++t) __builtin_amdgcn_s_sleep(1);
#endif
    __syncthreads();
    if (threadIdx.x == 0) g_tail_role = tail_claim_m(rw, epoch);
    __syncthreads();
    const uint32_t role = g_tail_role;
    if (role == 0) return;
    __syncthreads();
    if (threadIdx.x == 0) g_tail_role = tail_await_decision(rw, epoch, err);
    __syncthreads();
    if (g_tail_role != (kTailM0 | kTailM1)) return;  // the squarer went on alone
    if (BN_TAIL_STAMPS) TAIL_STAMP(role == 1 ? 25 : 27);
    ds_fe_last_m2(ch, (int)role - 1);
    if (BN_TAIL_STAMPS) TAIL_STAMP(role == 1 ? 26 : 28);
}
// the squarer: decides (both multipliers if both have claimed, else alone), runs the
// last chunk of d and writes the Gt image to *out (zero: BN_ERR_FE_ZERO, the zero image;
// *ok = 0 for zero, 1 otherwise, when ok is given)
__device__ __forceinline__ void tail_squarer(uint32_t d, uint32_t* rw, DsChan& ch, uint32_t epoch, int* err,
                                             bn_gt* out, const WL& w, uint8_t* ok = nullptr) {
    __syncthreads();
    if (threadIdx.x == 0) g_tail_role = tail_decide(rw, epoch);
    __syncthreads();
    if (g_tail_role == (kTailM0 | kTailM1))
        d = ds_fe_last_s2(d, ch);
    else
        d = ds_fe_last(d);
    if (BN_TAIL_STAMPS) TAIL_STAMP(8);
    const Fq<2> r = ds_to_w12(d);  // threads 0..11 get the value
    const bool z = w12_is_zero(r);
    if (threadIdx.x == 0) g_tail_zero = z ? 1u : 0u;
    __syncthreads();
    const bool zero = g_tail_zero != 0;
    if (zero && err && threadIdx.x == 0) err_or(err, BN_ERR_FE_ZERO);
    if (ok && threadIdx.x == 0) *ok = zero ? 0 : 1;
    uint32_t words[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (!zero && threadIdx.x < 12) fq_store_ref(r, words);
    if (threadIdx.x < 12) st_words(&out->c[w_gt_index(w)], words);
}
__global__ void __launch_bounds__(kTailThreads) k_seg_tail(const uint32_t* __restrict__ g, SegPlan plan,
                                                           bn_gt* __restrict__ out, int* __restrict__ err,
                                                           uint32_t* __restrict__ ws, uint32_t epoch) {
    fold_table_init();
    const WL w = wl();
    const int s = (int)blockIdx.x;
    uint64_t* const link = (uint64_t*)(ws + kLinkOff);
    DsChan ch = {(uint64_t*)(ws + kDsChanOff), err, 0, 0, false, epoch};  // its dead flag serves the chain too
    bool carrier = false;
    uint32_t d = 0;
    if (s < plan.S) {
        int e = 0;
        for (int t = s + 1; t < plan.S; ++t) e += plan.hi[t] - plan.lo[t];
        Fq<2> x = widen<2>(fq_zero());
        if (threadIdx.x < (unsigned)kWLanes) x = w_ld_split(g, (size_t)plan.S, (size_t)s, w);  // group 0
        if (BN_TAIL_STAMPS && s == 0) TAIL_STAMP(16);
        x = w12_fe_first_par(x);
        if (BN_TAIL_STAMPS && s == 0) TAIL_STAMP(17);
        ds_init();
        d = ds_from_w12(x);
#pragma unroll 1
        for (int k = 0; k < e; ++k) d = ds_cyc_body(d);
        if (BN_TAIL_STAMPS && s == 0) TAIL_STAMP(18);
        carrier = true;
        int k = s == plan.S - 1 ? s - 1 : s, side = s == plan.S - 1 ? 1 : 0;
#pragma unroll 1
        for (; k >= 0; --k, side = 1) {
            ds_chan_st(link + 128 * (2 * k + side), d, epoch);
            __syncthreads();  // every digit lane's store is issued before the arrival
            if (threadIdx.x == 0)
                g_tail_role = __hip_atomic_exchange((__attribute__((address_space(1))) uint32_t*)(ws + kLinkNodeOff + k),
                                                    epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __syncthreads();
            if (g_tail_role != epoch) {  // first at node k: the other side carries on
                carrier = false;
                break;
            }
            d = ds_mul(d, ds_chan_ld(link + 128 * (2 * k + 1 - side), ch), false);
        }
    } else {
        ds_init();
    }
    if (!carrier) {  // one of the last chunk's multipliers, if a role is still free
        tail_multiplier(ws + kRoleWord, ch, epoch, err);
        return;
    }
    // the carrier of P_0: the squarer
    if (BN_TAIL_STAMPS) TAIL_STAMP(1);
    tail_squarer(d, ws + kRoleWord, ch, epoch, err, &out[0], w);
}

// pairing_many's final exponentiations for batches of at most kFeDsMax pairs (after
// k_pairing_latency wrote the Miller values, f_out): with per = 3, pair i takes blocks
// 3i (the squarer, which runs the first chunk first, w12_fe_first_par) and 3i + 1,
// 3i + 2 (multiplier candidates); with per = 1 (more pairs than a third of the CUs) one
// block per pair, the squarer alone.  Each pair has its own role word and channel
// (kFeDsWords of ws, epoch-stamped as k_seg_tail's).  The digit-sliced last chunk with
// two multipliers against the latency kernel's 16-lane two-group one: ~0.24 ms shorter
// per pairing (profiles/r6q_latency_fe_ds.txt).
// f == 0 (the reference's final_exponentiation returns None): BN_ERR_FE_ZERO, the
// zero image and ok[i] = 0 (when ok is given), as the latency kernel and k_fe_wide.
__global__ void __launch_bounds__(kTailThreads) k_fe_ds(const uint32_t* __restrict__ f, size_t n,
                                                        bn_gt* __restrict__ out, uint8_t* __restrict__ ok,
                                                        int* __restrict__ err, uint32_t* __restrict__ ws,
                                                        uint32_t epoch, int per) {
    fold_table_init();
    const WL w = wl();
    const size_t i = blockIdx.x / (unsigned)per;
    if (i >= n) return;  // (block-uniform)
    uint32_t* pw = ws + i * (size_t)kFeDsWords;
    DsChan ch = {(uint64_t*)(pw + kDsChanOff), err, 0, 0, false, epoch};
    if (blockIdx.x % (unsigned)per != 0) {
        ds_init();
        tail_multiplier(pw + kRoleWord, ch, epoch, err);
        return;
    }
    Fq<2> x = widen<2>(fq_zero());
    if (threadIdx.x < (unsigned)kWLanes) x = w_ld_split(f, n, i, w);  // group 0
    x = w12_fe_first_par(x);
    ds_init();
    tail_squarer(ds_from_w12(x), pw + kRoleWord, ch, epoch, err, &out[i], w, ok ? ok + i : nullptr);
}
#endif

// g: the S segment values (element s of a split-layout array of stride S);
// segment s's value is raised to 2^(len_(s+1) + ... + len_(S-1)), the values are
// multiplied in a tree, then the final exponentiation's last chunk (do_fe:
// pairing_batch, after the first chunk on every segment) or the value itself
// (miller_loop_batch) goes to out[0].  zf (do_fe only): k_seg_fe1 has run the
// first chunk and the squarings already, zf[s] its zero flags.
__global__ void __launch_bounds__(kTailThreads) k_horner_tree2(const uint32_t* __restrict__ g, SegPlan plan,
                                                               int do_fe, bn_gt* __restrict__ out,
                                                               int* __restrict__ err,
                                                               const uint32_t* __restrict__ zf) {
    if (BN_TAIL_STAMPS) TAIL_STAMP(blockIdx.x == 0 ? 0 : 24);
    if (threadIdx.x == 0) g_tail_zero = 0;
    if (threadIdx.x < kTailDuo * 4) g_tail_cnt[threadIdx.x] = 0;
    __syncthreads();  // the resets are seen before any group can use them
    fold_table_init();
    const WL w = wl();
    const int grp = (int)threadIdx.x / kWLanes;
    const bool seg = grp < plan.S;
    Fq<2> x = fq_select(w.e == 0 && w.c == 0, widen<2>(fq_one()), widen<2>(fq_zero()));
    if (seg) x = w_ld_split(g, (size_t)plan.S, (size_t)grp, w);
    int e = 0, e0 = 0;  // this group's squarings (g_s^(2^e_s)) and group 0's (the most)
    for (int t = 1; t < plan.S; ++t) {
        e0 += plan.hi[t] - plan.lo[t];
        if (t > grp) e += plan.hi[t] - plan.lo[t];
    }
#if BN_TAIL_DS
    if (do_fe && zf && blockIdx.x == 1) {  // the multiplier block of the final exponentiation
#if BN_TAIL_LATE_M  // test build (`make chanfail`): M starts ~2 ms late, so the squarer must go on alone
        for (int t = 0; t < 40000; ++t) __builtin_amdgcn_s_sleep(1);
#endif
        if (threadIdx.x == 0) g_tail_role = tail_claim(const_cast<uint32_t*>(zf), kRoleM);
        __syncthreads();
        if (g_tail_role != 0) return;  // the squarer block has gone on alone
        if (BN_TAIL_STAMPS) TAIL_STAMP(25);
        ds_init();
        DsChan ch = {(uint64_t*)(const_cast<uint32_t*>(zf) + kDsChanOff), err, 0, 0, false, 1};
        ds_fe_last_m(ch);
        if (BN_TAIL_STAMPS) TAIL_STAMP(26);
        return;
    }
#endif
    if (do_fe && zf) {
        if (threadIdx.x < (unsigned)plan.S && zf[threadIdx.x]) g_tail_zero = 1;
        e0 = 0;  // k_seg_fe1 did the first chunk and the squarings
    } else if (do_fe) {
        if (seg && w12_is_zero(x) && w.l == 0) g_tail_zero = 1;
        x = w12_fe_first(x);  // first chunk; of one (groups past S): one
#pragma unroll 1
        for (int k = 0; k < e0; ++k) {
            const Fq<2> y = w12_cyc(x);
            x = k < e ? y : x;
        }
    } else {
#pragma unroll 1
        for (int k = 0; k < e0; ++k) {
            const Fq<2> y = w12_mul(x, x);
            x = k < e ? y : x;
        }
    }
    // the product tree: group g's value sits in its fourth operand array, which only
    // g's own w12_mul overwrites -- and at a level where group g multiplies, no group
    // reads g's slot (its readers are the groups g - h, and g < h) before the barrier
    // that ends the level
    auto slot = [&](int gi) { return g_wide + gi * kWGroupWords + 3 * kWArr; };
#pragma unroll 1
    for (int h = kWGroups / 2; h >= 1; h /= 2) {
        w_put(slot(grp), w.l, x);
        __syncthreads();
        if (grp < h) {
            const Fq<2> y = w12_mul(x, w_get<2>(slot(grp + h), w.l));
            if (grp + h < plan.S) x = y;  // groups past S hold one
        }
        __syncthreads();
    }
    // every group takes group 0's value
    if (grp == 0) w_put(slot(0), w.l, x);
    __syncthreads();
    x = w_get<2>(slot(0), w.l);
    __syncthreads();  // slot 0 is group 0's operand area again from here on
    uint32_t words[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#if BN_TAIL_DS
    if (do_fe) {
        const bool zero = g_tail_zero != 0;
        if (zero && err && threadIdx.x == 0) err_or(err, BN_ERR_FE_ZERO);
        if (BN_TAIL_STAMPS) TAIL_STAMP(1);
        ds_init();
        uint32_t d = ds_from_w12(x);
        bool duo = false;
        if (zf && gridDim.x == 2) {  // with the multiplier block (block 1), if it has started
            if (threadIdx.x == 0) g_tail_role = tail_claim(const_cast<uint32_t*>(zf), kRoleSolo);
            __syncthreads();
            duo = g_tail_role == kRoleM;
        }
        if (duo) {
            DsChan ch = {(uint64_t*)(const_cast<uint32_t*>(zf) + kDsChanOff), err, 0, 0, false, 1};
            d = ds_fe_last_s(d, ch);
        } else {
            d = ds_fe_last(d);
        }
        if (BN_TAIL_STAMPS) TAIL_STAMP(8);
        const Fq<2> r = ds_to_w12(d);  // every thread; threads 0..11 get the value
        if (!zero && threadIdx.x < 12) fq_store_ref(r, words);
    } else {
        fq_store_ref(x, words);
    }
    if (threadIdx.x < 12) st_words(&out[0].c[w_gt_index(w)], words);
#else
    if (do_fe) {
        if (grp >= 3 * kTailDuo) return;  // wave 3
        const bool m = grp >= 2 * kTailDuo;
        const int ch = m ? grp - 2 * kTailDuo : grp >> 1;
        WDuo d = {g_tail_ch + ch * kDuoWords, g_tail_cnt + 4 * ch, 0, 0, err};
        if (m) {
            w12_final_exp_m(d);
            return;
        }
        const bool zero = g_tail_zero != 0;
        if (zero && err && w.l == 0 && grp == 0) err_or(err, BN_ERR_FE_ZERO);
        const Fq<2> r = w12_fe_last_s(x, d);
        if (!zero) fq_store_ref(r, words);
    } else {
        fq_store_ref(x, words);
    }
    if (w.l < 12 && grp == 0) st_words(&out[0].c[w_gt_index(w)], words);
#endif
}

}  // namespace bn

BN_EXPORT_FOLD_CHECK(tail)

#if BN_TAIL_STAMPS
extern "C" int bn_dbg_tail_stamps(uint64_t out[32]) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(bn::g_tail_stamps), 32 * sizeof(uint64_t)) == hipSuccess ? 0 : -1;
}
#endif
