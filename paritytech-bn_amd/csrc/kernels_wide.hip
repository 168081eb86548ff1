// kernels_wide.hip -- latency kernels on the wide layout (fq12_wide.h: one Fq12
// over a 16-lane group): final exponentiation of a few values and the product
// reduction behind pairing_batch / miller_loop_batch (mod.rs:609-640, 904-926).
// Inputs and outputs use the lane-strided two-lane layout of the pairing path
// (kernels.h st_fq12/ld_fq12 with BN_SPLIT), so these kernels slot in after
// k_miller without a conversion.
#ifndef BN_FOLD_LDS
#define BN_FOLD_LDS 1
#endif
#include "fq.h"
#define BN_SPLIT 1
#include "fq12_wide.h"
#include "lines_wide.h"

namespace bn {

__device__ __forceinline__ size_t w_elem() { return lane_id() / kWLanes; }

// Element and role of this group in the final-exponentiation kernels: with
// BN_FE_DUO a block holds kWGroups / 2 elements, each with its squarer group in
// waves 0-1 and its multiplier group in waves 2-3 (fq12_wide.h), and channel
// `slot` of the block; else one element per group, every group a squarer.
struct WRole {
    size_t e;
    bool sq, duo;
    int slot;
};
constexpr int kDuoPerBlock = kWGroups / 2;
__device__ __forceinline__ WRole w_role(bool duo) {
#if BN_FE_DUO
    if (duo) {
        const int g = (int)threadIdx.x / kWLanes;
        return {(size_t)blockIdx.x * kDuoPerBlock + (size_t)(g % kDuoPerBlock), g < kDuoPerBlock, true, g % kDuoPerBlock};
    }
#endif
    (void)duo;
    return {w_elem(), true, false, 0};
}
#if BN_FE_DUO
__shared__ uint32_t g_wduo_ch[kDuoPerBlock * kDuoWords];  // 36 KB
__shared__ uint32_t g_wduo_cnt[kDuoPerBlock * 4];
#endif
// zero the block's channel counters (every thread of the block calls it)
__device__ __forceinline__ void w_duo_init() {
#if BN_FE_DUO
    if (threadIdx.x < kDuoPerBlock * 4) g_wduo_cnt[threadIdx.x] = 0;
    __syncthreads();
#endif
}
// the final exponentiation on S (with its M running w12_final_exp_m), or on
// the group alone
__device__ __forceinline__ Fq<2> w_final_exp(const WRole& r, const Fq<2>& x, int* err) {
#if BN_FE_DUO
    if (r.duo) {
        WDuo d = {g_wduo_ch + r.slot * kDuoWords, g_wduo_cnt + 4 * r.slot, 0, 0, err};
        return w12_final_exp_s(x, d);
    }
#endif
    (void)r;
    (void)err;
    return w12_final_exp(x);
}
// the last chunk only, of s = w12_fe_first(x) (k_horner_tree)
__device__ __forceinline__ Fq<2> w_fe_last(const WRole& r, const Fq<2>& s, int* err) {
#if BN_FE_DUO
    if (r.duo) {
        WDuo d = {g_wduo_ch + r.slot * kDuoWords, g_wduo_cnt + 4 * r.slot, 0, 0, err};
        return w12_fe_last_s(s, d);
    }
#endif
    (void)r;
    (void)err;
    return w12_fe_last(s);
}
// M's part; true if this group is M (and has done it)
__device__ __forceinline__ bool w_final_exp_m(const WRole& r, bool run, int* err) {
#if BN_FE_DUO
    if (r.sq) return false;
    if (run) {
        WDuo d = {g_wduo_ch + r.slot * kDuoWords, g_wduo_cnt + 4 * r.slot, 0, 0, err};
        w12_final_exp_m(d);
    }
    return true;
#else
    (void)r;
    (void)run;
    (void)err;
    return false;
#endif
}

// out[e] = final_exponentiation(f[e]) for e < n, f lane-strided (split layout,
// stride `stride`).  f == 0: zero image, ok = 0, error bit (fq12.rs:63-72;
// pairing() panics, mod.rs:900).  A skipped pair's Miller value is already
// Fq12::one() (k_miller), and FE(one) = one.
__global__ void __launch_bounds__(kBlock) k_fe_wide(const uint32_t* __restrict__ f, size_t stride, size_t n,
                                                    bn_gt* __restrict__ out, uint8_t* __restrict__ ok,
                                                    int* __restrict__ err, int duo) {
    fold_table_init();
    w_duo_init();
    const WRole role = w_role(duo != 0);
    // idle groups of the block (past n) repeat the last element instead of returning:
    // a wave whose other groups had returned ran its last group ~200 us slower
    const bool live = role.e < n;
    const size_t e = live ? role.e : n - 1;
    if (w_final_exp_m(role, true, err)) return;
    const WL w = wl();
    const Fq<2> x = w_ld_split(f, stride, e, w);
    const bool zero = w12_is_zero(x);
    if (ok && w.l == 0 && live) ok[e] = zero ? 0 : 1;
    if (zero && err && w.l == 0 && live) err_or(err, BN_ERR_FE_ZERO);
    const Fq<2> r = w_final_exp(role, x, err);
    uint32_t words[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (!zero) fq_store_ref(r, words);
    if (w.l < 12 && live) st_words(&out[e].c[w_gt_index(w)], words);
}

// one value per group for k_horner_tree's product tree
__shared__ uint32_t g_wval[kWGroups * kWLanes * kWSlot];  // 12 KB

// Recombination of segmented Miller loops (pairing.h miller_segment), one
// 16-lane group per element e < n: segment s of element e is element s * n + e
// of g (split layout, stride S * n, as k_miller_seg writes it).  x = g_0, then
// x = x^(2^len_s) * g_s for s = 1..S-1 (the generic squaring, as the reference's
// loop squares its accumulator), then the final exponentiation when do_fe
// (pairing / pairing_batch; zero -> zero image + error bit) or the Miller value
// itself (miller_loop_batch) -> out[e].
#ifndef BN_LAT_STAMPS
#define BN_LAT_STAMPS 0
#endif
#if BN_LAT_STAMPS
// diagnostic build: block 0's group 0 stamps s_memrealtime (100 MHz) at the
// phase boundaries of k_horner_wide (tools/lat_stamps.py --horner)
__device__ uint64_t g_hor_stamps[8];
#define HOR_STAMP(k)                                                                       \
    do {                                                                                   \
        if (blockIdx.x == 0 && threadIdx.x == 0) g_hor_stamps[k] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
#else
#define HOR_STAMP(k) ((void)0)
#endif
__global__ void __launch_bounds__(kBlock) k_horner_wide(const uint32_t* __restrict__ g, size_t n, SegPlan plan,
                                                        int do_fe, bn_gt* __restrict__ out, int* __restrict__ err,
                                                        int duo) {
    HOR_STAMP(0);  // start
    fold_table_init();
    w_duo_init();
    const WRole role = w_role(duo != 0);
    // idle groups of the block (past n) repeat the last element instead of returning:
    // a wave whose other groups had returned ran its last group ~200 us slower
    const bool live = role.e < n;
    const size_t e = live ? role.e : n - 1;
    if (w_final_exp_m(role, do_fe != 0, err)) return;
    const WL w = wl();
    const size_t stride = (size_t)plan.S * n;
    Fq<2> x = w_ld_split(g, stride, e, w);
    HOR_STAMP(1);  // g_0 in
#pragma unroll 1
    for (int s = 1; s < plan.S; ++s) {
#pragma unroll 1
        for (int k = plan.lo[s]; k < plan.hi[s]; ++k) x = w12_square(x);
        if (s == 1) HOR_STAMP(2);  // the first run of squarings
        x = w12_mul(x, w_ld_split(g, stride, (size_t)s * n + e, w));
        if (s == 1) HOR_STAMP(3);  // its load + product
    }
    HOR_STAMP(4);  // recombination done
    uint32_t words[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (do_fe) {
        const bool zero = w12_is_zero(x);
        if (zero && err && w.l == 0 && live) err_or(err, BN_ERR_FE_ZERO);
        const Fq<2> r = w_final_exp(role, x, err);
        HOR_STAMP(5);  // final exponentiation done
        if (!zero) fq_store_ref(r, words);
    } else {
        fq_store_ref(x, words);
    }
    if (w.l < 12 && live) st_words(&out[e].c[w_gt_index(w)], words);
}

// The same recombination for ONE element (n = 1: the product of pairing_batch /
// miller_loop_batch) on the S <= 16 groups of one block, as a tree.  Horner's
// value f = (..(g_0^(2^len_1) g_1)^(2^len_2)..)^(2^len_(S-1)) g_(S-1) is the
// product over s of g_s^(2^e_s), e_s = len_(s+1) + .. + len_(S-1), because
// squaring is a ring homomorphism; so group s loads g_s and squares it e_s times,
// and the sixteen values are multiplied in a tree through LDS (Fq12
// multiplication is commutative and associative).  The dependent chain is group
// 0's e_0 squarings and four products, instead of the same squarings, S - 1
// products and S - 1 global loads one after another.
// pairing_batch (do_fe): the first chunk of the final exponentiation E1(x) =
// x^((p^6 - 1)(p^2 + 1)) is a power map, so E1(f) = prod E1(g_s)^(2^e_s).  Every
// group runs E1 on its g_s (side by side) and then squares in the cyclotomic
// subgroup (Granger-Scott, w12_cyc: the same square as the generic one there, at
// about half its instructions); group 0 then runs only the last chunk, so the
// final exponentiation's value is the reference's.  f = 0 iff some g_s = 0 (a
// field), which sets the error bit and the zero image as before.
// miller_loop_batch: generic squarings and the Miller value itself.
// Every group of the block stays busy to the end (a wave whose other groups have
// returned runs its last group markedly slower): groups past S work
// on one, every group runs group 0's number of squarings and keeps its own
// count's result, every group computes each tree level's product and keeps it
// where the level needs it, and the last chunk then runs on every group pair --
// S groups 0-7 with M groups 8-15 (BN_FE_DUO) -- on copies of group 0's value;
// group 0 stores the result.
__shared__ uint32_t g_hor_zero;
__global__ void __launch_bounds__(kBlock) k_horner_tree(const uint32_t* __restrict__ g, SegPlan plan, int do_fe,
                                                        bn_gt* __restrict__ out, int* __restrict__ err, int duo) {
    HOR_STAMP(0);  // start
    if (threadIdx.x == 0) g_hor_zero = 0;
    __syncthreads();  // the reset is seen before any group can set the flag
    fold_table_init();
    w_duo_init();
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
    HOR_STAMP(1);  // g_0 in
    if (do_fe) {
        if (seg && w12_is_zero(x) && w.l == 0) g_hor_zero = 1;
        x = w12_fe_first(x);  // first chunk; of one (groups past S): one
        HOR_STAMP(3);         // group 0's first chunk done
#pragma unroll 1
        for (int k = 0; k < e0; ++k) {
            const Fq<2> y = w12_cyc(x);
            x = k < e ? y : x;
        }
    } else {
#pragma unroll 1
        for (int k = 0; k < e0; ++k) {
            const Fq<2> y = w12_square(x);
            x = k < e ? y : x;
        }
    }
    HOR_STAMP(2);  // group 0's squarings done
    uint32_t* mine = g_wval + (grp * kWLanes) * kWSlot;
#pragma unroll 1
    for (int h = kWGroups / 2; h >= 1; h /= 2) {
        w_put(mine, w.l, x);
        __syncthreads();
        const Fq<2> y = w12_mul(x, w_get<2>(g_wval + (((grp + h) % kWGroups) * kWLanes) * kWSlot, w.l));
        if (grp < h && grp + h < plan.S) x = y;  // groups past S hold one
        __syncthreads();
    }
    // every group takes group 0's value: the pairs (g, g + 8) run the last chunk side by side
    if (grp == 0) w_put(g_wval, w.l, x);
    __syncthreads();
    x = w_get<2>(g_wval, w.l);
    HOR_STAMP(4);  // recombination done
    const WRole role = w_role(duo != 0);  // group g < 8: S of channel g; group g + 8: its M
    if (w_final_exp_m(role, do_fe != 0, err)) return;
    uint32_t words[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (do_fe) {
        const bool zero = g_hor_zero != 0;
        if (zero && err && w.l == 0 && grp == 0) err_or(err, BN_ERR_FE_ZERO);
        const Fq<2> r = w_fe_last(role, x, err);
        HOR_STAMP(5);  // final exponentiation done
        if (!zero) fq_store_ref(r, words);
    } else {
        fq_store_ref(x, words);
    }
    if (w.l < 12 && grp == 0) st_words(&out[0].c[w_gt_index(w)], words);
}

}  // namespace bn
#include "latency_kernel.h"
namespace bn {

// *status = the bn_status of the device-side outcome bits in *err (bn_*_batch_dev)
__global__ void __launch_bounds__(kBlock) k_err_status(const int* __restrict__ err, int* __restrict__ status) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        const int b = *err;
        *status = (b & (1 << BN_ERR_INTERNAL))    ? BN_ERR_INTERNAL
                  : (b & (1 << BN_ERR_TO_AFFINE)) ? BN_ERR_TO_AFFINE
                  : (b & (1 << BN_ERR_FE_ZERO))   ? BN_ERR_FE_ZERO
                                                  : BN_OK;
    }
}

}  // namespace bn

#if BN_LAT_STAMPS
extern "C" int bn_dbg_lat_stamps(uint64_t out[8]) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(bn::g_lat_stamps), 8 * sizeof(uint64_t)) == hipSuccess ? 0 : -1;
}
extern "C" int bn_dbg_hor_stamps(uint64_t out[8]) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(bn::g_hor_stamps), 8 * sizeof(uint64_t)) == hipSuccess ? 0 : -1;
}
#endif

BN_EXPORT_FOLD_CHECK(wide)
