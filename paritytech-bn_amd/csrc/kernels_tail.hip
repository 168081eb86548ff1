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
#define BN_FOLD_LDS 1
#define BN_WIDE_ARRS 4
#define BN_S_CYC w12_cyc32
#include "fq.h"
#define BN_SPLIT 1
#include "fq12_wide.h"
#if BN_TAIL_DS
#include "fq12_ds.h"
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
__global__ void __launch_bounds__(kTailThreads) k_seg_fe1(uint32_t* __restrict__ g, SegPlan plan,
                                                          uint32_t* __restrict__ zf) {
    fold_table_init();
    const WL w = wl();
    const int s = (int)blockIdx.x;
    {  // k_horner_tree2's channel: every stamp cleared (the blocks share the words)
        uint64_t* ch = (uint64_t*)(zf + kDsChanOff);
        for (int i = s * kTailThreads + (int)threadIdx.x; i < kDsChanWords / 2; i += plan.S * kTailThreads)
            __hip_atomic_store(ch + i, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    int e = 0;
    for (int t = s + 1; t < plan.S; ++t) e += plan.hi[t] - plan.lo[t];
    Fq<2> x = widen<2>(fq_zero());
    if (threadIdx.x < (unsigned)kWLanes) {  // group 0
        x = w_ld_split(g, (size_t)plan.S, (size_t)s, w);
        const bool zero = w12_is_zero(x);
        if (threadIdx.x == 0) zf[s] = zero ? 1u : 0u;
        x = w12_fe_first(x);
    }
    ds_init();
    uint32_t d = ds_from_w12(x);
#pragma unroll 1
    for (int k = 0; k < e; ++k) d = ds_cyc(d);
    x = ds_to_w12(d);
    if (threadIdx.x < 12) w_st_split(g, (size_t)plan.S, (size_t)s, w, x);
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
        ds_init();
        DsChan ch = {(uint64_t*)(const_cast<uint32_t*>(zf) + kDsChanOff), err, 0, 0};
        ds_fe_last_m(ch);
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
        ds_init();
        uint32_t d = ds_from_w12(x);
        if (zf && gridDim.x == 2) {  // with the multiplier block (block 1)
            DsChan ch = {(uint64_t*)(const_cast<uint32_t*>(zf) + kDsChanOff), err, 0, 0};
            d = ds_fe_last_s(d, ch);
        } else {
            d = ds_fe_last(d);
        }
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
