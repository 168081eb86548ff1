// latency_kernel.h -- k_pairing_latency (pairing() of a few pairs in one launch,
// DESIGN.md §5), included by two translation units:
//  - kernels_wide.hip: the one-wave-per-SIMD build (batches up to 2,048 pairs:
//    one block of 8 pairs per CU);
//  - kernels_latency_w2.hip: the same kernel as k_pairing_latency_w2, built for
//    two waves per SIMD (every kernel of that unit has amdgpu_waves_per_eu(2, 2),
//    so the wide-layout functions it calls fit 256 registers) with the smaller
//    LDS footprint of BN_WIDE_ARRS = 4, BN_LAT_RING = 6, BN_DUO_RING = 1 (77.8 KB:
//    two blocks per CU), for 2,049-4,096 pairs in one round of blocks.
// A lone wave issues a v_mad_u64_u32 only every ~9.5 cycles (profiles/r3j_mad_issue.txt),
// so a second wave on the SIMD runs its own chain beside the first almost for free.
#pragma once
#ifndef BN_LAT_KERNEL_NAME
#define BN_LAT_KERNEL_NAME k_pairing_latency
#endif
#ifndef BN_LAT_KERNEL_ATTR
#define BN_LAT_KERNEL_ATTR
#endif

namespace bn {

// ---------------------------------------------------------------- k_pairing_latency
// pairing() of a few pairs in ONE launch, for latency (bn_pairing_many_dev
// batches of at most kLatencyMaxDefault pairs, capi.hip).  A block holds
// kLatPairs pairs and three waves (four with BN_FE_DUO):
//  - wave 0, the producer: to_affine and the 87 line coefficients of each pair
//    on eight lanes (lines_wide.h, as k_prepare_wide), each line scaled by P
//    (ell_vw * Py, ell_vv * Px: mod.rs:589) and put into the pair's LDS ring;
//  - waves 1-2, the consumers: one 16-lane group per pair runs the Miller loop
//    on the wide layout (fq12_wide.h) right behind the producer -- per digit
//    the generic square and the sparse product by each line as it arrives
//    (mod.rs:579-607's order, so the Miller value is the reference's) -- then
//    the final exponentiation (w12_final_exp), and stores the Gt image;
//  - BN_FE_DUO: the consumer is the squarer of the two-group final
//    exponentiation (fq12_wide.h w12_final_exp_s); the multiplier groups are
//    wave 0 once its lines are out (pairs 0-3) and wave 3 (pairs 4-7).
// The loop needs no segments and no Horner recombination, and the three
// kernels of the segmented latency path (k_prepare_wide, k_miller_seg,
// k_horner_wide) become one.  Hand-off: the producer writes a line, waits for
// its LDS writes (lgkmcnt(0)) and bumps the pair's `prod` counter; a consumer
// spins (s_sleep) until `prod` passes the line it needs and bumps `cons` after
// reading it; the producer keeps at most kLatRing lines ahead.  Both sides
// always progress, so every wave reaches the end; the spins are capped anyway, and
// a wait that runs out of its cap sets BN_ERR_INTERNAL (the call then fails).
// (the ring itself, g_lat_ring, is declared in fq12_wide.h beside w12_mul_line)
__shared__ uint32_t g_lat_prod[kLatPairs], g_lat_cons[kLatPairs], g_lat_skip[kLatPairs];
__shared__ uint32_t g_lat_duo[kLatPairs * 4];  // BN_FE_DUO: the counters of each pair's channel
static_assert(kDuoWords <= kLatRing * kLatLineWords, "the FE channel reuses the pair's line ring");
constexpr uint32_t kLatSpinCap = kSpinCap;  // fq12_wide.h: ~4 s of s_sleep 1, never reached while both sides run

// Diagnostic build (-DBN_LAT_STAMPS=1, tools/lat_stamps.py): block 0 records
// s_memrealtime (100 MHz) at the phase boundaries of its first pair into a
// buffer read by bn_dbg_lat_stamps(); the product build has none of it.
#ifndef BN_LAT_STAMPS
#define BN_LAT_STAMPS 0
#endif
#if BN_LAT_STAMPS
__device__ uint64_t g_lat_stamps[8];
#define LAT_STAMP(cond, k)                                                            \
    do {                                                                              \
        if (blockIdx.x == 0 && (cond)) g_lat_stamps[k] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
#else
#define LAT_STAMP(cond, k) ((void)0)
#endif

#if BN_FE_DUO
// the multiplier group of pair j (fq12_wide.h, two-group final exponentiation);
// its channel is the pair's line ring, free once the Miller loop has read every
// line -- before S hands over anything
__device__ __forceinline__ void lat_multiplier(int j, size_t base, size_t n, const uint32_t* f_out, int* err) {
    (void)base;
    (void)n;
    if (f_out) return;  // no final exponentiation here (idle groups pair up with their idle squarers)
    WDuo duo = {g_lat_ring + j * kLatRing * kLatLineWords, g_lat_duo + 4 * j, 0, 0, err};
    w12_final_exp_m(duo);
}
#endif

// f_out != null (pairing_batch / miller_loop_batch): the Miller values go to
// f_out (split layout, lane-strided, stride n; a zero-point pair's is one) for the
// product reduction, and no final exponentiation runs here; mode 1
// (miller_loop_batch) flags a zero point as BN_ERR_TO_AFFINE (lib.rs:629-630).
__global__ void __launch_bounds__(kLatThreads) BN_LAT_KERNEL_ATTR BN_LAT_KERNEL_NAME(const bn_g1* __restrict__ p,
                                                                 const bn_g2* __restrict__ q, size_t n,
                                                                 bn_gt* __restrict__ out, uint32_t* __restrict__ f_out,
                                                                 int mode, int* __restrict__ err) {
    fold_table_init();
    if (threadIdx.x < kLatPairs) {
        g_lat_prod[threadIdx.x] = 0;
        g_lat_cons[threadIdx.x] = 0;
        g_lat_skip[threadIdx.x] = 0;
    }
    if (threadIdx.x < kLatPairs * 4) g_lat_duo[threadIdx.x] = 0;
    __syncthreads();
    volatile uint32_t* prod = g_lat_prod;
    volatile uint32_t* cons = g_lat_cons;
    const size_t base = (size_t)blockIdx.x * kLatPairs;
    LAT_STAMP(threadIdx.x == 0, 0);  // start
    if (threadIdx.x < 64) {
        // ---- producer wave: pair j on lanes 8j..8j+7 (k_prepare_wide's layout)
        const int L = (int)threadIdx.x, j = L >> 3, c = L & 1;
        const bool valid = base + j < n;
        const size_t pi = valid ? base + j : n - 1;  // idle slots repeat a real pair
        const int k = pw_slot();
        const bool st = k == 0;
        const PairAffine a = pair_to_affine<true>(p, q, pi, pi * kL + c, nullptr, err, valid ? mode : 0);
        LAT_STAMP(threadIdx.x == 0, 1);  // producer: to_affine done
        if (st && c == 0) g_lat_skip[j] = a.skip ? 1u : 0u;
        bool dead = false;  // a wait of this wave ran out of its cap
        // the ring wait (the producer stays at most kLatRing lines ahead of its consumer)
        auto ring_wait = [&](int line) {
            uint32_t spins = 0;
            if (!dead)
                for (; BN_ANY(valid && line - (int)cons[j] >= kLatRing) && spins < kLatSpinCap; ++spins)
                    __builtin_amdgcn_s_sleep(1);
            if (BN_ANY(valid && line - (int)cons[j] >= kLatRing)) {  // ring overrun: fail the call
                dead = true;  // sticky for the wave: no later wait spins again
                if (L == 0 && err) err_or(err, BN_ERR_INTERNAL);
            }
            asm volatile("" ::: "memory");
        };
        // the operand forms c0, c1, -c1 of a coefficient (fq12_wide.h w12_mul_line) at ring words 3q..3q+2
        auto ring_put = [&](int line, int qq, const Fq2<kLine>& x) {
            uint32_t* ln = g_lat_ring + (j * kLatRing + line % kLatRing) * kLatLineWords;
            w_put(ln, 3 * qq + c, x.c);
            if (c) w_put(ln, 3 * qq + 2, fq_neg(x.c));
        };
        auto announce = [&](int line) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the line is in LDS before it is announced
            if (st && c == 0) prod[j] = (uint32_t)line + 1;
        };
        G2Proj r = {a.qa.x, a.qa.y, widen<kPt>(fq2_one())};
        const auto qy_neg = fq2_neg(a.qa.y);
        int line = 0;
#if BN_LINES_PRESCALED
        // the P products from the steps' free slots (lines_wide.h PwEll): slot 0 writes
        // ell_0, slot 2 ell_vw * Py (x4), slot 3 ell_vv * Px (x2), each from its own lanes
        // (one select and one ring write per lane at a per-slot offset, not a write per
        // slot under its own branch: that staged the values through scratch)
        auto emit = [&](int ln_i, const PwEll& e) {
            const Fq2<kLine> x = fq2_select(k == 0, e.e.ell_0, fq2_select(k == 2, e.vw_py, e.vv_px));
            ring_wait(ln_i);
            if (k != 1) ring_put(ln_i, k == 0 ? 0 : k - 1, x);
            announce(ln_i);
        };
        const Fq2<2> py_r = pw_real(a.py);
        const Fq2<2> px_r = pw_real(a.px);
        const auto px3_r = pw_real(fq_add(fq_add(a.px, a.px), a.px));
        const auto bxpy_q = fq2_scale(a.qa.x, a.py);
#pragma unroll 1
        for (int d = 0; d < BN_NAF_DIGITS; ++d) {
            emit(line++, pw_doubling_step_p(r, k, py_r, px3_r));
            if ((kNafNonzero >> d) & 1u) {
                const bool minus = (kNafMinus >> d) & 1u;
                const G2Aff<kPt> bq = {a.qa.x, fq2_select(minus, widen<kPt>(qy_neg), a.qa.y)};
                emit(line++, pw_mixed_addition_step_p(r, bq, bxpy_q, k, py_r, px_r));
            }
        }
        G2Aff<kPt> q1 = mul_by_q(a.qa);
        G2Aff<kPt> q2 = mul_by_q(q1);
        q2.y = narrow<kPt>(fq2_neg(q2.y));
        emit(line++, pw_mixed_addition_step_p(r, q1, fq2_scale(q1.x, a.py), k, py_r, px_r));
        emit(line++, pw_mixed_addition_step_p(r, q2, fq2_scale(q2.x, a.py), k, py_r, px_r));
#else
        auto emit = [&](int ln_i, const Ell& e) {
            // slots 0, 2 scale ell_vw by Py, slots 1, 3 ell_vv by Px (one product
            // per lane instead of two); slot 0 takes x2 from slot 1
            const bool odd_slot = (k & 1) != 0;
            const auto y = narrow<kLine>(fq2_scale(fq2_select(odd_slot, e.ell_vv, e.ell_vw), fq_select(odd_slot, a.px, a.py)));
            const auto x2 = pw_from(y, 1);
            ring_wait(ln_i);
            if (st) {
                ring_put(ln_i, 0, e.ell_0);
                ring_put(ln_i, 1, y);
                ring_put(ln_i, 2, x2);
            }
            announce(ln_i);
        };
#pragma unroll 1
        for (int d = 0; d < BN_NAF_DIGITS; ++d) {
            emit(line++, pw_doubling_step(r, k));
            if ((kNafNonzero >> d) & 1u) {
                const bool minus = (kNafMinus >> d) & 1u;
                const G2Aff<kPt> bq = {a.qa.x, fq2_select(minus, widen<kPt>(qy_neg), a.qa.y)};
                emit(line++, pw_mixed_addition_step(r, bq, k));
            }
        }
        G2Aff<kPt> q1 = mul_by_q(a.qa);
        G2Aff<kPt> q2 = mul_by_q(q1);
        q2.y = narrow<kPt>(fq2_neg(q2.y));
        emit(line++, pw_mixed_addition_step(r, q1, k));
        emit(line++, pw_mixed_addition_step(r, q2, k));
#endif
        LAT_STAMP(threadIdx.x == 0, 2);  // producer: last line out
#if BN_FE_DUO
        lat_multiplier((int)threadIdx.x / kWLanes, base, n, f_out, err);
#endif
        return;
    }
#if BN_FE_DUO
    if (threadIdx.x >= 64 + kLatPairs * kWLanes) {  // wave 3: the multipliers of pairs 4-7
        lat_multiplier(kLatPairs / 2 + ((int)threadIdx.x - 64 - kLatPairs * kWLanes) / kWLanes, base, n, f_out, err);
        return;
    }
#endif
    // ---- consumer groups: pair j on a 16-lane group of waves 1-2
    const int j = ((int)threadIdx.x - 64) / kWLanes;
    // idle groups repeat the block's last pair (the producer fills their rings
    // with it) and store nothing, so a wave runs the same number of groups
    // whatever n is
    const bool live = base + j < n;
    const size_t pi = live ? base + j : n - 1;
    const WL w = wl();
    auto ln = [&](int line) { return (uint32_t)((j * kLatRing + line % kLatRing) * kLatLineWords); };
    bool dead = false;  // a wait of this group ran out of its cap
    auto wait_line = [&](int line) {
        uint32_t spins = 0;
        if (!dead)
            for (; prod[j] <= (uint32_t)line && spins < kLatSpinCap; ++spins) __builtin_amdgcn_s_sleep(1);
        if (prod[j] <= (uint32_t)line) {  // line never published: fail the call
            dead = true;
            if (w.l == 0 && err) err_or(err, BN_ERR_INTERNAL);
        }
        asm volatile("" ::: "memory");
    };
    auto took = [&](int line) {  // the line's words have been read (the product has returned)
        asm volatile("" ::: "memory");
        if (w.l == 0) cons[j] = (uint32_t)line + 1;
    };
    int line = 0;
    wait_line(line);
    LAT_STAMP(threadIdx.x == 64, 3);  // consumer: first line in
    Fq<2> f = w12_from_line(ln(line));  // digit 0 from f = one: one^2 * line = the line
    took(line++);
#pragma unroll 1
    for (int d = 0; d < BN_NAF_DIGITS; ++d) {
        if (d > 0) {
            f = w12_square(f);  // the generic square, as the reference's loop
            wait_line(line);
            f = w12_mul_line(f, ln(line));
            took(line++);
        }
        if ((kNafNonzero >> d) & 1u) {
            wait_line(line);
            f = w12_mul_line(f, ln(line));
            took(line++);
        }
    }
#pragma unroll 1
    for (int t = 0; t < 2; ++t) {  // the lines of Q1 and -Q2 (mod.rs:600-604)
        wait_line(line);
        f = w12_mul_line(f, ln(line));
        took(line++);
    }
    LAT_STAMP(threadIdx.x == 64, 4);  // consumer: Miller loop done
    // a zero point: pairing() is Fq12::one() (mod.rs:896), and FE(one) = one
    const Fq<2> one = fq_select(w.e == 0 && w.c == 0, widen<2>(fq_one()), widen<2>(fq_zero()));
    const Fq<2> x = g_lat_skip[j] ? one : f;
    if (f_out) {  // the Miller value, for the product of pairing_batch / miller_loop_batch
        if (live) w_st_split(f_out, n, pi, w, x);
        return;
    }
    const bool zero = w12_is_zero(x);
    if (zero && err && w.l == 0 && live) err_or(err, BN_ERR_FE_ZERO);
#if BN_FE_DUO
    WDuo duo = {g_lat_ring + j * kLatRing * kLatLineWords, g_lat_duo + 4 * j, 0, 0, err};
    const Fq<2> res = w12_final_exp_s(x, duo);
#else
    const Fq<2> res = w12_final_exp(x);
#endif
    LAT_STAMP(threadIdx.x == 64, 5);  // consumer: final exponentiation done
    uint32_t words[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (!zero) fq_store_ref(res, words);
    if (w.l < 12 && live) st_words(&out[pi].c[w_gt_index(w)], words);
}


}  // namespace bn
