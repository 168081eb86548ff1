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

namespace bn {

__device__ __forceinline__ size_t w_elem() { return lane_id() / kWLanes; }

// this lane's coordinate of element e of a lane-strided split Fq12 array
// (stride = elements in the array)
__device__ __forceinline__ Fq<2> w_ld_split(const uint32_t* f, size_t stride, size_t e, const WL& w) {
    return ld_fq<2>(f, 2 * stride, 2 * e + w.c, w_tower_index(w));
}
__device__ __forceinline__ void w_st_split(uint32_t* f, size_t stride, size_t e, const WL& w, const Fq<2>& x) {
    if (w.l < 12) st_fq(f, 2 * stride, 2 * e + w.c, w_tower_index(w), x);
}

// out[e] = final_exponentiation(f[e]) for e < n, f lane-strided (split layout,
// stride `stride`).  f == 0: zero image, ok = 0, error bit (fq12.rs:63-72;
// pairing() panics, mod.rs:900).  A skipped pair's Miller value is already
// Fq12::one() (k_miller), and FE(one) = one.
__global__ void __launch_bounds__(kBlock) k_fe_wide(const uint32_t* __restrict__ f, size_t stride, size_t n,
                                                    bn_gt* __restrict__ out, uint8_t* __restrict__ ok,
                                                    int* __restrict__ err) {
    fold_table_init();
    const size_t e = w_elem();
    if (e >= n) return;
    const WL w = wl();
    const Fq<2> x = w_ld_split(f, stride, e, w);
    const bool zero = w12_is_zero(x);
    if (ok && w.l == 0) ok[e] = zero ? 0 : 1;
    if (zero && err && w.l == 0) atomicOr(err, 1 << BN_ERR_FE_ZERO);
    const Fq<2> r = w12_final_exp(x);
    uint32_t words[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (!zero) fq_store_ref(r, words);
    if (w.l < 12) st_words(&out[e].c[w_gt_index(w)], words);
}

// Product reduction of several independent sets (blockIdx.y = set y, the
// elements y * in_set + [0, n) of `in`, split layout, stride in_stride): block
// (b, y) multiplies the set's elements [32b, 32b + 32) -- one product per group
// of the two elements 2g, 2g + 1, then a tree over the 16 groups through LDS --
// and writes the block's product as element out_base + y * out_set + b of `out`
// (stride out_stride).  Elements past n count as one.  The order of the factors
// differs from the reference's left-to-right accumulation; Fq12 multiplication
// is commutative and associative, so the value is the same.
__shared__ uint32_t g_wval[kWGroups * kWLanes * kWSlot];  // 12 KB: one value per group

__global__ void __launch_bounds__(kBlock) k_fq12_reduce_wide(const uint32_t* __restrict__ in, size_t in_stride,
                                                             size_t n, size_t in_set, uint32_t* __restrict__ out,
                                                             size_t out_stride, size_t out_base, size_t out_set) {
    fold_table_init();
    const WL w = wl();
    const int g = (int)threadIdx.x / kWLanes;
    const size_t base = (size_t)blockIdx.x * 2 * kWGroups;
    const size_t e0 = base + 2 * g, e1 = e0 + 1, sb = (size_t)blockIdx.y * in_set;
    const Fq<2> one = fq_select(w.e == 0 && w.c == 0, widen<2>(fq_one()), widen<2>(fq_zero()));
    const Fq<2> a = e0 < n ? w_ld_split(in, in_stride, sb + e0, w) : one;
    const Fq<2> b = e1 < n ? w_ld_split(in, in_stride, sb + e1, w) : one;
    Fq<2> x = e1 < n ? w12_mul(a, b) : a;  // uniform per group
    uint32_t* mine = g_wval + (g * kWLanes) * kWSlot;
#pragma unroll 1
    for (int s = kWGroups / 2; s >= 1; s /= 2) {
        w_put(mine, w.l, x);
        __syncthreads();
        if (g < s) {
            const Fq<2> y = w_get<2>(g_wval + ((g + s) * kWLanes) * kWSlot, w.l);
            x = w12_mul(x, y);
        }
        __syncthreads();
    }
    if (g == 0) w_st_split(out, out_stride, out_base + blockIdx.y * out_set + blockIdx.x, w, x);
}

// Recombination of segmented Miller loops (pairing.h miller_segment), one
// 16-lane group per element e < n: segment s of element e is element s * n + e
// of g (split layout, stride S * n, as k_miller_seg writes it).  x = g_0, then
// x = x^(2^len_s) * g_s for s = 1..S-1 (the generic squaring, as the reference's
// loop squares its accumulator), then the final exponentiation when do_fe
// (pairing / pairing_batch; zero -> zero image + error bit) or the Miller value
// itself (miller_loop_batch) -> out[e].
__global__ void __launch_bounds__(kBlock) k_horner_wide(const uint32_t* __restrict__ g, size_t n, SegPlan plan,
                                                        int do_fe, bn_gt* __restrict__ out, int* __restrict__ err) {
    fold_table_init();
    const size_t e = w_elem();
    if (e >= n) return;
    const WL w = wl();
    const size_t stride = (size_t)plan.S * n;
    Fq<2> x = w_ld_split(g, stride, e, w);
#pragma unroll 1
    for (int s = 1; s < plan.S; ++s) {
#pragma unroll 1
        for (int k = plan.lo[s]; k < plan.hi[s]; ++k) x = w12_mul(x, x);
        x = w12_mul(x, w_ld_split(g, stride, (size_t)s * n + e, w));
    }
    uint32_t words[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (do_fe) {
        const bool zero = w12_is_zero(x);
        if (zero && err && w.l == 0) atomicOr(err, 1 << BN_ERR_FE_ZERO);
        const Fq<2> r = w12_final_exp(x);
        if (!zero) fq_store_ref(r, words);
    } else {
        fq_store_ref(x, words);
    }
    if (w.l < 12) st_words(&out[e].c[w_gt_index(w)], words);
}

// *status = the bn_status of the device-side outcome bits in *err (bn_*_batch_dev)
__global__ void __launch_bounds__(kBlock) k_err_status(const int* __restrict__ err, int* __restrict__ status) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        const int b = *err;
        *status = (b & (1 << BN_ERR_TO_AFFINE)) ? BN_ERR_TO_AFFINE : (b & (1 << BN_ERR_FE_ZERO)) ? BN_ERR_FE_ZERO : BN_OK;
    }
}

}  // namespace bn
