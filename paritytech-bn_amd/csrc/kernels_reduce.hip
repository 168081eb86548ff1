// kernels_reduce.hip -- k_fq12_reduce_wide, the product reduction behind
// pairing_batch / miller_loop_batch (mod.rs:609-640, 904-926), in its own
// translation unit: it multiplies with w12_mul only, so the wide layout needs
// four operand arrays per group, not five, and the block tree passes values
// through each group's fourth array instead of a separate one -- 55.9 KB of LDS
// per block instead of 81.5 KB, so two blocks share a CU (149 VGPRs).  Inputs and
// outputs use the lane-strided two-lane layout of the pairing path.
#define BN_FOLD_LDS 1
#define BN_WIDE_ARRS 4
#include "fq.h"
#define BN_SPLIT 1
#include "fq12_wide.h"

namespace bn {

// Product reduction of several independent sets (set y: the elements
// sets.off[y] + [0, sets.n[y]) of `in`, split layout, stride in_stride, taken by
// the blocks sets.blk[y] .. sets.blk[y + 1] - 1, so sets of different sizes need
// no padding blocks): block b of set y multiplies the set's elements
// [16Gb, 16Gb + 16G) (G = per_group) -- a
// chain of G factors per group (elements g, g + 16, ...), then a tree over the 16
// groups through LDS -- and writes the block's product as element out_base + y *
// out_set + b of `out` (stride out_stride).  Elements past n[y] count as one.  The
// order of the factors differs from the reference's left-to-right accumulation;
// Fq12 multiplication is commutative and associative, so the value is the same.
__global__ void __launch_bounds__(kBlock) k_fq12_reduce_wide(const uint32_t* __restrict__ in, size_t in_stride,
                                                             SetSpan sets, uint32_t* __restrict__ out,
                                                             size_t out_stride, size_t out_base, size_t out_set,
                                                             int per_group) {
    fold_table_init();
    const WL w = wl();
    const int g = (int)threadIdx.x / kWLanes;
    // group g multiplies elements e0 + 16t (t < per_group) of its block's range in
    // a chain -- at each step the block's 16 groups read 16 consecutive elements --
    // with the next factor's load issued before the product that precedes it
    // (factors past n are skipped), then the groups' values meet in the tree below
    int set = 0;
    while (set + 1 < sets.sets && blockIdx.x >= sets.blk[set + 1]) ++set;  // block-uniform
    const size_t b = blockIdx.x - sets.blk[set];
    const size_t e0 = b * kWGroups * (size_t)per_group + g, sb = sets.off[set];
    const size_t n = sets.n[set];
    const Fq<2> one = fq_select(w.e == 0 && w.c == 0, widen<2>(fq_one()), widen<2>(fq_zero()));
    Fq<2> x = e0 < n ? w_ld_split(in, in_stride, sb + e0, w) : one;
    Fq<2> y = e0 + kWGroups < n ? w_ld_split(in, in_stride, sb + e0 + kWGroups, w) : one;
#pragma unroll 1
    for (int t = 1; t < per_group; ++t) {
        const size_t e = e0 + (size_t)(t + 1) * kWGroups;
        const Fq<2> y_next = (t + 1 < per_group && e < n) ? w_ld_split(in, in_stride, sb + e, w) : one;
        if (e0 + (size_t)t * kWGroups < n) x = w12_mul(x, y);  // uniform per group
        y = y_next;
    }
    // the tree: group g's value sits in its fourth operand array, which only g's own
    // w12_mul overwrites -- and at a level where g multiplies, no group reads g's slot
    // (its readers are the groups g - s, and g < s) before the barrier that ends it
    auto slot = [&](int grp) { return g_wide + grp * kWGroupWords + 3 * kWArr; };
#pragma unroll 1
    for (int s = kWGroups / 2; s >= 1; s /= 2) {
        w_put(slot(g), w.l, x);
        __syncthreads();
        if (g < s) {
            const Fq<2> y2 = w_get<2>(slot(g + s), w.l);
            x = w12_mul(x, y2);
        }
        __syncthreads();
    }
    if (g == 0) w_st_split(out, out_stride, out_base + (size_t)set * out_set + b, w, x);
}

}  // namespace bn

BN_EXPORT_FOLD_CHECK(reduce)
