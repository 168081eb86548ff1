// kernels_util.hip -- product tree over Miller values and Gt image <-> lane-strided conversion.
// Pairing-path layout (BN_PATH_SPLIT: two lanes per element, kernels.h); n,
// m, half and stride count elements, the grid has kPathLanes threads each.
#include "fq.h"
#define BN_SPLIT BN_PATH_SPLIT
#include "kernels.h"

namespace bn {

constexpr size_t kL = BN_SPLIT ? 2 : 1;  // lanes per element in this translation unit

// f[e] *= f[e + half] for e + half < m: one level of the product tree (slot stride `stride` elements)
__global__ void BN_PATH_ATTR __launch_bounds__(kBlock) k_fq12_product(uint32_t* __restrict__ f, size_t stride, size_t m,
                                                                     size_t half) {
    fold_table_init();
    const size_t l = lane_id(), e = l / kL;
    if (e >= half || e + half >= m) return;
    Fq12<kF> a = ld_fq12_buf<kF>(f, kL * stride, l);
    Fq12<kF> b = ld_fq12_buf<kF>(f, kL * stride, l + kL * half);
    st_fq12_buf(f, kL * stride, l, mul12(a, b));
}

// Gt images <-> lane-strided internal Fq12
__global__ void BN_PATH_ATTR __launch_bounds__(kBlock) k_gt_load(const bn_gt* __restrict__ g, size_t n,
                                                                uint32_t* __restrict__ f) {
    fold_table_init();
    const size_t l = lane_id(), e = l / kL;
    if (e >= n) return;
    st_fq12(f, kL * n, l, ld_gt(g[e]));
}
__global__ void BN_PATH_ATTR __launch_bounds__(kBlock) k_gt_store(const uint32_t* __restrict__ f, size_t n, size_t stride,
                                                                 bn_gt* __restrict__ g) {
    fold_table_init();
    const size_t l = lane_id(), e = l / kL;
    if (e >= n) return;
    st_gt(g[e], ld_fq12<kF>(f, kL * stride, l));
}

}  // namespace bn

BN_EXPORT_FOLD_CHECK(util)
