// kernels_util.hip -- product tree over Miller values and Gt image <-> lane-strided conversion.
#include "kernels.h"

namespace bn {

// f[i] *= f[i + half] for i + half < m: one level of the product tree (array stride `stride`)
__global__ void __launch_bounds__(kBlock) k_fq12_product(uint32_t* __restrict__ f, size_t stride, size_t m, size_t half) {
    fold_table_init();
    const size_t i = lane_id();
    if (i >= half || i + half >= m) return;
    Fq12<kF> a = ld_fq12_buf<kF>(f, stride, i);
    Fq12<kF> b = ld_fq12_buf<kF>(f, stride, i + half);
    st_fq12_buf(f, stride, i, mul12(a, b));
}

// Gt images <-> lane-strided internal Fq12
__global__ void __launch_bounds__(kBlock) k_gt_load(const bn_gt* __restrict__ g, size_t n, uint32_t* __restrict__ f) {
    fold_table_init();
    const size_t i = lane_id();
    if (i >= n) return;
    st_fq12(f, n, i, ld_gt(g[i]));
}
__global__ void __launch_bounds__(kBlock) k_gt_store(const uint32_t* __restrict__ f, size_t n, size_t stride,
                                                     bn_gt* __restrict__ g) {
    fold_table_init();
    const size_t i = lane_id();
    if (i >= n) return;
    st_gt(g[i], ld_fq12<kF>(f, stride, i));
}

}  // namespace bn

BN_EXPORT_FOLD_CHECK(util)
