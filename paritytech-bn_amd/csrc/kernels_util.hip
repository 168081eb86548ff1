// kernels_util.hip -- Gt image <-> lane-strided conversion.
// Pairing-path layout (BN_PATH_SPLIT: two lanes per element, kernels.h); n,
// m, half and stride count elements, the grid has kPathLanes threads each.
#include "fq.h"
#define BN_SPLIT BN_PATH_SPLIT
#include "kernels.h"

namespace bn {

constexpr size_t kL = BN_SPLIT ? 2 : 1;  // lanes per element in this translation unit

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
