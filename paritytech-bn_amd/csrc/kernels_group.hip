// kernels_group.hip -- batched G1 scalar multiplication (mod.rs:272-292) and the
// G1/G2 group law (mod.rs:169-216, 294-358), one lane per element (G2 * Fr runs
// on the two-lane layout: kernels_pairing.hip k_g2_mul_split).
// fq_fold reads -q*p from an LDS table (fq.h; every kernel here calls
// fold_table_init first)
#ifndef BN_FOLD_LDS
#define BN_FOLD_LDS 1
#endif
#include "kernels.h"

namespace bn {

// ---------------------------------------------------------------- scalar multiplication
// Launched with kPairBlock threads per block when the batch gives every CU a
// whole block (kG1MulPairBlockMin, capi.hip), else kBlock: the issue balance of
// kernels.h between the two waves each SIMD then holds.  (1024-thread blocks,
// four waves per SIMD, cap the kernel at 128 VGPRs: 428 B of spills.)
__global__ void __launch_bounds__(kPairBlock) k_g1_mul(const bn_g1* __restrict__ p, const bn_fr* __restrict__ k, size_t n,
                                                     bn_g1* __restrict__ out) {
    fold_table_init();
    const Balance bal = balance_init();
    const size_t i = lane_id();
    if (i >= n) return;
    uint32_t s[8];
    fr_to_canonical(k[i], s);
    G1J a = {widen<kPt>(ld_ref(p[i].x)), widen<kPt>(ld_ref(p[i].y)), widen<kPt>(ld_ref(p[i].z))};
    G1J r = jac_mul(a, s, [&](int t) { balance_step(bal, (uint32_t)t); });
    st_ref(out[i].x, r.x);
    st_ref(out[i].y, r.y);
    st_ref(out[i].z, r.z);
}
// Two chains per lane (curve.h jac_mul2): lane i multiplies elements i and i + h,
// h = ceil(n / 2); the odd tail's second chain has the zero scalar.  The two bases
// and the two canonical scalars sit in LDS, word-major ([word][thread],
// conflict-free): 2 x (27 + 8) words per thread, 143 KB per 512-thread block
// besides the fold table.
constexpr int kMul2Words = 27;
constexpr int kMul2Slots = 2 * kMul2Words + 16;
__global__ void __launch_bounds__(kPairBlock) k_g1_mul2(const bn_g1* __restrict__ p, const bn_fr* __restrict__ k,
                                                      size_t n, bn_g1* __restrict__ out) {
    __shared__ uint32_t lds[kMul2Slots][kPairBlock];
    fold_table_init();
    const Balance bal = balance_init();
    const size_t h = (n + 1) / 2;
    const size_t i = lane_id();
    if (i >= h) return;
    const unsigned tid = threadIdx.x;
    const size_t j = i + h;
    const bool has1 = j < n;
    const size_t j1 = has1 ? j : i;
    bool z0, z1;
    int top0, top1;
    {
        uint32_t s0[8], s1[8];
        fr_to_canonical(k[i], s0);
        fr_to_canonical(k[j1], s1);
#pragma unroll
        for (int t = 0; t < 8; ++t) s1[t] = has1 ? s1[t] : 0u;
        top0 = scalar_top_bit(s0);
        top1 = scalar_top_bit(s1);
        const G1J a0 = {widen<kPt>(ld_ref(p[i].x)), widen<kPt>(ld_ref(p[i].y)), widen<kPt>(ld_ref(p[i].z))};
        const G1J a1 = {widen<kPt>(ld_ref(p[j1].x)), widen<kPt>(ld_ref(p[j1].y)), widen<kPt>(ld_ref(p[j1].z))};
        z0 = jac_is_zero(a0);
        z1 = jac_is_zero(a1);
#pragma unroll
        for (int w = 0; w < 9; ++w) {
            lds[w][tid] = a0.x.v[w];
            lds[9 + w][tid] = a0.y.v[w];
            lds[18 + w][tid] = a0.z.v[w];
            lds[kMul2Words + w][tid] = a1.x.v[w];
            lds[kMul2Words + 9 + w][tid] = a1.y.v[w];
            lds[kMul2Words + 18 + w][tid] = a1.z.v[w];
        }
#pragma unroll
        for (int w = 0; w < 8; ++w) {
            lds[2 * kMul2Words + w][tid] = s0[w];
            lds[2 * kMul2Words + 8 + w][tid] = s1[w];
        }
    }
    // each thread reads only its own column: no barrier needed
    auto base = [&](int c) {
        G1J b;
        const int o = c * kMul2Words;
#pragma unroll
        for (int w = 0; w < 9; ++w) {
            b.x.v[w] = lds[o + w][tid];
            b.y.v[w] = lds[o + 9 + w][tid];
            b.z.v[w] = lds[o + 18 + w][tid];
        }
        return b;
    };
    auto bit = [&](int c, int pos) { return ((lds[2 * kMul2Words + 8 * c + (pos >> 5)][tid] >> (pos & 31)) & 1u) != 0; };
    G1J r0, r1;
    jac_mul2<Fq>(base, bit, z0, z1, top0, top1, r0, r1, [&](int t) { balance_step(bal, (uint32_t)t); });
    st_ref(out[i].x, r0.x);
    st_ref(out[i].y, r0.y);
    st_ref(out[i].z, r0.z);
    if (has1) {
        st_ref(out[j].x, r1.x);
        st_ref(out[j].y, r1.y);
        st_ref(out[j].z, r1.z);
    }
}
// ---------------------------------------------------------------- group law
// Group::normalize (lib.rs:391-398, 542-549): to_affine (mod.rs:199-216), then
// to_jacobian (mod.rs:220-226: z = one); a zero point stays as it is.  The
// inverse is unique, so (x z^-2, y z^-3, 1) is the reference's image also when z
// is already one (its shortcut returns the same residues).
template <template <int> class F>
__device__ __forceinline__ Jac<F> jac_normalize(const Jac<F>& a) {
    const bool zero = jac_is_zero(a);
    const auto zinv = F_inv(a.z);  // F_inv(0) = 0; that result is discarded
    const auto zinv2 = F_sqr(zinv);
    const Jac<F> r = {narrow<kPt>(F_mul(a.x, zinv2)), narrow<kPt>(F_mul(a.y, F_mul(zinv2, zinv))),
                      F_widen<kPt>(F_one<F>())};
    return {F_select(zero, a.x, r.x), F_select(zero, a.y, r.y), F_select(zero, a.z, r.z)};
}
// PartialEq for G<P> (mod.rs:169-195): both zero, or neither and
// x1 z2^2 == x2 z1^2 and y1 z2^3 == y2 z1^3 (mod p)
template <template <int> class F>
__device__ __forceinline__ bool jac_eq(const Jac<F>& a, const Jac<F>& b) {
    const bool az = jac_is_zero(a), bz = jac_is_zero(b);
    const auto z1sq = F_sqr(a.z);
    const auto z2sq = F_sqr(b.z);
    const bool ex = F_is_zero(F_sub(F_mul(a.x, z2sq), F_mul(b.x, z1sq)));
    const auto z1cu = F_mul(a.z, z1sq);
    const auto z2cu = F_mul(b.z, z2sq);
    const bool ey = F_is_zero(F_sub(F_mul(a.y, z2cu), F_mul(b.y, z1cu)));
    return az ? bz : (!bz && ex && ey);
}
// out[i] = a[i] op b[i] (op: GroupOp, kernels.h; wave-uniform); kGroupEq writes
// eq[i] instead of out[i]
template <template <int> class F>
__device__ __forceinline__ Jac<F> group_apply(int op, const Jac<F>& x, const Jac<F>& y) {
    switch (op) {
        case kGroupAdd: return jac_add(x, y);                // mod.rs:294-334
        case kGroupSub: return jac_add(x, jac_neg(y));     // mod.rs:352-358: self + (-other)
        case kGroupNeg: return jac_neg(x);                 // mod.rs:336-350
        default: return jac_normalize(x);                     // kGroupNormalize
    }
}
__global__ void __launch_bounds__(kBlock) k_g1_op(int op, const bn_g1* a, const bn_g1* b, size_t n, bn_g1* out,
                                                  uint8_t* __restrict__ eq) {
    fold_table_init();
    const size_t i = lane_id();
    if (i >= n) return;
    const G1J x = {widen<kPt>(ld_ref(a[i].x)), widen<kPt>(ld_ref(a[i].y)), widen<kPt>(ld_ref(a[i].z))};
    G1J y = x;
    if (b) y = {widen<kPt>(ld_ref(b[i].x)), widen<kPt>(ld_ref(b[i].y)), widen<kPt>(ld_ref(b[i].z))};
    if (op == kGroupEq) {
        eq[i] = jac_eq(x, y) ? 1 : 0;
        return;
    }
    const G1J r = group_apply(op, x, y);
    st_ref(out[i].x, r.x);
    st_ref(out[i].y, r.y);
    st_ref(out[i].z, r.z);
}
__global__ void __launch_bounds__(kBlock) k_g2_op(int op, const bn_g2* a, const bn_g2* b, size_t n, bn_g2* out,
                                                  uint8_t* __restrict__ eq) {
    fold_table_init();
    const size_t i = lane_id();
    if (i >= n) return;
    const G2J x = {widen<kPt>(ld_ref2(a[i].x)), widen<kPt>(ld_ref2(a[i].y)), widen<kPt>(ld_ref2(a[i].z))};
    G2J y = x;
    if (b) y = {widen<kPt>(ld_ref2(b[i].x)), widen<kPt>(ld_ref2(b[i].y)), widen<kPt>(ld_ref2(b[i].z))};
    if (op == kGroupEq) {
        eq[i] = jac_eq(x, y) ? 1 : 0;
        return;
    }
    const G2J r = group_apply(op, x, y);
    st_ref2(out[i].x, r.x);
    st_ref2(out[i].y, r.y);
    st_ref2(out[i].z, r.z);
}

}  // namespace bn

BN_EXPORT_FOLD_CHECK(group)

#if defined(BN_MUL_STATS) && BN_MUL_STATS
// the G*Fr schedule counters of the diagnostic build (curve.h BN_MUL_STAT), read and cleared
extern "C" int bn_dbg_mul_stats(unsigned long long out[5]) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(bn::g_mul_stats), 5 * sizeof(unsigned long long)) != hipSuccess) return -1;
    const unsigned long long z[5] = {0, 0, 0, 0, 0};
    return hipMemcpyToSymbol(HIP_SYMBOL(bn::g_mul_stats), z, sizeof z) == hipSuccess ? 0 : -1;
}
#endif
