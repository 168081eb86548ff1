// kernels_pairing.hip -- to_affine + G2 line precomputation (mod.rs:199-216, 701-727) and the
// Miller loop (mod.rs:579-607).  Pairing-path layout (BN_PATH_SPLIT: two lanes
// per pairing, fq2_split.h; `n` counts pairings, the grid has kPathLanes
// threads per pairing).  G1 values (P, its affine form) are held by both lanes.
// fq_fold reads -q*p from an LDS table (fq.h; every kernel here calls
// fold_table_init first): 2-3 % faster on this path, measured
#ifndef BN_FOLD_LDS
#define BN_FOLD_LDS 1
#endif
#include "fq.h"
#define BN_SPLIT BN_PATH_SPLIT
#include "kernels.h"

namespace bn {

constexpr size_t kL = BN_SPLIT ? 2 : 1;  // lanes per pairing in this translation unit

// ---------------------------------------------------------------- pairing kernels
// to_affine of both points of pair i (mod.rs:199-216; the z == 1 shortcut yields
// the same values as the general path).  flags[lane]: 1 = skip (a zero point;
// pairing() returns Fq12::one(), mod.rs:896); mode 1 (miller_loop_batch): a zero
// point sets *err = BN_ERR_TO_AFFINE (lib.rs:629-630).
struct PairAffine {
    Fq<2> px, py;
    G2Aff<kPt> qa;
};
__device__ __forceinline__ PairAffine pair_to_affine(const bn_g1* __restrict__ p, const bn_g2* __restrict__ q, size_t i,
                                                     size_t l, uint8_t* __restrict__ flags, int* __restrict__ err,
                                                     int mode) {
    uint32_t w[8];
    ld_words(&p[i].z, w);
    const bool p_zero = words_zero(w);
    const Fq<2> pz = fq_load_ref(w);
#if BN_SPLIT
    uint32_t wz[8];
    ld_words(lane_odd() ? &q[i].z.c1 : &q[i].z.c0, wz);  // this lane's coordinate of z
    const uint32_t own_zero = words_zero(wz) ? 1u : 0u;
    const bool q_zero = (own_zero & swap_pair(own_zero)) != 0;
    const Fq2<2> qz = {fq_load_ref(wz)};
    const auto qz_sq = fq_sqr(qz.c);
    const auto nq = fq_add(qz_sq, fq_partner(qz_sq));  // N(qz) = z0^2 + z1^2, the same on both lanes
#else
    uint32_t w0[8], w1[8];
    ld_words(&q[i].z.c0, w0);
    ld_words(&q[i].z.c1, w1);
    const bool q_zero = words_zero(w0) && words_zero(w1);
    const Fq2<2> qz = {fq_load_ref(w0), fq_load_ref(w1)};
    const auto nq = fq_add(fq_sqr(qz.c0), fq_sqr(qz.c1));
#endif
    if ((p_zero || q_zero) && mode == 1 && (l % kL) == 0) atomicOr(err, 1 << BN_ERR_TO_AFFINE);
    flags[l] = (p_zero || q_zero) ? 1 : 0;

    // One inversion for both points (Montgomery's trick): t = (pz * N(qz))^-1 with
    // N(qz) = qz.c0^2 + qz.c1^2 (the norm fq2.rs:119-130 inverts), so pz^-1 = t * N(qz)
    // and qz^-1 = conj(qz) * (t * pz).  Inverses are unique: these are the values the
    // reference's two inversions give.  A zero z makes t = 0; that pair is skipped
    // (flags) or rejected (mode 1) and its values are never used.
    const Fq<2> t = fq_inv(fq_mul(pz, nq));
    const auto pzinv = fq_mul(t, nq);
    const auto ninv = fq_mul(t, pz);
    auto pzinv2 = fq_sqr(pzinv);
    PairAffine a;
    a.px = fq_mul(ld_ref(p[i].x), pzinv2);
    a.py = fq_mul(ld_ref(p[i].y), fq_mul(pzinv2, pzinv));
#if BN_SPLIT
    const auto zn = fq_mul(qz.c, ninv);
    const auto qzinv = wrap2(fq_select(lane_odd(), fq_neg(zn), zn));  // conj(qz) * ninv
#else
    const auto qzinv = mk2(fq_mul(qz.c0, ninv), fq_neg(fq_mul(qz.c1, ninv)));
#endif
    auto qzinv2 = fq2_sqr(qzinv);
    a.qa = {narrow<kPt>(fq2_mul(ld_ref2(q[i].x), qzinv2)), narrow<kPt>(fq2_mul(ld_ref2(q[i].y), fq2_mul(qzinv2, qzinv)))};
    return a;
}

// to_affine + the 87 line coefficients (AffineG2::precompute) -> HBM
__global__ void BN_PATH_ATTR __launch_bounds__(kBlock) k_prepare(const bn_g1* __restrict__ p, const bn_g2* __restrict__ q,
                                                                size_t n, uint32_t* __restrict__ coeffs,
                                                                uint32_t* __restrict__ paff, uint8_t* __restrict__ flags,
                                                                int* __restrict__ err, int mode) {
    fold_table_init();
    const size_t l = lane_id(), i = l / kL, nl = kL * n;
    if (i >= n) return;
    const PairAffine a = pair_to_affine(p, q, i, l, flags, err, mode);
    st_fq(paff, nl, l, 0, a.px);
    st_fq(paff, nl, l, 1, a.py);
    g2_precompute(a.qa, [&](int k, const Ell& e) {
        st_fq2(coeffs, nl, l, k * 6 + 0, e.ell_0);
        st_fq2(coeffs, nl, l, k * 6 + 2, e.ell_vw);
        st_fq2(coeffs, nl, l, k * 6 + 4, e.ell_vv);
    });
}

// The coefficients k_prepare wrote for pair i -> the reference images of its
// G2Precomp (mod.rs:566-577): 87 x {ell_0, ell_vw, ell_vv}, each a canonical Fq2
__global__ void BN_PATH_ATTR __launch_bounds__(kBlock) k_coeffs_store(const uint32_t* __restrict__ coeffs, size_t n,
                                                                     bn_fq2* __restrict__ out) {
    fold_table_init();
    const size_t l = lane_id(), i = l / kL, nl = kL * n;
    if (i >= n) return;
#pragma unroll 1
    for (int k = 0; k < BN_NUM_COEFFS; ++k)
#pragma unroll
        for (int j = 0; j < 3; ++j) st_ref2(out[(i * BN_NUM_COEFFS + k) * 3 + j], ld_fq2<kLine>(coeffs, nl, l, k * 6 + 2 * j));
}

// A/B form ("line coefficients"): to_affine, the line steps and the
// Miller loop fused in one kernel -- each coefficient is applied as soon as it is
// computed and never leaves registers (no 16.7 KB/pairing HBM round trip).  Same
// operations in the same order as k_prepare + k_miller, so the same Miller value.
__global__ void BN_PATH_ATTR __launch_bounds__(kBlock) k_pairing_fused(const bn_g1* __restrict__ p,
                                                                      const bn_g2* __restrict__ q, size_t n,
                                                                      uint8_t* __restrict__ flags,
                                                                      int* __restrict__ err, int mode,
                                                                      uint32_t* __restrict__ f_out) {
    fold_table_init();
    const size_t l = lane_id(), i = l / kL, nl = kL * n;
    if (i >= n) return;
    const PairAffine a = pair_to_affine(p, q, i, l, flags, err, mode);
    Fq12<kF> f = miller_fused(a.qa, a.px, a.py);
    if (flags[l]) f = widen<kF>(fq12_one());
    st_fq12(f_out, nl, l, f);
}

__global__ void BN_PATH_ATTR __launch_bounds__(kBlock) k_miller(const uint32_t* __restrict__ coeffs,
                                                               const uint32_t* __restrict__ paff,
                                                               const uint8_t* __restrict__ flags, size_t n,
                                                               uint32_t* __restrict__ f_out) {
    fold_table_init();
    const size_t l = lane_id(), i = l / kL, nl = kL * n;
    if (i >= n) return;
    const Fq<2> px = ld_fq<2>(paff, nl, l, 0);
    const Fq<2> py = ld_fq<2>(paff, nl, l, 1);
    Fq12<kF> f = miller_loop(px, py, [&](int k) {
        return Ell{ld_fq2<kLine>(coeffs, nl, l, k * 6 + 0), ld_fq2<kLine>(coeffs, nl, l, k * 6 + 2),
                   ld_fq2<kLine>(coeffs, nl, l, k * 6 + 4)};
    });
    if (flags[l]) f = widen<kF>(fq12_one());
    st_fq12(f_out, nl, l, f);
}

// Miller loop in segments (pairing_batch / miller_loop_batch with fewer pairs
// than fill the GPU): lane pair (segment s, pair i) -- segment-major, so a wave
// reads consecutive pairs' coefficients -- computes pair i's loop over the
// segment's digits (pairing.h miller_segment) into element s * n + i of `out`
// (split layout, stride S * n).  Segment values of a pair with a zero point are one.
__global__ void BN_PATH_ATTR __launch_bounds__(kBlock) k_miller_seg(const uint32_t* __restrict__ coeffs,
                                                                   const uint32_t* __restrict__ paff,
                                                                   const uint8_t* __restrict__ flags, size_t n,
                                                                   SegPlan plan, uint32_t* __restrict__ out) {
    fold_table_init();
    const size_t l = lane_id(), pr = l / kL, nl = kL * n;
    if (pr >= (size_t)plan.S * n) return;
    const int s = (int)(pr / n);
    const size_t lt = (pr % n) * kL + (l % kL);  // the pair's lane in the per-pair arrays
    const Fq<2> px = ld_fq<2>(paff, nl, lt, 0);
    const Fq<2> py = ld_fq<2>(paff, nl, lt, 1);
    Fq12<kF> f = miller_segment(px, py, plan.lo[s], plan.hi[s], plan.idx[s], [&](int k) {
        return Ell{ld_fq2<kLine>(coeffs, nl, lt, k * 6 + 0), ld_fq2<kLine>(coeffs, nl, lt, k * 6 + 2),
                   ld_fq2<kLine>(coeffs, nl, lt, k * 6 + 4)};
    });
    if (flags[lt]) f = widen<kF>(fq12_one());
    st_fq12(out, kL * plan.S * n, l, f);
}

}  // namespace bn

BN_EXPORT_FOLD_CHECK(pairing)
