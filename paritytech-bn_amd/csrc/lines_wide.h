// lines_wide.h -- the per-pair pieces shared by the line-producing kernels
// (kernels_pairing.hip: k_prepare, k_prepare_wide, k_pairing_fused, and
// kernels_wide.hip: k_pairing_latency): to_affine of a pair and the G2 line
// steps on eight lanes per pair.  Included inside namespace bn after kernels.h,
// by translation units with BN_SPLIT = 1.
#pragma once
#include <type_traits>

namespace bn {

constexpr size_t kL = BN_SPLIT ? 2 : 1;  // lanes per pairing in the including translation unit

// ---------------------------------------------------------------- pairing kernels
// to_affine of both points of pair i (mod.rs:199-216; the z == 1 shortcut yields
// the same values as the general path).  flags[lane]: 1 = skip (a zero point;
// pairing() returns Fq12::one(), mod.rs:896); mode 1 (miller_loop_batch): a zero
// point sets *err = BN_ERR_TO_AFFINE (lib.rs:629-630).  flags may be null.
struct PairAffine {
    Fq<2> px, py;
    G2Aff<kPt> qa;
    bool skip;  // a zero point: pairing() of the pair is Fq12::one()
};
// Quad: the four lanes of every quad work on the same pair (the eight-lane layouts):
// the inversion splits its updates over them (tower.h fq_inv_quad)
template <bool Quad = false>
__device__ __forceinline__ PairAffine pair_to_affine(const bn_g1* __restrict__ p, const bn_g2* __restrict__ q, size_t i,
                                                     size_t l, uint8_t* __restrict__ flags, int* __restrict__ err,
                                                     int mode) {
    uint32_t w[8];
    ld_words(&p[i].z, w);
    const bool p_zero = words_zero(w);
    const bool p_one = words_one(w);
    const Fq<2> pz = fq_load_ref(w);
#if BN_SPLIT
    uint32_t wz[8];
    ld_words(lane_odd() ? &q[i].z.c1 : &q[i].z.c0, wz);  // this lane's coordinate of z
    const uint32_t own_zero = words_zero(wz) ? 1u : 0u;
    const bool q_zero = (own_zero & swap_pair(own_zero)) != 0;
    const uint32_t own_one = (lane_odd() ? words_zero(wz) : words_one(wz)) ? 1u : 0u;  // z = one + 0 u
    const bool q_one = (own_one & swap_pair(own_one)) != 0;
    const Fq2<2> qz = {fq_load_ref(wz)};
    const auto qz_sq = fq_sqr(qz.c);
    const auto nq = fq_add(qz_sq, fq_partner(qz_sq));  // N(qz) = z0^2 + z1^2, the same on both lanes
#else
    uint32_t w0[8], w1[8];
    ld_words(&q[i].z.c0, w0);
    ld_words(&q[i].z.c1, w1);
    const bool q_zero = words_zero(w0) && words_zero(w1);
    const bool q_one = words_one(w0) && words_zero(w1);
    const Fq2<2> qz = {fq_load_ref(w0), fq_load_ref(w1)};
    const auto nq = fq_add(fq_sqr(qz.c0), fq_sqr(qz.c1));
#endif
    if ((p_zero || q_zero) && mode == 1 && (l % kL) == 0) err_or(err, BN_ERR_TO_AFFINE);
    if (flags) flags[l] = (p_zero || q_zero) ? 1 : 0;

    // One inversion for both points (Montgomery's trick): t = (pz * N(qz))^-1 with
    // N(qz) = qz.c0^2 + qz.c1^2 (the norm fq2.rs:119-130 inverts), so pz^-1 = t * N(qz)
    // and qz^-1 = conj(qz) * (t * pz).  Inverses are unique: these are the values the
    // reference's two inversions give.  A zero z makes t = 0; that pair is skipped
    // (flags) or rejected (mode 1) and its values are never used.
    // The reference's z == one branch (mod.rs:199-216: the affine point is (x, y) itself):
    // when every pair of the wave has both z == one (points that came in affine, e.g.
    // through AffineG1::new / AffineG2::new), t = (1 * 1)^-1 = 1 needs no inversion --
    // the binary GCD is ~25 k VALU per wave, ~17 % of k_prepare_wide.  The products
    // below then multiply by one: the same values.
    Fq<2> t;
    if (BN_ALL(p_one && q_one))  // wave-uniform
        t = widen<2>(fq_one());
    else
        t = fq_inv<Quad>(fq_mul(pz, nq));
    const auto pzinv = fq_mul(t, nq);
    const auto ninv = fq_mul(t, pz);
    auto pzinv2 = fq_sqr(pzinv);
    PairAffine a;
    a.skip = p_zero || q_zero;
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

#if BN_SPLIT
// ---------------------------------------------------------------- k_prepare_wide
// The same to_affine + 87 line coefficients for small batches, on EIGHT lanes
// per pair: four lane pairs ("slots") run each line step's independent Fq2
// products side by side -- the doubling step's ten products in three layers,
// the mixed addition's fourteen in four -- and exchange the results over
// ds_bpermute; the sums, halvings and narrowings between layers run on every
// slot alike.  A lone pair's 87 dependent steps are the latency of k_prepare
// (DESIGN.md §5); here each step issues about a third of the instructions per
// lane.  Same formulas (fq2_mul(x, x) for the squares: the same residues), so the
// coefficients are the same values; slot 0 stores them, in k_prepare's layout.
constexpr int kPW = kPrepareWideLanes;  // lanes per pair (kernels.h)
__device__ __forceinline__ int pw_slot() { return (int)((__lane_id() >> 1) & 3u); }
// this lane's coordinate of x as computed by slot j of its group
template <int B>
__device__ __forceinline__ Fq2<B> pw_from(const Fq2<B>& x, int j) {
    const int src = (int)((__lane_id() & ~7u) | ((unsigned)j << 1) | (__lane_id() & 1u));
    Fq2<B> r;
#pragma unroll
    for (int d = 0; d < 9; ++d) r.c.v[d] = (uint32_t)__shfl((int)x.c.v[d], src);
    return r;
}
// slot k's operand as a tree on the bits of k: where the four are two pairs of the
// same value (a0 == a2, a1 == a3) the compiler merges the outer select away
template <int B>
__device__ __forceinline__ Fq2<B> pw_pick(int k, const Fq2<B>& a0, const Fq2<B>& a1, const Fq2<B>& a2,
                                          const Fq2<B>& a3) {
    const bool b0 = (k & 1) != 0, b1 = (k & 2) != 0;
    return fq2_select(b1, fq2_select(b0, a3, a2), fq2_select(b0, a1, a0));
}
template <class T>
struct Fq2K;
template <int B>
struct Fq2K<Fq2<B>> {
    static constexpr int K = B;
};
// one layer: slot k computes x_k * y_k (each operand folded to bound <= 40 as
// fq2_mul would, then all joined to one static bound so the slots run one stream)
template <class X0, class Y0, class X1, class Y1, class X2, class Y2, class X3, class Y3>
__device__ __forceinline__ auto pw_mul(int k, const X0& x0_in, const Y0& y0_in, const X1& x1_in, const Y1& y1_in,
                                       const X2& x2_in, const Y2& y2_in, const X3& x3_in, const Y3& y3_in) {
    const auto x0 = pre<40>(x0_in);
    const auto y0 = pre<40>(y0_in);
    const auto x1 = pre<40>(x1_in);
    const auto y1 = pre<40>(y1_in);
    const auto x2 = pre<40>(x2_in);
    const auto y2 = pre<40>(y2_in);
    const auto x3 = pre<40>(x3_in);
    const auto y3 = pre<40>(y3_in);
    constexpr int JX = kjoin(kjoin(Fq2K<std::decay_t<decltype(x0)>>::K, Fq2K<std::decay_t<decltype(x1)>>::K),
                             kjoin(Fq2K<std::decay_t<decltype(x2)>>::K, Fq2K<std::decay_t<decltype(x3)>>::K));
    constexpr int JY = kjoin(kjoin(Fq2K<std::decay_t<decltype(y0)>>::K, Fq2K<std::decay_t<decltype(y1)>>::K),
                             kjoin(Fq2K<std::decay_t<decltype(y2)>>::K, Fq2K<std::decay_t<decltype(y3)>>::K));
    return fq2_mul(pw_pick(k, widen<JX>(x0), widen<JX>(x1), widen<JX>(x2), widen<JX>(x3)),
                   pw_pick(k, widen<JY>(y0), widen<JY>(y1), widen<JY>(y2), widen<JY>(y3)));
}
// doubling_step (curve.h) in three layers
__device__ __forceinline__ Ell pw_doubling_step(G2Proj& s, int k) {
    const auto l1 = pw_mul(k, s.x, s.y, s.y, s.y, s.z, s.z, s.x, s.x);  // x*y, y^2, z^2, x^2
    const auto a = fq2_half(pw_from(l1, 0));
    const auto b = pw_from(l1, 1);
    const auto c = pw_from(l1, 2);
    const auto j = pw_from(l1, 3);
    const auto d = fq2_add(fq2_add(c, c), c);
    const auto yz = fq2_add(s.y, s.z);
    const auto bc = g2_coeff_b();
    const auto l2 = pw_mul(k, bc, d, yz, yz, bc, d, yz, yz);  // e = b' * 3c, (y + z)^2
    const auto e = pw_from(l2, 0);
    const auto h = fq2_sub(pw_from(l2, 1), fq2_add(b, c));
    const auto f = fq2_add(fq2_add(e, e), e);
    const auto g = fq2_half(fq2_add(b, f));
    const auto i = fq2_sub(e, b);
    const auto l3 = pw_mul(k, a, fq2_sub(b, f), g, g, e, e, b, h);  // x', g^2, e^2, z'
    const auto e_sq = pw_from(l3, 2);
    s.x = narrow<kPt>(pw_from(l3, 0));
    s.y = narrow<kPt>(fq2_sub(pw_from(l3, 1), fq2_add(fq2_add(e_sq, e_sq), e_sq)));
    s.z = narrow<kPt>(pw_from(l3, 3));
    return {narrow<kLine>(fq2_mul_xi(i)), narrow<kLine>(fq2_neg(h)), narrow<kLine>(fq2_add(fq2_add(j, j), j))};
}
// mixed_addition_step (curve.h) in four layers
template <int BB>
__device__ __forceinline__ Ell pw_mixed_addition_step(G2Proj& s, const G2Aff<BB>& base, int k) {
    const auto l1 = pw_mul(k, s.z, base.x, s.z, base.y, s.z, base.x, s.z, base.y);  // z*bx, z*by
    const auto d = fq2_sub(s.x, pw_from(l1, 0));
    const auto e = fq2_sub(s.y, pw_from(l1, 1));
    const auto l2 = pw_mul(k, d, d, e, e, e, base.x, d, base.y);  // f = d^2, g = e^2, e*bx, d*by
    const auto f = pw_from(l2, 0);
    const auto g = pw_from(l2, 1);
    const auto l0 = fq2_mul_xi(fq2_sub(pw_from(l2, 2), pw_from(l2, 3)));
    const auto l3 = pw_mul(k, d, f, s.x, f, s.z, g, s.z, g);  // h = d*f, i = x*f, z*g
    const auto h = pw_from(l3, 0);
    const auto i = pw_from(l3, 1);
    const auto jj = fq2_sub(fq2_add(pw_from(l3, 2), h), fq2_add(i, i));
    const auto l4 = pw_mul(k, d, jj, e, fq2_sub(i, jj), h, s.y, s.z, h);  // nx, e*(i - j), h*y, nz
    s.x = narrow<kPt>(pw_from(l4, 0));
    s.y = narrow<kPt>(fq2_sub(pw_from(l4, 1), pw_from(l4, 2)));
    s.z = narrow<kPt>(pw_from(l4, 3));
    return {narrow<kLine>(l0), narrow<kLine>(d), narrow<kLine>(fq2_neg(e))};
}

// ---------------------------------------------------------------- P-scaled lines from the free slots
// The Miller loop multiplies by ell_0 + (ell_vw Py) w^3 + (ell_vv Px) w^4 (mod.rs:589).
// The doubling step's middle layer above runs two distinct products on four slots and
// the addition's first and third layers three, so the two P products fit into slots
// that were duplicates: the scaled coefficients cost the producer no extra layer, and
// the consumer (k_miller_seg, k_miller, the latency kernel's groups) no longer scales
// each line (two Fq products of its ~4,700 VALU per line).  Slot 2 ends up holding
// ell_vw * Py and slot 3 ell_vv * Px (each in its own lanes: stored from there, no
// exchange); every slot holds ell_0 and the reference's unscaled ell_vw, ell_vv (the
// G2Precomp export).  P products take P as the Fq2 (P, 0).
struct PwEll {
    Ell e;                       // the reference's coefficients
    Fq2<kLine> vw_py, vv_px;     // ell_vw * Py on slot 2's lanes, ell_vv * Px on slot 3's
};
// (x, 0): this lane's coordinate of an Fq as an Fq2 (the c1 lane holds zero)
template <int B>
__device__ __forceinline__ Fq2<B> pw_real(const Fq<B>& x) {
    return {fq_select(lane_odd(), widen<B>(fq_zero()), x)};
}
// doubling_step (curve.h) in three layers with the P products: h = (y + z)^2 - y^2 - z^2
// = 2 y z (the same field value), so y z joins layer 1 and x^2 moves to layer 2.
// L1: x y, y^2, z^2, y z;  L2: e = b' * 3c, j = x^2, y z * Py, z' = y^2 * h;
// L3: x' = a (b - f), g^2, e^2, j * 3Px
template <int PY, int PX>
__device__ __forceinline__ PwEll pw_doubling_step_p(G2Proj& s, int k, const Fq2<PY>& py_r, const Fq2<PX>& px3_r) {
    const auto l1 = pw_mul(k, s.x, s.y, s.y, s.y, s.z, s.z, s.y, s.z);  // x*y, y^2, z^2, y*z
    const auto a = fq2_half(pw_from(l1, 0));
    const auto b = pw_from(l1, 1);
    const auto c = pw_from(l1, 2);
    const auto yz = pw_from(l1, 3);
    const auto h = fq2_add(yz, yz);
    const auto d = fq2_add(fq2_add(c, c), c);
    const auto bc = g2_coeff_b();
    const auto l2 = pw_mul(k, bc, d, s.x, s.x, yz, py_r, b, h);  // e, j = x^2, yz * Py, z' = b * h
    const auto e = pw_from(l2, 0);
    const auto j = pw_from(l2, 1);
    const auto zn = pw_from(l2, 3);
    const auto f = fq2_add(fq2_add(e, e), e);
    const auto g = fq2_half(fq2_add(b, f));
    const auto i = fq2_sub(e, b);
    const auto l3 = pw_mul(k, a, fq2_sub(b, f), g, g, e, e, j, px3_r);  // x', g^2, e^2, j * 3Px
    const auto e_sq = pw_from(l3, 2);
    s.x = narrow<kPt>(pw_from(l3, 0));
    s.y = narrow<kPt>(fq2_sub(pw_from(l3, 1), fq2_add(fq2_add(e_sq, e_sq), e_sq)));
    s.z = narrow<kPt>(zn);
    const auto& yzpy = l2;  // slot 2: y z Py
    PwEll r;
    r.e = {narrow<kLine>(fq2_mul_xi(i)), narrow<kLine>(fq2_neg(h)), narrow<kLine>(fq2_add(fq2_add(j, j), j))};
    r.vw_py = narrow<kLine>(fq2_neg(fq2_add(yzpy, yzpy)));  // -h Py
    r.vv_px = narrow<kLine>(l3);                             // slot 3: 3 j Px
    return r;
}
// mixed_addition_step (curve.h) in four layers with the P products:
// L1: z bx, z by, x Py, z (bx Py)  (d Py = x Py - z bx Py);  L2: d^2, e^2, e bx, d by;
// L3: d f, x f, z g, e Px;  L4: as pw_mixed_addition_step.  bxpy = base.x * Py (per base)
template <int BB, int XB, int PY, int PX>
__device__ __forceinline__ PwEll pw_mixed_addition_step_p(G2Proj& s, const G2Aff<BB>& base, const Fq2<XB>& bxpy,
                                                          int k, const Fq2<PY>& py_r, const Fq2<PX>& px_r) {
    const auto l1 = pw_mul(k, s.z, base.x, s.z, base.y, s.x, py_r, s.z, bxpy);  // z*bx, z*by, x*Py, z*bxPy
    const auto d = fq2_sub(s.x, pw_from(l1, 0));
    const auto e = fq2_sub(s.y, pw_from(l1, 1));
    const auto zbxpy = pw_from(l1, 3);
    const auto l2 = pw_mul(k, d, d, e, e, e, base.x, d, base.y);  // f = d^2, g = e^2, e*bx, d*by
    const auto f = pw_from(l2, 0);
    const auto g = pw_from(l2, 1);
    const auto l0 = fq2_mul_xi(fq2_sub(pw_from(l2, 2), pw_from(l2, 3)));
    const auto l3 = pw_mul(k, d, f, s.x, f, s.z, g, e, px_r);  // h = d*f, i = x*f, z*g, e*Px
    const auto h = pw_from(l3, 0);
    const auto i = pw_from(l3, 1);
    const auto jj = fq2_sub(fq2_add(pw_from(l3, 2), h), fq2_add(i, i));
    const auto l4 = pw_mul(k, d, jj, e, fq2_sub(i, jj), h, s.y, s.z, h);  // nx, e*(i - j), h*y, nz
    s.x = narrow<kPt>(pw_from(l4, 0));
    s.y = narrow<kPt>(fq2_sub(pw_from(l4, 1), pw_from(l4, 2)));
    s.z = narrow<kPt>(pw_from(l4, 3));
    PwEll r;
    r.e = {narrow<kLine>(l0), narrow<kLine>(d), narrow<kLine>(fq2_neg(e))};
    r.vw_py = narrow<kLine>(fq2_sub(l1, zbxpy));  // slot 2: x Py - z bx Py = d Py
    r.vv_px = narrow<kLine>(fq2_neg(l3));         // slot 3: -e Px
    return r;
}


#endif  // BN_SPLIT

}  // namespace bn
