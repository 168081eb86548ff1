// host_emul.cpp -- TEST INFRASTRUCTURE: the engine's device arithmetic headers
// compiled for the host CPU, so tests can check the exact kernel formulas (and
// their static bound bookkeeping) against the oracle without a GPU.  Nothing
// in the product links this.
#include <stdint.h>
#include <string.h>

#include "../../paritytech-bn_amd/csrc/pairing.h"

using namespace bn;

static Fq<2> ld(const uint32_t* w) { return fq_load_ref(w); }
template <int B>
static void st(const Fq<B>& a, uint32_t* w) { fq_store_ref(a, w); }
static Fq2<2> ld2(const uint32_t* w) { return {ld(w), ld(w + 8)}; }
template <int B>
static void st2(const Fq2<B>& a, uint32_t* w) { st(a.c0, w); st(a.c1, w + 8); }
static Fq12<2> ld12(const uint32_t* w) {
    return {{ld2(w), ld2(w + 16), ld2(w + 32)}, {ld2(w + 48), ld2(w + 64), ld2(w + 80)}};
}
template <int B>
static void st12(const Fq12<B>& a, uint32_t* w) {
    st2(a.c0.c0, w); st2(a.c0.c1, w + 16); st2(a.c0.c2, w + 32);
    st2(a.c1.c0, w + 48); st2(a.c1.c1, w + 64); st2(a.c1.c2, w + 80);
}

extern "C" {
void he_fq_mul(const uint32_t* a, const uint32_t* b, uint32_t* o) { st(fq_mul(ld(a), ld(b)), o); }
void he_fq_add(const uint32_t* a, const uint32_t* b, uint32_t* o) { st(fq_add(ld(a), ld(b)), o); }
void he_fq_sub(const uint32_t* a, const uint32_t* b, uint32_t* o) { st(fq_sub(ld(a), ld(b)), o); }
void he_fq_neg(const uint32_t* a, uint32_t* o) { st(fq_neg(ld(a)), o); }
void he_fq_inv(const uint32_t* a, uint32_t* o) { st(fq_inv(ld(a)), o); }
void he_fq_fold(const uint32_t* a, uint32_t* o) {
    // exercise the fold on a large-bound value: a*37 + 90p-ish
    auto x = ld(a);
    auto big = fq_add(fq_mul_small<8>(fq_mul_small<8>(x)), fq_sub(x, widen<20>(x)));
    st(fq_fold(big), o);
}
void he_fq2_mul(const uint32_t* a, const uint32_t* b, uint32_t* o) { st2(fq2_mul(ld2(a), ld2(b)), o); }
void he_fq2_sqr(const uint32_t* a, uint32_t* o) { st2(fq2_sqr(ld2(a)), o); }
void he_fq2_inv(const uint32_t* a, uint32_t* o) { st2(fq2_inv(ld2(a)), o); }
void he_fq12_mul(const uint32_t* a, const uint32_t* b, uint32_t* o) { st12(fq12_mul(ld12(a), ld12(b)), o); }
void he_fq12_sqr(const uint32_t* a, uint32_t* o) { st12(fq12_sqr(ld12(a)), o); }
void he_fq12_inv(const uint32_t* a, uint32_t* o) { st12(fq12_inv(ld12(a)), o); }
void he_fq12_cyc_sqr(const uint32_t* a, uint32_t* o) { st12(fq12_cyclotomic_sqr(ld12(a)), o); }
void he_fq12_exp_by_neg_z(const uint32_t* a, uint32_t* o) { st12(exp_by_neg_z(widen<kF>(ld12(a))), o); }
void he_fq12_frob(const uint32_t* a, int power, uint32_t* o) {
    if (power == 1) st12(fq12_frobenius_map<1>(ld12(a)), o);
    else if (power == 2) st12(fq12_frobenius_map<2>(ld12(a)), o);
    else st12(fq12_frobenius_map<3>(ld12(a)), o);
}
void he_fq12_mul_by_024(const uint32_t* f, const uint32_t* e0, const uint32_t* evw, const uint32_t* evv, uint32_t* o) {
    st12(fq12_mul_by_024(ld12(f), ld2(e0), ld2(evw), ld2(evv)), o);
}
void he_final_exp(const uint32_t* f, uint32_t* o) {
    st12(fe_last_chunk(fe_first_chunk(widen<kF>(ld12(f)))), o);
}
// q affine (x.c0, x.c1, y.c0, y.c1) -> 87 x (ell_0, ell_vw, ell_vv) reference images
void he_g2_precompute(const uint32_t* q, uint32_t* out) {
    G2Aff<2> qa = {ld2(q), ld2(q + 16)};
    g2_precompute(qa, [&](int k, const Ell& e) {
        st2(e.ell_0, out + k * 48);
        st2(e.ell_vw, out + k * 48 + 16);
        st2(e.ell_vv, out + k * 48 + 32);
    });
}
void he_miller_loop(const uint32_t* coeffs, const uint32_t* px, const uint32_t* py, uint32_t* o) {
    Fq<2> x = ld(px), y = ld(py);
    auto f = miller_loop(x, y, [&](int k) {
        Ell e = {widen<kLine>(ld2(coeffs + k * 48)), widen<kLine>(ld2(coeffs + k * 48 + 16)),
                 widen<kLine>(ld2(coeffs + k * 48 + 32))};
        return e;
    });
    st12(f, o);
}
void he_g1_mul(const uint32_t* p, const uint32_t* k_canonical, uint32_t* o) {
    G1J a = {widen<kPt>(ld(p)), widen<kPt>(ld(p + 8)), widen<kPt>(ld(p + 16))};
    G1J r = jac_mul(a, k_canonical);
    st(r.x, o); st(r.y, o + 8); st(r.z, o + 16);
}
void he_g2_mul(const uint32_t* p, const uint32_t* k_canonical, uint32_t* o) {
    G2J a = {widen<kPt>(ld2(p)), widen<kPt>(ld2(p + 16)), widen<kPt>(ld2(p + 32))};
    G2J r = jac_mul(a, k_canonical);
    st2(r.x, o); st2(r.y, o + 16); st2(r.z, o + 32);
}
}
