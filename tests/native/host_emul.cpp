// host_emul.cpp -- TEST INFRASTRUCTURE: the engine's device arithmetic headers
// compiled for the host CPU, so tests can check the exact kernel formulas (and
// their static bound bookkeeping) against the oracle without a GPU.  Nothing
// in the product links this.
#include <stdint.h>
#include <string.h>

#include "../../paritytech-bn_amd/csrc/codec.h"
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
// fq_is_zero / fq_eq on multiples of p with lazy digits and on plain values:
// bit k of o[0] = test k (see tests/test_host_emul.py::test_fq_is_zero)
void he_fq_zero_checks(const uint32_t* a, const uint32_t* b, uint32_t* o) {
    auto x = ld(a), y = ld(b);
    auto z1 = fq_sub(x, x);               // (B+1) p with raised digits
    auto z2 = fq_add(z1, fq_sub(y, y));   // a larger multiple of p
    auto z3 = fq_mul_small<4>(z1);        // 4 (B+1) p, lazy digits
    auto z4 = fq_neg(x);                  // B p - x
    uint32_t r = 0;
    r |= (uint32_t)fq_is_zero(z1) << 0;
    r |= (uint32_t)fq_is_zero(z2) << 1;
    r |= (uint32_t)fq_is_zero(z3) << 2;
    r |= (uint32_t)fq_is_zero(x) << 3;
    r |= (uint32_t)fq_is_zero(fq_sub(x, y)) << 4;
    r |= (uint32_t)fq_eq(x, fq_add(x, z3)) << 5;
    r |= (uint32_t)fq_is_zero(fq_add(x, z4)) << 6;
    r |= (uint32_t)fq_eq(x, y) << 7;
    r |= (uint32_t)fq_is_zero(fq_zero()) << 8;
    o[0] = r;
    o[1] = 0;
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
// k_gt_pow's formulas (kernels_gtpow.hip): when x is a nonzero cyclotomic-subgroup
// member (x^(p^4) * x == x^(p^2)), as for a whole wave of such elements on the
// device, signed 5-bit windows (Booth digits -16..16 from bits 5i - 1 .. 5i + 4,
// negative digits by the conjugate) over a table x^0..x^16 with cyclotomic
// squarings; otherwise unsigned 4-bit windows over x^0..x^15 with generic
// squarings.  e = canonical scalar words.  Returns 1 when the cyclotomic chain ran.
int he_gt_pow(const uint32_t* a, const uint32_t* e_in, uint32_t* o) {
    Fq12<kF> tab[17];
    tab[0] = widen<kF>(fq12_one());
    tab[1] = widen<kF>(ld12(a));
    for (int j = 2; j < 17; ++j) tab[j] = mul12(tab[j - 1], tab[1]);
    const Fq12<kF> x2 = narrow12<kF>(fq12_frobenius_map<2>(tab[1]));
    const Fq12<kF> x4x = mul12(narrow12<kF>(fq12_frobenius_map<2>(x2)), tab[1]);
    const bool cyc = fq12_is_zero(fq12_sub(x4x, x2)) && !fq12_is_zero(tab[1]);
    uint32_t e[8];
    memcpy(e, e_in, sizeof e);
    if (cyc) {
        for (int s = 7; s > 0; --s) e[s] = (e[s] << 1) | (e[s - 1] >> 31);
        e[0] <<= 1;
        auto entry = [&](uint32_t f) {
            const uint32_t v = (f >> 1) + (f & 1u);
            const bool neg = (f & 32u) != 0 && v != 32u;
            const uint32_t mag = (f & 32u) ? 32u - v : v;
            return neg ? Fq12<kF>(fq12_conj(tab[mag])) : tab[mag];
        };
        Fq12<kF> acc = entry(e[7] >> 26);
        for (int w = 49; w >= 0; --w) {
            for (int s = 7; s > 0; --s) e[s] = (e[s] << 5) | (e[s - 1] >> 27);
            e[0] <<= 5;
            for (int s = 0; s < 5; ++s) acc = cyc_sqr(acc);
            acc = mul12(acc, entry(e[7] >> 26));
        }
        st12(acc, o);
        return 1;
    }
    Fq12<kF> acc = tab[e[7] >> 28];
    for (int w = 62; w >= 0; --w) {
        for (int s = 7; s > 0; --s) e[s] = (e[s] << 4) | (e[s - 1] >> 28);
        e[0] <<= 4;
        for (int s = 0; s < 4; ++s) acc = narrow12<kF>(fq12_sqr(acc));
        acc = mul12(acc, tab[e[7] >> 28]);
    }
    st12(acc, o);
    return 0;
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
// ---- codec.h (encodings, sqrt, validation, decompression)
int he_fq_from_slice(const uint8_t* be, uint32_t* o) {
    uint32_t w[8];
    words_from_be<8>(be, w);
    Fq<2> x;
    bool ok = fq_new_plain(w, x);
    st(x, o);
    return ok ? ST_OK : ST_FIELD_NOT_MEMBER;
}
void he_fq_to_be(const uint32_t* a, uint8_t* be) {
    uint32_t w[8];
    fq_plain_words(ld(a), w);
    be_from_words<8>(w, be);
}
int he_fq2_from_slice(const uint8_t* be, uint32_t* o) {
    uint32_t v[16];
    words_from_be<16>(be, v);
    Fq2<2> x;
    bool ok = fq2_from_u512(v, x);
    st2(x, o);
    return ok ? ST_OK : ST_FIELD_NOT_MEMBER;
}
void he_fr_from_slice(const uint8_t* be, uint32_t* o) {
    uint32_t w[8];
    words_from_be<8>(be, w);
    fr_from_plain_words(w, o);
}
int he_fq_sqrt(const uint32_t* a, uint32_t* o) {
    Fq<2> r;
    bool some = fq_sqrt(ld(a), r);
    st(r, o);
    return some;
}
int he_fq2_sqrt(const uint32_t* a, uint32_t* o) {
    Fq2<kPt> r;
    bool some = fq2_sqrt(ld2(a), r);
    st2(r, o);
    return some;
}
int he_g2_affine_new(const uint32_t* xy, uint32_t* o) {
    Fq2<kPt> x = widen<kPt>(ld2(xy)), y = widen<kPt>(ld2(xy + 16));
    if (!g2_on_curve(x, y)) return ST_GROUP_NOT_ON_CURVE;
    if (!g2_in_subgroup(x, y)) return ST_GROUP_NOT_IN_SUBGROUP;
    st2(x, o); st2(y, o + 16); st2(fq2_one(), o + 32);
    return ST_OK;
}
int he_g1_from_compressed(const uint8_t* b, uint32_t* o) {
    Fq<2> x, y;
    uint8_t s = g1_decompress(b, x, y);
    if (s == ST_OK) { st(x, o); st(y, o + 8); st(fq_one(), o + 16); }
    return s;
}
int he_g2_from_compressed(const uint8_t* b, uint32_t* o) {
    Fq2<kPt> x, y;
    uint8_t s = g2_decompress(b, x, y);
    if (s == ST_OK) { st2(x, o); st2(y, o + 16); st2(fq2_one(), o + 32); }
    return s;
}
}
