// san_emul.cpp -- TEST INFRASTRUCTURE: the subset of the engine's device
// arithmetic (host compilation of the csrc headers) that tests/native/san_main.cpp
// runs under AddressSanitizer + UndefinedBehaviorSanitizer.  The whole of
// host_emul.cpp does not fit a sanitizer build (the final exponentiation and
// Gt::pow inline into functions the instrumented compile takes > 15 min on), so
// this unit keeps the building blocks they are made of: the Fq12 product,
// inverse and cyclotomic square, the sparse line product, the 87-line G2
// precomputation and Miller loop, and the codec's decoding and square roots.
#include <stdint.h>

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
void se_fq12_mul(const uint32_t* a, const uint32_t* b, uint32_t* o) { st12(fq12_mul(ld12(a), ld12(b)), o); }
void se_fq12_inv(const uint32_t* a, uint32_t* o) { st12(fq12_inv(ld12(a)), o); }
void se_fq12_cyc_sqr(const uint32_t* a, uint32_t* o) { st12(fq12_cyclotomic_sqr(ld12(a)), o); }
// q affine (x.c0, x.c1, y.c0, y.c1) -> 87 x (ell_0, ell_vw, ell_vv) reference images
void se_g2_precompute(const uint32_t* q, uint32_t* out) {
    G2Aff<2> qa = {ld2(q), ld2(q + 16)};
    g2_precompute(qa, [&](int k, const Ell& e) {
        st2(e.ell_0, out + k * 48);
        st2(e.ell_vw, out + k * 48 + 16);
        st2(e.ell_vv, out + k * 48 + 32);
    });
}
void se_miller_loop(const uint32_t* coeffs, const uint32_t* px, const uint32_t* py, uint32_t* o) {
    Fq<2> x = ld(px), y = ld(py);
    auto f = miller_loop(x, y, [&](int k) {
        return Ell{widen<kLine>(ld2(coeffs + k * 48)), widen<kLine>(ld2(coeffs + k * 48 + 16)),
                   widen<kLine>(ld2(coeffs + k * 48 + 32))};
    });
    st12(f, o);
}
int se_fq_from_slice(const uint8_t* be, uint32_t* o) {
    uint32_t w[8];
    words_from_be<8>(be, w);
    Fq<2> x;
    bool ok = fq_new_plain(w, x);
    st(x, o);
    return ok ? ST_OK : ST_FIELD_NOT_MEMBER;
}
int se_g1_from_compressed(const uint8_t* b, uint32_t* o) {
    Fq<2> x, y;
    uint8_t s = g1_decompress(b, x, y);
    if (s == ST_OK) { st(x, o); st(y, o + 8); st(fq_one(), o + 16); }
    return s;
}
int se_fq2_sqrt(const uint32_t* a, uint32_t* o) {
    Fq2<kPt> r;
    bool some = fq2_sqrt(ld2(a), r);
    st2(r, o);
    return some;
}
}
