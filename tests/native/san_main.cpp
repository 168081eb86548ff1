// san_main.cpp -- sanitizer driver (TEST INFRASTRUCTURE ONLY).
// Built by tests/test_sanitizers.py with -fsanitize=address,undefined together
// with the CPU oracle (oracle/bn_oracle.c) and the host compilation of the
// engine's device headers (tests/native/san_emul.cpp), it cross-checks the two
// on a few inputs of every kind the pairing path handles, so any out-of-bounds
// access, use-after-free or undefined integer
// operation in either shows up as a sanitizer report (non-zero exit).
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "../../oracle/bn_oracle.h"

extern "C" {
void se_fq12_mul(const uint32_t* a, const uint32_t* b, uint32_t* o);
void se_fq12_inv(const uint32_t* a, uint32_t* o);
void se_fq12_cyc_sqr(const uint32_t* a, uint32_t* o);
void se_g2_precompute(const uint32_t* q, uint32_t* out);
void se_miller_loop(const uint32_t* coeffs, const uint32_t* px, const uint32_t* py, uint32_t* o);
int se_fq_from_slice(const uint8_t* be, uint32_t* o);
int se_g1_from_compressed(const uint8_t* b, uint32_t* o);
int se_fq2_sqrt(const uint32_t* a, uint32_t* o);
}

static uint64_t g_state = 0x9e3779b97f4a7c15ull;
static uint64_t next64() {
    uint64_t z = (g_state += 0x9e3779b97f4a7c15ull);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}
static orc_fe rnd_fe() {  // canonical value below p, then its Montgomery image
    orc_fe c, m;
    for (int i = 0; i < 4; ++i) c.l[i] = next64();
    c.l[3] &= 0x2fffffffffffffffull;
    orc_fe_from_canonical(0, &c, &m);
    return m;
}
static orc_fq12 rnd_fq12() {
    orc_fq12 f;
    orc_fe* e = (orc_fe*)&f;
    for (int i = 0; i < 12; ++i) e[i] = rnd_fe();
    return f;
}
static int g_fail = 0;
static void check(const char* what, const void* a, const void* b, size_t n) {
    if (memcmp(a, b, n) != 0) {
        fprintf(stderr, "MISMATCH: %s\n", what);
        g_fail = 1;
    }
}

int main() {
    // tower: product, inverse, cyclotomic squaring
    for (int k = 0; k < 4; ++k) {
        orc_fq12 a = rnd_fq12(), b = rnd_fq12(), want, got;
        orc_fq12_mul(&a, &b, &want);
        se_fq12_mul((const uint32_t*)&a, (const uint32_t*)&b, (uint32_t*)&got);
        check("fq12 mul", &want, &got, sizeof want);
        orc_fq12_inverse(&a, &want);
        se_fq12_inv((const uint32_t*)&a, (uint32_t*)&got);
        check("fq12 inv", &want, &got, sizeof want);
        orc_fq12_cyclotomic_squared(&a, &want);
        se_fq12_cyc_sqr((const uint32_t*)&a, (uint32_t*)&got);
        check("fq12 cyclotomic square", &want, &got, sizeof want);
    }
    // Miller value of (s G1, t G2): oracle vs host-compiled precompute + Miller loop
    orc_g1 g1;
    orc_g2 g2;
    orc_g1_one(&g1);
    orc_g2_one(&g2);
    orc_fe s = rnd_fe(), t = rnd_fe();
    orc_g1 P;
    orc_g2 Q;
    orc_g1_mul(&g1, &s, &P);
    orc_g2_mul(&g2, &t, &Q);
    {
        orc_fq12 want, f;
        orc_g2_affine qa;
        orc_fe px, py;
        orc_g2_to_affine(&Q, &qa);
        orc_g1_to_affine(&P, &px, &py);
        static uint32_t coeffs[ORC_NUM_COEFFS * 48];
        se_g2_precompute((const uint32_t*)&qa, coeffs);
        orc_ell_coeffs oc[ORC_NUM_COEFFS];
        orc_g2_precompute(&qa, oc);
        check("g2 precompute (87 coefficients)", oc, coeffs, sizeof oc);
        se_miller_loop(coeffs, (const uint32_t*)&px, (const uint32_t*)&py, (uint32_t*)&f);
        orc_miller_loop(oc, &px, &py, &want);
        check("Miller loop", &want, &f, sizeof want);
    }
    // threaded oracle helpers (the CPU baselines)
    {
        enum { N = 6 };
        orc_g1 ps[N];
        orc_g2 qs[N];
        for (int i = 0; i < N; ++i) {
            orc_fe a = rnd_fe(), b = rnd_fe();
            orc_g1_mul(&g1, &a, &ps[i]);
            orc_g2_mul(&g2, &b, &qs[i]);
        }
        orc_fq12 many[N], one[N], b1, b3;
        orc_pairing_many(ps, qs, N, many, 3);
        for (int i = 0; i < N; ++i) orc_pairing(&ps[i], &qs[i], &one[i]);
        check("pairing_many (3 threads)", many, one, sizeof many);
        orc_pairing_batch(ps, qs, N, &b1);
        orc_pairing_batch_mt(ps, qs, N, &b3, 3);
        check("pairing_batch_mt (3 threads)", &b1, &b3, sizeof b1);
    }
    // encodings / decompression / square roots at their edges
    {
        uint8_t be[32];
        memset(be, 0xff, sizeof be);
        orc_fe o1;
        uint32_t o2[8];
        const int r1 = orc_fq_from_slice(be, &o1), r2 = se_fq_from_slice(be, o2);
        if ((r1 != 0) != (r2 != 0)) {
            fprintf(stderr, "MISMATCH: Fq::from_slice(2^256-1) status\n");
            g_fail = 1;
        }
        uint8_t rec[33];
        rec[0] = 2;  // compressed G1::one(): x = 1, even y
        memset(rec + 1, 0, 32);
        rec[32] = 1;
        orc_g1 w1;
        uint32_t w2[24];
        const int c1 = orc_g1_from_compressed(rec, sizeof rec, &w1), c2 = se_g1_from_compressed(rec, w2);
        if (c1 != c2) {
            fprintf(stderr, "MISMATCH: G1::from_compressed status %d vs %d\n", c1, c2);
            g_fail = 1;
        } else if (c1 == 0) {
            check("G1::from_compressed", &w1, w2, sizeof w1);
        }
        orc_fq2 x = {rnd_fe(), rnd_fe()}, sq, r;
        orc_fq2_squared(&x, &sq);
        const int q1 = orc_fq2_sqrt(&sq, &r);
        uint32_t r2w[16];
        const int q2 = se_fq2_sqrt((const uint32_t*)&sq, r2w);
        if ((q1 == 0) != (q2 != 0)) {  // oracle: 0 = Some; host emulation: 1 = Some
            fprintf(stderr, "MISMATCH: Fq2::sqrt status\n");
            g_fail = 1;
        } else if (q1 == 0) {
            check("Fq2::sqrt", &r, r2w, sizeof r);
        }
    }
    if (g_fail) return 1;
    printf("san ok\n");
    return 0;
}
