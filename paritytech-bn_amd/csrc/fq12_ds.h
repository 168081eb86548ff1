// fq12_ds.h -- digit-sliced Fq12: ONE element spread over a 256-thread block,
// one 26-bit digit (or product column) per lane, for the latency-bound chain of
// a single final exponentiation (pairing_batch's tail, kernels_tail.hip).
//
// Why: on the 16-lane layout (fq12_wide.h) each lane owns a whole Fq coordinate,
// so a cyclotomic squaring is ~780 instructions of one lane's stream (251
// v_mad_u64_u32, the rest carries, folds, selects): ~2 us on a lone wave, and the
// final exponentiation is ~190 of them in a row.  A lone wave issues about one
// instruction per 5-9.5 cycles whatever the dependences
// (profiles/r3j_mad_issue.txt), so the chain's length is its instruction count.
// Here coordinate cid (= 2e + c, as the w12 lane l) is a 21-lane SLOT (three per
// wave, four waves: one per SIMD -- six waves of two 32-lane slots put two waves on
// two SIMDs and ran no faster than the 16-lane squaring, tools/ds_check) and each
// lane holds one digit: a product's column j is lane j's ten-term MAD chain, the
// Montgomery reduction is column-parallel (m = T * p' mod R as a truncated
// product, then T + m p, the exact low-part quotient from three lanes), carries
// move one lane up per DPP wave_shr:1, and additions are one instruction per lane.
// A squaring is ~40 MAD and ~200 other instructions per lane, two barriers.
//
// Representation: 26-bit digits, ten per value, Montgomery R = 2^260 (the
// 16-lane layout's values x * 2^261 are halved on the way in and doubled on the
// way out).  Digit k of a value sits at lane 10 + k (kDsB); lane 19 (kDsTop) is a
// signed sink that takes every carry out of the lanes below it.  Stored values
// (the operands of products) are "folded": digits 0..8 in [0, 2^26 + 2], the top
// digit in [0, 2^23), value in [0, 5p).  Product outputs are signed digits; the
// linear parts of the Granger-Scott squaring run on signed 64-bit digits and one
// fold per output brings them back (top-digit quotient estimate, subtract q p, a
// spread multiple of p for non-negative digits).  Every bound below was checked
// lane by lane, with random and maximal-digit inputs, by tools/ds_model.py, which
// is this file's algorithm in Python.
//
// Bit-exactness: every operation computes the field value of the reference
// operation it replaces (fq12.rs:198-247 Granger-Scott squaring, 319-327 product,
// 112-128 Frobenius and conjugation); images are canonicalized at the boundary.
#pragma once
#include "fq12_wide.h"

namespace bn {

constexpr int kDsThreads = 256;                  // 4 waves of 3 slots of 21 lanes
constexpr int kDsDig = 26;
constexpr uint32_t kDsM = (1u << kDsDig) - 1;
constexpr int kDsB = 10;                         // lane of digit 0
constexpr int kDsTop = kDsB + 9;                 // lane of digit 9: the sink
// p, p' = -p^-1 mod 2^260, 3p and 8p with digits 0..8 raised by 2^26 (the next
// digit pays), all in 26-bit digits (tools/ds_model.py)
constexpr uint32_t kDsP[10] = {0x07cfd47u, 0x02305b6u, 0x0a8d3c2u, 0x245a1c7u, 0x197816au,
                               0x0605617u, 0x1045b68u, 0x280a6e1u, 0x272e131u, 0x00c1913u};
constexpr uint32_t kDsPinv[10] = {0x0866389u, 0x081e0b9u, 0x2ac987du, 0x1947b29u, 0x09ede7du,
                                  0x20cf6a0u, 0x2fcbd01u, 0x231af62u, 0x2b79188u, 0x3fd5e88u};
constexpr uint32_t kDsS3[10] = {0x0576f7d5u, 0x04691121u, 0x05fa7b45u, 0x06d0e554u, 0x04c6843eu,
                                0x05210245u, 0x070d1237u, 0x0781f4a2u, 0x0758a393u, 0x00244b39u};
constexpr uint32_t kDsS8[10] = {0x07e7ea38u, 0x05182dafu, 0x05469e0fu, 0x062d0e38u, 0x04bc0b53u,
                                0x0702b0bau, 0x0422db3fu, 0x04053709u, 0x0797098cu, 0x0060c89bu};
// 8p with digits 0..8 raised by 2^27 (the next digit pays 2): K p - b for a folded b
constexpr uint32_t kDsS8b[10] = {0x0be7ea38u, 0x09182daeu, 0x09469e0eu, 0x0a2d0e37u, 0x08bc0b52u,
                                 0x0b02b0b9u, 0x0822db3eu, 0x08053708u, 0x0b97098bu, 0x0060c89au};
// the Granger-Scott output of slot cid as products of the squaring's slots:
// y = A PR[i1] + B PR[i2] + C PR[i3] + E a (fq12_wide.h w12_cyc's table with xi P
// written out: xi (P0, P1) = (9 P0 - P1, 9 P1 + P0))
struct DsComb {
    int8_t i1, a, i2, b, i3, c, e, pad;
};
constexpr DsComb kDsComb[12] = {
    {6, 3, 0, -30, 1, 3, -2, 0}, {7, 3, 1, -30, 0, -3, -2, 0},  // w^0: 3 (Q0 - P0 - xi P0) - 2a
    {4, 54, 5, -6, 0, 0, 2, 0},  {5, 54, 4, 6, 0, 0, 2, 0},     // w^1: 6 xi P2 + 2a
    {8, 3, 2, -30, 3, 3, -2, 0}, {9, 3, 3, -30, 2, -3, -2, 0},  // w^2: 3 (Q1 - P1 - xi P1) - 2a
    {0, 6, 0, 0, 0, 0, 2, 0},    {1, 6, 0, 0, 0, 0, 2, 0},      // w^3: 6 P0 + 2a
    {10, 3, 4, -30, 5, 3, -2, 0}, {11, 3, 5, -30, 4, -3, -2, 0}, // w^4: 3 (Q2 - P2 - xi P2) - 2a
    {2, 6, 0, 0, 0, 0, 2, 0},    {3, 6, 0, 0, 0, 0, 2, 0},      // w^5: 6 P1 + 2a
};
// floor(x_top * 2^234 / p) estimate factor, rounded 2^-18 low so q never overshoots
// on a non-negative value (fq_fold's rule)
constexpr float kDsFoldC = 0x1.52917cp-20f;
// gamma_(K,e).c = fq6 frobenius_coeffs_c(e/2)(K) * fq12 frobenius_coeffs_c1(K)^(e%2)
// (fq6.rs:8-87, fq12.rs:9-45), K = 1..3, e = 0..5, c = 0..1, as x * 2^260 mod p
constexpr uint32_t kDsFrob[3 * 12][10] = {
    {0x2fce4b4u, 0x082203du, 0x09a8455u, 0x126eaa6u, 0x2498908u, 0x063c052u, 0x29201d8u, 0x1c93e16u, 0x24e1bb7u, 0x007c590u},
    {0x0000000u, 0x0000000u, 0x0000000u, 0x0000000u, 0x0000000u, 0x0000000u, 0x0000000u, 0x0000000u, 0x0000000u, 0x0000000u},
    {0x1449070u, 0x29a58ccu, 0x38aaf9bu, 0x0e1ebedu, 0x0a6b1d7u, 0x228821fu, 0x1ed5ef0u, 0x29f046fu, 0x351a1f3u, 0x00bcd35u},
    {0x221e4bdu, 0x20970a2u, 0x20f7f58u, 0x1b96e94u, 0x10b6915u, 0x19d7626u, 0x2ddd94bu, 0x0d134a5u, 0x12cd2a1u, 0x0061ffau},
    {0x252c8c8u, 0x3d41364u, 0x30e1766u, 0x3fd5c5fu, 0x28bedc7u, 0x1b57589u, 0x04e4be3u, 0x135e776u, 0x1ea0e94u, 0x0049256u},
    {0x0c8961cu, 0x0d835f9u, 0x157816cu, 0x01ee8ceu, 0x387b6b8u, 0x2ff1fd1u, 0x2df8519u, 0x0e91b2au, 0x25259dbu, 0x0087853u},
    {0x18f833cu, 0x1cfec1bu, 0x2e1f7a3u, 0x174b798u, 0x098fe17u, 0x10d4482u, 0x19d6e18u, 0x02f79dbu, 0x287c1bcu, 0x003a8d7u},
    {0x111a28eu, 0x009418au, 0x0a00d3bu, 0x08f30d0u, 0x231ebfdu, 0x0b6bc64u, 0x080280au, 0x0a9faf4u, 0x1e00d39u, 0x008bd6du},
    {0x040fc2fu, 0x268d616u, 0x15da913u, 0x0e26092u, 0x33728d3u, 0x25633c2u, 0x100b172u, 0x37696fcu, 0x0b791a1u, 0x002ceeau},
    {0x3b0b53cu, 0x25010a5u, 0x37670c5u, 0x2257bc0u, 0x312a19bu, 0x17341ccu, 0x052c12bu, 0x2377b60u, 0x07088cbu, 0x000df3fu},
    {0x3a30ec6u, 0x0d29ac0u, 0x316d2e4u, 0x2a80fa7u, 0x096fac2u, 0x0cf6317u, 0x0cc4713u, 0x30c6368u, 0x01f63deu, 0x002147eu},
    {0x3992367u, 0x3673756u, 0x272a4e9u, 0x0165147u, 0x070fe03u, 0x37f3875u, 0x162b070u, 0x30cedb9u, 0x2982b40u, 0x0070f88u},
    {0x2fce4b4u, 0x082203du, 0x09a8455u, 0x126eaa6u, 0x2498908u, 0x063c052u, 0x29201d8u, 0x1c93e16u, 0x24e1bb7u, 0x007c590u},
    {0x0000000u, 0x0000000u, 0x0000000u, 0x0000000u, 0x0000000u, 0x0000000u, 0x0000000u, 0x0000000u, 0x0000000u, 0x0000000u},
    {0x324c1d9u, 0x1dd0e4du, 0x2c0f6cbu, 0x2d48b1eu, 0x174dbf6u, 0x3d4ba4cu, 0x30e1644u, 0x338dca6u, 0x3e8cc53u, 0x0048b29u},
    {0x0000000u, 0x0000000u, 0x0000000u, 0x0000000u, 0x0000000u, 0x0000000u, 0x0000000u, 0x0000000u, 0x0000000u, 0x0000000u},
    {0x0a4da6cu, 0x17df3c6u, 0x2cf4638u, 0x3f3423fu, 0x0c2d458u, 0x3d15011u, 0x1806fd4u, 0x3f04571u, 0x00d91cdu, 0x008deadu},
    {0x0000000u, 0x0000000u, 0x0000000u, 0x0000000u, 0x0000000u, 0x0000000u, 0x0000000u, 0x0000000u, 0x0000000u, 0x0000000u},
    {0x1801893u, 0x3a0e578u, 0x00e4f6cu, 0x11eb721u, 0x34df862u, 0x3fc95c4u, 0x272598fu, 0x0b768cau, 0x024c57au, 0x0045383u},
    {0x0000000u, 0x0000000u, 0x0000000u, 0x0000000u, 0x0000000u, 0x0000000u, 0x0000000u, 0x0000000u, 0x0000000u, 0x0000000u},
    {0x1583b6eu, 0x245f768u, 0x1e7dcf6u, 0x37116a8u, 0x022a573u, 0x08b9bcbu, 0x1f64523u, 0x347ca3au, 0x28a14ddu, 0x0078de9u},
    {0x0000000u, 0x0000000u, 0x0000000u, 0x0000000u, 0x0000000u, 0x0000000u, 0x0000000u, 0x0000000u, 0x0000000u, 0x0000000u},
    {0x3d822dbu, 0x2a511efu, 0x1d98d89u, 0x2525f87u, 0x0d4ad11u, 0x08f0606u, 0x383eb93u, 0x290616fu, 0x2654f63u, 0x0033a66u},
    {0x0000000u, 0x0000000u, 0x0000000u, 0x0000000u, 0x0000000u, 0x0000000u, 0x0000000u, 0x0000000u, 0x0000000u, 0x0000000u},
    {0x2fce4b4u, 0x082203du, 0x09a8455u, 0x126eaa6u, 0x2498908u, 0x063c052u, 0x29201d8u, 0x1c93e16u, 0x24e1bb7u, 0x007c590u},
    {0x0000000u, 0x0000000u, 0x0000000u, 0x0000000u, 0x0000000u, 0x0000000u, 0x0000000u, 0x0000000u, 0x0000000u, 0x0000000u},
    {0x3739d42u, 0x01255ccu, 0x04d8ecfu, 0x329eecdu, 0x1806e54u, 0x37f7aa5u, 0x39e78f9u, 0x2478ba4u, 0x3b277bdu, 0x008138eu},
    {0x3e5b43cu, 0x3879a84u, 0x395c4c6u, 0x29f0799u, 0x0bfdf29u, 0x2382268u, 0x1ec49abu, 0x321d439u, 0x3fc70b1u, 0x0087428u},
    {0x1f4d60au, 0x32da33du, 0x01a841au, 0x3da57d1u, 0x3460958u, 0x15fc2e8u, 0x083d2d1u, 0x2da01afu, 0x3016849u, 0x007a235u},
    {0x37242ebu, 0x03872bcu, 0x152317au, 0x18e0485u, 0x2ccb918u, 0x0910f56u, 0x30b790cu, 0x39365d5u, 0x37b9de7u, 0x004ccd2u},
    {0x2ed7a0bu, 0x253199au, 0x1c6dc1eu, 0x0d0ea2eu, 0x0fe8353u, 0x3531195u, 0x366ed4fu, 0x2512d05u, 0x3eb1f75u, 0x008703bu},
    {0x36b5ab9u, 0x019c42bu, 0x008c687u, 0x1b670f7u, 0x365956du, 0x3a999b2u, 0x084335du, 0x1d6abedu, 0x092d3f8u, 0x0035ba6u},
    {0x17c3362u, 0x2088a81u, 0x18d9d06u, 0x0befbecu, 0x0ce600au, 0x1aea5bcu, 0x2ed193eu, 0x214e853u, 0x3ed850bu, 0x0028ecdu},
    {0x128801fu, 0x276aaf8u, 0x10160cbu, 0x2ae5098u, 0x2f5cafdu, 0x0d86122u, 0x0d06082u, 0x2a81d24u, 0x194257eu, 0x007827bu},
    {0x18a6cffu, 0x03761dcu, 0x172166eu, 0x188e8c7u, 0x0ff01aau, 0x3c79ad7u, 0x26425b9u, 0x35b0fe5u, 0x1bb55eeu, 0x002888bu},
    {0x19dbb1cu, 0x21ab273u, 0x3894010u, 0x3c3202bu, 0x29686e4u, 0x0a54455u, 0x10ccaceu, 0x211137cu, 0x3bba202u, 0x002593au},
};


// A right operand is read as a WINDOW: lane j reads words j+1 .. j+10 of a
// 48-word array whose words 10..19 hold the ten digits (the rest stay zero), so
// its column j = sum_i u_i v_(j-i) is a ten-term MAD chain with u broadcast.
constexpr int kDsWin = 48;
constexpr int kDsSlot = 21;  // lanes per slot: columns 0..18, carries to 19, 20
struct DsLds {
    uint32_t E[12][16];           // left operands of the products (words 10..15: scratch of non-digit lanes)
    uint32_t X[12][16];           // xi * left operand
    uint32_t BW[12][kDsWin];      // right operands of ds_mul (windows)
    uint32_t U0[12][16], U1[12][16];      // per-slot operands of the squaring / Frobenius
    uint32_t V0[12][kDsWin], V1[12][kDsWin];
    uint32_t GW[3][12][kDsWin];   // Frobenius constants (windows)
    int32_t D[12][16], MM[12][16];  // per-slot broadcasts of the reduction
    int32_t PR[12][16];           // the squaring's twelve products
    uint32_t CV[12][16];          // layout conversion (16-lane group <-> slots)
    // per lane j of a slot: p'_(j-i) (j < 10, else 0) and p_(j-i) for i = 0..9 (0
    // outside the digit range), and digit k = j - 10 of p, 3p, 8p (2^26 spread) and
    // 8p (2^27 spread)
    int32_t KPI[24][12], KP[24][12];
    uint32_t KOWN[24][4];
    DsComb KC[12];
};
__shared__ DsLds g_ds;

// this thread's place: slot cid (coordinate 2e + c, as the w12 lane l) = three per
// wave, lane j of the slot (lane 63 of a wave is lane 21 of its third slot: no
// digit, no column), digit k = j - 10 (a digit lane when 0 <= k < 10).
// Operations are called by every thread of the block (kDsThreads) in the same
// order; the arrays a slot's lanes share are one wave's, so they need no barrier,
// and every array another wave reads is behind a barrier before its next write.
struct DsLane {
    int cid, j, e, c, k, s;
    bool dl;
};
__device__ __forceinline__ DsLane ds_lane() {
    DsLane x;
    const int t = (int)threadIdx.x;
    const int l = t & 63;
    x.s = l >= 2 * kDsSlot ? 2 : l >= kDsSlot ? 1 : 0;
    x.j = l - kDsSlot * x.s;
    x.cid = 3 * (t >> 6) + x.s;
    x.e = x.cid >> 1;
    x.c = x.cid & 1;
    x.k = x.j - kDsB;
    x.dl = (unsigned)x.k < 10u;
    return x;
}
// the word a lane writes for digit k of a 16-word row: non-digit lanes write
// into the row's spare words 10..15
__device__ __forceinline__ int ds_wk(const DsLane& x) { return x.dl ? x.k : 10 + (x.j & 3); }

// ---------------------------------------------------------------- lanes
__device__ __forceinline__ uint32_t ds_shr1(uint32_t v) {  // lane l <- lane l - 1 (lane 0 of the wave <- 0)
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x138, 0xf, 0xf, true);
}
__device__ __forceinline__ uint32_t ds_shl1(uint32_t v) {  // lane l <- lane l + 1
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x130, 0xf, 0xf, true);
}
__device__ __forceinline__ int64_t ds_shr1_64(int64_t v) {
    const uint64_t u = (uint64_t)v;
    return (int64_t)(((uint64_t)ds_shr1((uint32_t)(u >> 32)) << 32) | ds_shr1((uint32_t)u));
}
__device__ __forceinline__ int64_t ds_shl1_64(int64_t v) {
    const uint64_t u = (uint64_t)v;
    return (int64_t)(((uint64_t)ds_shl1((uint32_t)(u >> 32)) << 32) | ds_shl1((uint32_t)u));
}
// the LDS accesses of a slot's lanes are one wave's: in order; this keeps the
// compiler from moving them across each other
__device__ __forceinline__ void ds_order() { asm volatile("" ::: "memory"); }
__device__ __forceinline__ int64_t ds_mad_i(int32_t a, int32_t b, int64_t c) { return (int64_t)a * (int64_t)b + c; }

// x = c0 + c1 2^26 + c2 2^52 (c0, c1 in [0, 2^26), c2 signed); digit j = c0_j +
// c1_(j-1) + c2_(j-2).  With the sink: lane kDsTop keeps its whole value and the
// lane below it hands up its whole quotient (the true top digit fits 32 bits, so
// the wrapped 32-bit sum is exact).  What lane 0 of a slot receives from the slot
// below (lanes 19, 20) is zero wherever it is used (tools/ds_model.py).
__device__ __forceinline__ int32_t ds_split64(int64_t x, int j, bool sink) {
    const uint64_t u = (uint64_t)x;
    const uint32_t lo = (uint32_t)u, hi = (uint32_t)(u >> 32);
    uint32_t c0 = lo & kDsM;
    uint32_t c1 = __builtin_amdgcn_alignbit(hi, lo, kDsDig) & kDsM;
    uint32_t c2 = (uint32_t)((int32_t)hi >> (2 * kDsDig - 32));
    if (sink) {
        const bool top = j == kDsTop, below = j == kDsTop - 1;
        c0 = top ? lo : c0;
        c1 = top ? 0u : below ? __builtin_amdgcn_alignbit(hi, lo, kDsDig) : c1;  // the whole x >> 26, truncated
        c2 = (top || below) ? 0u : c2;
    }
    return (int32_t)(c0 + ds_shr1(c1 + ds_shr1(c2)));  // c0_j + c1_(j-1) + c2_(j-2)
}
__device__ __forceinline__ int32_t ds_split32(int32_t d, int j, bool sink) {
    uint32_t lo = (uint32_t)d & kDsM;
    uint32_t hi = (uint32_t)(d >> kDsDig);
    if (sink) {
        lo = j == kDsTop ? (uint32_t)d : lo;
        hi = j == kDsTop ? 0u : hi;
    }
    return (int32_t)(lo + ds_shr1(hi));
}

// ---------------------------------------------------------------- setup
// every thread of the block (kDsThreads) calls this; ends with a barrier
__device__ void ds_init() {
    const int t = (int)threadIdx.x;
    if (t < 24) {
#pragma unroll
        for (int i = 0; i < 10; ++i) {
            const int a = t - i;
            g_ds.KPI[t][i] = (int32_t)((t < 10 && a >= 0) ? kDsPinv[a < 10 ? a : 0] : 0u);
            g_ds.KP[t][i] = (int32_t)((a >= 0 && a < 10) ? kDsP[a < 10 ? a : 0] : 0u);
        }
        const int k = t - kDsB;
        const bool dl = (unsigned)k < 10u;
        const int kk = dl ? k : 0;
        g_ds.KOWN[t][0] = dl ? kDsP[kk] : 0u;
        g_ds.KOWN[t][1] = dl ? kDsS3[kk] : 0u;
        g_ds.KOWN[t][2] = dl ? kDsS8[kk] : 0u;
        g_ds.KOWN[t][3] = dl ? kDsS8b[kk] : 0u;
    }
    if (t < 12) g_ds.KC[t] = kDsComb[t];
    // windows: zero everywhere, then the Frobenius constants' digits
    for (int w = t; w < 12 * kDsWin; w += kDsThreads) {
        (&g_ds.BW[0][0])[w] = 0;
        (&g_ds.V0[0][0])[w] = 0;
        (&g_ds.V1[0][0])[w] = 0;
    }
    for (int w = t; w < 3 * 12 * kDsWin; w += kDsThreads) {
        const int r = w / kDsWin, o = w % kDsWin;
        (&g_ds.GW[0][0][0])[w] = (o >= kDsB && o < kDsB + 10) ? kDsFrob[r][o - kDsB] : 0u;
    }
    __syncthreads();
}

// ---------------------------------------------------------------- reduction and fold
template <class T>
__device__ __forceinline__ void ds_ld10(const T* p, T (&v)[10]) {
    const uint4 a = *(const uint4*)p, b = *(const uint4*)(p + 4);
    const uint2 c = *(const uint2*)(p + 8);
    v[0] = (T)a.x; v[1] = (T)a.y; v[2] = (T)a.z; v[3] = (T)a.w;
    v[4] = (T)b.x; v[5] = (T)b.y; v[6] = (T)b.z; v[7] = (T)b.w;
    v[8] = (T)c.x; v[9] = (T)c.y;
}
// T: this lane's signed 64-bit column (lanes 0..18) of a sum of products ->
// T / 2^260 mod p as signed digits at lanes 10..19 (0 elsewhere; lane 19 the
// top).  Value in (-3p, T/R + 3p).
__device__ __forceinline__ int32_t ds_redc(int64_t T, const DsLane& x) {
    int32_t kpi[10], kp[10];
    ds_ld10(&g_ds.KPI[x.j][0], kpi);
    ds_ld10(&g_ds.KP[x.j][0], kp);
    const int32_t d = ds_split64(T, x.j, false);  // lanes 0..20
    g_ds.D[x.cid][x.j < 10 ? x.j : 10 + (x.j & 3)] = d;
    ds_order();
    int32_t dv[10];
    ds_ld10(&g_ds.D[x.cid][0], dv);
    int64_t m = 0;
#pragma unroll
    for (int i = 0; i < 10; ++i) m = ds_mad_i(dv[i], kpi[i], m);
    int32_t mm = ds_split64(m, x.j, false);
    mm = x.j < 10 ? mm : 0;  // m mod 2^260, digits in [-2^11, 2^27]
    g_ds.MM[x.cid][x.j < 10 ? x.j : 10 + (x.j & 3)] = mm;
    ds_order();
    int32_t mv[10];
    ds_ld10(&g_ds.MM[x.cid][0], mv);
    int64_t s = d;
#pragma unroll
    for (int i = 0; i < 10; ++i) s = ds_mad_i(mv[i], kp[i], s);
    // T + m p = 0 mod 2^260.  Lane 20 (weight 2^260 above the sink) joins lane 19,
    // one split with the sink, then the low part's quotient q (lanes 0..9 of the
    // split hold q * 2^260 exactly) from lanes 7..9 in 32-bit arithmetic (the rest
    // weighs < 2^-24 of a unit), added to digit 0 of the result (lane 10)
    const int64_t up = ds_shl1_64(s);
    s += x.j == kDsTop ? (int64_t)((uint64_t)up << kDsDig) : 0;
    s = x.j > kDsTop ? 0 : s;
    const int32_t r = ds_split64(s, x.j, true);
    const int32_t b = r + (int32_t)ds_shr1((uint32_t)(r >> kDsDig));
    const int32_t t = r + (int32_t)ds_shr1((uint32_t)(b >> kDsDig));
    const int32_t qs = (int32_t)ds_shr1((uint32_t)((t + 2) >> kDsDig));
    return x.j < kDsB ? 0 : x.j == kDsB ? r + qs : r;
}

// d: signed digits at lanes 10..19 (0 elsewhere; lane 19 the top, |value| < 2^31 p)
// -> the folded value: digits 0..8 in [0, 2^26 + 2], top in [0, 2^22), value in
// [0, 5p), same residue
__device__ __forceinline__ uint32_t ds_fold_digits(int32_t d, const DsLane& x) {
    const uint4 own = *(const uint4*)&g_ds.KOWN[x.j][0];
    const int qi = (int)__builtin_floorf((float)d * kDsFoldC);  // meaningful on the sink lanes
    const int q0 = __builtin_amdgcn_readlane(qi, kDsTop), q1 = __builtin_amdgcn_readlane(qi, kDsSlot + kDsTop),
              q2 = __builtin_amdgcn_readlane(qi, 2 * kDsSlot + kDsTop);
    const int q = x.s == 0 ? q0 : x.s == 1 ? q1 : q2;
    const int64_t z = ds_mad_i(-q, (int32_t)own.x, (int64_t)d);
    int32_t zz = ds_split32(ds_split64(z, x.j, true), x.j, true);
    const uint32_t r = (uint32_t)zz + own.y;  // digits >= 0 now; lanes outside 10..19 stay 0
    return (uint32_t)ds_split32((int32_t)r, x.j, true);
}
// y: signed 64-bit digits at lanes 10..19 (0 elsewhere) -> the folded value:
// digits 0..8 in [0, 2^26 + 2], top in [0, 2^22), value in [0, 5p), same residue
__device__ __forceinline__ uint32_t ds_fold(int64_t y, const DsLane& x) {
    return ds_fold_digits(ds_split64(y, x.j, true), x);
}

// ---------------------------------------------------------------- operations
// Diagnostic (tools/ds_check.hip built with -DBN_DS_STAMPS=1): thread 0 adds the
// clocks of each phase of ds_cyc to g_ds_stamp[phase]
#if defined(BN_DS_STAMPS) && BN_DS_STAMPS
__shared__ unsigned long long g_ds_stamp[8];
#define DS_STAMP(i)                                                 \
    do {                                                            \
        const unsigned long long t_ = clock64();                    \
        if (threadIdx.x == 0) g_ds_stamp[i] += t_ - ds_t0;           \
        ds_t0 = t_;                                                 \
    } while (0)
#define DS_STAMP_INIT unsigned long long ds_t0 = clock64()
#else
#define DS_STAMP(i) ((void)0)
#define DS_STAMP_INIT ((void)0)
#endif
// this lane's column of u * v: u broadcast (ten digits), v's window at w (words j+1..j+10)
__device__ __forceinline__ uint64_t ds_col(const uint32_t (&u)[10], const uint32_t* w, uint64_t a = 0) {
#pragma unroll
    for (int i = 0; i < 10; ++i) a += (uint64_t)u[i] * w[9 - i];
    return a;
}

// Granger-Scott cyclotomic squaring (fq12.rs:198-247, as fq12_wide.h w12_cyc):
// slot (e, c), e < 3: P_e = x y of pair e = (w^e, w^(e+3)); e >= 3: Q = (x + y)(xi y + x)
// of pair e - 3; then every output coordinate from them (kDsComb)
__device__ __forceinline__ uint32_t ds_cyc_body(uint32_t a) {
    DS_STAMP_INIT;
    const DsLane x = ds_lane();
    const int wk = ds_wk(x);
    g_ds.E[x.cid][wk] = a;
    __syncthreads();
    DS_STAMP(0);
    const bool hi = x.e >= 3;
    const int kk = hi ? x.e - 3 : x.e;
    {
        const uint32_t x0 = g_ds.E[2 * kk][wk], x1 = g_ds.E[2 * kk + 1][wk], y0 = g_ds.E[2 * kk + 6][wk],
                       y1 = g_ds.E[2 * kk + 7][wk];
        const uint32_t u0 = hi ? x0 + y0 : x0, u1 = hi ? x1 + y1 : x1;
        const uint32_t v0 = hi ? 9u * y0 - y1 + g_ds.KOWN[x.j][2] + x0 : y0;  // (xi y + x).c0 + 8p
        const uint32_t v1 = hi ? 9u * y1 + y0 + x1 : y1;                    // (xi y + x).c1
        g_ds.U0[x.cid][wk] = u0;
        g_ds.U1[x.cid][wk] = u1;
        if (x.dl) {
            g_ds.V0[x.cid][kDsB + x.k] = x.c ? v1 : v0;  // own coordinate of v
            g_ds.V1[x.cid][kDsB + x.k] = x.c ? v0 : v1;  // the other
        }
    }
    ds_order();
    DS_STAMP(1);
    uint32_t u0[10], u1[10];
    ds_ld10(&g_ds.U0[x.cid][0], u0);
    ds_ld10(&g_ds.U1[x.cid][0], u1);
    const uint64_t a1 = ds_col(u0, &g_ds.V0[x.cid][x.j + 1]);
    const uint64_t a2 = ds_col(u1, &g_ds.V1[x.cid][x.j + 1]);
    // c0 = u0 v0 - u1 v1, c1 = u0 v1 + u1 v0
    const int64_t T = (int64_t)a1 + (x.c ? (int64_t)a2 : -(int64_t)a2);
    DS_STAMP(2);
    const int32_t p = ds_redc(T, x);
    g_ds.PR[x.cid][wk] = p;
    const DsComb cb = g_ds.KC[x.cid];
    DS_STAMP(3);
    __syncthreads();
    DS_STAMP(4);
    int64_t y = ds_mad_i(cb.e, (int32_t)a, 0);
    y = ds_mad_i(cb.a, g_ds.PR[cb.i1][wk], y);
    y = ds_mad_i(cb.b, g_ds.PR[cb.i2][wk], y);
    y = ds_mad_i(cb.c, g_ds.PR[cb.i3][wk], y);
    DS_STAMP(5);
    const uint32_t r = ds_fold(x.dl ? y : 0, x);
    DS_STAMP(6);
    return r;
}
// the out-of-line form (most call sites); the squaring chains of the tail (ds_exp_sq,
// k_seg_fe1's squarings) inline ds_cyc_body: a call saves and reloads registers through
// scratch, and the reload's s_waitcnt vmcnt also waits for the hand-off stores issued
// before it (gfx950 counts stores in vmcnt)
__device__ __noinline__ uint32_t ds_cyc(uint32_t a) { return ds_cyc_body(a); }

// a * b (fq12.rs:319-327) on the w-basis: out_e = sum_i a'_i b_(e - i mod 6) with
// a'_i = xi a_i where the index wraps (w^6 = xi); conj_b: b's conjugate (its odd
// coefficients negated, fq12.rs:126-128), written as 8p - b into the window
__device__ __noinline__ uint32_t ds_mul(uint32_t a, uint32_t b, bool conj_b) {
    const DsLane x = ds_lane();
    const int wk = ds_wk(x);
    const uint4 own = *(const uint4*)&g_ds.KOWN[x.j][0];
    g_ds.E[x.cid][wk] = a;
    if (x.dl) g_ds.BW[x.cid][kDsB + x.k] = (conj_b && (x.e & 1)) ? own.w - b : b;
    __syncthreads();
    {
        const uint32_t ap = g_ds.E[x.cid ^ 1][wk];  // the other coordinate of this lane's Fq2
        g_ds.X[x.cid][wk] = x.c ? 9u * a + ap : 9u * a - ap + own.z;
    }
    __syncthreads();
    uint64_t pp = 0, qq = 0;
#ifndef BN_DS_MUL_UNROLL
#define BN_DS_MUL_UNROLL 2
#endif
#pragma unroll BN_DS_MUL_UNROLL
    for (int i = 0; i < 6; ++i) {
        const bool wrap = i > x.e;
        const int jj = wrap ? x.e - i + 6 : x.e - i;
        uint32_t u0[10], u1[10];
        ds_ld10(wrap ? &g_ds.X[2 * i][0] : &g_ds.E[2 * i][0], u0);
        ds_ld10(wrap ? &g_ds.X[2 * i + 1][0] : &g_ds.E[2 * i + 1][0], u1);
        // c0: x0 y0 - x1 y1; c1: x0 y1 + x1 y0
        pp = ds_col(u0, &g_ds.BW[2 * jj + x.c][x.j + 1], pp);
        qq = ds_col(u1, &g_ds.BW[2 * jj + 1 - x.c][x.j + 1], qq);
    }
    __syncthreads();  // every wave is done reading E, X, BW before the next operation writes them
    const int64_t T = (int64_t)pp + (x.c ? (int64_t)qq : -(int64_t)qq);
    return ds_fold_digits(ds_redc(T, x), x);
}

// frobenius_map(K) (fq12.rs:112-119): coefficient e -> conj^K(a_e) * gamma_(K,e)
template <int K>
__device__ __noinline__ uint32_t ds_frob(uint32_t a) {
    const DsLane x = ds_lane();
    g_ds.E[x.cid][ds_wk(x)] = a;
    __syncthreads();
    uint32_t u0[10], u1[10];
    ds_ld10(&g_ds.E[2 * x.e][0], u0);  // this Fq2's c0 and c1
    ds_ld10(&g_ds.E[2 * x.e + 1][0], u1);
    // c0 = x0 g0 - s x1 g1, c1 = x0 g1 + s x1 g0 (s = -1: odd K conjugates)
    const uint64_t A1 = ds_col(u0, &g_ds.GW[K - 1][2 * x.e + x.c][x.j + 1]);
    const uint64_t A2 = ds_col(u1, &g_ds.GW[K - 1][2 * x.e + 1 - x.c][x.j + 1]);
    __syncthreads();  // E is read before the next operation writes it
    const bool neg2 = (x.c == 0) != ((K & 1) != 0);
    const int64_t T = (int64_t)A1 + (neg2 ? -(int64_t)A2 : (int64_t)A2);
    return ds_fold_digits(ds_redc(T, x), x);
}

// unitary inverse (fq12.rs:126-128): the odd coefficients negate
__device__ __forceinline__ uint32_t ds_conj(uint32_t a) {
    const DsLane x = ds_lane();
    return ds_fold_digits((x.e & 1) ? -(int32_t)a : (int32_t)a, x);
}

// ---------------------------------------------------------------- layout conversion
// group 0 of the 16-lane layout (threads 0..11 hold coordinate l = threadIdx.x,
// value X = x 2^261 mod p) -> slots: X / 2 = x 2^260 mod p in 26-bit digits.
// Every thread calls; ends with the slot value.
__device__ uint32_t ds_from_w12(const Fq<2>& v) {
    const DsLane x = ds_lane();
    if (threadIdx.x < 12) {
        const auto h = fq_half(v);  // an integer below 2^260
#pragma unroll
        for (int k = 0; k < 10; ++k) {
            const int bit = kDsDig * k, i = bit / 29, s = bit % 29;
            uint64_t w = (uint64_t)h.v[i] >> s;
            if (i + 1 < 9) w |= (uint64_t)h.v[i + 1] << (29 - s);
            g_ds.CV[threadIdx.x][k] = (uint32_t)w & kDsM;
        }
    }
    __syncthreads();
    const uint32_t r = x.dl ? g_ds.CV[x.cid][x.k] : 0u;
    __syncthreads();  // CV is free again
    return r;
}
// slots -> threads 0..11: 2 * value (x 2^261), bound 10p, folded to Fq<2>.
// Every thread calls.
__device__ Fq<2> ds_to_w12(uint32_t a) {
    const DsLane x = ds_lane();
    if (x.dl) g_ds.CV[x.cid][x.k] = a;
    __syncthreads();
    Fq<2> r = widen<2>(fq_zero());
    if (threadIdx.x < 12) {
        uint32_t v[9];
        uint64_t acc = 0;
        int pos = 0, k = 0;
#pragma unroll
        for (int i = 0; i < 9; ++i) {
#pragma unroll
            for (int t = 0; t < 2; ++t)
                if (k < 10 && pos < 29) {
                    acc += (uint64_t)g_ds.CV[threadIdx.x][k] << pos;
                    pos += kDsDig;
                    ++k;
                }
            v[i] = i < 8 ? (uint32_t)acc & M29 : (uint32_t)acc;
            acc >>= 29;
            pos -= 29;
        }
        r = fq_fold(fq_dbl(Fq<5>{{v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7], v[8]}}));
    }
    __syncthreads();  // CV is free again
    return r;
}

// ---------------------------------------------------------------- final exponentiation
// exp_by_neg_z (fq12.rs:121-124) with the signed width-4 windows of w12_exp_by_neg_z
__device__ __noinline__ uint32_t ds_exp_by_neg_z(uint32_t xx) {
    const uint32_t x2 = ds_cyc(xx);
    const uint32_t x3 = ds_mul(xx, x2, false);
    const uint32_t x5 = ds_mul(x3, x2, false);
    const uint32_t x7 = ds_mul(x5, x2, false);
    auto val = [&](int d) {
        const int m = d < 0 ? -d : d;
        return m == 1 ? xx : m == 3 ? x3 : m == 5 ? x5 : x7;
    };
    uint32_t r = val(kZWin.d[0]);
    if (kZWin.d[0] < 0) r = ds_conj(r);
#pragma unroll 1
    for (int t = 1; t < kZWin.n; ++t) {
#pragma unroll 1
        for (int s = 0; s < kZWin.run[t]; ++s) r = ds_cyc(r);
        r = ds_mul(r, val(kZWin.d[t]), kZWin.d[t] < 0);
    }
#pragma unroll 1
    for (int s = 0; s < kZWin.tail; ++s) r = ds_cyc(r);
    return ds_conj(r);
}
// the last chunk of the final exponentiation (fq12.rs:75-105) of s =
// w12_fe_first(f), as w12_fe_last (products with a conjugate factor take it on
// the right: the product commutes)
__device__ __noinline__ uint32_t ds_fe_last(uint32_t s) {
    const uint32_t a = ds_exp_by_neg_z(s);
    const uint32_t b = ds_cyc(a);
    const uint32_t c = ds_cyc(b);
    const uint32_t d = ds_mul(c, b, false);
    const uint32_t e = ds_exp_by_neg_z(d);
    const uint32_t f1 = ds_cyc(e);
    const uint32_t g = ds_exp_by_neg_z(f1);
    const uint32_t j = ds_mul(e, g, true);   // conj(g) * e
    const uint32_t k = ds_mul(j, d, true);   // j * conj(d)
    const uint32_t l = ds_mul(k, b, false);
    const uint32_t m = ds_mul(k, e, false);
    const uint32_t n = ds_mul(s, m, false);
    const uint32_t o = ds_frob<1>(l);
    const uint32_t p = ds_mul(o, n, false);
    const uint32_t q = ds_frob<2>(k);
    const uint32_t r = ds_mul(q, p, false);
    const uint32_t t = ds_mul(l, s, true);   // conj(s) * l
    const uint32_t u = ds_frob<3>(t);
    return ds_mul(u, r, false);
}

// ---------------------------------------------------------------- squarer and multiplier blocks
// The same last chunk on TWO blocks of one launch (k_horner_tree2 after k_seg_fe1):
// the squarer block S runs the chain of squarings and hands x^(2^k) at each nonzero
// NAF digit of u to the multiplier block M through global memory; M multiplies
// them into its accumulator and hands the result back (fq12_wide.h's two-group
// final exponentiation, here between CUs of different XCDs).  Every item has its
// own slot (kDsItems of them, no reuse within a call) and every word carries its
// stamp: each digit lane stores (1 << 32 | digit) as one agent-scope 64-bit atomic
// (coherent across the XCDs' L2s) and goes on -- the producer never waits for its
// stores -- and the consumer's lanes poll their own words until the stamp is there.
// k_seg_fe1 zeroes the channel before each tail.  A poll that runs out of its cap
// sets BN_ERR_INTERNAL (the call fails, as fq12_wide.h duo_wait) and marks the
// wave's channel dead: every later take of that wave reads its words once and does
// not spin again, so a lost stamp or a stalled partner costs one capped wait per
// wave, not one per item.  (Counters with release / acquire
// cost the producer ~1.5 us per hand-off, tools/xblock_probe.)
constexpr int kDsItems = 80;    // S -> M: 3 x 24 powers + b + k
constexpr int kDsResults = 8;   // M -> S: a, e, g, o, u
constexpr int kDsChanWords = 2 * 128 * (kDsItems + kDsResults);  // 32-bit words
// Failure injection for tests/test_gpu_failure.py only (`make chanfail`): the
// producer's stores are dropped, so every take runs out of its cap.
#ifndef BN_DS_DROP_STAMPS
#define BN_DS_DROP_STAMPS 0
#endif
struct DsChan {
    uint64_t* w;  // (kDsItems + kDsResults) x 128 stamped words of global memory
    int* err;
    uint32_t items, results;
    bool dead;       // wave-uniform: a take of this wave has run out of its cap
    uint32_t epoch;  // the stamp: a word is there when its high half equals it (never 0)
};
__device__ __forceinline__ void ds_chan_st(uint64_t* slot, uint32_t a, uint32_t epoch) {
    const DsLane x = ds_lane();
    typedef __attribute__((address_space(1))) uint64_t g64;  // global: global_ (not flat) instructions
    if (x.dl && !BN_DS_DROP_STAMPS)
        __hip_atomic_store((g64*)(slot + 10 * x.cid + x.k), ((uint64_t)epoch << 32) | a, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}
// every lane of the wave takes part (the spin condition is a wave-wide vote, so
// `dead` stays wave-uniform); digit lanes poll their own word, the others return 0
__device__ __forceinline__ uint32_t ds_chan_ld(const uint64_t* slot, DsChan& ch) {
    const DsLane x = ds_lane();
    typedef const __attribute__((address_space(1))) uint64_t g64;
    g64* p = (g64*)(slot + 10 * x.cid + (x.dl ? x.k : 0));
    uint64_t v = x.dl ? __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : ((uint64_t)ch.epoch << 32);
    if (!ch.dead)
        for (uint32_t spins = 0; __any((uint32_t)(v >> 32) != ch.epoch) && spins < kSpinCap; ++spins) {
            __builtin_amdgcn_s_sleep(1);
            if (x.dl) v = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    if (__any((uint32_t)(v >> 32) != ch.epoch)) {  // decided on the words themselves: one that arrived during the last sleep counts
        if (!ch.dead && ch.err && (threadIdx.x & 63u) == 0) err_or(ch.err, BN_ERR_INTERNAL);
        ch.dead = true;
    }
    return x.dl ? (uint32_t)v : 0u;
}
__device__ __forceinline__ void ds_put(DsChan& ch, uint32_t a) {  // S
    ds_chan_st(ch.w + 128 * (ch.items++), a, ch.epoch);
}
__device__ __forceinline__ uint32_t ds_take(DsChan& ch) {  // M
    return ds_chan_ld(ch.w + 128 * (ch.items++), ch);
}
__device__ __forceinline__ void ds_put_result(DsChan& ch, uint32_t a) {  // M
    ds_chan_st(ch.w + 128 * (kDsItems + ch.results++), a, ch.epoch);
}
__device__ __forceinline__ uint32_t ds_get_result(DsChan& ch) {  // S
    return ds_chan_ld(ch.w + 128 * (kDsItems + ch.results++), ch);
}
// Diagnostic (-DBN_TAIL_STAMPS=1, tools/tail_stamps.py): thread 0 of a block records
// s_memrealtime (100 MHz) at the phase boundaries of the product's tail
// (k_seg_fe1's segment 0, and k_horner_tree2's squarer and multiplier blocks)
#ifndef BN_TAIL_STAMPS
#define BN_TAIL_STAMPS 0
#endif
#if BN_TAIL_STAMPS
__device__ uint64_t g_tail_stamps[32];
#define TAIL_STAMP(i)                                                                      \
    do {                                                                                   \
        if (threadIdx.x == 0) g_tail_stamps[i] = __builtin_amdgcn_s_memrealtime();       \
    } while (0)
#else
#define TAIL_STAMP(i) ((void)0)
#endif
// S's side of exp_by_neg_z: x^(2^k) handed over at each nonzero NAF digit of u
// (force-inlined, as ds_exp_mul and the two last-chunk drivers below: the channel state
// then lives in registers; as __noinline__ functions they took DsChan by reference, i.e.
// through the stack, and every put and take paid two scratch round trips behind an
// s_waitcnt vmcnt(0) that also waited for the previous put's store -- S's squarings ran
// 1.39 us each against 1.17 us without hand-offs, tools/tail_stamps.py)
__device__ __forceinline__ uint32_t ds_exp_sq(uint32_t xx, DsChan& ch, int stamp = -1) {
#pragma unroll 1
    for (int k = 0;; ++k) {
        if ((kZNaf.nz >> k) & 1u) ds_put(ch, xx);
        if (k == kZNaf.top) break;
        xx = ds_cyc_body(xx);
    }
    if (BN_TAIL_STAMPS && stamp >= 0) TAIL_STAMP(stamp);  // the squarings are done; M's product is awaited
    return ds_get_result(ch);
}
// M's side: the product of the handed-over powers (x^-1 = conj(x) in the cyclotomic
// subgroup); returns the first item (x itself)
__device__ __forceinline__ uint32_t ds_exp_mul(DsChan& ch) {
    const uint32_t x0 = ds_take(ch);
    uint32_t acc = (kZNaf.minus & 1u) ? ds_conj(x0) : x0;
#pragma unroll 1
    for (int k = 1; k <= kZNaf.top; ++k) {
        if (!((kZNaf.nz >> k) & 1u)) continue;
        const uint32_t y = ds_take(ch);
        acc = ds_mul(acc, y, ((kZNaf.minus >> k) & 1u) != 0);
    }
    ds_put_result(ch, ds_conj(acc));
    return x0;
}
// the last chunk (fq12.rs:75-105) of s on S, with M (ds_fe_last_m) beside it: the
// hand-overs are [24 powers of s], b, [24 powers of d], [24 powers of f1], k; M
// returns a, e, g, then o = frob(k b) and u = frob^3(conj(s) k b) (fq12_wide.h
// w12_fe_last_s / w12_final_exp_m, the reference's names)
__device__ __forceinline__ uint32_t ds_fe_last_s(uint32_t s, DsChan& ch) {
    const uint32_t a = ds_exp_sq(s, ch, 2);
    TAIL_STAMP(3);
    const uint32_t b = ds_cyc(a);
    ds_put(ch, b);
    const uint32_t c = ds_cyc(b);
    const uint32_t d = ds_mul(c, b, false);
    const uint32_t e = ds_exp_sq(d, ch, 4);
    TAIL_STAMP(5);
    const uint32_t f1 = ds_cyc(e);
    const uint32_t g = ds_exp_sq(f1, ch, 6);
    TAIL_STAMP(7);
    const uint32_t j = ds_mul(e, g, true);  // conj(g) * e
    const uint32_t k = ds_mul(j, d, true);  // j * conj(d)
    ds_put(ch, k);
    const uint32_t m = ds_mul(k, e, false);
    const uint32_t n = ds_mul(s, m, false);
    const uint32_t q = ds_frob<2>(k);
    const uint32_t o = ds_get_result(ch);
    const uint32_t p = ds_mul(o, n, false);
    const uint32_t r = ds_mul(q, p, false);
    const uint32_t u = ds_get_result(ch);
    return ds_mul(u, r, false);
}
__device__ __forceinline__ void ds_fe_last_m(DsChan& ch) {
    const uint32_t s = ds_exp_mul(ch);  // a
    const uint32_t b = ds_take(ch);
    (void)ds_exp_mul(ch);               // e
    (void)ds_exp_mul(ch);               // g
    const uint32_t k = ds_take(ch);
    const uint32_t l = ds_mul(k, b, false);
    ds_put_result(ch, ds_frob<1>(l));   // o
    const uint32_t t = ds_mul(l, s, true);  // conj(s) * l
    ds_put_result(ch, ds_frob<3>(t));   // u
}

// ---------------------------------------------------------------- two multiplier blocks
// One multiplier falls behind the squarer: its 23 products per exponentiation (~3 us
// each) take longer than S's 62 squarings (~0.93 us), so S waited ~15 us for each
// exponentiation's result (tools/tail_stamps.py, profiles/r6i_tail_stamps.json).  With
// two, M_0 multiplies the even and M_1 the odd hand-overs of each exponentiation (the
// same slots: item numbers as ds_fe_last_s), each returns its partial product
// conjugated, and S multiplies the two (conj is multiplicative and the product
// commutes: the value of ds_exp_sq).  Results: exponentiation e's partials in slots
// 2e and 2e + 1, then o and u (M_0) in 6 and 7.
static_assert(kDsResults >= 8, "three pairs of partials, o and u");
__device__ __forceinline__ uint32_t ds_exp_sq2(uint32_t xx, DsChan& ch, int stamp = -1) {
#pragma unroll 1
    for (int k = 0;; ++k) {
        if ((kZNaf.nz >> k) & 1u) ds_put(ch, xx);
        if (k == kZNaf.top) break;
        xx = ds_cyc_body(xx);
    }
    if (BN_TAIL_STAMPS && stamp >= 0) TAIL_STAMP(stamp);
    const uint32_t r0 = ds_get_result(ch);
    const uint32_t r1 = ds_get_result(ch);
    return ds_mul(r0, r1, false);
}
// M_par's share of exponentiation e (its hand-overs from item ch.items on); returns
// the first hand-over (x itself) on M_0
__device__ __forceinline__ uint32_t ds_exp_mul2(DsChan& ch, int par, int e) {
    uint32_t acc = 0, x0 = 0;
    int j = 0;
#pragma unroll 1
    for (int k = 0; k <= kZNaf.top; ++k) {
        if (!((kZNaf.nz >> k) & 1u)) continue;
        if ((j & 1) == par) {
            const uint32_t y = ds_chan_ld(ch.w + 128 * (ch.items + j), ch);
            const bool cj = ((kZNaf.minus >> k) & 1u) != 0;
            if (j == par) {
                x0 = y;
                acc = cj ? ds_conj(y) : y;
            } else {
                acc = ds_mul(acc, y, cj);
            }
        }
        ++j;
    }
    ch.items += j;
    ds_chan_st(ch.w + 128 * (kDsItems + 2 * e + par), ds_conj(acc), ch.epoch);
    return x0;
}
__device__ __forceinline__ uint32_t ds_fe_last_s2(uint32_t s, DsChan& ch) {
    const uint32_t a = ds_exp_sq2(s, ch, 2);
    TAIL_STAMP(3);
    const uint32_t b = ds_cyc(a);
    ds_put(ch, b);
    const uint32_t c = ds_cyc(b);
    const uint32_t d = ds_mul(c, b, false);
    const uint32_t e = ds_exp_sq2(d, ch, 4);
    TAIL_STAMP(5);
    const uint32_t f1 = ds_cyc(e);
    const uint32_t g = ds_exp_sq2(f1, ch, 6);
    TAIL_STAMP(7);
    const uint32_t j = ds_mul(e, g, true);  // conj(g) * e
    const uint32_t k = ds_mul(j, d, true);  // j * conj(d)
    ds_put(ch, k);
    const uint32_t m = ds_mul(k, e, false);
    const uint32_t n = ds_mul(s, m, false);
    const uint32_t q = ds_frob<2>(k);
    const uint32_t o = ds_get_result(ch);
    const uint32_t p = ds_mul(o, n, false);
    const uint32_t r = ds_mul(q, p, false);
    const uint32_t u = ds_get_result(ch);
    return ds_mul(u, r, false);
}
__device__ __forceinline__ void ds_fe_last_m2(DsChan& ch, int par) {
    const uint32_t s = ds_exp_mul2(ch, par, 0);  // a's partial; s on M_0
    uint32_t b = 0;
    if (par == 0) b = ds_take(ch); else ++ch.items;
    (void)ds_exp_mul2(ch, par, 1);              // e
    (void)ds_exp_mul2(ch, par, 2);              // g
    if (par != 0) return;
    const uint32_t k = ds_take(ch);
    const uint32_t l = ds_mul(k, b, false);
    ds_chan_st(ch.w + 128 * (kDsItems + 6), ds_frob<1>(l), ch.epoch);     // o
    const uint32_t t = ds_mul(l, s, true);                                  // conj(s) * l
    ds_chan_st(ch.w + 128 * (kDsItems + 7), ds_frob<3>(t), ch.epoch);     // u
}

}  // namespace bn
