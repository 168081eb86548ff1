// kernels.h -- shared device helpers and the kernel declarations of the engine
// (definitions in kernels_*.hip; launched from capi.hip).
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/bn254mi.h"
#include "pairing.h"

namespace bn {

// 256 threads = 4 waves: the dispatcher puts one such workgroup per CU, one wave
// per SIMD (measured census, profiles/r1_ubench3.jsonl); 64-thread workgroups
// left 104 of 1024 SIMDs with two waves while others idled.
constexpr int kBlock = 256;
// The pairing-path kernels (kernels_pairing/fe/util.hip) run two lanes per
// element (fq2_split.h: 2^16 pairings -> 2048 waves, two per SIMD); the host
// launches kPathLanes threads per element.  Built with -DBN_PATH_SPLIT=0 they
// run the one-lane layout (the round-1 form, kept for A/B measurements).
constexpr int kPathLanes = BN_PATH_SPLIT ? 2 : 1;
// words of one Fq12 slot per lane of the translation unit's own layout
constexpr int kSlotLaneWords = BN_SPLIT ? 54 : 108;
#if BN_SPLIT
// two waves per SIMD: the kernel must fit 256 registers (three or four waves: the
// spills cost 20-40 %, profiles/r2u_ab_waves_per_simd.txt)
#define BN_PATH_ATTR __attribute__((amdgpu_waves_per_eu(2, 2)))
#else
#define BN_PATH_ATTR
#endif
constexpr int kCoeffFq = BN_NUM_COEFFS * 6;  // Fq elements of line coefficients per pairing
constexpr size_t kChunk = size_t(1) << 18;   // pairings per launch set (~5 GB workspace)
constexpr int kSlotWords = 108;              // one Fq12: 12 Fq x 9 digits
// Gt::pow's window table (kernels_gtpow.hip): x^0..x^16 for the signed 5-bit
// windows of cyclotomic-subgroup waves (x^0..x^15 otherwise), in the context's
// Fq12 slots
constexpr int kGtPowEntries = 17;

// ---------------------------------------------------------------- lane-strided storage
template <int B>
__device__ __forceinline__ void st_fq(uint32_t* base, size_t n, size_t i, int j, const Fq<B>& x) {
#pragma unroll
    for (int l = 0; l < 9; ++l) base[((size_t)j * 9 + l) * n + i] = x.v[l];
}
template <int B>
__device__ __forceinline__ Fq<B> ld_fq(const uint32_t* base, size_t n, size_t i, int j) {
    Fq<B> x;
#pragma unroll
    for (int l = 0; l < 9; ++l) x.v[l] = base[((size_t)j * 9 + l) * n + i];
    return x;
}
#if BN_SPLIT
// Two lanes per element (fq2_split.h): `n` counts LANES and `i` is the lane;
// an Fq2 "slot" j (even, as in the one-lane layout) holds the lane's own
// coordinate at word ((j/2)*9 + l)*n + i, so a wave touches 256 contiguous bytes.
template <int B>
__device__ __forceinline__ void st_fq2(uint32_t* base, size_t n, size_t i, int j, const Fq2<B>& x) {
    st_fq(base, n, i, j / 2, x.c);
}
template <int B>
__device__ __forceinline__ Fq2<B> ld_fq2(const uint32_t* base, size_t n, size_t i, int j) {
    return {ld_fq<B>(base, n, i, j / 2)};
}
#else
template <int B>
__device__ __forceinline__ void st_fq2(uint32_t* base, size_t n, size_t i, int j, const Fq2<B>& x) {
    st_fq(base, n, i, j, x.c0);
    st_fq(base, n, i, j + 1, x.c1);
}
template <int B>
__device__ __forceinline__ Fq2<B> ld_fq2(const uint32_t* base, size_t n, size_t i, int j) {
    return {ld_fq<B>(base, n, i, j), ld_fq<B>(base, n, i, j + 1)};
}
#endif
template <int B>
__device__ __forceinline__ void st_fq12(uint32_t* base, size_t n, size_t i, const Fq12<B>& f) {
    st_fq2(base, n, i, 0, f.c0.c0);
    st_fq2(base, n, i, 2, f.c0.c1);
    st_fq2(base, n, i, 4, f.c0.c2);
    st_fq2(base, n, i, 6, f.c1.c0);
    st_fq2(base, n, i, 8, f.c1.c1);
    st_fq2(base, n, i, 10, f.c1.c2);
}
template <int B>
__device__ __forceinline__ Fq12<B> ld_fq12(const uint32_t* base, size_t n, size_t i) {
    return {{ld_fq2<B>(base, n, i, 0), ld_fq2<B>(base, n, i, 2), ld_fq2<B>(base, n, i, 4)},
            {ld_fq2<B>(base, n, i, 6), ld_fq2<B>(base, n, i, 8), ld_fq2<B>(base, n, i, 10)}};
}

// In the step machine, Fq12 slots go through a buffer descriptor (the *_buf forms):
// one 32-bit VGPR offset (the lane) serves all 108 words, and the word offset
// w * n * 4 is the uniform scalar soffset.  Plain global loads of a
// lane-strided element need a 64-bit VGPR address per word.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t slot_rsrc(const uint32_t* base) {
    return __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, 0x7fffffff, 0x00020000);
}
template <int B>
__device__ __forceinline__ Fq<B> ld_fq_buf(__amdgpu_buffer_rsrc_t rs, int vo, size_t n, int j) {
    Fq<B> x;
#pragma unroll
    for (int l = 0; l < 9; ++l) x.v[l] = __builtin_amdgcn_raw_buffer_load_b32(rs, vo, (int)(((size_t)j * 9 + l) * n * 4), 0);
    return x;
}
template <int B>
__device__ __forceinline__ void st_fq_buf(__amdgpu_buffer_rsrc_t rs, int vo, size_t n, int j, const Fq<B>& x) {
#pragma unroll
    for (int l = 0; l < 9; ++l) __builtin_amdgcn_raw_buffer_store_b32(x.v[l], rs, vo, (int)(((size_t)j * 9 + l) * n * 4), 0);
}
#if BN_SPLIT
template <int B>
__device__ __forceinline__ void st_fq12_buf(uint32_t* base, size_t n, size_t i, const Fq12<B>& f) {
    const auto rs = slot_rsrc(base);
    const int vo = (int)(i * 4);
    const Fq2<B>* c[6] = {&f.c0.c0, &f.c0.c1, &f.c0.c2, &f.c1.c0, &f.c1.c1, &f.c1.c2};
#pragma unroll
    for (int k = 0; k < 6; ++k) st_fq_buf(rs, vo, n, k, c[k]->c);
}
template <int B>
__device__ __forceinline__ Fq12<B> ld_fq12_buf(const uint32_t* base, size_t n, size_t i) {
    const auto rs = slot_rsrc(base);
    const int vo = (int)(i * 4);
    auto q = [&](int k) { return Fq2<B>{ld_fq_buf<B>(rs, vo, n, k)}; };
    return {{q(0), q(1), q(2)}, {q(3), q(4), q(5)}};
}
#else
template <int B>
__device__ __forceinline__ void st_fq12_buf(uint32_t* base, size_t n, size_t i, const Fq12<B>& f) {
    const auto rs = slot_rsrc(base);
    const int vo = (int)(i * 4);
    const Fq2<B>* c[6] = {&f.c0.c0, &f.c0.c1, &f.c0.c2, &f.c1.c0, &f.c1.c1, &f.c1.c2};
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        st_fq_buf(rs, vo, n, 2 * k, c[k]->c0);
        st_fq_buf(rs, vo, n, 2 * k + 1, c[k]->c1);
    }
}
template <int B>
__device__ __forceinline__ Fq12<B> ld_fq12_buf(const uint32_t* base, size_t n, size_t i) {
    const auto rs = slot_rsrc(base);
    const int vo = (int)(i * 4);
    auto q = [&](int k) { return Fq2<B>{ld_fq_buf<B>(rs, vo, n, 2 * k), ld_fq_buf<B>(rs, vo, n, 2 * k + 1)}; };
    return {{q(0), q(1), q(2)}, {q(3), q(4), q(5)}};
}

#endif  // BN_SPLIT

// Per-lane slot selection (Gt::pow's window table): the descriptor is built
// from the uniform workspace base and the lane's slot goes into the VGPR
// offset, so the resource stays wave-uniform.  A descriptor built from a
// lane-divergent pointer makes the compiler wrap every load in a readfirstlane
// waterfall loop whose per-lane pointer lives in VGPRs across partial-exec
// regions; round 1's k_gt_pow faulted with an illegal address in that form
// (DESIGN.md §3).  vo_bytes = (slot * kSlotWords * n + i) * 4 must stay below
// 2^31 (checked by the host launcher).
#if !BN_SPLIT
template <int B>
__device__ __forceinline__ Fq12<B> ld_fq12_buf_sel(const uint32_t* ws, size_t n, uint32_t vo_bytes) {
    const auto rs = slot_rsrc(ws);
    const int vo = (int)vo_bytes;
    auto q = [&](int k) { return Fq2<B>{ld_fq_buf<B>(rs, vo, n, 2 * k), ld_fq_buf<B>(rs, vo, n, 2 * k + 1)}; };
    return {{q(0), q(1), q(2)}, {q(3), q(4), q(5)}};
}
#else
// two lanes per element: `n` counts lanes, the lane's own coordinates
template <int B>
__device__ __forceinline__ Fq12<B> ld_fq12_buf_sel(const uint32_t* ws, size_t n, uint32_t vo_bytes) {
    const auto rs = slot_rsrc(ws);
    const int vo = (int)vo_bytes;
    auto q = [&](int k) { return Fq2<B>{ld_fq_buf<B>(rs, vo, n, k)}; };
    return {{q(0), q(1), q(2)}, {q(3), q(4), q(5)}};
}
#endif

template <int B>
__device__ __forceinline__ Fq6<B> ld_fq6(const uint32_t* base, size_t n, size_t i, int h) {
    return {ld_fq2<B>(base, n, i, 6 * h), ld_fq2<B>(base, n, i, 6 * h + 2), ld_fq2<B>(base, n, i, 6 * h + 4)};
}

// No memory operation may move across this point (compiler barrier only).
__device__ __forceinline__ void mem_fence() { asm volatile("" ::: "memory"); }

// Fq6 product (fq6.rs:197-207, the same Karatsuba as fq6_mul) with operand b
// supplied per Fq2 coordinate by g(j), fetched right before each product that
// needs it (mem_fence keeps the loads from being hoisted), so b never has to be
// held in registers.
template <int A, class G>
__device__ __forceinline__ auto fq6_mul_g(const Fq6<A>& a, G&& g) {
    if constexpr (kv(A) > 20) {
        return fq6_mul_g(fq6_fold(a), g);
    } else {
        mem_fence();
        auto a_a = fq2_mul(a.c0, g(0));
        mem_fence();
        auto b_b = fq2_mul(a.c1, g(1));
        mem_fence();
        auto c_c = fq2_mul(a.c2, g(2));
        mem_fence();
        auto t0 = fq2_sub(fq2_sub(fq2_mul(fq2_add(a.c1, a.c2), fq2_add(g(1), g(2))), b_b), c_c);
        mem_fence();
        auto t1 = fq2_sub(fq2_sub(fq2_mul(fq2_add(a.c0, a.c1), fq2_add(g(0), g(1))), a_a), b_b);
        mem_fence();
        auto t2 = fq2_sub(fq2_mul(fq2_add(a.c0, a.c2), fq2_add(g(0), g(2))), a_a);
        return mk6(fq2_add(fq2_mul_xi(t0), a_a), fq2_add(t1, fq2_mul_xi(c_c)), fq2_sub(fq2_add(t2, b_b), c_c));
    }
}

#if !BN_SPLIT
// a * b (fq12.rs:319-327 Karatsuba) with b read per Fq2 from `y`, the calling
// lane's strided copy of an Fq12 (word w at y[w * stride]: an LDS image with
// stride kBlock, or a lane-strided HBM slot with stride n); conj_b multiplies
// by conj(b) instead (fq12.rs:126-128).  b is never held in registers whole.
__device__ __forceinline__ Fq12<kF> mul12_strided(const Fq12<kF>& a, const uint32_t* y, size_t stride, bool conj_b) {
    auto ld = [&](int j) {  // Fq2 coordinate j of b (0..2: b.c0, 3..5: b.c1)
        Fq2<kF> r;
#pragma unroll
        for (int l = 0; l < 9; ++l) {
            r.c0.v[l] = y[((2 * j) * 9 + l) * stride];
            r.c1.v[l] = y[((2 * j + 1) * 9 + l) * stride];
        }
        return r;
    };
    auto g0 = [&](int j) { return ld(j); };
    auto g1 = [&](int j) {
        Fq2<kF> r = ld(3 + j);
        if (conj_b) r = fq2_neg(r);
        return r;
    };
    auto gs = [&](int j) { return fq2_add(g0(j), g1(j)); };
    const auto aa = fq6_fold(fq6_mul_g(a.c0, g0));
    const auto s = fq6_add(a.c0, a.c1);
    const auto bb = fq6_fold(fq6_mul_g(a.c1, g1));
    const auto t = fq6_mul_g(s, gs);
    return narrow12<kF>(mk12(fq6_add(fq6_mul_by_nonresidue(bb), aa), fq6_sub(fq6_sub(t, aa), bb)));
}
__device__ __forceinline__ Fq12<kF> mul12_lds(const Fq12<kF>& a, const uint32_t* yl, bool conj_b) {
    return mul12_strided(a, yl, kBlock, conj_b);
}

#endif

// Asynchronous copy of a lane-strided Fq12 (108 words, stride n) from global
// memory into the block's LDS image (stride kBlock) with buffer_load ... lds:
// no VGPRs and no vector ALU (SGPR offsets, M0 = the wave's LDS base).  The
// caller waits with lds_copy_wait() before reading.
__device__ __forceinline__ void lds_copy_fq12(const uint32_t* src_block, size_t n, uint32_t* yl_block) {
    // src_block = slot base + blockIdx.x * kBlock; yl_block = LDS image base
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void*)src_block, 0, 0x7fffffff, 0x00020000);
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x & ~63u);
    const int lane_off = (int)(threadIdx.x & 63u) * 4 + (int)wave * 4;
#pragma unroll
    for (int w = 0; w < kSlotWords; ++w)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rs, (__attribute__((address_space(3))) void*)(yl_block + w * kBlock + wave), 4, lane_off,
            (int)((size_t)w * n * 4), 0, 0);
}
__device__ __forceinline__ void lds_copy_wait() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// ---------------------------------------------------------------- reference images
__device__ __forceinline__ void ld_words(const bn_fq* src, uint32_t w[8]) {
    const uint4* s = reinterpret_cast<const uint4*>(src);
    uint4 a = s[0], b = s[1];
    w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w;
    w[4] = b.x; w[5] = b.y; w[6] = b.z; w[7] = b.w;
}
__device__ __forceinline__ void st_words(bn_fq* dst, const uint32_t w[8]) {
    uint4* d = reinterpret_cast<uint4*>(dst);
    d[0] = make_uint4(w[0], w[1], w[2], w[3]);
    d[1] = make_uint4(w[4], w[5], w[6], w[7]);
}
__device__ __forceinline__ bool words_zero(const uint32_t w[8]) {
    return (w[0] | w[1] | w[2] | w[3] | w[4] | w[5] | w[6] | w[7]) == 0;
}
// the reference's Montgomery image of one (R mod p, little-endian 32-bit words): the
// value `z == one` compares against in to_affine (mod.rs:199-216)
__device__ __forceinline__ bool words_one(const uint32_t w[8]) {
    return ((w[0] ^ 0xc58f0d9du) | (w[1] ^ 0xd35d438du) | (w[2] ^ 0xf5c70b3du) | (w[3] ^ 0x0a78eb28u) |
            (w[4] ^ 0x7879462cu) | (w[5] ^ 0x666ea36fu) | (w[6] ^ 0x9a07df2fu) | (w[7] ^ 0x0e0a77c1u)) == 0;
}
__device__ __forceinline__ Fq<2> ld_ref(const bn_fq& a) {
    uint32_t w[8];
    ld_words(&a, w);
    return fq_load_ref(w);
}
template <int B>
__device__ __forceinline__ void st_ref(bn_fq& a, const Fq<B>& x) {
    uint32_t w[8];
    fq_store_ref(x, w);
    st_words(&a, w);
}
#if BN_SPLIT
// this lane's coordinate of a reference Fq2 image (c0 on even lanes, c1 on odd)
__device__ __forceinline__ Fq2<2> ld_ref2(const bn_fq2& a) { return {ld_ref(lane_odd() ? a.c1 : a.c0)}; }
template <int B>
__device__ __forceinline__ void st_ref2(bn_fq2& a, const Fq2<B>& x) {
    st_ref(lane_odd() ? a.c1 : a.c0, x.c);
}
#else
__device__ __forceinline__ Fq2<2> ld_ref2(const bn_fq2& a) { return {ld_ref(a.c0), ld_ref(a.c1)}; }
template <int B>
__device__ __forceinline__ void st_ref2(bn_fq2& a, const Fq2<B>& x) {
    st_ref(a.c0, x.c0);
    st_ref(a.c1, x.c1);
}
#endif
#if BN_SPLIT
// Gt image: coefficient 2k + (lane parity) is the lane's coordinate of Fq2 k in
// the order c0.c0, c0.c1, c0.c2, c1.c0, c1.c1, c1.c2 (fq12.rs:52-55)
template <int B>
__device__ __forceinline__ void st_gt(bn_gt& g, const Fq12<B>& f) {
    const int o = lane_odd() ? 1 : 0;
    st_ref(g.c[0 + o], f.c0.c0.c);
    st_ref(g.c[2 + o], f.c0.c1.c);
    st_ref(g.c[4 + o], f.c0.c2.c);
    st_ref(g.c[6 + o], f.c1.c0.c);
    st_ref(g.c[8 + o], f.c1.c1.c);
    st_ref(g.c[10 + o], f.c1.c2.c);
}
__device__ __forceinline__ Fq12<2> ld_gt(const bn_gt& g) {
    const int o = lane_odd() ? 1 : 0;
    auto q = [&](int k) { return Fq2<2>{ld_ref(g.c[2 * k + o])}; };
    return {{q(0), q(1), q(2)}, {q(3), q(4), q(5)}};
}
// the lane's half of the zero image
__device__ __forceinline__ void st_gt_zero(bn_gt& g) {
    uint32_t z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const int o = lane_odd() ? 1 : 0;
#pragma unroll
    for (int k = 0; k < 6; ++k) st_words(&g.c[2 * k + o], z);
}
#else
template <int B>
__device__ __forceinline__ void st_gt(bn_gt& g, const Fq12<B>& f) {
    // coefficient order c0.c0.c0, c0.c0.c1, c0.c1.c0, ... (fq12.rs:52-55); no array
    // of pointers (a private array would live in scratch)
    st_ref(g.c[0], f.c0.c0.c0);
    st_ref(g.c[1], f.c0.c0.c1);
    st_ref(g.c[2], f.c0.c1.c0);
    st_ref(g.c[3], f.c0.c1.c1);
    st_ref(g.c[4], f.c0.c2.c0);
    st_ref(g.c[5], f.c0.c2.c1);
    st_ref(g.c[6], f.c1.c0.c0);
    st_ref(g.c[7], f.c1.c0.c1);
    st_ref(g.c[8], f.c1.c1.c0);
    st_ref(g.c[9], f.c1.c1.c1);
    st_ref(g.c[10], f.c1.c2.c0);
    st_ref(g.c[11], f.c1.c2.c1);
}
__device__ __forceinline__ Fq12<2> ld_gt(const bn_gt& g) {
    auto q = [&](int k) { return Fq2<2>{ld_ref(g.c[2 * k]), ld_ref(g.c[2 * k + 1])}; };
    return {{q(0), q(1), q(2)}, {q(3), q(4), q(5)}};
}
__device__ __forceinline__ void st_gt_zero(bn_gt& g) {
    uint32_t z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < 12; ++k) st_words(&g.c[k], z);
}
#endif  // BN_SPLIT

// Fr Montgomery image -> canonical scalar words: U256::from(Fr), fp.rs:13-20
// (one REDC by r with 32-bit digits; once per scalar product)
__device__ __forceinline__ void fr_to_canonical(const bn_fr& k, uint32_t out[8]) {
    constexpr uint32_t R[8] = {0xf0000001u, 0x43e1f593u, 0x79b97091u, 0x2833e848u,
                               0x8181585du, 0xb85045b6u, 0xe131a029u, 0x30644e72u};
    uint32_t t[9];
    ld_words(reinterpret_cast<const bn_fq*>(&k), t);
    t[8] = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const uint32_t m = t[0] * 0xefffffffu;
        uint64_t c = ((uint64_t)m * R[0] + t[0]) >> 32;
#pragma unroll
        for (int j = 1; j < 8; ++j) {
            const uint64_t s = (uint64_t)m * R[j] + t[j] + c;
            t[j - 1] = (uint32_t)s;
            c = s >> 32;
        }
        const uint64_t s = (uint64_t)t[8] + c;
        t[7] = (uint32_t)s;
        t[8] = (uint32_t)(s >> 32);
    }
    uint32_t d[8];
    int64_t br = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int64_t s = (int64_t)t[j] - R[j] + br;
        d[j] = (uint32_t)s;
        br = s >> 32;
    }
    const bool ge = (t[8] != 0) || (br == 0);
#pragma unroll
    for (int j = 0; j < 8; ++j) out[j] = ge ? d[j] : t[j];
}

__device__ __forceinline__ size_t lane_id() { return (size_t)blockIdx.x * blockDim.x + threadIdx.x; }

// ---------------------------------------------------------------- issue balance
// The throughput kernels run several identical, VALU-issue-bound waves per SIMD
// (k_pairing_fused, k_fq12_vm, k_gt_pow, k_miller_seg, k_g1_mul: two).  The SIMD arbitrates VALU issue between them by priority, then age
// (MI355X_MICROARCH.md, "Two waves per SIMD"), so at equal priority the older
// wave runs ahead and the younger one finishes ALONE, at the lone-wave issue
// rate: the measured average wave lifetime was ~0.77 of the kernel
// (profiles/pmc_summary.json).
// Balance: such a kernel launches one workgroup holding every wave of its CU
// (kPairBlock = 512 threads for two waves per SIMD; up to 1024 supported).  Each wave
// publishes its program position in LDS at every step of its main loop and sets
// its priority (s_setprio) to the number of waves on its SIMD (found from
// HW_ID's SIMD field at start) that are AHEAD of it, so laggards issue first and
// the waves finish together.  Scheduling only: no value depends on it.
// Without it: 7.6 instead of 8.3 M pairings/s (profiles/r3a_ab_balance.txt).
constexpr int kPairBlock = 512;
constexpr int kMaxBlock = 1024;
struct Balance {
    uint32_t w = 0;        // this wave's index in the block
    uint32_t partner = 0;  // the first other wave of the block on this wave's SIMD (itself if none)
    uint32_t more = 0;     // any further ones (bit j = wave j): more than two waves per SIMD
};
#if defined(__HIP_DEVICE_COMPILE__)
__shared__ uint32_t g_bal_prog[kMaxBlock / 64];
__shared__ uint32_t g_bal_simd[kMaxBlock / 64];
// every thread of the block calls this (it has a barrier), before any early return
__device__ __forceinline__ Balance balance_init() {
    Balance b;
    b.w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // HW_ID (hwreg 4): bits 5:4 = the SIMD this wave runs on
    const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);
    g_bal_simd[b.w] = (hw >> 4) & 3u;
    g_bal_prog[b.w] = 0;
    __syncthreads();
    const uint32_t nw = blockDim.x >> 6;
    uint32_t m = 0;
    for (uint32_t j = 0; j < nw; ++j)
        if (j != b.w && g_bal_simd[j] == g_bal_simd[b.w]) m |= 1u << j;
    m = __builtin_amdgcn_readfirstlane(m);
    b.partner = m ? (uint32_t)__builtin_ctz(m) : b.w;
    b.more = m & (m - 1);
    return b;
}
// `pos`: this wave's position in the (shared) program, non-decreasing.  The
// priority is the number of other waves on the SIMD not behind this one (a tie
// counts: two tied waves both run at 1, and age decides between them).
// The position words are read and written as relaxed workgroup-scope atomics:
// they become plain LDS operations (ds_read / ds_write).  Through a volatile
// generic pointer they were flat_load/flat_store sc0 sc1 (rounds 3-4), and in
// k_pairing_full the backend then emitted an illegal VOPC for the LDS-to-flat
// cast as soon as the unit's code changed ("Operand has incorrect register
// class", V_CMP_NE_U32_e32 0, src_shared_base).
__device__ __forceinline__ uint32_t bal_ld(uint32_t j) {
    return __hip_atomic_load(&g_bal_prog[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void balance_step(const Balance& b, uint32_t pos) {
    __hip_atomic_store(&g_bal_prog[b.w], pos, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    uint32_t ahead = __builtin_amdgcn_readfirstlane(bal_ld(b.partner)) >= pos && b.partner != b.w ? 1u : 0u;
    if (b.more) {
        for (uint32_t m = b.more; m; m &= m - 1)
            ahead += __builtin_amdgcn_readfirstlane(bal_ld(__builtin_ctz(m))) >= pos ? 1u : 0u;
        if (ahead >= 3) __builtin_amdgcn_s_setprio(3);
        else if (ahead == 2) __builtin_amdgcn_s_setprio(2);
    }
    if (ahead == 1) __builtin_amdgcn_s_setprio(1);
    else if (ahead == 0) __builtin_amdgcn_s_setprio(0);
}
#else
__device__ __forceinline__ Balance balance_init() { return Balance{}; }
__device__ __forceinline__ void balance_step(const Balance&, uint32_t) {}
#endif


// BN_DEVICE_CHECKS builds: export this translation unit's fold-bound
// violation counter (fq.h) as bn_dbg_fold_bad_<tu>().
#if BN_DEVICE_CHECKS
#define BN_EXPORT_FOLD_CHECK(tu)                                                  \
    extern "C" unsigned bn_dbg_fold_bad_##tu(void) {                              \
        unsigned h = 0;                                                           \
        if (hipMemcpyFromSymbol(&h, HIP_SYMBOL(bn::g_fold_bad), sizeof h) != hipSuccess) \
            return 0xffffffffu;                                                   \
        return h;                                                                 \
    }
#else
#define BN_EXPORT_FOLD_CHECK(tu)
#endif

inline unsigned grid_for(size_t n) { return (unsigned)((n + kBlock - 1) / kBlock); }
inline unsigned grid_pair(size_t n) { return (unsigned)((n + kPairBlock - 1) / kPairBlock); }

// ---------------------------------------------------------------- Fq12 step machine
// The final exponentiation is ~300 Fq12 operations; compiled inline it is one
// enormous kernel (minutes to build, scratch spills).  Instead k_fq12_vm runs a
// step program over lane-strided Fq12 slots in HBM: each step loads its
// operands, computes in registers, stores the result.  Every operation's code
// exists once.  The opcode is wave-uniform.  A step is two words:
//   w0 = op | d << 8 | a << 16 | b << 24,   w1 = k | flags << 8
// OP_CYC:  d = cyc^k(a)                       (k cyclotomic squarings in registers)
// OP_MUL:  d = [conj] (cyc^k(a) * [conj] b)   (kFlagConjB, kFlagConjOut)
// so a whole run of an exponent chain (zeros then a digit) is one step and the
// slot traffic is paid once per nonzero digit, not once per squaring.  The
// previous step's result stays in registers: kFlagAccA takes operand a from
// there instead of its slot, and kFlagNoStore skips the store of a result that
// no later step reads from its slot.
enum Fq12Op : uint32_t {
    OP_MOV = 0, OP_MUL = 1, OP_SQR = 2, OP_CYC = 3, OP_CONJ = 4,
    OP_FROB1 = 5, OP_FROB2 = 6, OP_FROB3 = 7, OP_INV = 8
};
constexpr uint32_t kFlagConjB = 1, kFlagConjOut = 2, kFlagAccA = 4, kFlagNoStore = 8;
inline void vm_step(uint32_t out[2], uint32_t op, uint32_t d, uint32_t a, uint32_t b, uint32_t k, uint32_t flags) {
    out[0] = op | (d << 8) | (a << 16) | (b << 24);
    out[1] = k | (flags << 8);
}

// Segments of the Miller loop's 64 NAF digits (k_miller_seg / k_horner_wide):
// segment s covers digits [lo[s], hi[s]) and starts at line coefficient idx[s]
constexpr int kMaxSeg = 16;
// K[s]: pairs per lane pair of segment s -- the reference's shared-squaring
// multi-Miller loop (mod.rs:609-640): lane pair g of segment s squares its
// accumulator once per digit and multiplies in the lines of pairs g, g + G[s],
// ..., g + (K[s]-1) G[s] (G[s] = ceil(n / K[s])); K = 1 for pairing_many's
// per-pair loops.  Segment s's lane pairs are [off[s], off[s] + G[s]) of `total`
// (k_miller_seg writes element off[s] + g); a pairing_batch plan pads each
// segment's range to whole 512-thread blocks, so no block mixes two segments.
struct SegPlan {
    int S;
    int lo[kMaxSeg], hi[kMaxSeg], idx[kMaxSeg];
    int K[kMaxSeg];
    uint32_t G[kMaxSeg], off[kMaxSeg], total;
};
// the element ranges of the sets k_fq12_reduce_wide multiplies (set y: elements
// off[y] .. off[y] + n[y] - 1 of its input) and the blocks that take them (set y:
// blocks blk[y] .. blk[y + 1] - 1 of the launch, one output element each)
struct SetSpan {
    uint32_t off[kMaxSeg], n[kMaxSeg], blk[kMaxSeg + 1];
    int sets;
};

// ---------------------------------------------------------------- kernels
__global__ void __launch_bounds__(kPairBlock) k_miller_seg(const uint32_t* __restrict__ coeffs,
                                                       const uint32_t* __restrict__ paff,
                                                       const uint8_t* __restrict__ flags, size_t n, SegPlan plan,
                                                       uint32_t* __restrict__ out);
// out[e] = Horner recombination of element e's S segment values (element s * n + e of g,
// split layout, stride S * n): x = g0; x = x^(2^len_s) * g_s; then the final
// exponentiation when do_fe
__global__ void __launch_bounds__(kBlock) k_horner_wide(const uint32_t* __restrict__ g, size_t n, SegPlan plan,
                                                        int do_fe, bn_gt* __restrict__ out, int* __restrict__ err, int duo);
// the same for ONE element (n = 1) on the S groups of one block: group s raises g_s
// to 2^(len_(s+1) + ... + len_(S-1)), then a product tree; out[0]
__global__ void __launch_bounds__(kBlock) k_horner_tree(const uint32_t* __restrict__ g, SegPlan plan, int do_fe,
                                                        bn_gt* __restrict__ out, int* __restrict__ err, int duo);
__global__ void __launch_bounds__(kPairBlock) k_prepare(const bn_g1* __restrict__ p, const bn_g2* __restrict__ q, size_t n,
                          uint32_t* __restrict__ coeffs, uint32_t* __restrict__ paff, uint8_t* __restrict__ flags,
                          int* __restrict__ err, int mode, int scale);
// the same outputs on kPrepareWideLanes lanes per pair (kernels_pairing.hip): four
// lane pairs run each line step's independent products side by side.  scale = 1: the
// lines as the Miller loop multiplies by them (ell_vw Py, ell_vv Px; the consumers of
// coeffs expect that form in a BN_LINES_PRESCALED build), 0: the reference's
// coefficients (the G2Precomp export)
constexpr int kPrepareWideLanes = 8;
// BN_LINES_PRESCALED: the producers store each line as the Miller loop multiplies by it
// (ell_0, ell_vw * Py, ell_vv * Px; mod.rs:589), so k_miller_seg / k_miller apply it
// without scaling, and the latency kernel's producer writes it to its ring that way
// (lines_wide.h PwEll: the eight-lane steps take the two P products in slots their
// layers left duplicated); `scale` = 0 keeps the reference's G2Precomp coefficients
// (the bn_g2_precompute export).  0: the consumers scale.
#ifndef BN_LINES_PRESCALED
#define BN_LINES_PRESCALED 1
#endif
__global__ void __launch_bounds__(kPairBlock) k_prepare_wide(const bn_g1* __restrict__ p, const bn_g2* __restrict__ q,
                                                         size_t n, uint32_t* __restrict__ coeffs,
                                                         uint32_t* __restrict__ paff, uint8_t* __restrict__ flags,
                                                         int* __restrict__ err, int mode, int scale);
__global__ void __launch_bounds__(kBlock) k_coeffs_store(const uint32_t* __restrict__ coeffs, size_t n,
                                                         bn_fq2* __restrict__ out);
__global__ void __launch_bounds__(kPairBlock) k_pairing_fused(const bn_g1* __restrict__ p, const bn_g2* __restrict__ q,
                                                          size_t n, uint8_t* __restrict__ flags, int* __restrict__ err,
                                                          int mode, uint32_t* __restrict__ f_out);
__global__ void __launch_bounds__(kBlock) k_miller(const uint32_t* __restrict__ coeffs, const uint32_t* __restrict__ paff,
                         const uint8_t* __restrict__ flags, size_t n, uint32_t* __restrict__ f_out);
__global__ void __launch_bounds__(kPairBlock) k_fq12_vm(const uint32_t* __restrict__ prog, int nsteps, uint32_t* slots, size_t n);
__global__ void __launch_bounds__(kPairBlock) k_pairing_full(const bn_g1* __restrict__ p, const bn_g2* __restrict__ q,
                                                          size_t n, const uint32_t* __restrict__ prog, int nsteps,
                                                          uint32_t* __restrict__ slots, bn_gt* __restrict__ out,
                                                          int* __restrict__ err);
__global__ void __launch_bounds__(kBlock) k_fe_out(const uint32_t* __restrict__ slots, size_t n, int out_slot, const uint8_t* __restrict__ flags,
                         bn_gt* __restrict__ out, uint8_t* __restrict__ ok, int* __restrict__ err);
// kernels_wide.hip (fq12_wide.h): final exponentiation and product reduction on 16-lane groups
__global__ void __launch_bounds__(kBlock) k_fe_wide(const uint32_t* __restrict__ f, size_t stride, size_t n,
                                                    bn_gt* __restrict__ out, uint8_t* __restrict__ ok,
                                                    int* __restrict__ err, int duo);
__global__ void __launch_bounds__(kBlock) k_fq12_reduce_wide(const uint32_t* __restrict__ in, size_t in_stride,
                                                             SetSpan sets, uint32_t* __restrict__ out,
                                                             size_t out_stride, size_t out_base, size_t out_set, int per_group);
// kernels_tail.hip: k_horner_tree's recombination + final exponentiation of ONE
// product, the final exponentiation's squarer on a pair of 16-lane groups (w12_cyc32)
constexpr int kTailBlock = 256;
__global__ void __launch_bounds__(kTailBlock) k_horner_tree2(const uint32_t* __restrict__ g, SegPlan plan, int do_fe,
                                                             bn_gt* __restrict__ out, int* __restrict__ err,
                                                             const uint32_t* __restrict__ zf);
// words of the workspace region behind zf: the zero flags and the channel between
// k_horner_tree2's squarer and multiplier blocks (fq12_ds.h DsChan)
constexpr int kTailChanWords = 1024 + 2 * 128 * 88;
// pairing_batch with several segments: one block per segment runs the first chunk of
// the final exponentiation and the segment's Horner squarings (digit-sliced, fq12_ds.h)
// in place, zf[s] = segment s's value is zero; then k_horner_tree2 with zf on two
// blocks (the final exponentiation's squarer and multiplier)
__global__ void __launch_bounds__(kTailBlock) k_seg_fe1(uint32_t* __restrict__ g, SegPlan plan,
                                                        uint32_t* __restrict__ zf);
// pairing_batch's whole tail in one launch of max(S, 3) blocks (k_seg_fe1, the
// segments' product as a chain of nodes completed by whichever block arrives second,
// the last chunk on the squarer and two multipliers): ws = bn_ctx.tail_ws, every word
// it polls stamped with `epoch` (1 .. 2^29 - 1, a new one per launch)
constexpr int kTailWsWords = kTailChanWords + 2 * kMaxSeg * 256;
__global__ void __launch_bounds__(kTailBlock) k_seg_tail(const uint32_t* __restrict__ g, SegPlan plan,
                                                         bn_gt* __restrict__ out, int* __restrict__ err,
                                                         uint32_t* __restrict__ ws, uint32_t epoch);
// pairing_many's final exponentiations of n <= kFeDsMax Miller values (split layout,
// stride n) on `per` blocks per pair (3: squarer + two multiplier candidates, 1: the
// squarer alone; digit-sliced) into out[0..n); ws = bn_ctx.fe_ds_ws (kFeDsWords per pair,
// zeroed at creation)
constexpr int kFeDsMax = 256;
constexpr int kFeDsWords = kTailChanWords;  // role word (kernels_tail.hip kRoleWord) + channel
__global__ void __launch_bounds__(kTailBlock) k_fe_ds(const uint32_t* __restrict__ f, size_t n,
                                                      bn_gt* __restrict__ out, uint8_t* __restrict__ ok,
                                                      int* __restrict__ err, uint32_t* __restrict__ ws,
                                                      uint32_t epoch, int per);
// kernels_wide.hip: the whole pairing of kLatPairs pairs per block in one launch
// (a producer wave for the lines, consumer groups for the wide Miller loop + FE)
constexpr int kLatPairs = 8;
#ifndef BN_FE_DUO
#define BN_FE_DUO 1  // the latency kernels' final exponentiation on two groups (fq12_wide.h)
#endif
// one producer wave, two consumer waves (+ with BN_FE_DUO a wave of multiplier groups)
constexpr int kLatThreads = 64 + kLatPairs * 16 + (BN_FE_DUO ? 64 : 0);
// k_fe_wide / k_horner_wide: the two-group final exponentiation (8 elements per
// block) while the blocks fit one round on the 256 CUs (the channel makes it one
// block per CU); above, one group per element (16 per block)
constexpr size_t kWideDuoMax = 2048;
inline bool wide_duo(size_t n) { return BN_FE_DUO && n <= kWideDuoMax; }
inline unsigned wide_blocks(size_t n) { return (unsigned)(wide_duo(n) ? (n + 7) / 8 : (n + 15) / 16); }
__global__ void __launch_bounds__(kLatThreads) k_pairing_latency(const bn_g1* __restrict__ p,
                                                                 const bn_g2* __restrict__ q, size_t n,
                                                                 bn_gt* __restrict__ out, uint32_t* __restrict__ f_out,
                                                                 int mode, int* __restrict__ err);
// the same kernel built for two waves per SIMD (kernels_latency_w2.hip)
__global__ void __launch_bounds__(kLatThreads) __attribute__((amdgpu_waves_per_eu(2, 2)))
k_pairing_latency_w2(const bn_g1* __restrict__ p, const bn_g2* __restrict__ q, size_t n, bn_gt* __restrict__ out,
                     uint32_t* __restrict__ f_out, int mode, int* __restrict__ err);
__global__ void __launch_bounds__(kBlock) k_err_status(const int* __restrict__ err, int* __restrict__ status);
__global__ void __launch_bounds__(kBlock) k_gt_load(const bn_gt* __restrict__ g, size_t n, uint32_t* __restrict__ f);
__global__ void __launch_bounds__(kBlock) k_gt_store(const uint32_t* __restrict__ f, size_t n, size_t stride, bn_gt* __restrict__ g);
__global__ void __launch_bounds__(kPairBlock) k_g1_mul(const bn_g1* __restrict__ p, const bn_fr* __restrict__ k, size_t n, bn_g1* __restrict__ out);
__global__ void __launch_bounds__(kPairBlock) k_g1_mul2(const bn_g1* __restrict__ p, const bn_fr* __restrict__ k, size_t n, bn_g1* __restrict__ out);
__global__ void BN_PATH_ATTR __launch_bounds__(kPairBlock) k_g2_mul_split(const bn_g2* __restrict__ p, const bn_fr* __restrict__ k, size_t n, bn_g2* __restrict__ out);
// the group law (kernels_group.hip): op codes of k_g1_op / k_g2_op (b may be null for neg / normalize)
enum GroupOp { kGroupAdd = 0, kGroupSub = 1, kGroupNeg = 2, kGroupNormalize = 3, kGroupEq = 4 };
__global__ void __launch_bounds__(kBlock) k_g1_op(int op, const bn_g1* a, const bn_g1* b, size_t n, bn_g1* out,
                                                  uint8_t* __restrict__ eq);
__global__ void __launch_bounds__(kBlock) k_g2_op(int op, const bn_g2* a, const bn_g2* b, size_t n, bn_g2* out,
                                                  uint8_t* __restrict__ eq);
__global__ void __launch_bounds__(kPairBlock) k_gt_pow(const bn_gt* __restrict__ a, const bn_fr* __restrict__ k, size_t n,
                                                   bn_gt* __restrict__ out, uint32_t* __restrict__ ws);
// kernels_codec.hip (codec.h): encodings, square roots, validation, decompression
__global__ void __launch_bounds__(kBlock) k_fq_from_slice(const uint8_t* __restrict__ be, size_t n, bn_fq* __restrict__ out, uint8_t* __restrict__ st);
__global__ void __launch_bounds__(kBlock) k_fq_to_be(const bn_fq* __restrict__ a, size_t n, uint8_t* __restrict__ be);
__global__ void __launch_bounds__(kBlock) k_fq2_from_slice(const uint8_t* __restrict__ be, size_t n, bn_fq2* __restrict__ out, uint8_t* __restrict__ st);
__global__ void __launch_bounds__(kBlock) k_fr_from_slice(const uint8_t* __restrict__ be, size_t n, bn_fr* __restrict__ out);
__global__ void __launch_bounds__(kBlock) k_fr_to_be(const bn_fr* __restrict__ a, size_t n, uint8_t* __restrict__ be);
__global__ void __launch_bounds__(kBlock) k_fq_sqrt(const bn_fq* __restrict__ a, size_t n, bn_fq* __restrict__ out, uint8_t* __restrict__ ok);
__global__ void __launch_bounds__(kBlock) k_fq2_sqrt(const bn_fq2* __restrict__ a, size_t n, bn_fq2* __restrict__ out, uint8_t* __restrict__ ok);
__global__ void __launch_bounds__(kBlock) k_g1_affine_new(const bn_fq* __restrict__ x, const bn_fq* __restrict__ y, size_t n, bn_g1* __restrict__ out, uint8_t* __restrict__ st);
__global__ void __launch_bounds__(kBlock) k_g2_affine_new(const bn_fq2* __restrict__ x, const bn_fq2* __restrict__ y, size_t n, bn_g2* __restrict__ out, uint8_t* __restrict__ st);
__global__ void __launch_bounds__(kBlock) k_g1_from_compressed(const uint8_t* __restrict__ b, size_t n, bn_g1* __restrict__ out, uint8_t* __restrict__ st);
__global__ void __launch_bounds__(kBlock) k_g2_from_compressed(const uint8_t* __restrict__ b, size_t n, bn_g2* __restrict__ out, uint8_t* __restrict__ st);

}  // namespace bn
