// kernels_codec.hip -- batched encodings, square roots, point validation and
// decompression (codec.h), one lane per element.  Invalid elements get an
// all-zero output image and their status (bn_elem_status).
#include "codec.h"
#include "kernels.h"

namespace bn {

// 32 big-endian bytes (32-byte aligned records) <-> little-endian words
__device__ __forceinline__ void ld_be32(const uint8_t* src, uint32_t w[8]) {
    const uint4* s = reinterpret_cast<const uint4*>(src);
    const uint4 a = s[0], b = s[1];
    const uint32_t raw[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
    for (int i = 0; i < 8; ++i) w[i] = __builtin_bswap32(raw[7 - i]);
}
__device__ __forceinline__ void st_be32(uint8_t* dst, const uint32_t w[8]) {
    uint32_t raw[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) raw[i] = __builtin_bswap32(w[7 - i]);
    uint4* d = reinterpret_cast<uint4*>(dst);
    d[0] = make_uint4(raw[0], raw[1], raw[2], raw[3]);
    d[1] = make_uint4(raw[4], raw[5], raw[6], raw[7]);
}
__device__ __forceinline__ void zero_fq(bn_fq& a) {
    const uint32_t z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    st_words(&a, z);
}

// Fq::from_slice (lib.rs:154-159)
__global__ void __launch_bounds__(kBlock) k_fq_from_slice(const uint8_t* __restrict__ be, size_t n, bn_fq* __restrict__ out,
                                                          uint8_t* __restrict__ st) {
    fold_table_init();
    const size_t i = lane_id();
    if (i >= n) return;
    uint32_t w[8];
    ld_be32(be + 32 * i, w);
    Fq<2> x;
    const bool ok = fq_new_plain(w, x);
    st[i] = ok ? ST_OK : ST_FIELD_NOT_MEMBER;
    if (ok) st_ref(out[i], x); else zero_fq(out[i]);
}
// Fq::to_big_endian (lib.rs:160-170): the canonical integer
__global__ void __launch_bounds__(kBlock) k_fq_to_be(const bn_fq* __restrict__ a, size_t n, uint8_t* __restrict__ be) {
    fold_table_init();
    const size_t i = lane_id();
    if (i >= n) return;
    uint32_t w[8];
    fq_plain_words(ld_ref(a[i]), w);
    st_be32(be + 32 * i, w);
}
// Fq2::from_slice (lib.rs:260-267)
__global__ void __launch_bounds__(kBlock) k_fq2_from_slice(const uint8_t* __restrict__ be, size_t n, bn_fq2* __restrict__ out,
                                                           uint8_t* __restrict__ st) {
    fold_table_init();
    const size_t i = lane_id();
    if (i >= n) return;
    uint32_t v[16];
    ld_be32(be + 64 * i + 32, v);  // low half of the U512
    ld_be32(be + 64 * i, v + 8);
    Fq2<2> x;
    const bool ok = fq2_from_u512(v, x);
    st[i] = ok ? ST_OK : ST_FIELD_NOT_MEMBER;
    if (ok) {
        st_ref2(out[i], x);
    } else {
        zero_fq(out[i].c0);
        zero_fq(out[i].c1);
    }
}
// Fr::from_slice (lib.rs:45-49: new_mul_factor, reduces mod r)
__global__ void __launch_bounds__(kBlock) k_fr_from_slice(const uint8_t* __restrict__ be, size_t n, bn_fr* __restrict__ out) {
    fold_table_init();
    const size_t i = lane_id();
    if (i >= n) return;
    uint32_t w[8], m[8];
    ld_be32(be + 32 * i, w);
    fr_from_plain_words(w, m);
    st_words(reinterpret_cast<bn_fq*>(&out[i]), m);
}
// Fr::to_big_endian (lib.rs:50-55): the RAW Montgomery image, as the reference writes it
__global__ void __launch_bounds__(kBlock) k_fr_to_be(const bn_fr* __restrict__ a, size_t n, uint8_t* __restrict__ be) {
    fold_table_init();
    const size_t i = lane_id();
    if (i >= n) return;
    uint32_t w[8];
    ld_words(reinterpret_cast<const bn_fq*>(&a[i]), w);
    st_be32(be + 32 * i, w);
}

// Fq::sqrt / Fq2::sqrt (fp.rs:245-260, fq2.rs:208-224); ok[i] = 0 for None
__global__ void __launch_bounds__(kBlock) k_fq_sqrt(const bn_fq* __restrict__ a, size_t n, bn_fq* __restrict__ out,
                                                    uint8_t* __restrict__ ok) {
    fold_table_init();
    const size_t i = lane_id();
    if (i >= n) return;
    Fq<2> r;
    const bool some = fq_sqrt(ld_ref(a[i]), r);
    ok[i] = some;
    if (some) st_ref(out[i], r); else zero_fq(out[i]);
}
__global__ void __launch_bounds__(kBlock) k_fq2_sqrt(const bn_fq2* __restrict__ a, size_t n, bn_fq2* __restrict__ out,
                                                     uint8_t* __restrict__ ok) {
    fold_table_init();
    const size_t i = lane_id();
    if (i >= n) return;
    Fq2<kPt> r;
    const bool some = fq2_sqrt(ld_ref2(a[i]), r);
    ok[i] = some;
    if (some) {
        st_ref2(out[i], r);
    } else {
        zero_fq(out[i].c0);
        zero_fq(out[i].c1);
    }
}

// AffineG::new (mod.rs:95-113) -> to_jacobian (mod.rs:220-226)
__global__ void __launch_bounds__(kBlock) k_g1_affine_new(const bn_fq* __restrict__ x, const bn_fq* __restrict__ y, size_t n,
                                                          bn_g1* __restrict__ out, uint8_t* __restrict__ st) {
    fold_table_init();
    const size_t i = lane_id();
    if (i >= n) return;
    const Fq<2> X = ld_ref(x[i]), Y = ld_ref(y[i]);
    const bool ok = g1_on_curve(X, Y);
    st[i] = ok ? ST_OK : ST_GROUP_NOT_ON_CURVE;
    if (ok) {
        st_ref(out[i].x, X);
        st_ref(out[i].y, Y);
        st_ref(out[i].z, fq_one());
    } else {
        zero_fq(out[i].x);
        zero_fq(out[i].y);
        zero_fq(out[i].z);
    }
}
template <int B>
__device__ __forceinline__ void st_g2_affine(bn_g2& o, const Fq2<B>& x, const Fq2<B>& y, bool ok) {
    if (ok) {
        st_ref2(o.x, x);
        st_ref2(o.y, y);
        st_ref2(o.z, fq2_one());
    } else {
        const uint32_t z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        bn_fq* f = &o.x.c0;
#pragma unroll
        for (int k = 0; k < 6; ++k) st_words(f + k, z);
    }
}
__global__ void __launch_bounds__(kBlock) k_g2_affine_new(const bn_fq2* __restrict__ x, const bn_fq2* __restrict__ y, size_t n,
                                                          bn_g2* __restrict__ out, uint8_t* __restrict__ st) {
    fold_table_init();
    const size_t i = lane_id();
    if (i >= n) return;
    const Fq2<kPt> X = widen<kPt>(ld_ref2(x[i])), Y = widen<kPt>(ld_ref2(y[i]));
    const bool on = g2_on_curve(X, Y);
    const bool in = g2_in_subgroup(X, Y);
    const uint8_t s = !on ? ST_GROUP_NOT_ON_CURVE : !in ? ST_GROUP_NOT_IN_SUBGROUP : ST_OK;
    st[i] = s;
    st_g2_affine(out[i], X, Y, s == ST_OK);
}

// G1::from_compressed / G2::from_compressed (lib.rs:359-375, 506-526); records of 33 / 65 bytes
__global__ void __launch_bounds__(kBlock) k_g1_from_compressed(const uint8_t* __restrict__ b, size_t n, bn_g1* __restrict__ out,
                                                               uint8_t* __restrict__ st) {
    fold_table_init();
    const size_t i = lane_id();
    if (i >= n) return;
    uint8_t rec[33];
#pragma unroll
    for (int k = 0; k < 33; ++k) rec[k] = b[33 * i + k];
    Fq<2> x, y;
    const uint8_t s = g1_decompress(rec, x, y);
    st[i] = s;
    if (s == ST_OK) {
        st_ref(out[i].x, x);
        st_ref(out[i].y, y);
        st_ref(out[i].z, fq_one());
    } else {
        zero_fq(out[i].x);
        zero_fq(out[i].y);
        zero_fq(out[i].z);
    }
}
__global__ void __launch_bounds__(kBlock) k_g2_from_compressed(const uint8_t* __restrict__ b, size_t n, bn_g2* __restrict__ out,
                                                               uint8_t* __restrict__ st) {
    fold_table_init();
    const size_t i = lane_id();
    if (i >= n) return;
    uint8_t rec[65];
#pragma unroll
    for (int k = 0; k < 65; ++k) rec[k] = b[65 * i + k];
    Fq2<kPt> x, y;
    const uint8_t s = g2_decompress(rec, x, y);
    st[i] = s;
    st_g2_affine(out[i], x, y, s == ST_OK);
}

}  // namespace bn

BN_EXPORT_FOLD_CHECK(codec)
