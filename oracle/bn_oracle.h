/*
 * bn_oracle.h -- CPU restatement of substrate-bn 0.6.0 (risc0/paritytech-bn).
 *
 * TEST INFRASTRUCTURE ONLY.  This is the parity oracle and the CPU baseline
 * ("kind": "port") for the MI355X pairing engine.  Only tests/, the smoke()
 * entry of __graft_entry__.py and bench.py's cpu_baseline leg may load it.
 * The product library (libbn254mi.so) never links or calls it.
 *
 * All values use the reference's memory image: an Fq/Fr is 32 bytes, the
 * canonical Montgomery residue a*2^256 mod m as four little-endian u64 limbs
 * (== U256([u128;2]) of src/arith.rs:9-11 on x86_64).
 *
 * Parity is pinned: tests/test_oracle.py checks this restatement against every
 * known-answer vector the reference's own tests hold for the pairing path
 * (src/groups/mod.rs:643-691, 780-892, 929-999; src/fields/mod.rs:94-344).
 */
#ifndef BN_ORACLE_H
#define BN_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct { uint64_t l[4]; } orc_fe;          /* Fq or Fr, Montgomery  */
typedef struct { orc_fe c0, c1; } orc_fq2;
typedef struct { orc_fq2 c0, c1, c2; } orc_fq6;
typedef struct { orc_fq6 c0, c1; } orc_fq12;       /* 384 B, == Gt          */
typedef struct { orc_fe x, y, z; } orc_g1;         /* Jacobian, 96 B        */
typedef struct { orc_fq2 x, y, z; } orc_g2;        /* Jacobian, 192 B       */
typedef struct { orc_fq2 x, y; } orc_g2_affine;
typedef struct { orc_fq2 ell_0, ell_vw, ell_vv; } orc_ell_coeffs;

#define ORC_NUM_COEFFS 87

/* ---- Fq / Fr element ops (src/fields/fp.rs, src/arith.rs) ---- */
/* field: 0 = Fq, 1 = Fr */
void orc_fe_from_canonical(int field, const orc_fe* a, orc_fe* out); /* Fp::new  */
void orc_fe_to_canonical(int field, const orc_fe* a, orc_fe* out);   /* U256::from(Fp) */
void orc_fe_add(int field, const orc_fe* a, const orc_fe* b, orc_fe* out);
void orc_fe_sub(int field, const orc_fe* a, const orc_fe* b, orc_fe* out);
void orc_fe_mul(int field, const orc_fe* a, const orc_fe* b, orc_fe* out);
void orc_fe_neg(int field, const orc_fe* a, orc_fe* out);
int  orc_fe_inverse(int field, const orc_fe* a, orc_fe* out);       /* 0 ok, 1 zero */

/* ---- tower (src/fields/fq2.rs, fq6.rs, fq12.rs) ---- */
void orc_fq2_mul(const orc_fq2* a, const orc_fq2* b, orc_fq2* out);
void orc_fq2_squared(const orc_fq2* a, orc_fq2* out);
int  orc_fq2_inverse(const orc_fq2* a, orc_fq2* out);
void orc_fq6_mul(const orc_fq6* a, const orc_fq6* b, orc_fq6* out);
void orc_fq6_squared(const orc_fq6* a, orc_fq6* out);
int  orc_fq6_inverse(const orc_fq6* a, orc_fq6* out);
void orc_fq12_mul(const orc_fq12* a, const orc_fq12* b, orc_fq12* out);
void orc_fq12_squared(const orc_fq12* a, orc_fq12* out);
void orc_fq12_add(const orc_fq12* a, const orc_fq12* b, orc_fq12* out);
void orc_fq12_sub(const orc_fq12* a, const orc_fq12* b, orc_fq12* out);
void orc_fq12_neg(const orc_fq12* a, orc_fq12* out);
int  orc_fq12_inverse(const orc_fq12* a, orc_fq12* out);
void orc_fq12_frobenius_map(const orc_fq12* a, int power, orc_fq12* out);
void orc_fq12_cyclotomic_squared(const orc_fq12* a, orc_fq12* out);
void orc_fq12_exp_by_neg_z(const orc_fq12* a, orc_fq12* out);
void orc_fq12_mul_by_024(const orc_fq12* f, const orc_fq2* ell_0, const orc_fq2* ell_vw,
                         const orc_fq2* ell_vv, orc_fq12* out);
void orc_fq12_pow(const orc_fq12* a, const orc_fe* exp_canonical, orc_fq12* out);
int  orc_final_exponentiation(const orc_fq12* f, orc_fq12* out);   /* 0 ok, 1 f==0 */

/* ---- groups (src/groups/mod.rs) ---- */
void orc_g1_one(orc_g1* out);
void orc_g2_one(orc_g2* out);
void orc_g1_add(const orc_g1* a, const orc_g1* b, orc_g1* out);
void orc_g1_double(const orc_g1* a, orc_g1* out);
void orc_g1_neg(const orc_g1* a, orc_g1* out);
void orc_g1_mul(const orc_g1* p, const orc_fe* fr_mont, orc_g1* out);
int  orc_g1_eq(const orc_g1* a, const orc_g1* b);
int  orc_g1_to_affine(const orc_g1* p, orc_fe* x, orc_fe* y);       /* 0 ok, 1 zero */
void orc_g2_add(const orc_g2* a, const orc_g2* b, orc_g2* out);
void orc_g2_double(const orc_g2* a, orc_g2* out);
void orc_g2_neg(const orc_g2* a, orc_g2* out);
void orc_g2_mul(const orc_g2* p, const orc_fe* fr_mont, orc_g2* out);
int  orc_g2_eq(const orc_g2* a, const orc_g2* b);
int  orc_g2_to_affine(const orc_g2* p, orc_g2_affine* out);
int  orc_g1_on_curve_affine(const orc_fe* x, const orc_fe* y);

/* ---- pairing path ---- */
void orc_g2_precompute(const orc_g2_affine* q, orc_ell_coeffs out[ORC_NUM_COEFFS]);
void orc_miller_loop(const orc_ell_coeffs c[ORC_NUM_COEFFS], const orc_fe* px,
                     const orc_fe* py, orc_fq12* out);
void orc_pairing(const orc_g1* p, const orc_g2* q, orc_fq12* out);
void orc_pairing_batch(const orc_g1* p, const orc_g2* q, size_t n, orc_fq12* out);
int  orc_miller_loop_batch(const orc_g2* q, const orc_g1* p, size_t n, orc_fq12* out);

/* ---- multi-threaded batch helpers (CPU baseline) ---- */
void orc_pairing_many(const orc_g1* p, const orc_g2* q, size_t n, orc_fq12* out, int nthreads);
void orc_g1_mul_many(const orc_g1* p, const orc_fe* k, size_t n, orc_g1* out, int nthreads);
void orc_g2_mul_many(const orc_g2* p, const orc_fe* k, size_t n, orc_g2* out, int nthreads);
/* pairing_batch with the shared loop split over threads (same result as orc_pairing_batch) */
void orc_pairing_batch_mt(const orc_g1* p, const orc_g2* q, size_t n, orc_fq12* out, int nthreads);


/* ---- encodings / validation / decompression / Gt::pow ----
 * per-element status, same values as bn_elem_status in include/bn254mi.h */
enum {
    ORC_OK = 0,
    ORC_FIELD_INVALID_SLICE_LENGTH = 1, /* FieldError::InvalidSliceLength (lib.rs:99-104) */
    ORC_FIELD_INVALID_U512 = 2,         /* FieldError::InvalidU512Encoding */
    ORC_FIELD_NOT_MEMBER = 3,           /* FieldError::NotMember */
    ORC_CURVE_INVALID_ENCODING = 4,     /* CurveError::InvalidEncoding (lib.rs:106-112) */
    ORC_CURVE_NOT_MEMBER = 5,           /* CurveError::NotMember */
    ORC_GROUP_NOT_ON_CURVE = 6,         /* groups::Error::NotOnCurve (mod.rs:89-92) */
    ORC_GROUP_NOT_IN_SUBGROUP = 7       /* groups::Error::NotInSubgroup */
};
int  orc_fq_from_slice(const uint8_t* be32, orc_fe* out);
void orc_fq_to_big_endian(const orc_fe* a, uint8_t* be32);
int  orc_fq2_from_slice(const uint8_t* be64, orc_fq2* out);
void orc_fr_from_slice(const uint8_t* be32, orc_fe* out);
void orc_fr_to_big_endian(const orc_fe* a, uint8_t* be32);
int  orc_u512_divrem(const uint8_t* be64, orc_fe* q, orc_fe* r);
int  orc_fq_sqrt(const orc_fe* a, orc_fe* out);                   /* 0 Some, 1 None */
int  orc_fq2_sqrt(const orc_fq2* a, orc_fq2* out);
int  orc_g1_affine_new(const orc_fe* x, const orc_fe* y, orc_g1* out);
int  orc_g2_affine_new(const orc_fq2* x, const orc_fq2* y, orc_g2* out);
int  orc_g1_from_compressed(const uint8_t* bytes, size_t len, orc_g1* out);
int  orc_g2_from_compressed(const uint8_t* bytes, size_t len, orc_g2* out);
void orc_gt_pow(const orc_fq12* a, const orc_fe* fr_mont, orc_fq12* out);
/* kind 0: G1 compressed (33 B), 1: G2 compressed (65 B), 2: G2 affine (x, y) validation */
void orc_decode_many(int kind, const uint8_t* in, size_t n, void* out, uint8_t* status, int nthreads);

#ifdef __cplusplus
}
#endif
#endif
