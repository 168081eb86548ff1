/*
 * bn254mi.h -- C ABI of the MI355X BN254 pairing engine (libbn254mi.so).
 *
 * Drop-in boundary for the batched hot path of risc0/paritytech-bn
 * (crate substrate-bn 0.6.0).  The reference has no FFI; its boundary is the
 * public Rust API in src/lib.rs.  Each entry point below names the reference
 * function it replaces (file:line under /root/reference).  INTEGRATION.md shows
 * the Rust-side `extern "C"` binding a maintainer adds to keep
 * `pairing()/pairing_batch()/miller_loop_batch()/G1 * Fr` source-compatible.
 *
 * Value types are byte-identical to the reference's #[repr(C)] memory images,
 * so Rust slices pass zero-copy:
 *   bn_fq  == fields::Fq  == U256([u128;2]) : canonical x*2^256 mod p, little endian
 *   bn_fr  == fields::Fr  (Montgomery mod r, same layout)
 *   bn_g1  == groups::G1  == G<G1Params>{x,y,z}  (Jacobian; zero is z == 0)
 *   bn_g2  == groups::G2  (Jacobian over Fq2 {c0,c1})
 *   bn_gt  == Gt(Fq12)    12 Fq in order c0.c0.c0, c0.c0.c1, c0.c1.c0, ... c1.c2.c1
 *
 * Every call returns BN_OK (0) or a bn_status code.  Host-buffer calls block
 * until the result is in the caller's buffer (the Rust API is synchronous).
 * *_dev calls take device pointers and enqueue on `stream` (a hipStream_t, or
 * NULL for the context's own stream) without synchronizing.
 */
#ifndef BN254MI_H
#define BN254MI_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct { uint64_t l[4]; } bn_fq;
typedef struct { bn_fq c0, c1; } bn_fq2;
typedef struct { uint64_t l[4]; } bn_fr;
typedef struct { bn_fq x, y, z; } bn_g1;
typedef struct { bn_fq2 x, y, z; } bn_g2;
typedef struct { bn_fq c[12]; } bn_gt;

typedef enum {
    BN_OK = 0,
    BN_ERR_INVALID_ARGUMENT = 1,
    BN_ERR_TO_AFFINE = 2,     /* CurveError::ToAffineConversion (lib.rs:629-630) */
    BN_ERR_FE_ZERO = 3,       /* final exponentiation of zero: fq12.rs:63-72 None; pairing panics (mod.rs:900) */
    BN_ERR_HIP = 4,           /* a HIP runtime error; see bn_last_error() */
    BN_ERR_NO_DEVICE = 5,
    BN_ERR_INTERNAL = 6       /* a device-side hand-off between waves ran out of its wait cap; the result is
                                 not trusted and the call fails (never seen in normal operation) */
} bn_status;

typedef struct bn_ctx bn_ctx;

/* One context per device.  A context may be shared by host threads: each call holds
 * it for its whole duration (staging, kernels, readback).  *_dev calls enqueued on
 * different streams run on the device in call order (the context's workspace is
 * shared; each call's stream waits for the previous call's work).  The reference
 * is reentrant from any thread (lib.rs:303-305, Group: Send + Sync). */
int bn_ctx_create(int device, bn_ctx** out);
int bn_ctx_destroy(bn_ctx* ctx);
const char* bn_last_error(const bn_ctx* ctx);
/* the stream *_dev calls use when given NULL */
void* bn_ctx_stream(bn_ctx* ctx);
/* The sticky device outcome of the *_dev calls without a status word (bn_pairing_many_dev,
 * bn_pairing_many_allgather_dev): synchronizes `stream` (NULL: the context's stream), returns
 * BN_ERR_INTERNAL or BN_ERR_FE_ZERO (a Miller value was zero: the reference panics, mod.rs:900)
 * if any such call since the last bn_dev_status (or host-buffer call, which starts from a clear
 * word) set it, else BN_OK, and clears it.  On a multi-device context it checks every device,
 * each on its own context stream, and `stream` must be NULL (else BN_ERR_INVALID_ARGUMENT). */
int bn_dev_status(bn_ctx* ctx, void* stream);

/* ---- several devices of the node in one process ----
 * A multi-device context shards the host-buffer calls bn_pairing_many,
 * bn_final_exponentiation_many, bn_miller_loop_many, bn_g1_mul_many and
 * bn_g2_mul_many contiguously (device k takes bn_shard_range(n, D, k)), runs the
 * shards concurrently and writes each into the caller's output: the same bytes
 * as one device.  bn_pairing_batch / bn_miller_loop_batch reduce each shard to
 * one Miller value, multiply the partials on the first device in device order
 * (pairing_batch then runs one final exponentiation): the reference's shared
 * loop value exactly (mod.rs:609-640).  Other calls need a single-device
 * context: bn_ctx_device(ctx, k) returns device k's (owned by ctx). */
int bn_ctx_create_multi(const int* devices, int ndev, bn_ctx** out);
int bn_ctx_num_devices(const bn_ctx* ctx);
bn_ctx* bn_ctx_device(bn_ctx* ctx, int k);
/* [*lo, *hi) = shard k of n elements over ndev devices: [k*n/ndev, (k+1)*n/ndev) */
void bn_shard_range(size_t n, int ndev, int k, size_t* lo, size_t* hi);
/* BASELINE config 4 in one process: device k computes out = pairing(d_p[k][i], d_q[k][i])
 * for its n_per_dev HBM-resident pairs, then one RCCL all-gather over xGMI leaves
 * every d_out[k] (ndev * n_per_dev Gt on device k) holding all results in device
 * order.  streams[k] (or NULL / a NULL array: the device context's stream) orders
 * the work on device k.  RCCL (librccl.so.1) is loaded on first use. */
int bn_pairing_many_allgather_dev(bn_ctx* ctx, const bn_g1* const* d_p, const bn_g2* const* d_q, size_t n_per_dev,
                                  bn_gt* const* d_out, void* const* streams);

/* ---- pairing path (src/groups/mod.rs:894-926, src/lib.rs:611-633) ---- */

/* out[i] = pairing(p[i], q[i]) for i < n                     (lib.rs:611-613, mod.rs:894-902)
 * Zero input point -> Gt::one().  BN_ERR_FE_ZERO if a Miller value is 0 (the reference panics). */
int bn_pairing_many(bn_ctx* ctx, const bn_g1* p, const bn_g2* q, size_t n, bn_gt* out);
int bn_pairing_many_dev(bn_ctx* ctx, const bn_g1* d_p, const bn_g2* d_q, size_t n, bn_gt* d_out, void* stream);

/* *out = pairing_batch(&[(p[i], q[i])])                       (lib.rs:615-623, mod.rs:904-926)
 * Pairs with a zero point are skipped; n == 0 or all skipped -> Gt::one(). */
int bn_pairing_batch(bn_ctx* ctx, const bn_g1* p, const bn_g2* q, size_t n, bn_gt* out);

/* *out = miller_loop_batch(&[(q[i], p[i])]) -- note the (G2, G1) order (lib.rs:625-633,
 * mod.rs:609-640).  No final exponentiation.  BN_ERR_TO_AFFINE if any point is zero. */
int bn_miller_loop_batch(bn_ctx* ctx, const bn_g2* q, const bn_g1* p, size_t n, bn_gt* out);

/* Device-pointer forms (BASELINE config 5 with HBM-resident inputs): *d_out (one Gt
 * on the device) = pairing_batch / miller_loop_batch of the n pairs, enqueued on
 * `stream` without synchronizing.  The per-pair Miller values are reduced on the
 * device (kernels_wide.hip) and pairing_batch's one final exponentiation runs on
 * a 16-lane group.  Outcomes that depend on the data are written to *d_status
 * (a device int, may be NULL) when the work completes: BN_OK, BN_ERR_TO_AFFINE
 * (miller_loop_batch: a zero point, lib.rs:629-630; *d_out is then unspecified)
 * or BN_ERR_FE_ZERO (pairing_batch: the reference panics; *d_out is zero). */
int bn_pairing_batch_dev(bn_ctx* ctx, const bn_g1* d_p, const bn_g2* d_q, size_t n, bn_gt* d_out, int* d_status,
                         void* stream);
int bn_miller_loop_batch_dev(bn_ctx* ctx, const bn_g2* d_q, const bn_g1* d_p, size_t n, bn_gt* d_out,
                             int* d_status, void* stream);

/* out[i] = Gt::final_exponentiation(f[i]) (lib.rs:598-600, fq12.rs:107-110);
 * ok[i] = 0 where f[i] == 0 (the reference returns None), out[i] then zero. */
int bn_final_exponentiation_many(bn_ctx* ctx, const bn_gt* f, size_t n, bn_gt* out, uint8_t* ok);

/* per-pair Miller values G2Precomp::miller_loop (mod.rs:579-607) after to_affine +
 * precompute; a pair with a zero point gives Fq12::one() */
int bn_miller_loop_many(bn_ctx* ctx, const bn_g1* p, const bn_g2* q, size_t n, bn_gt* out);

/* the line coefficients of AffineG2::precompute (mod.rs:701-727) of q[i] after
 * to_affine: out[(i * 87 + k) * 3 + j] = coefficient k's (ell_0, ell_vw, ell_vv)[j]
 * (G2Precomp / EllCoeffs, mod.rs:566-577).  BN_ERR_TO_AFFINE if a q is zero. */
int bn_g2_precompute_many(bn_ctx* ctx, const bn_g2* q, size_t n, bn_fq2* out);

/* ---- group path (src/groups/mod.rs:250-334, lib.rs:425-431) ---- */

/* out[i] = p[i] * k[i]: the reference's double-and-add chain (mod.rs:272-292), so the
 * Jacobian output is bit-identical, not merely an equal point. */
int bn_g1_mul_many(bn_ctx* ctx, const bn_g1* p, const bn_fr* k, size_t n, bn_g1* out);
int bn_g1_mul_many_dev(bn_ctx* ctx, const bn_g1* d_p, const bn_fr* d_k, size_t n, bn_g1* d_out, void* stream);
int bn_g2_mul_many(bn_ctx* ctx, const bn_g2* p, const bn_fr* k, size_t n, bn_g2* out);
int bn_g2_mul_many_dev(bn_ctx* ctx, const bn_g2* d_p, const bn_fr* d_k, size_t n, bn_g2* d_out, void* stream);

/* ---- group law (lib.rs:388-423, 539-574; src/groups/mod.rs:169-216, 294-358) ----
 * Batched forms of the G1 / G2 operators, each lane running the reference's own
 * Jacobian formulas, so the output images are bit-identical (not merely equal points):
 *   add        out = a + b      (mod.rs:294-334: both zero shortcuts, the doubling when a == b)
 *   sub        out = a - b      (mod.rs:352-358: a + (-b))
 *   neg        out = -a         (mod.rs:336-350: zero unchanged, else (x, -y, z))
 *   normalize  out = a.normalize() (lib.rs:391-398: to_affine then to_jacobian, z = one,
 *              mod.rs:199-226; zero unchanged)
 *   eq         eq[i] = (a == b) (PartialEq, mod.rs:169-195: projective equality) as 0 / 1 */
int bn_g1_add_many(bn_ctx* ctx, const bn_g1* a, const bn_g1* b, size_t n, bn_g1* out);
int bn_g1_sub_many(bn_ctx* ctx, const bn_g1* a, const bn_g1* b, size_t n, bn_g1* out);
int bn_g1_neg_many(bn_ctx* ctx, const bn_g1* a, size_t n, bn_g1* out);
int bn_g1_normalize_many(bn_ctx* ctx, const bn_g1* a, size_t n, bn_g1* out);
int bn_g1_eq_many(bn_ctx* ctx, const bn_g1* a, const bn_g1* b, size_t n, uint8_t* eq);
int bn_g2_add_many(bn_ctx* ctx, const bn_g2* a, const bn_g2* b, size_t n, bn_g2* out);
int bn_g2_sub_many(bn_ctx* ctx, const bn_g2* a, const bn_g2* b, size_t n, bn_g2* out);
int bn_g2_neg_many(bn_ctx* ctx, const bn_g2* a, size_t n, bn_g2* out);
int bn_g2_normalize_many(bn_ctx* ctx, const bn_g2* a, size_t n, bn_g2* out);
int bn_g2_eq_many(bn_ctx* ctx, const bn_g2* a, const bn_g2* b, size_t n, uint8_t* eq);
int bn_g1_add_many_dev(bn_ctx* ctx, const bn_g1* d_a, const bn_g1* d_b, size_t n, bn_g1* d_out, void* stream);
int bn_g1_sub_many_dev(bn_ctx* ctx, const bn_g1* d_a, const bn_g1* d_b, size_t n, bn_g1* d_out, void* stream);
int bn_g1_neg_many_dev(bn_ctx* ctx, const bn_g1* d_a, size_t n, bn_g1* d_out, void* stream);
int bn_g1_normalize_many_dev(bn_ctx* ctx, const bn_g1* d_a, size_t n, bn_g1* d_out, void* stream);
int bn_g1_eq_many_dev(bn_ctx* ctx, const bn_g1* d_a, const bn_g1* d_b, size_t n, uint8_t* d_eq, void* stream);
int bn_g2_add_many_dev(bn_ctx* ctx, const bn_g2* d_a, const bn_g2* d_b, size_t n, bn_g2* d_out, void* stream);
int bn_g2_sub_many_dev(bn_ctx* ctx, const bn_g2* d_a, const bn_g2* d_b, size_t n, bn_g2* d_out, void* stream);
int bn_g2_neg_many_dev(bn_ctx* ctx, const bn_g2* d_a, size_t n, bn_g2* d_out, void* stream);
int bn_g2_normalize_many_dev(bn_ctx* ctx, const bn_g2* d_a, size_t n, bn_g2* d_out, void* stream);
int bn_g2_eq_many_dev(bn_ctx* ctx, const bn_g2* d_a, const bn_g2* d_b, size_t n, uint8_t* d_eq, void* stream);

/* ---- Gt / Fq12 element operations (src/fields/fq12.rs) for batched callers and tests ---- */
typedef enum {
    BN_FQ12_MUL = 0,          /* a * b          fq12.rs:319-327 (Gt * Gt, lib.rs:603-609) */
    BN_FQ12_SQR = 1,          /* a^2            fq12.rs:295-303 */
    BN_FQ12_INV = 2,          /* a^-1 (0 -> 0)  fq12.rs:305-313 */
    BN_FQ12_CYC_SQR = 3,      /* cyclotomic_squared fq12.rs:198-247 */
    BN_FQ12_EXP_BY_NEG_Z = 4, /* fq12.rs:121-124 */
    BN_FQ12_FROB1 = 5, BN_FQ12_FROB2 = 6, BN_FQ12_FROB3 = 7 /* fq12.rs:112-119 */
} bn_fq12_op;
int bn_fq12_op_many(bn_ctx* ctx, int op, const bn_gt* a, const bn_gt* b, size_t n, bn_gt* out);

/* ---- encodings, validation, square roots, decompression, Gt::pow ----
 * Batched forms of the reference's per-element API.  Each element gets a status
 * (bn_elem_status) where the reference returns a Result/Option; an element that
 * fails has an all-zero output image.  Byte records are the reference's slices:
 * 32-byte big-endian Fq/Fr, 64-byte big-endian Fq2 (a U512 = c1 * p + c0),
 * 33-byte compressed G1, 65-byte compressed G2, packed back to back.  The host
 * forms copy through the context; the _dev forms take device pointers and
 * enqueue on `stream` (NULL: the context's stream) without synchronizing. */
typedef enum {
    BN_ST_OK = 0,
    BN_ST_FIELD_INVALID_SLICE_LENGTH = 1, /* FieldError::InvalidSliceLength (lib.rs:99-104) */
    BN_ST_FIELD_INVALID_U512 = 2,         /* FieldError::InvalidU512Encoding */
    BN_ST_FIELD_NOT_MEMBER = 3,           /* FieldError::NotMember */
    BN_ST_CURVE_INVALID_ENCODING = 4,     /* CurveError::InvalidEncoding (lib.rs:106-112) */
    BN_ST_CURVE_NOT_MEMBER = 5,           /* CurveError::NotMember */
    BN_ST_GROUP_NOT_ON_CURVE = 6,         /* groups::Error::NotOnCurve (mod.rs:89-92) */
    BN_ST_GROUP_NOT_IN_SUBGROUP = 7       /* groups::Error::NotInSubgroup */
} bn_elem_status;

/* Fq::from_slice (lib.rs:154-159): NotMember unless the value is below p */
int bn_fq_from_slice_many(bn_ctx* ctx, const uint8_t* be32, size_t n, bn_fq* out, uint8_t* status);
/* Fq::to_big_endian (lib.rs:160-170): the canonical integer */
int bn_fq_to_big_endian_many(bn_ctx* ctx, const bn_fq* a, size_t n, uint8_t* be32);
/* Fq2::from_slice (lib.rs:260-267): c0 = v mod p, c1 = v div p; NotMember when v >= p^2 */
int bn_fq2_from_slice_many(bn_ctx* ctx, const uint8_t* be64, size_t n, bn_fq2* out, uint8_t* status);
/* Fr::from_slice (lib.rs:45-49): new_mul_factor, reduces any 256-bit value mod r */
int bn_fr_from_slice_many(bn_ctx* ctx, const uint8_t* be32, size_t n, bn_fr* out);
/* Fr::to_big_endian (lib.rs:50-55): writes the RAW Montgomery image, as the reference does */
int bn_fr_to_big_endian_many(bn_ctx* ctx, const bn_fr* a, size_t n, uint8_t* be32);
/* Fq::sqrt / Fq2::sqrt (fp.rs:245-260, fq2.rs:208-224): ok[i] = 0 where the reference returns None */
int bn_fq_sqrt_many(bn_ctx* ctx, const bn_fq* a, size_t n, bn_fq* out, uint8_t* ok);
int bn_fq2_sqrt_many(bn_ctx* ctx, const bn_fq2* a, size_t n, bn_fq2* out, uint8_t* ok);
/* AffineG1::new / AffineG2::new (lib.rs:413-415, 549-551; mod.rs:95-113) then into G1/G2
 * (to_jacobian, mod.rs:220-226).  G2 includes the order check [r]P == 0. */
int bn_g1_affine_new_many(bn_ctx* ctx, const bn_fq* x, const bn_fq* y, size_t n, bn_g1* out, uint8_t* status);
int bn_g2_affine_new_many(bn_ctx* ctx, const bn_fq2* x, const bn_fq2* y, size_t n, bn_g2* out, uint8_t* status);
int bn_g2_affine_new_many_dev(bn_ctx* ctx, const bn_fq2* d_x, const bn_fq2* d_y, size_t n, bn_g2* d_out,
                              uint8_t* d_status, void* stream);
/* G1::from_compressed (lib.rs:359-375, 33-byte records) and G2::from_compressed
 * (lib.rs:506-526, 65-byte records, includes the G2 order check) */
int bn_g1_from_compressed_many(bn_ctx* ctx, const uint8_t* b33, size_t n, bn_g1* out, uint8_t* status);
int bn_g2_from_compressed_many(bn_ctx* ctx, const uint8_t* b65, size_t n, bn_g2* out, uint8_t* status);
int bn_g1_from_compressed_many_dev(bn_ctx* ctx, const uint8_t* d_b33, size_t n, bn_g1* d_out, uint8_t* d_status,
                                   void* stream);
int bn_g2_from_compressed_many_dev(bn_ctx* ctx, const uint8_t* d_b65, size_t n, bn_g2* d_out, uint8_t* d_status,
                                   void* stream);
/* out[i] = Gt::pow(a[i], k[i]) (lib.rs:592-594; generic Fq12 pow, fields/mod.rs:35-46) */
int bn_gt_pow_many(bn_ctx* ctx, const bn_gt* a, const bn_fr* k, size_t n, bn_gt* out);
int bn_gt_pow_many_dev(bn_ctx* ctx, const bn_gt* d_a, const bn_fr* d_k, size_t n, bn_gt* d_out, void* stream);

/* ---- measurement ---- */
/* enable HIP-event timing of each kernel phase of bn_pairing_many_dev (events are
 * recorded on the launch stream between the kernels) */
int bn_set_phase_timing(bn_ctx* ctx, int enable);
/* Batches of at most n elements take the latency path: bn_pairing_many_dev runs
 * k_pairing_latency (up to bn_set_latency_max pairs) or the segmented Miller loop with
 * the recombination + final exponentiation on 16-lane groups, bn_final_exponentiation_many
 * the 16-lane final exponentiation (kernels_wide.hip); larger batches take the throughput
 * path (k_pairing_full: to_affine, lines, Miller loop and the two-lane final-exponentiation
 * step machine in one launch).  Default 8192 (the measured crossover) or
 * $BN254MI_FE_WIDE_MAX; results are identical either way.  On a multi-device
 * context it applies to every device. */
int bn_set_fe_wide_max(bn_ctx* ctx, size_t n);
/* Within the latency path, bn_pairing_many_dev batches of at most n pairs run the
 * whole pairing in ONE launch (k_pairing_latency: a wave computing the 87 lines of
 * each pair feeds, through an LDS ring, 16-lane groups running the Miller loop and
 * the final exponentiation; above 2,048 pairs its two-wave build, two blocks per CU);
 * larger ones the segmented three-kernel form.  pairing_batch / miller_loop_batch take
 * the same kernel for their Miller values up to n pairs.
 * Default 4096 or $BN254MI_LATENCY_MAX; 0 disables it; results are identical. */
int bn_set_latency_max(bn_ctx* ctx, size_t n);
/* device milliseconds per phase of bn_pairing_many_dev since the last read, per chunk
 * launch set: the default throughput form is one kernel (k_pairing_full) and the
 * latency form one kernel (k_pairing_latency), both timed whole in ms[0] (ms[1..3] = 0);
 * the three-launch forms ($BN254MI_MILLER_FORM 0-2) split it as ms[0] k_prepare or
 * k_pairing_fused, ms[1] k_miller / k_miller_seg, ms[2] k_fq12_vm, ms[3] k_fe_out;
 * the segmented latency path ms[0] k_prepare_wide, ms[1] k_miller_seg, ms[2] k_horner_wide.
 * *launches = launch sets measured */
int bn_get_phase_times(bn_ctx* ctx, float ms[4], int* launches);

/* ---- workspace ---- */
/* device bytes the context holds for a batch of n pairings (allocated on first use) */
size_t bn_workspace_bytes(size_t n);
/* pre-size the context workspace for batches up to n (avoids allocation inside timed loops) */
int bn_reserve(bn_ctx* ctx, size_t n);

#ifdef __cplusplus
}
#endif
#endif
