// ctx.h -- the bn_ctx behind the C ABI (host side, shared by capi.hip and
// capi_multi.hip).  Not a public header.
#pragma once
#include <hip/hip_runtime.h>

#include <array>
#include <mutex>
#include <string>
#include <vector>

struct bn_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    std::mutex mu;
    // last error message; a multi-device context's host-buffer calls write it
    // without holding `mu` (their sub-contexts do the locking), so writes there
    // take err_mu
    std::mutex err_mu;
    std::string err;
    // workspace (device)
    size_t cap = 0;  // pairings
    uint32_t* coeffs = nullptr;
    uint32_t* paff = nullptr;
    uint32_t* slots = nullptr;  // Fq12 slots of the step machine; slot 0 = Miller values
    uint8_t* flags = nullptr;
    uint32_t* d_prog = nullptr; // final-exponentiation step program
    // optional per-phase timing of bn_pairing_many_dev (HIP events on the launch stream)
    bool timing = false;
    std::vector<hipEvent_t> ev_pool;
    std::vector<std::array<hipEvent_t, 5>> ev_marks;
    int fe_steps = 0;
    int fe_out = 0;
    bool fe_last_out = false;  // the program's last step writes fe_out (k_pairing_full)
    // batches of at most this many elements run the final exponentiation on the
    // wide layout (kernels_wide.hip, 16 lanes per element: latency) instead of
    // the step machine (k_fq12_vm, 2 lanes per element: throughput)
    size_t fe_wide_max = 0;
    // A/B switch ($BN254MI_MILLER_FORM) for bn_pairing_many_dev batches above the
    // wide threshold: 1 (default, measured fastest) = to_affine,
    // line steps and Miller loop fused in one kernel (k_pairing_fused, no
    // coefficient traffic); 0 = k_prepare (line coefficients to HBM) + k_miller;
    // 2 = k_prepare + k_miller_seg with one segment
    int miller_form = 3;  // 3: k_pairing_full; 1: k_pairing_fused + k_fq12_vm + k_fe_out; 0/2: k_prepare + k_miller(_seg) + ...
    // bn_pairing_many_dev batches of at most this many pairs run k_pairing_latency
    size_t latency_max = 0;
    bool latency_w2 = true;  // above lat_w1_max pairs the one-launch path runs the two-wave build
    size_t lat_w1_max = 2048;  // CU count x kLatPairs (bn_ctx_create): one round of one-wave blocks
    // batches of at most this many pairs take k_prepare_wide (8 lanes per pair)
    size_t prepare_wide_max = 0;
    int* d_err = nullptr;
    // pairing_batch's one-launch tail (kernels_tail.hip k_seg_tail): its own words
    // (kTailWsWords, zeroed at creation), every word it polls stamped with the
    // launch's epoch, so no clearing between products
    uint32_t* tail_ws = nullptr;
    uint32_t tail_epoch = 0;
    // pairing_many of at most fe_ds_max pairs: k_pairing_latency's Miller values, then
    // k_fe_ds (three digit-sliced blocks per pair); its words (kFeDsMax pairs, zeroed)
    uint32_t* fe_ds_ws = nullptr;
    size_t fe_ds_max = 0;
    // staging for host-buffer calls (device)
    size_t stage_bytes = 0;
    void* stage = nullptr;
    // bn_pairing_many's host pipeline (capi.hip): two pinned bounce buffers, the
    // copy streams and the per-buffer events (created with the context);
    // $BN254MI_HOST_PIPELINE: 1 (default) pipeline above one piece, 0 never
    // (pageable A/B form), 2 always
    int host_pipeline = 1;
    size_t host_piece = 0;  // pairs per piece (kHostPiece; $BN254MI_HOST_PIECE, at most kChunk)
    size_t pin_bytes = 0;
    void* pin = nullptr;
    hipStream_t h2d = nullptr, d2h = nullptr;
    hipEvent_t ev_in[2] = {}, ev_comp[2] = {}, ev_out[2] = {};
    // The workspace (coeffs, paff, slots, flags, d_err, stage) is shared by every
    // call on this context.  Host-side, the mutex serializes the calls; device-side,
    // every workspace user records ws_event on its stream when it has enqueued its
    // work, and the next user's stream waits on that event first (WsUse), so _dev
    // calls on different caller streams run in call order instead of racing on the
    // same buffers.  No caller stream is remembered past its call.
    hipEvent_t ws_event = nullptr;
    bool ws_pending = false;
    // multi-device context (bn_ctx_create_multi): one single-device sub-context
    // per listed device; `device` is -1 and the fields above are unused
    std::vector<bn_ctx*> subs;
    std::vector<int> devices;
    void* comms = nullptr;  // RCCL communicators (capi_multi.hip), created on first use
};


// capi_multi.hip: the multi-device forms of the host-buffer entry points
#include "../../include/bn254mi.h"
#define BN_HIDDEN __attribute__((visibility("hidden")))
extern "C" {  // internal (not in bn254mi.h); C linkage matches their definitions' scope
BN_HIDDEN int bn_multi_pairing_many(bn_ctx* c, const bn_g1* p, const bn_g2* q, size_t n, bn_gt* out);
BN_HIDDEN int bn_multi_pairing_batch(bn_ctx* c, const bn_g1* p, const bn_g2* q, size_t n, bn_gt* out);
BN_HIDDEN int bn_multi_miller_loop_batch(bn_ctx* c, const bn_g2* q, const bn_g1* p, size_t n, bn_gt* out);
BN_HIDDEN int bn_multi_final_exponentiation_many(bn_ctx* c, const bn_gt* f, size_t n, bn_gt* out, uint8_t* ok);
BN_HIDDEN int bn_multi_miller_loop_many(bn_ctx* c, const bn_g1* p, const bn_g2* q, size_t n, bn_gt* out);
BN_HIDDEN int bn_multi_g1_mul_many(bn_ctx* c, const bn_g1* p, const bn_fr* k, size_t n, bn_g1* out);
BN_HIDDEN int bn_multi_g2_mul_many(bn_ctx* c, const bn_g2* p, const bn_fr* k, size_t n, bn_g2* out);
BN_HIDDEN int bn_multi_destroy(bn_ctx* c);
// capi.hip internals used by capi_multi.hip
BN_HIDDEN int bn_internal_miller_product(bn_ctx* c, const bn_g1* p, const bn_g2* q, size_t n, int mode, bn_gt* result);
BN_HIDDEN void bn_internal_gt_one(bn_gt* out);
}
