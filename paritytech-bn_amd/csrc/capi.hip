// capi.hip -- host side of the C ABI (include/bn254mi.h): context, workspace,
// chunking, the final-exponentiation step program, and kernel launches.
#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <array>
#include <initializer_list>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "kernels.h"

using namespace bn;

#include "ctx.h"

namespace {

int fail(bn_ctx* c, int code, const std::string& msg) {
    if (c) c->err = msg;
    return code;
}
#define HIPCHK(ctx, x)                                                                   \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess)                                                            \
            return fail(ctx, BN_ERR_HIP, std::string(#x ": ") + hipGetErrorString(e_)); \
    } while (0)

#define RET_IF(x)              \
    do {                       \
        int r_ = (x);          \
        if (r_) return r_;     \
    } while (0)

// order this call's device work after the workspace's previous user (see bn_ctx)
int ws_acquire(bn_ctx* c, hipStream_t s) {
    if (c->ws_pending) HIPCHK(c, hipStreamWaitEvent(s, c->ws_event, 0));
    return BN_OK;
}
// ... and mark this call's work as the workspace's latest user (scope exit)
struct WsUse {
    bn_ctx* c;
    hipStream_t s;
    ~WsUse() {
        if (hipEventRecord(c->ws_event, s) == hipSuccess) c->ws_pending = true;
    }
};
// before freeing workspace buffers: wait until no queued work can still read them
int ws_drain(bn_ctx* c) {
    if (c->ws_pending) HIPCHK(c, hipEventSynchronize(c->ws_event));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return BN_OK;
}

constexpr int kFeSlots = 32;  // slot 0: Miller value, 1: easy-part result, 2..: temporaries
// batches up to this size take the latency path (segmented Miller loop, Horner
// + final exponentiation on 16-lane groups); measured crossover with the
// throughput path: 8192 pairs 3.58 vs 5.43 ms, 16384 pairs 6.05 vs 5.43 ms
// (profiles/r2j_latency_sweep.jsonl).  BN254MI_FE_WIDE_MAX or bn_set_fe_wide_max override.
constexpr size_t kFeWideMaxDefault = 8192;
// batches up to this size run the one-launch latency kernel (k_pairing_latency:
// a line-producer wave feeding the wide Miller loop and final exponentiation);
// BN254MI_LATENCY_MAX or bn_set_latency_max override (0: never)
// (above 2,048 pairs the two-wave build k_pairing_latency_w2: 4,096 pairs 1.60 ms against 1.94 ms for
// the segmented path and 2.18 ms for the one-wave build's two rounds, profiles/r4a_latency_w2_vs_w1.jsonl)
constexpr size_t kLatencyMaxDefault = 4096;  // one-wave crossover: 2048 pairs 1.27 vs 1.92 ms (profiles/r3e_latency.jsonl)
// batches up to this size run k_prepare_wide (8 lanes per pair: 2^14 pairs fill
// the GPU at two waves per SIMD).  BN254MI_PREPARE_WIDE_MAX overrides (0: never).
constexpr size_t kPrepareWideMaxDefault = 16384;

size_t ws_bytes(size_t n) {
    return n * ((size_t)kCoeffFq * 9 * 4 + kPathLanes * (2 * 9 * 4 + 1) + (size_t)kFeSlots * kSlotWords * 4) + 64;
}

// ---------------------------------------------------------------- FE step program
struct Prog {
    std::vector<uint32_t> s;  // two words per step (kernels.h)
    uint32_t next = 2;
    uint32_t tmp() { return next++; }
    int steps() const { return (int)(s.size() / 2); }
    void op(Fq12Op o, uint32_t d, uint32_t a, uint32_t b = 0, uint32_t k = 0, uint32_t flags = 0) {
        uint32_t w[2];
        vm_step(w, o, d, a, b, o == OP_CYC && k == 0 ? 1 : k, flags);
        s.push_back(w[0]);
        s.push_back(w[1]);
    }
    // x^e for a signed-digit chain (digit, position), top digit first and
    // positive.  pow[d] is the slot holding x^d for each odd |d| used; each run
    // "square k times, multiply by x^|d| or its conjugate" is one step, and the
    // last step conjugates when `conj_out`.
    uint32_t chain(const uint32_t* pow, const std::vector<std::pair<int, int>>& digits, bool conj_out) {
        const uint32_t r = tmp();
        int pos = digits[0].second;
        uint32_t src = pow[digits[0].first];
        bool wrote = false;
        for (size_t t = 1; t < digits.size(); ++t) {
            const int d = digits[t].first;
            const bool last = t + 1 == digits.size() && digits[t].second == 0;
            op(OP_MUL, r, src, pow[d < 0 ? -d : d], (uint32_t)(pos - digits[t].second),
               (d < 0 ? kFlagConjB : 0) | (last && conj_out ? kFlagConjOut : 0));
            pos = digits[t].second;
            src = r;
            wrote = true;
        }
        if (pos > 0) {
            op(OP_CYC, r, src, 0, (uint32_t)pos);
            if (conj_out) op(OP_CONJ, r, r);
        } else if (!wrote) {  // a single digit at position 0
            op(conj_out ? OP_CONJ : OP_MOV, r, src);
        }
        return r;
    }
    // exp_by_neg_z, fq12.rs:121-124: conj(cyclotomic_pow(u)) with
    // u = 0x44e992b44a6909f1 (fq12.rs:249-266).
    // windowed = width-4 signed window (digits +-1, 3, 5, 7: 13 chain products
    // + 3 for x^3, x^5, x^7, instead of the 27 of the binary chain), valid when
    // x is in the cyclotomic subgroup (there conj(x) = x^-1) -- always true
    // inside the final exponentiation.  The generic op (bn_fq12_op_many) keeps
    // the reference's binary chain so its output matches for any input.
    uint32_t exp_by_neg_z(uint32_t x, bool windowed = false) {
        constexpr int W = 4;
        uint64_t u = 4965661367192848881ull;
        std::vector<std::pair<int, int>> d;  // (digit, position), low to high
        for (int pos = 0; u; ++pos, u >>= 1) {
            if (!(u & 1)) continue;
            int z = 1;
            if (windowed) {
                z = (int)(u & ((1u << W) - 1));
                if (z >= (1 << (W - 1))) z -= 1 << W;
            }
            d.push_back({z, pos});
            u -= (uint64_t)(int64_t)z;  // u - z is divisible by 2^W (or 2)
        }
        std::reverse(d.begin(), d.end());
        uint32_t pow[1 << (W - 1)] = {0};
        pow[1] = x;
        if (windowed) {
            if (!win2) win2 = tmp(), win[3] = tmp(), win[5] = tmp(), win[7] = tmp();  // shared by the three calls
            op(OP_CYC, win2, x, 0, 1);
            op(OP_MUL, win[3], x, win2);
            op(OP_MUL, win[5], win[3], win2);
            op(OP_MUL, win[7], win[5], win2);
            pow[3] = win[3], pow[5] = win[5], pow[7] = win[7];
        }
        return chain(pow, d, true);
    }
    uint32_t win2 = 0, win[8] = {0};
    // Register forwarding: a step whose operand a is the previous step's
    // destination reads it from registers (kFlagAccA); a result that no later
    // step reads from its slot, and that is not a program output still in
    // place at the end, is not stored (kFlagNoStore).
    void finalize(const std::vector<uint32_t>& outputs) {
        const int n = steps();
        auto D = [&](int t) { return (s[2 * t] >> 8) & 0xff; };
        auto A = [&](int t) { return (s[2 * t] >> 16) & 0xff; };
        auto Bo = [&](int t) { return s[2 * t] >> 24; };
        auto reads_b = [&](int t) { return (s[2 * t] & 0xff) == OP_MUL; };
        for (int t = 1; t < n; ++t)
            if (A(t) == D(t - 1)) s[2 * t + 1] |= kFlagAccA << 8;
        for (int t = 0; t < n; ++t) {
            const uint32_t d = D(t);
            bool needed = true;  // stays true if d is an output never overwritten
            bool overwritten = false;
            bool read = false;
            for (int u = t + 1; u < n && !overwritten; ++u) {
                const bool via_acc = u == t + 1 && ((s[2 * u + 1] >> 8) & kFlagAccA);
                if ((A(u) == d && !via_acc) || (reads_b(u) && Bo(u) == d)) read = true;
                if (D(u) == d) overwritten = true;
            }
            bool is_out = false;
            for (uint32_t o : outputs) is_out |= o == d;
            needed = read || (is_out && !overwritten);
            if (!needed) s[2 * t + 1] |= kFlagNoStore << 8;
        }
    }
};
// final_exponentiation (fq12.rs:107-110) of slot 0; returns the result slot.
// Same operations as the reference; conjugations ride on the multiplies.
uint32_t build_final_exp(Prog& P) {
    // first chunk, fq12.rs:62-73
    const uint32_t b = P.tmp(), c = P.tmp(), d = P.tmp();
    P.op(OP_INV, b, 0);
    P.op(OP_MUL, c, b, 0, 0, kFlagConjB);  // c = conj(f) * f^-1
    P.op(OP_FROB2, d, c);
    P.op(OP_MUL, 1, d, c);  // slot 1 = self of the last chunk
    // last chunk, fq12.rs:75-105
    const uint32_t A = P.exp_by_neg_z(1, true);
    const uint32_t B = P.tmp(), D = P.tmp();
    P.op(OP_CYC, B, A, 0, 1);
    P.op(OP_MUL, D, B, B, 1);  // d = cyc(b) * b
    const uint32_t E = P.exp_by_neg_z(D, true);
    const uint32_t F = P.tmp();
    P.op(OP_CYC, F, E, 0, 1);
    const uint32_t G = P.exp_by_neg_z(F, true);
    const uint32_t J = P.tmp(), K = P.tmp(), L = P.tmp(), M = P.tmp(), N = P.tmp();
    P.op(OP_MUL, J, E, G, 0, kFlagConjB);  // j = conj(g) * e
    P.op(OP_MUL, K, J, D, 0, kFlagConjB);  // k = j * conj(d)
    P.op(OP_MUL, L, K, B);
    P.op(OP_MUL, M, K, E);
    P.op(OP_MUL, N, 1, M);
    const uint32_t O = P.tmp(), Pp = P.tmp(), Q = P.tmp(), R = P.tmp(), T = P.tmp(), U = P.tmp(), V = P.tmp();
    P.op(OP_FROB1, O, L);
    P.op(OP_MUL, Pp, O, N);
    P.op(OP_FROB2, Q, K);
    P.op(OP_MUL, R, Q, Pp);
    P.op(OP_MUL, T, L, 1, 0, kFlagConjB);  // t = conj(self) * l
    P.op(OP_FROB3, U, T);
    P.op(OP_MUL, V, U, R);
    return V;
}

int reserve(bn_ctx* c, size_t n) {
    if (n <= c->cap) return BN_OK;
    n = n < 1024 ? 1024 : n;
    if (c->cap) {
        int r = ws_drain(c);
        if (r) return r;
    }
    if (c->coeffs) HIPCHK(c, hipFree(c->coeffs));
    if (c->paff) HIPCHK(c, hipFree(c->paff));
    if (c->slots) HIPCHK(c, hipFree(c->slots));
    if (c->flags) HIPCHK(c, hipFree(c->flags));
    c->coeffs = nullptr; c->paff = nullptr; c->slots = nullptr; c->flags = nullptr; c->cap = 0;
    HIPCHK(c, hipMalloc(&c->coeffs, n * (size_t)kCoeffFq * 9 * 4));
    HIPCHK(c, hipMalloc(&c->paff, n * kPathLanes * 2 * 9 * 4));
    HIPCHK(c, hipMalloc(&c->slots, n * (size_t)kFeSlots * kSlotWords * 4));
    HIPCHK(c, hipMalloc(&c->flags, n * kPathLanes));
    c->cap = n;
    return BN_OK;
}
int stage(bn_ctx* c, size_t bytes) {
    if (bytes <= c->stage_bytes) return BN_OK;
    if (c->stage) {
        int r = ws_drain(c);
        if (r) return r;
        HIPCHK(c, hipFree(c->stage));
    }
    c->stage = nullptr;
    c->stage_bytes = 0;
    HIPCHK(c, hipMalloc(&c->stage, bytes));
    c->stage_bytes = bytes;
    return BN_OK;
}
hipStream_t pick(bn_ctx* c, void* s) { return s ? (hipStream_t)s : c->stream; }

// ---------------------------------------------------------------- host pipeline helpers
// pairs per piece of bn_pairing_many's host pipeline: 2^17 once a call has two
// such pieces, else 2^16 (the pipeline starts above one 2^16 piece).  Piece-size
// A/B on host buffers (profiles/r2av_host_piece_ab.jsonl): 2^17 pieces 159-162 ms
// at 2^20 pairs and 81-83 ms at 2^19, against 168-177 / 97 ms for 2^16 pieces and
// 163-172 / 83 ms for 2^18.
constexpr size_t kHostPiece = size_t(1) << 17;
constexpr size_t kHostPieceSmall = size_t(1) << 16;
size_t round256(size_t b) { return (b + 255) & ~(size_t)255; }
// pinned bounce buffers of bn_pairing_many (grown, never shrunk); the caller
// has drained the copy streams, which are the buffers' only device users
int pin_reserve(bn_ctx* c, size_t bytes) {
    if (bytes <= c->pin_bytes) return BN_OK;
    if (c->pin) HIPCHK(c, hipHostFree(c->pin));
    c->pin = nullptr;
    c->pin_bytes = 0;
    HIPCHK(c, hipHostMalloc(&c->pin, bytes, hipHostMallocDefault));
    c->pin_bytes = bytes;
    return BN_OK;
}
// memcpy split over up to 8 host threads for large copies (a single thread
// moves ~10 GB/s, a 2^16-pair piece is 44 MB)
void par_copy(void* dst, const void* src, size_t bytes) {
    constexpr size_t kPerThread = size_t(4) << 20;
    const size_t nt = std::min<size_t>(8, bytes / kPerThread);
    if (nt <= 1) {
        memcpy(dst, src, bytes);
        return;
    }
    const size_t per = ((bytes + nt - 1) / nt + 63) & ~(size_t)63;
    std::vector<std::thread> th;
    for (size_t t = 1; t < nt; ++t) {
        const size_t lo = t * per;
        if (lo >= bytes) break;
        th.emplace_back([=] { memcpy((uint8_t*)dst + lo, (const uint8_t*)src + lo, std::min(per, bytes - lo)); });
    }
    memcpy(dst, src, std::min(per, bytes));
    for (auto& t : th) t.join();
}

// to_affine + the 87 line coefficients of m pairs into c->coeffs / paff / flags:
// eight lanes per pair (k_prepare_wide, about a third of the step latency) while
// the batch leaves the GPU underfilled, two lanes per pair (k_prepare) otherwise
// (scale: 1 for the Miller-loop consumers, 0 for the coefficient export)
static int prepare(bn_ctx* c, const bn_g1* d_p, const bn_g2* d_q, size_t m, int mode, hipStream_t s, int scale = 1) {
    if (m <= c->prepare_wide_max)
        k_prepare_wide<<<grid_pair(kPrepareWideLanes * m), kPairBlock, 0, s>>>(d_p, d_q, m, c->coeffs, c->paff,
                                                                              c->flags, c->d_err, mode, scale);
    else
        k_prepare<<<grid_pair(kPathLanes * m), kPairBlock, 0, s>>>(d_p, d_q, m, c->coeffs, c->paff, c->flags, c->d_err,
                                                                   mode, scale);
    HIPCHK(c, hipGetLastError());
    return BN_OK;
}

// Miller values of n pairs into slot 0 (lane-strided, stride = n); n <= c->cap
int miller_values(bn_ctx* c, const bn_g1* d_p, const bn_g2* d_q, size_t n, int mode, hipStream_t s) {
    RET_IF(prepare(c, d_p, d_q, n, mode, s));
    k_miller<<<grid_for(kPathLanes * n), kBlock, 0, s>>>(c->coeffs, c->paff, c->flags, n, c->slots);
    HIPCHK(c, hipGetLastError());
    return BN_OK;
}
// the region of Fq12 slot k of the workspace (room for c->cap split-layout elements)
uint32_t* slot_region(bn_ctx* c, int k) { return c->slots + (size_t)k * kSlotWords * c->cap; }
constexpr int kRegionA = 1, kRegionB = 2;  // ping-pong regions of the product reduction
constexpr int kRegionParts = 3;            // per-chunk partial products
constexpr int kRegionResult = 4;           // the final product (element 0, stride 1)
constexpr size_t kWideGroups = kBlock / 16;  // k_fq12_reduce_wide: 16-lane groups per block
constexpr size_t kReduceBlocksMax = 512;      // one round of 256-thread blocks, two per CU (kernels_reduce.hip)
// BN_REDUCE_LAST: a level whose sets all fit one block with chains of up to 8 factors
// finishes there (config 5: 80 + 24 + 19 -> 85 + 30 us, profiles/r5af_ab_reduce_last.txt)
#ifndef BN_REDUCE_LAST
#define BN_REDUCE_LAST 1
#endif
constexpr int kReduceLastMax = 8;  // the longest chain a finishing level may take

// sets y < `sets` of n elements each at y * n
static SetSpan uniform_span(int sets, size_t n) {
    SetSpan sp{};
    sp.sets = sets;
    for (int y = 0; y < sets; ++y) {
        sp.off[y] = (uint32_t)(y * n);
        sp.n[y] = (uint32_t)n;
    }
    return sp;
}
// Multiply each of `sets` (<= kMaxSeg) sets of split-layout values together on
// the wide layout (k_fq12_reduce_wide, all sets in one launch per level): set y
// is elements span.off[y] + [0, span.n[y]) of `in` (stride in_stride), its product goes to
// element out_base + y * out_set of `out` (stride out_stride).  `in` must not
// be a ping-pong region.  Each set takes its own number of blocks (one flat grid),
// so sets of different sizes (the per-segment K of batch_plan) need no padding.
// Each level's chain length per group G is the smallest
// power of two >= 2 that needs at most 512 blocks: config 5's 16 x 4,096
// segment values take two launches (G = 8, then 2) instead of three of G = 2 --
// 2.20 against 2.25-2.26 ms per product; G = 16 2.21-2.27, G = 32 2.27-2.30
// (profiles/r4e_ab_reduce.txt, one block per CU then); with two blocks per CU
// (kernels_reduce.hip) G = 8 stays ahead of G = 4 (profiles/r4q_ab_reduce_lds.txt).
int product_wide(bn_ctx* c, const uint32_t* in, size_t in_stride, SetSpan span, int sets, uint32_t* out,
                 size_t out_stride, size_t out_base, size_t out_set, hipStream_t s) {
    if (sets < 1 || sets > kMaxSeg) return fail(c, BN_ERR_INTERNAL, "product reduction: bad set count");
    span.sets = sets;
    const uint32_t* src = in;
    size_t sstride = in_stride;
    bool a = true;
    for (;;) {
        // G (per_group): the smallest power of two >= 2 with at most kReduceBlocksMax
        // blocks over all sets, each set taking ceil(n[y] / (16 G)) blocks
        auto blocks_for = [&](int pg) {
            size_t t = 0;
            for (int y = 0; y < sets; ++y) t += (span.n[y] + kWideGroups * pg - 1) / (kWideGroups * pg);
            return t;
        };
        int per_group = 2;
        while (per_group < 64 && blocks_for(per_group) > kReduceBlocksMax) per_group *= 2;
#if BN_REDUCE_LAST
        // a level whose every set fits one block with chains of <= kReduceLastMax factors
        // finishes there instead of leaving a few blocks per set for one more launch
        size_t nmax = 0;
        for (int y = 0; y < sets; ++y) nmax = std::max<size_t>(nmax, span.n[y]);
        if (nmax > kWideGroups * (size_t)per_group && nmax <= kWideGroups * (size_t)kReduceLastMax)
            while (kWideGroups * (size_t)per_group < nmax) per_group *= 2;
#endif
        const size_t per_block = kWideGroups * (size_t)per_group;
        size_t bmax = 0;
        span.blk[0] = 0;
        for (int y = 0; y < sets; ++y) {
            const size_t by = std::max<size_t>(1, (span.n[y] + per_block - 1) / per_block);  // an empty set: one
            span.blk[y + 1] = span.blk[y] + (uint32_t)by;
            bmax = std::max(bmax, by);
        }
        const unsigned grid = span.blk[sets];
        if (bmax == 1) {
            k_fq12_reduce_wide<<<grid, kBlock, 0, s>>>(src, sstride, span, out, out_stride, out_base, out_set,
                                                       per_group);
            HIPCHK(c, hipGetLastError());
            return BN_OK;
        }
        uint32_t* dst = slot_region(c, a ? kRegionA : kRegionB);
        if ((size_t)sets * bmax > c->cap) return fail(c, BN_ERR_INTERNAL, "product reduction exceeds the workspace");
        k_fq12_reduce_wide<<<grid, kBlock, 0, s>>>(src, sstride, span, dst, sets * bmax, 0, bmax, per_group);
        HIPCHK(c, hipGetLastError());
        // next level: set y holds its blocks' products at y * bmax (stride sets * bmax)
        SetSpan nx{};
        nx.sets = sets;
        for (int y = 0; y < sets; ++y) {
            nx.off[y] = (uint32_t)(y * bmax);
            nx.n[y] = span.blk[y + 1] - span.blk[y];
        }
        span = nx;
        src = dst;
        sstride = sets * bmax;
        a = !a;
    }
}

// k_fe_ds over n <= c->fe_ds_max split-layout values of f (stride n): three blocks per
// value while they fit one round (one 84 KB block per CU), else one
static void launch_fe_ds(bn_ctx* c, const uint32_t* f, size_t n, bn_gt* out, uint8_t* ok, hipStream_t s) {
    c->tail_epoch = c->tail_epoch + 1 < (1u << 29) ? c->tail_epoch + 1 : 1u;
    const int per = 3 * n * kLatPairs <= c->lat_w1_max ? 3 : 1;  // (lat_w1_max = CUs x kLatPairs)
    k_fe_ds<<<(unsigned)(per * n), kTailBlock, 0, s>>>(f, n, out, ok, c->d_err, c->fe_ds_ws, c->tail_epoch, per);
}
// final exponentiation of the n split-layout values of `f` (stride n) -> out
// (device Gt images): the wide layout for small batches, else the step machine
// (whose program reads and writes the slots from slot 0: f must be slot 0)
int run_fe(bn_ctx* c, const uint32_t* f, size_t n, const uint8_t* flags, bn_gt* out, uint8_t* ok, hipStream_t s) {
    if (n <= c->fe_ds_max && n <= c->fe_wide_max) {  // digit-sliced blocks per value (kernels_tail.hip k_fe_ds)
        launch_fe_ds(c, f, n, out, ok, s);
        HIPCHK(c, hipGetLastError());
        return BN_OK;
    }
    if (n <= c->fe_wide_max) {
        k_fe_wide<<<wide_blocks(n), kBlock, 0, s>>>(f, n, n, out, ok, c->d_err, wide_duo(n) ? 1 : 0);
        HIPCHK(c, hipGetLastError());
        return BN_OK;
    }
    if (f != c->slots) return fail(c, BN_ERR_INVALID_ARGUMENT, "internal: step-machine FE input must be slot 0");
    k_fq12_vm<<<grid_pair(kPathLanes * n), kPairBlock, 0, s>>>(c->d_prog, c->fe_steps, c->slots, n);
    HIPCHK(c, hipGetLastError());
    k_fe_out<<<grid_for(kPathLanes * n), kBlock, 0, s>>>(c->slots, n, c->fe_out, flags, out, ok, c->d_err);
    HIPCHK(c, hipGetLastError());
    return BN_OK;
}

// ---- pairing_batch / miller_loop_batch: segmented Miller loop + device reduction
constexpr int kRegionSeg = 8;  // k_miller_seg output: plan.total elements from region kRegionSeg on

// Work of one lane pair in segment [d, e) of the 64 digits with K pairs: a
// squaring per digit but the first (36 Fq-mul) and K lines per line of a pair
// (39 each; two at a nonzero digit, and the last segment's two closing lines).
static int seg_sq(int d, int e) { return e - d - 1; }
static int seg_lines(int d, int e) {  // (digits + nonzero digits in [d, e), by popcount)
    const uint64_t in = (e >= 64 ? ~0ull : (1ull << e) - 1ull) & ~((1ull << d) - 1ull);
    return (e == BN_NAF_DIGITS ? 2 : 0) + (e - d) + __builtin_popcountll(kNafNonzero & in);
}
// (weights from the ISA -- 5,338 VALU per squaring against 4,730 plus the loads per
// line -- and three settings between them planned no better on the GPU,
// profiles/r5e_ab_segment_plan.txt)
constexpr int kSegWSqDefault = 36, kSegWLineDefault = 39;
// BN254MI_SEG_WEIGHTS="sq,line" overrides the two weights (A/B of the plan's cost model)
static int seg_weight(int which) {
    struct W {
        int v[2];
    };
    static const W w = [] {  // read once (thread-safe static initialization)
        W r = {{kSegWSqDefault, kSegWLineDefault}};
        if (const char* e = getenv("BN254MI_SEG_WEIGHTS")) {
            int x = 0, y = 0;
            if (sscanf(e, "%d,%d", &x, &y) == 2 && x > 0 && y > 0) r = {{x, y}};
        }
        return r;
    }();
    return w.v[which];
}
#define kSegWSq seg_weight(0)
#define kSegWLine seg_weight(1)
static int seg_cost(int d, int e, int K) { return kSegWSq * seg_sq(d, e) + kSegWLine * K * seg_lines(d, e); }
static void plan_index(SegPlan& p) {
    for (int k = 0; k < p.S; ++k)
        p.idx[k] = p.lo[k] + __builtin_popcountll(kNafNonzero & ((p.lo[k] ? (1ull << p.lo[k]) : 1ull) - 1ull));
}
// cut the 64 digits into S segments of about equal work for K pairs per lane pair
static SegPlan cut_plan(int S, int K) {
    SegPlan p{};
    p.S = S;
    auto cost = [K](int d) { return 36 + 39 * K + (((kNafNonzero >> d) & 1u) ? 39 * K : 0); };
    int total = 2 * 39 * K;
    for (int d = 0; d < BN_NAF_DIGITS; ++d) total += cost(d);
    int g = 0, acc = 0;
    p.lo[0] = 0;
    for (int d = 0; d < BN_NAF_DIGITS; ++d) {
        acc += cost(d);
        if (g + 1 < S && acc * S >= total * (g + 1) && d + 1 < BN_NAF_DIGITS) {
            p.hi[g] = d + 1;
            p.lo[++g] = d + 1;
        }
    }
    p.hi[g] = BN_NAF_DIGITS;
    p.S = g + 1;
    for (int k = 0; k < p.S; ++k) p.K[k] = K;
    plan_index(p);
    return p;
}
// the lane-pair layout of a plan over n pairs: segment s gets G[s] = ceil(n / K[s])
// lane pairs from off[s] on, each range rounded up to `align` lane pairs
static SegPlan plan_layout(SegPlan p, size_t n, uint32_t align) {
    uint32_t off = 0;
    for (int k = 0; k < p.S; ++k) {
        p.G[k] = (uint32_t)((n + (size_t)p.K[k] - 1) / (size_t)p.K[k]);
        p.off[k] = off;
        off += (p.G[k] + align - 1) / align * align;
    }
    p.total = off;
    return p;
}
// pairing_many's latency path: one pair per lane pair (K = 1); S doubles while
// S*n lane pairs leave the GPU underfilled; 16 segments only for the smallest
// batches (profiles/r2ac_latency_seg16.txt: 16 helps up to ~1024 pairs, costs
// at 4096 through the longer Horner recombination of every pair).  Unpadded:
// element s * n + e (k_horner_wide's layout).
SegPlan seg_plan(size_t n) {
    int S = 1;
    while (S < kMaxSeg && (size_t)S * n < ((size_t)1 << 16) && !(S >= 8 && (size_t)S * n >= ((size_t)1 << 14))) S *= 2;
    return plan_layout(cut_plan(S, 1), n, 1);
}
// pairing_batch / miller_loop_batch (one recombination for the whole product):
// up to 16 digit segments, each with its own number K[s] of pairs per lane pair
// sharing one squaring per digit (mod.rs:609-640).  The lane-pair budget is the
// uniform plan's: 16 ceil(n / K0) with K0 the largest power of two <= 16 that
// still leaves at least 2^16 lane pairs (two waves per SIMD; K0 = 4 at 2^14 terms).
// Within it the digits and the K[s] minimize the largest segment's work (the
// kernel runs as long as its heaviest lane pair): a dynamic program over the
// digit boundaries for a target work T, each segment taking the largest K that
// keeps it within T, binary-searched on T.  At 2^14 terms: 1,008 against the
// uniform plan's 1,236 (K = 4 everywhere: 696 to 1,236 per segment).  Each
// segment's lane pairs are padded to whole 512-thread blocks (256 lane pairs).
static SegPlan batch_plan_solve(size_t n);
// The plan depends on n alone: the last few are kept per host thread, so repeated
// products of one size (config 5) solve it once.
SegPlan batch_plan(size_t n) {
    struct Entry {
        size_t n;
        SegPlan p;
    };
    static thread_local Entry cache[4];
    static thread_local int used = 0, next = 0;
    for (int i = 0; i < used; ++i)
        if (cache[i].n == n) return cache[i].p;
    const SegPlan p = batch_plan_solve(n);
    cache[next] = {n, p};
    next = (next + 1) % 4;
    if (used < 4) ++used;
    return p;
}
static SegPlan batch_plan_solve(size_t n) {
    int K0 = 1;
    while (K0 < 16 && (size_t)kMaxSeg * ((n + 2 * K0 - 1) / (2 * K0)) >= ((size_t)1 << 16)) K0 *= 2;
    const size_t align = kPairBlock / kPathLanes;
    auto padded = [&](int K) { return ((n + (size_t)K - 1) / (size_t)K + align - 1) / align * align; };
    const size_t budget = (size_t)kMaxSeg * padded(K0);
    constexpr int D = BN_NAF_DIGITS;
    constexpr size_t kInf = ~(size_t)0;
    // dp[e][k]: fewest lane pairs covering digits [0, e) with k segments of work <= T
    auto solve = [&](int T, SegPlan* out) {
        static thread_local size_t dp[D + 1][kMaxSeg + 1];
        static thread_local int from[D + 1][kMaxSeg + 1], kof[D + 1][kMaxSeg + 1];
        for (auto& r : dp)
            for (auto& v : r) v = kInf;
        dp[0][0] = 0;
        for (int d = 0; d < D; ++d)
            for (int k = 0; k < kMaxSeg; ++k) {
                if (dp[d][k] == kInf) continue;
                for (int e = d + 1; e <= D; ++e) {
                    const int sq = seg_sq(d, e), L = seg_lines(d, e);
                    if (kSegWSq * sq + kSegWLine * L > T) break;  // even K = 1 is over T (and grows with e)
                    int K = (T - kSegWSq * sq) / (kSegWLine * L);
                    if (K > 64) K = 64;
                    if ((size_t)K > n) K = n > 0 ? (int)n : 1;  // no lane pair of dummy one-lines only
                    const size_t v = dp[d][k] + padded(K);
                    if (v < dp[e][k + 1]) {
                        dp[e][k + 1] = v;
                        from[e][k + 1] = d;
                        kof[e][k + 1] = K;
                    }
                }
            }
        int best = -1;
        for (int k = 1; k <= kMaxSeg; ++k)
            if (dp[D][k] <= budget && (best < 0 || dp[D][k] < dp[D][best])) best = k;
        if (best < 0) return false;
        if (out) {
            SegPlan p{};
            p.S = best;
            for (int e = D, k = best; k > 0; --k) {
                const int d = from[e][k];
                p.lo[k - 1] = d;
                p.hi[k - 1] = e;
                p.K[k - 1] = kof[e][k];
                e = d;
            }
            plan_index(p);
            *out = p;
        }
        return true;
    };
    SegPlan uni = cut_plan(kMaxSeg, K0);
    int hi = 0;
    for (int k = 0; k < uni.S; ++k) hi = std::max(hi, seg_cost(uni.lo[k], uni.hi[k], K0));
    int lo = 1;
    if (!solve(hi, nullptr)) return plan_layout(uni, n, (uint32_t)align);
    while (lo < hi) {
        const int mid = (lo + hi) / 2;
        if (solve(mid, nullptr)) hi = mid; else lo = mid + 1;
    }
    SegPlan p{};
    solve(hi, &p);
    return plan_layout(p, n, (uint32_t)align);
}

// Segment values of m <= kChunk device pairs (mode 0: a pair with a zero point
// counts as one; mode 1: a zero point sets the BN_ERR_TO_AFFINE bit), each
// segment reduced over the pairs into element g * nchunks + k (stride
// S * nchunks) of `parts`
int chunk_product(bn_ctx* c, const bn_g1* d_p, const bn_g2* d_q, size_t m, int mode, const SegPlan& plan,
                  uint32_t* parts, size_t nchunks, size_t k, hipStream_t s) {
    RET_IF(prepare(c, d_p, d_q, m, mode, s));
    const SegPlan lay = plan_layout(plan, m, kPairBlock / kPathLanes);  // this chunk's lane pairs
    // k_miller_seg writes lay.total elements from region kRegionSeg to the end of the slots
    if ((size_t)lay.total > (size_t)(kFeSlots - kRegionSeg) * c->cap)
        return fail(c, BN_ERR_INTERNAL, "segment layout exceeds the workspace");
    k_miller_seg<<<grid_pair(kPathLanes * (size_t)lay.total), kPairBlock, 0, s>>>(c->coeffs, c->paff, c->flags, m, lay,
                                                                              slot_region(c, kRegionSeg));
    HIPCHK(c, hipGetLastError());
    SetSpan sp{};
    for (int k2 = 0; k2 < lay.S; ++k2) {
        sp.off[k2] = lay.off[k2];
        sp.n[k2] = lay.G[k2];
    }
    return product_wide(c, slot_region(c, kRegionSeg), lay.total, sp, lay.S, parts, plan.S * nchunks, k, nchunks, s);
}
// where chunk partials go: straight into the result region (element g, stride S)
// for one chunk, else the parts region
uint32_t* parts_region(bn_ctx* c, size_t nchunks) {
    return nchunks == 1 ? slot_region(c, kRegionResult) : slot_region(c, kRegionParts);
}
// the S segment values of ONE product (result region, element s, stride S) ->
// their recombination, then the final exponentiation (do_fe) or the Miller value,
// into *d_out: k_horner_tree (the squarings of the segments side by side and a
// product tree); BN254MI_HORNER_TREE=0 selects k_horner_wide (one group, Horner's
// rule), kept for A/B
// Build parameters (A/B builds, tools/build_variant.sh): BN_TAIL_DS=0 builds the tail
// without the digit-sliced layout (kernels_tail.hip), BN_SEG_FE1=0 keeps the segments'
// first chunks and squarings inside k_horner_tree2
#ifndef BN_TAIL_DS
#define BN_TAIL_DS 1
#endif
#ifndef BN_SEG_FE1
#define BN_SEG_FE1 1
#endif
// BN_TAIL_M=0: the final exponentiation after k_seg_fe1 on one block (no multiplier block)
#ifndef BN_TAIL_M
#define BN_TAIL_M 1
#endif
// (g: the segment values, element s at stride S; default the result region)
static int recombine_one(bn_ctx* c, const SegPlan& plan, int do_fe, bn_gt* d_out, hipStream_t s,
                         uint32_t* g = nullptr) {
    if (!g) g = slot_region(c, kRegionResult);
    const char* env = getenv("BN254MI_HORNER_TREE");
    const int tree = env ? atoi(env) : 2;  // 2: k_horner_tree2 (default), 1: k_horner_tree, 0: k_horner_wide
    static const bool fused = [] {  // $BN254MI_TAIL_FUSED=0: k_seg_fe1 + k_horner_tree2 (A/B)
        const char* e = getenv("BN254MI_TAIL_FUSED");
        return !(e && atoi(e) == 0);
    }();
    if (tree == 2 && BN_FE_DUO && BN_TAIL_DS && BN_SEG_FE1 && BN_TAIL_M && fused && do_fe && plan.S >= 1 &&
        plan.S <= kMaxSeg) {
        // pairing_batch: the whole tail in one launch (kernels_tail.hip k_seg_tail)
        c->tail_epoch = c->tail_epoch + 1 < (1u << 29) ? c->tail_epoch + 1 : 1u;  // (epoch * 8 fits the role word)
        k_seg_tail<<<plan.S > 3 ? plan.S : 3, kTailBlock, 0, s>>>(g, plan, d_out, c->d_err,
                                                                  c->tail_ws, c->tail_epoch);
    } else if (tree == 2 && BN_FE_DUO && plan.S <= kMaxSeg) {
        // pairing_batch: the segments' first chunks and squarings one block each
        // (k_seg_fe1), the zero flags and the squarer <-> multiplier channel of
        // k_horner_tree2's two blocks at the start of the reduction's ping-pong region
        // A (free once the reduction has written the result region)
        const uint32_t* zf = nullptr;
        if (BN_TAIL_DS && BN_SEG_FE1 && do_fe && plan.S >= 1 && (size_t)kSlotWords * c->cap >= (size_t)kTailChanWords) {
            uint32_t* z = slot_region(c, kRegionA);
            k_seg_fe1<<<plan.S, kTailBlock, 0, s>>>(g, plan, z);
            HIPCHK(c, hipGetLastError());
            zf = z;
        }
        // two blocks: the squarer (block 0) and the multiplier (block 1) of the last
        // chunk hand values over by polling global memory, which needs both resident.
        // HIP does not promise co-residency, so the blocks claim their roles through a
        // word k_seg_fe1 clears (kernels_tail.hip tail_claim): a multiplier that has not
        // started when the squarer gets there is not waited for -- the squarer runs
        // the chunk alone (the same value) and the late block returns.
        k_horner_tree2<<<zf && BN_TAIL_M ? 2 : 1, kTailBlock, 0, s>>>(g, plan, do_fe, d_out, c->d_err,
                                                          zf);
    }
    else if (tree != 0)
        k_horner_tree<<<1, kBlock, 0, s>>>(g, plan, do_fe, d_out, c->d_err,
                                           wide_duo(1) ? 1 : 0);
    else
        k_horner_wide<<<1, kBlock, 0, s>>>(g, 1, plan, do_fe, d_out, c->d_err,
                                           wide_duo(1) ? 1 : 0);
    HIPCHK(c, hipGetLastError());
    return BN_OK;
}
// per segment, the chunk partials -> the result region; then the Horner
// recombination (+ the final exponentiation for pairing_batch) into *d_out
int finish_product(bn_ctx* c, const SegPlan& plan, size_t nchunks, int do_fe, bn_gt* d_out, hipStream_t s) {
    if (nchunks > 1)
        RET_IF(product_wide(c, slot_region(c, kRegionParts), plan.S * nchunks, uniform_span(plan.S, nchunks), plan.S,
                            slot_region(c, kRegionResult), plan.S, 0, 1, s));
    return recombine_one(c, plan, do_fe, d_out, s);
}
// The product of n <= c->latency_max device pairs: their Miller values from the
// one-launch k_pairing_latency (no FE), the product reduction, then one group's
// final exponentiation (do_fe: pairing_batch) or the Miller value itself
// (miller_loop_batch) into *d_out
// The one-launch latency kernel over m pairs (out: Gt images, or f_out: the Miller
// values): the one-wave build while its blocks (8 pairs each, one per CU) fit one
// round, above that the two-wave build (kernels_latency_w2.hip: two blocks per CU),
// unless $BN254MI_LATENCY_W2=0 (A/B)
// (lat_w1_max = the device's CU count x kLatPairs, set at context creation: 2,048
// on MI355X's 256 CUs)
static void launch_latency(bn_ctx* c, const bn_g1* d_p, const bn_g2* d_q, size_t m, bn_gt* out, uint32_t* f_out,
                           int mode, hipStream_t s) {
    const unsigned blocks = (unsigned)((m + kLatPairs - 1) / kLatPairs);
    if (m <= c->lat_w1_max || !c->latency_w2)
        k_pairing_latency<<<blocks, kLatThreads, 0, s>>>(d_p, d_q, m, out, f_out, mode, c->d_err);
    else
        k_pairing_latency_w2<<<blocks, kLatThreads, 0, s>>>(d_p, d_q, m, out, f_out, mode, c->d_err);
}
int latency_product(bn_ctx* c, const bn_g1* d_p, const bn_g2* d_q, size_t n, int mode, int do_fe, bn_gt* d_out,
                    hipStream_t s) {
    RET_IF(reserve(c, n));
    launch_latency(c, d_p, d_q, n, nullptr, slot_region(c, kRegionSeg), mode, s);
    HIPCHK(c, hipGetLastError());
    // one pair: its Miller value is the product, read in place (no reduction launch, ~15 us)
    if (n == 1) return recombine_one(c, cut_plan(1, 1), do_fe, d_out, s, slot_region(c, kRegionSeg));
    RET_IF(product_wide(c, slot_region(c, kRegionSeg), n, uniform_span(1, n), 1, slot_region(c, kRegionResult), 1, 0,
                        1, s));
    return recombine_one(c, cut_plan(1, 1), do_fe, d_out, s);  // one segment: the FE of the product when do_fe
}
// (at most one chunk: the one-launch path reserves workspace for all n pairs)
bool use_latency_product(const bn_ctx* c, size_t n) {
    return n <= c->latency_max && n <= c->fe_wide_max && n <= kChunk;
}

// the whole product of n device pairs into *d_out; the caller holds the workspace
int miller_product_dev(bn_ctx* c, const bn_g1* d_p, const bn_g2* d_q, size_t n, int mode, bn_gt* d_out,
                       hipStream_t s) {
    if (use_latency_product(c, n)) return latency_product(c, d_p, d_q, n, mode, mode == 0, d_out, s);
    const size_t nchunks = (n + kChunk - 1) / kChunk;
    const size_t m0 = n < kChunk ? n : kChunk;
    const SegPlan plan = batch_plan(m0);
    RET_IF(reserve(c, m0));
    if (nchunks * plan.S > c->cap) return fail(c, BN_ERR_INVALID_ARGUMENT, "too many chunks");
    uint32_t* parts = parts_region(c, nchunks);
    for (size_t k = 0; k < nchunks; ++k) {
        const size_t off = k * kChunk, m = (n - off) < kChunk ? (n - off) : kChunk;
        RET_IF(chunk_product(c, d_p + off, d_q + off, m, mode, plan, parts, nchunks, k, s));
    }
    return finish_product(c, plan, nchunks, mode == 0, d_out, s);
}

// the device outcome bits of the calls since the last clear; a wave hand-off that
// ran out of its wait cap (BN_ERR_INTERNAL) fails the call here, whatever else is set
int check_err(bn_ctx* c, hipStream_t s, int* out_bits) {
    int h = 0;
    HIPCHK(c, hipMemcpyAsync(&h, c->d_err, sizeof(int), hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipStreamSynchronize(s));
    *out_bits = h;
    if (h & (1 << BN_ERR_INTERNAL)) return fail(c, BN_ERR_INTERNAL, "device wave hand-off timed out; result discarded");
    return BN_OK;
}
int clear_err(bn_ctx* c, hipStream_t s) {
    HIPCHK(c, hipMemsetAsync(c->d_err, 0, sizeof(int), s));
    return BN_OK;
}

}  // namespace

#define CTX_GUARD(ctx)                                 \
    if (!(ctx)) return BN_ERR_INVALID_ARGUMENT;        \
    if (!(ctx)->subs.empty())                          \
        return fail((ctx), BN_ERR_INVALID_ARGUMENT,    \
                    "not available on a multi-device context; use bn_ctx_device()"); \
    std::lock_guard<std::mutex> lock_((ctx)->mu);      \
    HIPCHK(ctx, hipSetDevice((ctx)->device))
// host-buffer entry points: the lock for the whole call, and the context stream
// ordered after the workspace's previous user
#define CTX_GUARD_HOST(ctx)                \
    CTX_GUARD(ctx);                        \
    RET_IF(ws_acquire((ctx), (ctx)->stream)); \
    WsUse ws_use_{(ctx), (ctx)->stream}

// k_g1_mul2 (two chains per lane) once half the batch gives every CU one
// kPairBlock-thread block: 8.82 -> 8.36 ms at config 3's 2^18
// (profiles/r4c_ab_g1mul2.txt); below that k_g1_mul, one chain per lane, in
// kPairBlock-thread blocks (two waves on every SIMD, kernels.h issue balance)
// once the batch gives every CU one such block, else kBlock
constexpr size_t kG1MulPairBlockMin = (size_t)256 * kPairBlock;
static void g1_mul_launch(const bn_g1* d_p, const bn_fr* d_k, size_t n, bn_g1* d_out, hipStream_t s) {
    if ((n + 1) / 2 >= kG1MulPairBlockMin)
        k_g1_mul2<<<grid_pair((n + 1) / 2), kPairBlock, 0, s>>>(d_p, d_k, n, d_out);
    else if (n >= kG1MulPairBlockMin)
        k_g1_mul<<<grid_pair(n), kPairBlock, 0, s>>>(d_p, d_k, n, d_out);
    else
        k_g1_mul<<<grid_for(n), kBlock, 0, s>>>(d_p, d_k, n, d_out);
}
// G2 * Fr on the two-lane layout: 6.97 -> 6.22 ms per 2^16 against the one-lane
// kernel of rounds 1-3 (profiles/r4m_ab_g2_split.txt)
// (two chains per lane pair, as k_g1_mul2, measured 15 % slower at 2^16: one wave per
// SIMD; profiles/r5s_ab_g2_mul2.txt, removed after the A/B)
static void g2_mul_launch(const bn_g2* d_p, const bn_fr* d_k, size_t n, bn_g2* d_out, hipStream_t s) {
    k_g2_mul_split<<<grid_pair(kPathLanes * n), kPairBlock, 0, s>>>(d_p, d_k, n, d_out);
}

template <typename P, typename K>
static int host_mul(bn_ctx* c, const P* p, const bn_fr* k, size_t n, P* out, K launch) {
    CTX_GUARD_HOST(c);
    if (n == 0) return BN_OK;
    if (!p || !k || !out) return fail(c, BN_ERR_INVALID_ARGUMENT, "null buffer");
    RET_IF(stage(c, n * (2 * sizeof(P) + sizeof(bn_fr))));
    P* dp = (P*)c->stage;
    P* dout = dp + n;
    bn_fr* dk = (bn_fr*)(dout + n);
    HIPCHK(c, hipMemcpyAsync(dp, p, n * sizeof(P), hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(dk, k, n * sizeof(bn_fr), hipMemcpyHostToDevice, c->stream));
    launch(dp, dk, n, dout, c->stream);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipMemcpyAsync(out, dout, n * sizeof(P), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return BN_OK;
}

// ---------------------------------------------------------------- staged per-element calls
// Host-buffer form of a one-lane-per-element kernel: chunks of kChunk elements
// are copied in, `launch(dev, m, stream)` runs, outputs are copied back.  Each
// buffer is described by its per-element byte size.
struct HostIn { const void* p; size_t elem; };
struct HostOut { void* p; size_t elem; };
template <class Launch>
static int staged(bn_ctx* c, size_t n, std::initializer_list<HostIn> ins, std::initializer_list<HostOut> outs,
                  Launch&& launch) {
    if (n == 0) return BN_OK;
    for (const auto& b : ins)
        if (!b.p) return fail(c, BN_ERR_INVALID_ARGUMENT, "null buffer");
    for (const auto& b : outs)
        if (!b.p) return fail(c, BN_ERR_INVALID_ARGUMENT, "null buffer");
    for (size_t off = 0; off < n; off += kChunk) {
        const size_t m = (n - off) < kChunk ? (n - off) : kChunk;
        size_t bytes = 0;
        for (const auto& b : ins) bytes += (b.elem * m + 255) & ~(size_t)255;
        for (const auto& b : outs) bytes += (b.elem * m + 255) & ~(size_t)255;
        RET_IF(stage(c, bytes));
        std::vector<void*> dev;
        uint8_t* at = (uint8_t*)c->stage;
        for (const auto& b : ins) {
            HIPCHK(c, hipMemcpyAsync(at, (const uint8_t*)b.p + off * b.elem, m * b.elem, hipMemcpyHostToDevice, c->stream));
            dev.push_back(at);
            at += (b.elem * m + 255) & ~(size_t)255;
        }
        for (const auto& b : outs) {
            dev.push_back(at);
            at += (b.elem * m + 255) & ~(size_t)255;
        }
        RET_IF(launch(dev.data(), m, c->stream));
        HIPCHK(c, hipGetLastError());
        size_t k = ins.size();
        for (const auto& b : outs) {
            HIPCHK(c, hipMemcpyAsync((uint8_t*)b.p + off * b.elem, dev[k++], m * b.elem, hipMemcpyDeviceToHost, c->stream));
        }
        HIPCHK(c, hipStreamSynchronize(c->stream));
    }
    return BN_OK;
}
#define KL(kernel, ...) kernel<<<grid_for(m), kBlock, 0, s>>>(__VA_ARGS__)

static void ctx_teardown(bn_ctx* c);

extern "C" {

int bn_ctx_create(int device, bn_ctx** out) {
    if (!out) return BN_ERR_INVALID_ARGUMENT;
    *out = nullptr;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return BN_ERR_NO_DEVICE;
    if (device < 0 || device >= count) return BN_ERR_INVALID_ARGUMENT;
    bn_ctx* c = new bn_ctx();
    c->device = device;
    c->fe_wide_max = kFeWideMaxDefault;
    if (const char* e = getenv("BN254MI_FE_WIDE_MAX")) c->fe_wide_max = (size_t)strtoull(e, nullptr, 10);
    if (const char* e = getenv("BN254MI_MILLER_FORM")) c->miller_form = atoi(e);
    if (const char* e = getenv("BN254MI_HOST_PIPELINE")) c->host_pipeline = atoi(e);
    c->host_piece = kHostPiece;
    if (const char* e = getenv("BN254MI_HOST_PIECE")) {
        const size_t v = (size_t)strtoull(e, nullptr, 10);
        if (v > 0 && v <= kChunk) c->host_piece = v;
    }
    c->latency_max = kLatencyMaxDefault;
    if (const char* e = getenv("BN254MI_LATENCY_MAX")) c->latency_max = (size_t)strtoull(e, nullptr, 10);
    if (const char* e = getenv("BN254MI_LATENCY_W2")) c->latency_w2 = atoi(e) != 0;
    {  // one block of kLatPairs pairs per CU: the one-wave latency build's single round
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && cus > 0)
            c->lat_w1_max = (size_t)cus * kLatPairs;
    }
    c->prepare_wide_max = kPrepareWideMaxDefault;
    // $BN254MI_FE_DS_MAX: pairing_many batches up to this size take k_fe_ds for the
    // final exponentiations (0: the latency kernel's own 16-lane FE; A/B)
    c->fe_ds_max = kFeDsMax;
    if (const char* e = getenv("BN254MI_FE_DS_MAX")) {
        const size_t v = (size_t)strtoull(e, nullptr, 10);
        c->fe_ds_max = v < (size_t)kFeDsMax ? v : (size_t)kFeDsMax;
    }
    if (const char* e = getenv("BN254MI_PREPARE_WIDE_MAX")) c->prepare_wide_max = (size_t)strtoull(e, nullptr, 10);
    Prog P;
    c->fe_out = (int)build_final_exp(P);
    P.finalize({(uint32_t)c->fe_out});
    c->fe_steps = P.steps();
    // k_pairing_full returns the last step's result as the Gt: it must be fe_out
    c->fe_last_out = c->fe_steps > 0 && (int)((P.s[2 * (c->fe_steps - 1)] >> 8) & 0xff) == c->fe_out;
    if (P.next > (uint32_t)kFeSlots) {
        delete c;  // nothing created yet
        return BN_ERR_INVALID_ARGUMENT;
    }
    bool events_ok = true;
    if (hipSetDevice(device) == hipSuccess)
        for (hipEvent_t* e : {&c->ev_in[0], &c->ev_in[1], &c->ev_comp[0], &c->ev_comp[1], &c->ev_out[0], &c->ev_out[1]})
            events_ok = events_ok && hipEventCreateWithFlags(e, hipEventDisableTiming) == hipSuccess;
    if (!events_ok || hipSetDevice(device) != hipSuccess ||
        hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&c->h2d, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&c->d2h, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&c->ws_event, hipEventDisableTiming) != hipSuccess ||
        hipMalloc(&c->d_err, sizeof(int)) != hipSuccess || hipMemset(c->d_err, 0, sizeof(int)) != hipSuccess ||
        hipMalloc(&c->tail_ws, kTailWsWords * 4) != hipSuccess || hipMemset(c->tail_ws, 0, kTailWsWords * 4) != hipSuccess ||
        hipMalloc(&c->fe_ds_ws, (size_t)kFeDsMax * kFeDsWords * 4) != hipSuccess ||
        hipMemset(c->fe_ds_ws, 0, (size_t)kFeDsMax * kFeDsWords * 4) != hipSuccess ||
        hipMalloc(&c->d_prog, P.s.size() * 4) != hipSuccess ||
        hipMemcpy(c->d_prog, P.s.data(), P.s.size() * 4, hipMemcpyHostToDevice) != hipSuccess) {
        ctx_teardown(c);  // releases whatever was created (null handles are skipped)
        return BN_ERR_HIP;
    }
    *out = c;
    return BN_OK;
}

int bn_ctx_destroy(bn_ctx* c) {
    if (!c) return BN_ERR_INVALID_ARGUMENT;
    if (!c->subs.empty()) return bn_multi_destroy(c);
    ctx_teardown(c);
    return BN_OK;
}

}  // extern "C"

// releases every resource of a single-device context (also a partially created
// one: null handles are skipped) and deletes it
static void ctx_teardown(bn_ctx* c) {
    (void)hipSetDevice(c->device);
    if (c->ws_pending) (void)hipEventSynchronize(c->ws_event);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    for (hipStream_t s : {c->h2d, c->d2h})
        if (s) (void)hipStreamSynchronize(s);
    if (c->ws_event) (void)hipEventDestroy(c->ws_event);
    for (hipEvent_t e : {c->ev_in[0], c->ev_in[1], c->ev_comp[0], c->ev_comp[1], c->ev_out[0], c->ev_out[1]})
        if (e) (void)hipEventDestroy(e);
    if (c->pin) (void)hipHostFree(c->pin);
    for (hipStream_t s : {c->h2d, c->d2h})
        if (s) (void)hipStreamDestroy(s);
    for (void* p : {(void*)c->coeffs, (void*)c->paff, (void*)c->slots, (void*)c->flags, (void*)c->d_err,
                    (void*)c->d_prog, c->stage, (void*)c->tail_ws, (void*)c->fe_ds_ws})
        if (p) (void)hipFree(p);
    for (auto& ev : c->ev_marks)
        for (auto e : ev) c->ev_pool.push_back(e);
    for (auto e : c->ev_pool)
        if (e) (void)hipEventDestroy(e);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

extern "C" {

const char* bn_last_error(const bn_ctx* c) { return c ? c->err.c_str() : "null context"; }
void* bn_ctx_stream(bn_ctx* c) { return c ? (void*)c->stream : nullptr; }
size_t bn_workspace_bytes(size_t n) { return ws_bytes(n); }

int bn_reserve(bn_ctx* c, size_t n) {
    if (c && !c->subs.empty()) {
        for (bn_ctx* d : c->subs) RET_IF(bn_reserve(d, n / c->subs.size() + 1));
        return BN_OK;
    }
    CTX_GUARD(c);
    return reserve(c, n < kChunk ? n : kChunk);
}

static hipEvent_t take_event(bn_ctx* c) {
    if (c->ev_pool.empty()) {
        hipEvent_t e;
        if (hipEventCreate(&e) != hipSuccess) return nullptr;
        return e;
    }
    hipEvent_t e = c->ev_pool.back();
    c->ev_pool.pop_back();
    return e;
}

// n pairings of device arrays on stream s; the caller holds the lock
static int pairing_many_dev_impl(bn_ctx* c, const bn_g1* d_p, const bn_g2* d_q, size_t n, bn_gt* d_out,
                                 hipStream_t s) {
    if (n == 0) return BN_OK;
    if (!d_p || !d_q || !d_out) return fail(c, BN_ERR_INVALID_ARGUMENT, "null buffer");
    RET_IF(reserve(c, n < kChunk ? n : kChunk));
    RET_IF(ws_acquire(c, s));
    WsUse use{c, s};
    for (size_t off = 0; off < n; off += kChunk) {
        const size_t m = (n - off) < kChunk ? (n - off) : kChunk;
        std::array<hipEvent_t, 5> ev{};
        if (c->timing)
            for (auto& e : ev) e = take_event(c);
        auto mark = [&](int k) {
            if (c->timing && ev[k]) (void)hipEventRecord(ev[k], s);
        };
        mark(0);
        if (m <= c->fe_wide_max && m <= c->latency_max && m <= c->fe_ds_max) {
            // the Miller values in one launch (k_pairing_latency), then each pairing's final
            // exponentiation on three digit-sliced blocks (kernels_tail.hip k_fe_ds)
            launch_latency(c, d_p + off, d_q + off, m, nullptr, slot_region(c, kRegionSeg), 0, s);
            HIPCHK(c, hipGetLastError());
            launch_fe_ds(c, slot_region(c, kRegionSeg), m, d_out + off, nullptr, s);
            mark(1);
            mark(2);
            mark(3);
            mark(4);
            HIPCHK(c, hipGetLastError());
            if (c->timing) c->ev_marks.push_back(ev);
            continue;
        }
        if (m <= c->fe_wide_max && m <= c->latency_max) {
            // the whole pairing in one launch: line producer + wide Miller loop and FE
            // (kernels_wide.hip k_pairing_latency)
            launch_latency(c, d_p + off, d_q + off, m, d_out + off, nullptr, 0, s);
            mark(1);
            mark(2);
            mark(3);
            mark(4);
            HIPCHK(c, hipGetLastError());
            if (c->timing) c->ev_marks.push_back(ev);
            continue;
        }
        if (m <= c->fe_wide_max) {
            // latency path: the Miller loop in segments on 2 * S lanes per pairing,
            // recombined and exponentiated on a 16-lane group per pairing
            const SegPlan plan = seg_plan(m);
            RET_IF(prepare(c, d_p + off, d_q + off, m, 0, s));
            mark(1);
            k_miller_seg<<<grid_pair(kPathLanes * (size_t)plan.total), kPairBlock, 0, s>>>(c->coeffs, c->paff, c->flags, m, plan,
                                                                               slot_region(c, kRegionSeg));
            mark(2);
            k_horner_wide<<<wide_blocks(m), kBlock, 0, s>>>(slot_region(c, kRegionSeg), m, plan, 1, d_out + off,
                                                              c->d_err, wide_duo(m) ? 1 : 0);
            mark(3);
            mark(4);
            HIPCHK(c, hipGetLastError());
            if (c->timing) c->ev_marks.push_back(ev);
            continue;
        }
        if (c->miller_form == 3 && c->fe_last_out) {
            k_pairing_full<<<grid_pair(kPathLanes * m), kPairBlock, 0, s>>>(d_p + off, d_q + off, m, c->d_prog,
                                                                       c->fe_steps, c->slots, d_out + off, c->d_err);
            mark(1);
            mark(2);
            mark(3);
            mark(4);
            HIPCHK(c, hipGetLastError());
            if (c->timing) c->ev_marks.push_back(ev);
            continue;
        }
        if (c->miller_form == 1 || c->miller_form == 3) {  // form 3 without fe_last_out: the fused form
            k_pairing_fused<<<grid_pair(kPathLanes * m), kPairBlock, 0, s>>>(d_p + off, d_q + off, m, c->flags, c->d_err, 0,
                                                                        c->slots);
            mark(1);
        } else {
            k_prepare<<<grid_pair(kPathLanes * m), kPairBlock, 0, s>>>(d_p + off, d_q + off, m, c->coeffs, c->paff, c->flags,
                                                                  c->d_err, 0, 1);
            mark(1);
            if (c->miller_form == 2) {  // the segment kernel with one segment: the whole loop
                const SegPlan whole = plan_layout(cut_plan(1, 1), m, 1);  // one segment: the whole loop
                k_miller_seg<<<grid_pair(kPathLanes * m), kPairBlock, 0, s>>>(c->coeffs, c->paff, c->flags, m, whole,
                                                                          c->slots);
            } else {
                k_miller<<<grid_for(kPathLanes * m), kBlock, 0, s>>>(c->coeffs, c->paff, c->flags, m, c->slots);
            }
        }
        mark(2);
        // (m > fe_wide_max here: smaller chunks took the latency path above)
        k_fq12_vm<<<grid_pair(kPathLanes * m), kPairBlock, 0, s>>>(c->d_prog, c->fe_steps, c->slots, m);
        mark(3);
        k_fe_out<<<grid_for(kPathLanes * m), kBlock, 0, s>>>(c->slots, m, c->fe_out, c->flags, d_out + off, nullptr,
                                                             c->d_err);
        mark(4);
        HIPCHK(c, hipGetLastError());
        if (c->timing) c->ev_marks.push_back(ev);
    }
    return BN_OK;
}

int bn_pairing_many_dev(bn_ctx* c, const bn_g1* d_p, const bn_g2* d_q, size_t n, bn_gt* d_out, void* stream) {
    CTX_GUARD(c);
    return pairing_many_dev_impl(c, d_p, d_q, n, d_out, pick(c, stream));
}

int bn_dev_status(bn_ctx* c, void* stream) {
    if (c && !c->subs.empty()) {
        // one caller stream cannot order the work of several devices: each device is
        // checked on its own context stream (ws_event orders it after every _dev call)
        if (stream) {
            std::lock_guard<std::mutex> g(c->err_mu);
            return fail(c, BN_ERR_INVALID_ARGUMENT, "bn_dev_status: stream must be NULL on a multi-device context");
        }
        int rc = BN_OK;
        for (bn_ctx* d : c->subs) {
            const int r = bn_dev_status(d, nullptr);
            if (r != BN_OK && (rc == BN_OK || r == BN_ERR_INTERNAL)) rc = r;
        }
        return rc;
    }
    CTX_GUARD(c);
    const hipStream_t s = pick(c, stream);
    RET_IF(ws_acquire(c, s));  // after every workspace user, on any stream
    WsUse use{c, s};
    int bits = 0;
    const int rc = check_err(c, s, &bits);
    RET_IF(clear_err(c, s));
    HIPCHK(c, hipStreamSynchronize(s));
    if (rc) return rc;
    if (bits & (1 << BN_ERR_FE_ZERO)) return fail(c, BN_ERR_FE_ZERO, "miller loop cannot produce zero");
    return BN_OK;
}

int bn_set_phase_timing(bn_ctx* c, int enable) {
    CTX_GUARD(c);
    c->timing = enable != 0;
    return BN_OK;
}

// per-phase device time of the bn_pairing_many_dev calls since the last read:
// ms[0..3] = k_prepare, k_miller, k_fq12_vm (final exponentiation), k_fe_out;
// *launches = chunk launch sets measured.  Synchronizes on the recorded events.
int bn_get_phase_times(bn_ctx* c, float* ms, int* launches) {
    CTX_GUARD(c);
    if (!ms || !launches) return fail(c, BN_ERR_INVALID_ARGUMENT, "null buffer");
    for (int k = 0; k < 4; ++k) ms[k] = 0.f;
    *launches = 0;
    for (auto& ev : c->ev_marks) {
        HIPCHK(c, hipEventSynchronize(ev[4]));
        for (int k = 0; k < 4; ++k) {
            float t = 0.f;
            HIPCHK(c, hipEventElapsedTime(&t, ev[k], ev[k + 1]));
            ms[k] += t;
        }
        ++*launches;
        for (auto e : ev) c->ev_pool.push_back(e);
    }
    c->ev_marks.clear();
    return BN_OK;
}

// bn_pairing_many on host buffers: pieces of 2^16 or 2^17 pairs flow
// through two pinned bounce buffers and two device staging halves.  Piece k's
// inputs are copied by host threads into pinned half k&1, DMA'd on the h2d
// stream, computed on the context stream and DMA'd back on the d2h stream,
// while the host copies piece k+1 in and piece k-1 out (A/B against pageable
// hipMemcpyAsync of the caller's buffers: DESIGN.md §8).  The caller's lock is
// held throughout.
static int pairing_many_host(bn_ctx* c, const bn_g1* p, const bn_g2* q, size_t n, bn_gt* out) {
    const size_t piece = n >= 2 * c->host_piece ? c->host_piece : std::min(n, kHostPieceSmall);
    const size_t o_q = round256(piece * sizeof(bn_g1));
    const size_t o_out = o_q + round256(piece * sizeof(bn_g2));
    const size_t half = o_out + round256(piece * sizeof(bn_gt));
    RET_IF(stage(c, 2 * half));
    RET_IF(pin_reserve(c, 2 * half));
    RET_IF(clear_err(c, c->stream));
    // the copy streams start after the workspace's previous users (CTX_GUARD_HOST
    // ordered c->stream after them); ev_comp doubles as "stage half free"
    for (int b = 0; b < 2; ++b) HIPCHK(c, hipEventRecord(c->ev_comp[b], c->stream));
    const size_t np = (n + piece - 1) / piece;
    auto rows = [&](size_t k) { return std::min(piece, n - k * piece); };
    auto drain = [&](size_t k) -> int {  // piece k's results: pinned -> caller
        const int b = (int)(k & 1);
        HIPCHK(c, hipEventSynchronize(c->ev_out[b]));
        par_copy(out + k * piece, (uint8_t*)c->pin + b * half + o_out, rows(k) * sizeof(bn_gt));
        return BN_OK;
    };
    for (size_t k = 0; k < np; ++k) {
        const int b = (int)(k & 1);
        const size_t off = k * piece, m = rows(k);
        if (k >= 2) RET_IF(drain(k - 2));  // frees pinned half b (and its D2H source)
        uint8_t* hp = (uint8_t*)c->pin + b * half;
        uint8_t* dp = (uint8_t*)c->stage + b * half;
        par_copy(hp, p + off, m * sizeof(bn_g1));
        par_copy(hp + o_q, q + off, m * sizeof(bn_g2));
        HIPCHK(c, hipStreamWaitEvent(c->h2d, c->ev_comp[b], 0));  // piece k-2 has read stage half b
        HIPCHK(c, hipMemcpyAsync(dp, hp, m * sizeof(bn_g1), hipMemcpyHostToDevice, c->h2d));
        HIPCHK(c, hipMemcpyAsync(dp + o_q, hp + o_q, m * sizeof(bn_g2), hipMemcpyHostToDevice, c->h2d));
        HIPCHK(c, hipEventRecord(c->ev_in[b], c->h2d));
        HIPCHK(c, hipStreamWaitEvent(c->stream, c->ev_in[b], 0));
        RET_IF(pairing_many_dev_impl(c, (const bn_g1*)dp, (const bn_g2*)(dp + o_q), m, (bn_gt*)(dp + o_out),
                                     c->stream));
        HIPCHK(c, hipEventRecord(c->ev_comp[b], c->stream));
        HIPCHK(c, hipStreamWaitEvent(c->d2h, c->ev_comp[b], 0));
        HIPCHK(c, hipMemcpyAsync(hp + o_out, dp + o_out, m * sizeof(bn_gt), hipMemcpyDeviceToHost, c->d2h));
        HIPCHK(c, hipEventRecord(c->ev_out[b], c->d2h));
    }
    for (size_t k = np >= 2 ? np - 2 : 0; k < np; ++k) RET_IF(drain(k));
    int bits = 0;
    RET_IF(check_err(c, c->stream, &bits));
    if (bits & (1 << BN_ERR_FE_ZERO)) return fail(c, BN_ERR_FE_ZERO, "miller loop cannot produce zero");
    return BN_OK;
}

// the A/B form ($BN254MI_HOST_PIPELINE=0): hipMemcpyAsync straight from and to
// the caller's (pageable) buffers, one chunk at a time on the context stream
static int pairing_many_pageable(bn_ctx* c, const bn_g1* p, const bn_g2* q, size_t n, bn_gt* out) {
    for (size_t off = 0; off < n; off += kChunk) {
        const size_t m = (n - off) < kChunk ? (n - off) : kChunk;
        RET_IF(stage(c, m * (sizeof(bn_g1) + sizeof(bn_g2) + sizeof(bn_gt))));
        bn_g1* dp = (bn_g1*)c->stage;
        bn_g2* dq = (bn_g2*)(dp + m);
        bn_gt* dout = (bn_gt*)(dq + m);
        RET_IF(clear_err(c, c->stream));
        HIPCHK(c, hipMemcpyAsync(dp, p + off, m * sizeof(bn_g1), hipMemcpyHostToDevice, c->stream));
        HIPCHK(c, hipMemcpyAsync(dq, q + off, m * sizeof(bn_g2), hipMemcpyHostToDevice, c->stream));
        RET_IF(pairing_many_dev_impl(c, dp, dq, m, dout, c->stream));
        HIPCHK(c, hipMemcpyAsync(out + off, dout, m * sizeof(bn_gt), hipMemcpyDeviceToHost, c->stream));
        int bits = 0;
        RET_IF(check_err(c, c->stream, &bits));
        if (bits & (1 << BN_ERR_FE_ZERO)) return fail(c, BN_ERR_FE_ZERO, "miller loop cannot produce zero");
    }
    return BN_OK;
}

int bn_pairing_many(bn_ctx* c, const bn_g1* p, const bn_g2* q, size_t n, bn_gt* out) {
    if (c && !c->subs.empty()) return bn_multi_pairing_many(c, p, q, n, out);
    CTX_GUARD_HOST(c);  // held for the whole call: staging, kernels, readback
    if (n == 0) return BN_OK;
    if (!p || !q || !out) return fail(c, BN_ERR_INVALID_ARGUMENT, "null buffer");
    // one piece has nothing to overlap, and the runtime's own pageable copies
    // measured ~6 % faster there (12.0 vs 12.6 ms at 2^16 pairs); the pipeline
    // wins from two pieces on (2^20: 171 vs 191-199 ms; profiles/r2ak_host_e2e_ab.jsonl)
    const bool pipe = c->host_pipeline == 2 || (c->host_pipeline == 1 && n > kHostPieceSmall);
    const int rc = pipe ? pairing_many_host(c, p, q, n, out) : pairing_many_pageable(c, p, q, n, out);
    // an early error may leave copies queued: nothing may still touch the pinned
    // or staging buffers when the call returns
    (void)hipStreamSynchronize(c->h2d);
    (void)hipStreamSynchronize(c->d2h);
    (void)hipStreamSynchronize(c->stream);
    return rc;
}

// The Miller product of n host pairs -> *out (host image), then pairing_batch's
// final exponentiation when do_fe; mode 0 skips pairs with a zero point, mode 1
// (miller_loop_batch) rejects them.  Chunks of kChunk pairs are staged in turn.
// BN_ERR_TO_AFFINE / BN_ERR_FE_ZERO come from the device bits.
static int batch_host(bn_ctx* c, const bn_g1* p, const bn_g2* q, size_t n, int mode, bool do_fe, bn_gt* out) {
    RET_IF(clear_err(c, c->stream));
    if (use_latency_product(c, n)) {
        RET_IF(stage(c, n * (sizeof(bn_g1) + sizeof(bn_g2)) + sizeof(bn_gt)));
        bn_g1* dp = (bn_g1*)c->stage;
        bn_g2* dq = (bn_g2*)(dp + n);
        bn_gt* d = (bn_gt*)(dq + n);
        HIPCHK(c, hipMemcpyAsync(dp, p, n * sizeof(bn_g1), hipMemcpyHostToDevice, c->stream));
        HIPCHK(c, hipMemcpyAsync(dq, q, n * sizeof(bn_g2), hipMemcpyHostToDevice, c->stream));
        RET_IF(latency_product(c, dp, dq, n, mode, do_fe ? 1 : 0, d, c->stream));
        HIPCHK(c, hipMemcpyAsync(out, d, sizeof(bn_gt), hipMemcpyDeviceToHost, c->stream));
        int bits = 0;
        RET_IF(check_err(c, c->stream, &bits));
        if (bits & (1 << BN_ERR_TO_AFFINE)) return fail(c, BN_ERR_TO_AFFINE, "ToAffineConversion");
        if (bits & (1 << BN_ERR_FE_ZERO)) return fail(c, BN_ERR_FE_ZERO, "miller loop cannot produce zero");
        return BN_OK;
    }
    const size_t nchunks = (n + kChunk - 1) / kChunk;
    const size_t m0 = n < kChunk ? n : kChunk;
    const SegPlan plan = batch_plan(m0);
    RET_IF(reserve(c, m0));
    if (nchunks * plan.S > c->cap) return fail(c, BN_ERR_INVALID_ARGUMENT, "too many chunks");
    uint32_t* parts = parts_region(c, nchunks);
    for (size_t k = 0; k < nchunks; ++k) {
        const size_t off = k * kChunk, m = (n - off) < kChunk ? (n - off) : kChunk;
        RET_IF(stage(c, m * (sizeof(bn_g1) + sizeof(bn_g2)) + sizeof(bn_gt)));
        bn_g1* dp = (bn_g1*)c->stage;
        bn_g2* dq = (bn_g2*)(dp + m);
        HIPCHK(c, hipMemcpyAsync(dp, p + off, m * sizeof(bn_g1), hipMemcpyHostToDevice, c->stream));
        HIPCHK(c, hipMemcpyAsync(dq, q + off, m * sizeof(bn_g2), hipMemcpyHostToDevice, c->stream));
        RET_IF(chunk_product(c, dp, dq, m, mode, plan, parts, nchunks, k, c->stream));
        if (k + 1 < nchunks) HIPCHK(c, hipStreamSynchronize(c->stream));  // the stage is reused
    }
    bn_gt* d = (bn_gt*)c->stage;  // the stage holds at least one Gt past the inputs
    RET_IF(finish_product(c, plan, nchunks, do_fe, d, c->stream));
    HIPCHK(c, hipMemcpyAsync(out, d, sizeof(bn_gt), hipMemcpyDeviceToHost, c->stream));
    int bits = 0;
    RET_IF(check_err(c, c->stream, &bits));
    if (bits & (1 << BN_ERR_TO_AFFINE)) return fail(c, BN_ERR_TO_AFFINE, "ToAffineConversion");
    if (bits & (1 << BN_ERR_FE_ZERO)) return fail(c, BN_ERR_FE_ZERO, "miller loop cannot produce zero");
    return BN_OK;
}

// the Miller product of n host pairs on one single-device context (its lock held)
int bn_internal_miller_product(bn_ctx* c, const bn_g1* p, const bn_g2* q, size_t n, int mode, bn_gt* result) {
    CTX_GUARD_HOST(c);
    return batch_host(c, p, q, n, mode, false, result);
}

void bn_internal_gt_one(bn_gt* out);
static void gt_one(bn_gt* out) { bn_internal_gt_one(out); }
void bn_internal_gt_one(bn_gt* out) {  // Fq12::one() image: c0.c0.c0 = R mod p
    memset(out, 0, sizeof(bn_gt));
    out->c[0].l[0] = 0xd35d438dc58f0d9dull;
    out->c[0].l[1] = 0x0a78eb28f5c70b3dull;
    out->c[0].l[2] = 0x666ea36f7879462cull;
    out->c[0].l[3] = 0x0e0a77c19a07df2full;
}

// final exponentiation of n host images; ok may be null
static int final_exp_host(bn_ctx* c, const bn_gt* f, size_t n, bn_gt* out, uint8_t* ok, int* zero_seen) {
    *zero_seen = 0;
    for (size_t off = 0; off < n; off += kChunk) {
        const size_t m = (n - off) < kChunk ? (n - off) : kChunk;
        RET_IF(reserve(c, m));
        RET_IF(stage(c, m * (2 * sizeof(bn_gt) + 1)));
        bn_gt* din = (bn_gt*)c->stage;
        bn_gt* dout = din + m;
        uint8_t* dok = (uint8_t*)(dout + m);
        HIPCHK(c, hipMemcpyAsync(din, f + off, m * sizeof(bn_gt), hipMemcpyHostToDevice, c->stream));
        k_gt_load<<<grid_for(kPathLanes * m), kBlock, 0, c->stream>>>(din, m, c->slots);
        HIPCHK(c, hipGetLastError());
        RET_IF(run_fe(c, c->slots, m, nullptr, dout, dok, c->stream));
        HIPCHK(c, hipMemcpyAsync(out + off, dout, m * sizeof(bn_gt), hipMemcpyDeviceToHost, c->stream));
        if (ok) HIPCHK(c, hipMemcpyAsync(ok + off, dok, m, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
    }
    int bits = 0;
    RET_IF(check_err(c, c->stream, &bits));
    *zero_seen = (bits & (1 << BN_ERR_FE_ZERO)) != 0;
    return BN_OK;
}

int bn_pairing_batch(bn_ctx* c, const bn_g1* p, const bn_g2* q, size_t n, bn_gt* out) {
    if (c && !c->subs.empty()) return bn_multi_pairing_batch(c, p, q, n, out);
    CTX_GUARD_HOST(c);
    if (!out || (n && (!p || !q))) return fail(c, BN_ERR_INVALID_ARGUMENT, "null buffer");
    if (n == 0) {  // mod.rs:922-924
        gt_one(out);
        return BN_OK;
    }
    return batch_host(c, p, q, n, 0, true, out);
}

int bn_miller_loop_batch(bn_ctx* c, const bn_g2* q, const bn_g1* p, size_t n, bn_gt* out) {
    if (c && !c->subs.empty()) return bn_multi_miller_loop_batch(c, q, p, n, out);
    CTX_GUARD_HOST(c);
    if (!out || (n && (!p || !q))) return fail(c, BN_ERR_INVALID_ARGUMENT, "null buffer");
    if (n == 0) {  // the shared loop starts from Fq12::one() (mod.rs:610)
        gt_one(out);
        return BN_OK;
    }
    return batch_host(c, p, q, n, 1, false, out);
}

// ---- device-pointer forms of pairing_batch / miller_loop_batch (config 5 with HBM-resident inputs)
static int batch_dev(bn_ctx* c, const bn_g1* d_p, const bn_g2* d_q, size_t n, bn_gt* d_out, int* d_status,
                     int mode, hipStream_t s) {
    if (!d_out || (n && (!d_p || !d_q))) return fail(c, BN_ERR_INVALID_ARGUMENT, "null buffer");
    RET_IF(reserve(c, n == 0 ? 1 : n < kChunk ? n : kChunk));
    RET_IF(ws_acquire(c, s));
    WsUse use{c, s};
    HIPCHK(c, hipMemsetAsync(c->d_err, 0, sizeof(int), s));
    if (n == 0) {  // pairing_batch: mod.rs:922-924; the shared loop starts from one (mod.rs:610)
        // a constant-initialized, read-only image: no thread ever writes it
        static const bn_gt kGtOne = {{{{0xd35d438dc58f0d9dull, 0x0a78eb28f5c70b3dull, 0x666ea36f7879462cull,
                                        0x0e0a77c19a07df2full}}}};
        HIPCHK(c, hipMemcpyAsync(d_out, &kGtOne, sizeof(bn_gt), hipMemcpyHostToDevice, s));
    } else {
        RET_IF(miller_product_dev(c, d_p, d_q, n, mode, d_out, s));
    }
    if (d_status) {
        k_err_status<<<1, 64, 0, s>>>(c->d_err, d_status);
        HIPCHK(c, hipGetLastError());
    }
    return BN_OK;
}
int bn_pairing_batch_dev(bn_ctx* c, const bn_g1* d_p, const bn_g2* d_q, size_t n, bn_gt* d_out, int* d_status,
                         void* stream) {
    CTX_GUARD(c);
    return batch_dev(c, d_p, d_q, n, d_out, d_status, 0, pick(c, stream));
}
int bn_miller_loop_batch_dev(bn_ctx* c, const bn_g2* d_q, const bn_g1* d_p, size_t n, bn_gt* d_out, int* d_status,
                             void* stream) {
    CTX_GUARD(c);
    return batch_dev(c, d_p, d_q, n, d_out, d_status, 1, pick(c, stream));
}
int bn_set_latency_max(bn_ctx* c, size_t n) {
    if (c && !c->subs.empty()) {
        for (bn_ctx* d : c->subs) RET_IF(bn_set_latency_max(d, n));
        return BN_OK;
    }
    CTX_GUARD(c);
    c->latency_max = n;
    return BN_OK;
}
int bn_set_fe_wide_max(bn_ctx* c, size_t n) {
    if (c && !c->subs.empty()) {
        for (bn_ctx* d : c->subs) RET_IF(bn_set_fe_wide_max(d, n));
        return BN_OK;
    }
    CTX_GUARD(c);
    c->fe_wide_max = n;
    return BN_OK;
}

int bn_final_exponentiation_many(bn_ctx* c, const bn_gt* f, size_t n, bn_gt* out, uint8_t* ok) {
    if (c && !c->subs.empty()) return bn_multi_final_exponentiation_many(c, f, n, out, ok);
    CTX_GUARD_HOST(c);
    if (n == 0) return BN_OK;
    if (!f || !out) return fail(c, BN_ERR_INVALID_ARGUMENT, "null buffer");
    RET_IF(clear_err(c, c->stream));
    int zero = 0;
    return final_exp_host(c, f, n, out, ok, &zero);
}

int bn_miller_loop_many(bn_ctx* c, const bn_g1* p, const bn_g2* q, size_t n, bn_gt* out) {
    if (c && !c->subs.empty()) return bn_multi_miller_loop_many(c, p, q, n, out);
    CTX_GUARD_HOST(c);
    if (n == 0) return BN_OK;
    if (!p || !q || !out) return fail(c, BN_ERR_INVALID_ARGUMENT, "null buffer");
    for (size_t off = 0; off < n; off += kChunk) {
        const size_t m = (n - off) < kChunk ? (n - off) : kChunk;
        RET_IF(reserve(c, m));
        RET_IF(stage(c, m * (sizeof(bn_g1) + sizeof(bn_g2) + sizeof(bn_gt))));
        bn_g1* dp = (bn_g1*)c->stage;
        bn_g2* dq = (bn_g2*)(dp + m);
        bn_gt* dout = (bn_gt*)(dq + m);
        HIPCHK(c, hipMemcpyAsync(dp, p + off, m * sizeof(bn_g1), hipMemcpyHostToDevice, c->stream));
        HIPCHK(c, hipMemcpyAsync(dq, q + off, m * sizeof(bn_g2), hipMemcpyHostToDevice, c->stream));
        RET_IF(miller_values(c, dp, dq, m, 0, c->stream));
        k_gt_store<<<grid_for(kPathLanes * m), kBlock, 0, c->stream>>>(c->slots, m, m, dout);
        HIPCHK(c, hipGetLastError());
        HIPCHK(c, hipMemcpyAsync(out + off, dout, m * sizeof(bn_gt), hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
    }
    return BN_OK;
}

int bn_g2_precompute_many(bn_ctx* c, const bn_g2* q, size_t n, bn_fq2* out) {
    CTX_GUARD_HOST(c);
    if (n == 0) return BN_OK;
    if (!q || !out) return fail(c, BN_ERR_INVALID_ARGUMENT, "null buffer");
    RET_IF(clear_err(c, c->stream));
    bn_g1 one;  // k_prepare converts a G1 point too; G1::one() (z = 1) is never zero
    memset(&one, 0, sizeof one);
    one.x.l[0] = 0xd35d438dc58f0d9dull, one.x.l[1] = 0x0a78eb28f5c70b3dull;  // Fq::one(): R mod p
    one.x.l[2] = 0x666ea36f7879462cull, one.x.l[3] = 0x0e0a77c19a07df2full;
    one.z = one.x;
    for (size_t off = 0; off < n; off += kChunk) {
        const size_t m = (n - off) < kChunk ? (n - off) : kChunk;
        RET_IF(reserve(c, m));
        const size_t out_bytes = m * (size_t)BN_NUM_COEFFS * 3 * sizeof(bn_fq2);
        RET_IF(stage(c, m * (sizeof(bn_g1) + sizeof(bn_g2)) + out_bytes));
        bn_g1* dp = (bn_g1*)c->stage;
        bn_g2* dq = (bn_g2*)(dp + m);
        bn_fq2* dout = (bn_fq2*)(dq + m);
        std::vector<bn_g1> ones(m, one);
        HIPCHK(c, hipMemcpyAsync(dp, ones.data(), m * sizeof(bn_g1), hipMemcpyHostToDevice, c->stream));
        HIPCHK(c, hipMemcpyAsync(dq, q + off, m * sizeof(bn_g2), hipMemcpyHostToDevice, c->stream));
        RET_IF(prepare(c, dp, dq, m, 1, c->stream, 0));  // the reference's (unscaled) coefficients
        k_coeffs_store<<<grid_for(kPathLanes * m), kBlock, 0, c->stream>>>(c->coeffs, m, dout);
        HIPCHK(c, hipGetLastError());
        HIPCHK(c, hipMemcpyAsync(out + off * BN_NUM_COEFFS * 3, dout, out_bytes, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
    }
    int bits = 0;
    RET_IF(check_err(c, c->stream, &bits));
    if (bits & (1 << BN_ERR_TO_AFFINE)) return fail(c, BN_ERR_TO_AFFINE, "ToAffineConversion");
    return BN_OK;
}

int bn_g1_mul_many_dev(bn_ctx* c, const bn_g1* d_p, const bn_fr* d_k, size_t n, bn_g1* d_out, void* stream) {
    CTX_GUARD(c);
    if (n == 0) return BN_OK;
    if (!d_p || !d_k || !d_out) return fail(c, BN_ERR_INVALID_ARGUMENT, "null buffer");
    g1_mul_launch(d_p, d_k, n, d_out, pick(c, stream));
    HIPCHK(c, hipGetLastError());
    return BN_OK;
}
int bn_g2_mul_many_dev(bn_ctx* c, const bn_g2* d_p, const bn_fr* d_k, size_t n, bn_g2* d_out, void* stream) {
    CTX_GUARD(c);
    if (n == 0) return BN_OK;
    if (!d_p || !d_k || !d_out) return fail(c, BN_ERR_INVALID_ARGUMENT, "null buffer");
    g2_mul_launch(d_p, d_k, n, d_out, pick(c, stream));
    HIPCHK(c, hipGetLastError());
    return BN_OK;
}
int bn_g1_mul_many(bn_ctx* c, const bn_g1* p, const bn_fr* k, size_t n, bn_g1* out) {
    if (c && !c->subs.empty()) return bn_multi_g1_mul_many(c, p, k, n, out);
    return host_mul(c, p, k, n, out, g1_mul_launch);
}
int bn_g2_mul_many(bn_ctx* c, const bn_g2* p, const bn_fr* k, size_t n, bn_g2* out) {
    if (c && !c->subs.empty()) return bn_multi_g2_mul_many(c, p, k, n, out);
    return host_mul(c, p, k, n, out, g2_mul_launch);
}

int bn_fq12_op_many(bn_ctx* c, int op, const bn_gt* a, const bn_gt* b, size_t n, bn_gt* out) {
    CTX_GUARD_HOST(c);
    if (n == 0) return BN_OK;
    if (op < 0 || op > BN_FQ12_FROB3) return fail(c, BN_ERR_INVALID_ARGUMENT, "bad op");
    if (!a || !out || (op == BN_FQ12_MUL && !b)) return fail(c, BN_ERR_INVALID_ARGUMENT, "null buffer");
    for (size_t off = 0; off < n; off += kChunk) {
        const size_t m = (n - off) < kChunk ? (n - off) : kChunk;
        RET_IF(reserve(c, m));
        RET_IF(stage(c, m * 3 * sizeof(bn_gt) + 4096));
        bn_gt* da = (bn_gt*)c->stage;
        bn_gt* db = da + m;
        bn_gt* dout = db + m;
        uint32_t* dprog = (uint32_t*)(dout + m);
        HIPCHK(c, hipMemcpyAsync(da, a + off, m * sizeof(bn_gt), hipMemcpyHostToDevice, c->stream));
        k_gt_load<<<grid_for(kPathLanes * m), kBlock, 0, c->stream>>>(da, m, c->slots + (size_t)1 * kSlotWords * m);
        if (op == BN_FQ12_MUL) {
            HIPCHK(c, hipMemcpyAsync(db, b + off, m * sizeof(bn_gt), hipMemcpyHostToDevice, c->stream));
            k_gt_load<<<grid_for(kPathLanes * m), kBlock, 0, c->stream>>>(db, m, c->slots + (size_t)2 * kSlotWords * m);
        }
        Prog P;
        P.next = 3;
        uint32_t res = P.tmp();
        switch (op) {
            case BN_FQ12_MUL: P.op(OP_MUL, res, 1, 2); break;
            case BN_FQ12_SQR: P.op(OP_SQR, res, 1); break;
            case BN_FQ12_INV: P.op(OP_INV, res, 1); break;
            case BN_FQ12_CYC_SQR: P.op(OP_CYC, res, 1); break;
            case BN_FQ12_EXP_BY_NEG_Z: res = P.exp_by_neg_z(1); break;
            case BN_FQ12_FROB1: P.op(OP_FROB1, res, 1); break;
            case BN_FQ12_FROB2: P.op(OP_FROB2, res, 1); break;
            default: P.op(OP_FROB3, res, 1); break;
        }
        P.finalize({res});
        HIPCHK(c, hipMemcpyAsync(dprog, P.s.data(), P.s.size() * 4, hipMemcpyHostToDevice, c->stream));
        k_fq12_vm<<<grid_pair(kPathLanes * m), kPairBlock, 0, c->stream>>>(dprog, P.steps(), c->slots, m);
        k_gt_store<<<grid_for(kPathLanes * m), kBlock, 0, c->stream>>>(c->slots + (size_t)res * kSlotWords * m, m, m, dout);
        HIPCHK(c, hipGetLastError());
        HIPCHK(c, hipMemcpyAsync(out + off, dout, m * sizeof(bn_gt), hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
    }
    return BN_OK;
}

// ---------------------------------------------------------------- encodings / validation
int bn_fq_from_slice_many(bn_ctx* c, const uint8_t* be32, size_t n, bn_fq* out, uint8_t* st) {
    CTX_GUARD_HOST(c);
    return staged(c, n, {{be32, 32}}, {{out, sizeof(bn_fq)}, {st, 1}}, [&](void** d, size_t m, hipStream_t s) -> int {
        KL(k_fq_from_slice, (const uint8_t*)d[0], m, (bn_fq*)d[1], (uint8_t*)d[2]);
        return BN_OK;
    });
}
int bn_fq_to_big_endian_many(bn_ctx* c, const bn_fq* a, size_t n, uint8_t* be32) {
    CTX_GUARD_HOST(c);
    return staged(c, n, {{a, sizeof(bn_fq)}}, {{be32, 32}}, [&](void** d, size_t m, hipStream_t s) -> int {
        KL(k_fq_to_be, (const bn_fq*)d[0], m, (uint8_t*)d[1]);
        return BN_OK;
    });
}
int bn_fq2_from_slice_many(bn_ctx* c, const uint8_t* be64, size_t n, bn_fq2* out, uint8_t* st) {
    CTX_GUARD_HOST(c);
    return staged(c, n, {{be64, 64}}, {{out, sizeof(bn_fq2)}, {st, 1}}, [&](void** d, size_t m, hipStream_t s) -> int {
        KL(k_fq2_from_slice, (const uint8_t*)d[0], m, (bn_fq2*)d[1], (uint8_t*)d[2]);
        return BN_OK;
    });
}
int bn_fr_from_slice_many(bn_ctx* c, const uint8_t* be32, size_t n, bn_fr* out) {
    CTX_GUARD_HOST(c);
    return staged(c, n, {{be32, 32}}, {{out, sizeof(bn_fr)}}, [&](void** d, size_t m, hipStream_t s) -> int {
        KL(k_fr_from_slice, (const uint8_t*)d[0], m, (bn_fr*)d[1]);
        return BN_OK;
    });
}
int bn_fr_to_big_endian_many(bn_ctx* c, const bn_fr* a, size_t n, uint8_t* be32) {
    CTX_GUARD_HOST(c);
    return staged(c, n, {{a, sizeof(bn_fr)}}, {{be32, 32}}, [&](void** d, size_t m, hipStream_t s) -> int {
        KL(k_fr_to_be, (const bn_fr*)d[0], m, (uint8_t*)d[1]);
        return BN_OK;
    });
}
int bn_fq_sqrt_many(bn_ctx* c, const bn_fq* a, size_t n, bn_fq* out, uint8_t* ok) {
    CTX_GUARD_HOST(c);
    return staged(c, n, {{a, sizeof(bn_fq)}}, {{out, sizeof(bn_fq)}, {ok, 1}}, [&](void** d, size_t m, hipStream_t s) -> int {
        KL(k_fq_sqrt, (const bn_fq*)d[0], m, (bn_fq*)d[1], (uint8_t*)d[2]);
        return BN_OK;
    });
}
int bn_fq2_sqrt_many(bn_ctx* c, const bn_fq2* a, size_t n, bn_fq2* out, uint8_t* ok) {
    CTX_GUARD_HOST(c);
    return staged(c, n, {{a, sizeof(bn_fq2)}}, {{out, sizeof(bn_fq2)}, {ok, 1}}, [&](void** d, size_t m, hipStream_t s) -> int {
        KL(k_fq2_sqrt, (const bn_fq2*)d[0], m, (bn_fq2*)d[1], (uint8_t*)d[2]);
        return BN_OK;
    });
}
int bn_g1_affine_new_many(bn_ctx* c, const bn_fq* x, const bn_fq* y, size_t n, bn_g1* out, uint8_t* st) {
    CTX_GUARD_HOST(c);
    return staged(c, n, {{x, sizeof(bn_fq)}, {y, sizeof(bn_fq)}}, {{out, sizeof(bn_g1)}, {st, 1}},
                  [&](void** d, size_t m, hipStream_t s) -> int {
                      KL(k_g1_affine_new, (const bn_fq*)d[0], (const bn_fq*)d[1], m, (bn_g1*)d[2], (uint8_t*)d[3]);
                      return BN_OK;
                  });
}
int bn_g2_affine_new_many(bn_ctx* c, const bn_fq2* x, const bn_fq2* y, size_t n, bn_g2* out, uint8_t* st) {
    CTX_GUARD_HOST(c);
    return staged(c, n, {{x, sizeof(bn_fq2)}, {y, sizeof(bn_fq2)}}, {{out, sizeof(bn_g2)}, {st, 1}},
                  [&](void** d, size_t m, hipStream_t s) -> int {
                      KL(k_g2_affine_new, (const bn_fq2*)d[0], (const bn_fq2*)d[1], m, (bn_g2*)d[2], (uint8_t*)d[3]);
                      return BN_OK;
                  });
}
int bn_g2_affine_new_many_dev(bn_ctx* c, const bn_fq2* d_x, const bn_fq2* d_y, size_t n, bn_g2* d_out, uint8_t* d_st,
                              void* stream) {
    CTX_GUARD(c);
    if (n == 0) return BN_OK;
    if (!d_x || !d_y || !d_out || !d_st) return fail(c, BN_ERR_INVALID_ARGUMENT, "null buffer");
    k_g2_affine_new<<<grid_for(n), kBlock, 0, pick(c, stream)>>>(d_x, d_y, n, d_out, d_st);
    HIPCHK(c, hipGetLastError());
    return BN_OK;
}
int bn_g1_from_compressed_many(bn_ctx* c, const uint8_t* b33, size_t n, bn_g1* out, uint8_t* st) {
    CTX_GUARD_HOST(c);
    return staged(c, n, {{b33, 33}}, {{out, sizeof(bn_g1)}, {st, 1}}, [&](void** d, size_t m, hipStream_t s) -> int {
        KL(k_g1_from_compressed, (const uint8_t*)d[0], m, (bn_g1*)d[1], (uint8_t*)d[2]);
        return BN_OK;
    });
}
int bn_g2_from_compressed_many(bn_ctx* c, const uint8_t* b65, size_t n, bn_g2* out, uint8_t* st) {
    CTX_GUARD_HOST(c);
    return staged(c, n, {{b65, 65}}, {{out, sizeof(bn_g2)}, {st, 1}}, [&](void** d, size_t m, hipStream_t s) -> int {
        KL(k_g2_from_compressed, (const uint8_t*)d[0], m, (bn_g2*)d[1], (uint8_t*)d[2]);
        return BN_OK;
    });
}
int bn_g1_from_compressed_many_dev(bn_ctx* c, const uint8_t* d_b, size_t n, bn_g1* d_out, uint8_t* d_st, void* stream) {
    CTX_GUARD(c);
    if (n == 0) return BN_OK;
    if (!d_b || !d_out || !d_st) return fail(c, BN_ERR_INVALID_ARGUMENT, "null buffer");
    k_g1_from_compressed<<<grid_for(n), kBlock, 0, pick(c, stream)>>>(d_b, n, d_out, d_st);
    HIPCHK(c, hipGetLastError());
    return BN_OK;
}
int bn_g2_from_compressed_many_dev(bn_ctx* c, const uint8_t* d_b, size_t n, bn_g2* d_out, uint8_t* d_st, void* stream) {
    CTX_GUARD(c);
    if (n == 0) return BN_OK;
    if (!d_b || !d_out || !d_st) return fail(c, BN_ERR_INVALID_ARGUMENT, "null buffer");
    k_g2_from_compressed<<<grid_for(n), kBlock, 0, pick(c, stream)>>>(d_b, n, d_out, d_st);
    HIPCHK(c, hipGetLastError());
    return BN_OK;
}
// Gt::pow: the per-lane window table lives in the context's Fq12 slots (kGtPowEntries
// of kFeSlots); k_gt_pow addresses a lane's entry by a 32-bit buffer offset
// (ld_fq12_buf_sel): entry t < kGtPowEntries starts at t * kSlotWords * kChunk * 4
// bytes and its lane copies lie below (t + 1) * kSlotWords * kChunk * 4
static_assert(kGtPowEntries <= kFeSlots, "k_gt_pow's window table must fit the context's Fq12 slots");
static_assert((unsigned long long)kGtPowEntries * kSlotWords * kChunk * 4 < (1ull << 31),
              "k_gt_pow window-table offsets must fit the buffer descriptor's 31-bit range");
int bn_gt_pow_many_dev(bn_ctx* c, const bn_gt* d_a, const bn_fr* d_k, size_t n, bn_gt* d_out, void* stream) {
    CTX_GUARD(c);
    if (n == 0) return BN_OK;
    if (!d_a || !d_k || !d_out) return fail(c, BN_ERR_INVALID_ARGUMENT, "null buffer");
    RET_IF(reserve(c, n < kChunk ? n : kChunk));
    hipStream_t s = pick(c, stream);
    RET_IF(ws_acquire(c, s));
    WsUse use{c, s};
    for (size_t off = 0; off < n; off += kChunk) {
        const size_t m = (n - off) < kChunk ? (n - off) : kChunk;
        k_gt_pow<<<grid_pair(kPathLanes * m), kPairBlock, 0, s>>>(d_a + off, d_k + off, m, d_out + off, c->slots);
        HIPCHK(c, hipGetLastError());
    }
    return BN_OK;
}
int bn_gt_pow_many(bn_ctx* c, const bn_gt* a, const bn_fr* k, size_t n, bn_gt* out) {
    CTX_GUARD_HOST(c);
    return staged(c, n, {{a, sizeof(bn_gt)}, {k, sizeof(bn_fr)}}, {{out, sizeof(bn_gt)}},
                  [&](void** d, size_t m, hipStream_t s) -> int {
                      RET_IF(reserve(c, m));
                      k_gt_pow<<<grid_pair(kPathLanes * m), kPairBlock, 0, s>>>((const bn_gt*)d[0], (const bn_fr*)d[1], m, (bn_gt*)d[2],
                                                                         c->slots);
                      return BN_OK;
                  });
}

}  // extern "C"

// ---------------------------------------------------------------- group law
// (lib.rs:388-423, 539-574; mod.rs:169-216, 294-358): one lane per element,
// k_g1_op / k_g2_op.  Host forms stage chunks of kChunk elements through the
// context; _dev forms enqueue on the stream.  b is read for add / sub / eq only.
template <class P>
static void group_launch(int op, const P* a, const P* b, size_t n, P* out, uint8_t* eq, hipStream_t s) {
    if constexpr (sizeof(P) == sizeof(bn_g1))
        k_g1_op<<<grid_for(n), kBlock, 0, s>>>(op, a, b, n, out, eq);
    else
        k_g2_op<<<grid_for(n), kBlock, 0, s>>>(op, a, b, n, out, eq);
}
static bool group_binary(int op) { return op == kGroupAdd || op == kGroupSub || op == kGroupEq; }
template <class P>
static int group_host(bn_ctx* c, int op, const P* a, const P* b, size_t n, P* out, uint8_t* eq) {
    CTX_GUARD_HOST(c);
    const bool two = group_binary(op);
    auto run = [&](void** d, size_t m, hipStream_t s) -> int {
        const P* db = two ? (const P*)d[1] : nullptr;
        void* o = d[two ? 2 : 1];
        group_launch<P>(op, (const P*)d[0], db, m, op == kGroupEq ? nullptr : (P*)o,
                        op == kGroupEq ? (uint8_t*)o : nullptr, s);
        return BN_OK;
    };
    const HostOut dst = op == kGroupEq ? HostOut{eq, 1} : HostOut{out, sizeof(P)};
    if (two) return staged(c, n, {{a, sizeof(P)}, {b, sizeof(P)}}, {dst}, run);
    return staged(c, n, {{a, sizeof(P)}}, {dst}, run);
}
template <class P>
static int group_dev(bn_ctx* c, int op, const P* d_a, const P* d_b, size_t n, P* d_out, uint8_t* d_eq, void* stream) {
    CTX_GUARD(c);
    if (n == 0) return BN_OK;
    if (!d_a || (group_binary(op) && !d_b) || (op == kGroupEq ? !d_eq : !d_out))
        return fail(c, BN_ERR_INVALID_ARGUMENT, "null buffer");
    group_launch<P>(op, d_a, group_binary(op) ? d_b : nullptr, n, d_out, d_eq, pick(c, stream));
    HIPCHK(c, hipGetLastError());
    return BN_OK;
}

extern "C" {

int bn_g1_add_many(bn_ctx* c, const bn_g1* a, const bn_g1* b, size_t n, bn_g1* out) {
    return group_host(c, kGroupAdd, a, b, n, out, nullptr);
}
int bn_g1_sub_many(bn_ctx* c, const bn_g1* a, const bn_g1* b, size_t n, bn_g1* out) {
    return group_host(c, kGroupSub, a, b, n, out, nullptr);
}
int bn_g1_neg_many(bn_ctx* c, const bn_g1* a, size_t n, bn_g1* out) {
    return group_host<bn_g1>(c, kGroupNeg, a, nullptr, n, out, nullptr);
}
int bn_g1_normalize_many(bn_ctx* c, const bn_g1* a, size_t n, bn_g1* out) {
    return group_host<bn_g1>(c, kGroupNormalize, a, nullptr, n, out, nullptr);
}
int bn_g1_eq_many(bn_ctx* c, const bn_g1* a, const bn_g1* b, size_t n, uint8_t* eq) {
    return group_host<bn_g1>(c, kGroupEq, a, b, n, nullptr, eq);
}
int bn_g2_add_many(bn_ctx* c, const bn_g2* a, const bn_g2* b, size_t n, bn_g2* out) {
    return group_host(c, kGroupAdd, a, b, n, out, nullptr);
}
int bn_g2_sub_many(bn_ctx* c, const bn_g2* a, const bn_g2* b, size_t n, bn_g2* out) {
    return group_host(c, kGroupSub, a, b, n, out, nullptr);
}
int bn_g2_neg_many(bn_ctx* c, const bn_g2* a, size_t n, bn_g2* out) {
    return group_host<bn_g2>(c, kGroupNeg, a, nullptr, n, out, nullptr);
}
int bn_g2_normalize_many(bn_ctx* c, const bn_g2* a, size_t n, bn_g2* out) {
    return group_host<bn_g2>(c, kGroupNormalize, a, nullptr, n, out, nullptr);
}
int bn_g2_eq_many(bn_ctx* c, const bn_g2* a, const bn_g2* b, size_t n, uint8_t* eq) {
    return group_host<bn_g2>(c, kGroupEq, a, b, n, nullptr, eq);
}
int bn_g1_add_many_dev(bn_ctx* c, const bn_g1* d_a, const bn_g1* d_b, size_t n, bn_g1* d_out, void* stream) {
    return group_dev(c, kGroupAdd, d_a, d_b, n, d_out, nullptr, stream);
}
int bn_g1_sub_many_dev(bn_ctx* c, const bn_g1* d_a, const bn_g1* d_b, size_t n, bn_g1* d_out, void* stream) {
    return group_dev(c, kGroupSub, d_a, d_b, n, d_out, nullptr, stream);
}
int bn_g1_neg_many_dev(bn_ctx* c, const bn_g1* d_a, size_t n, bn_g1* d_out, void* stream) {
    return group_dev<bn_g1>(c, kGroupNeg, d_a, nullptr, n, d_out, nullptr, stream);
}
int bn_g1_normalize_many_dev(bn_ctx* c, const bn_g1* d_a, size_t n, bn_g1* d_out, void* stream) {
    return group_dev<bn_g1>(c, kGroupNormalize, d_a, nullptr, n, d_out, nullptr, stream);
}
int bn_g1_eq_many_dev(bn_ctx* c, const bn_g1* d_a, const bn_g1* d_b, size_t n, uint8_t* d_eq, void* stream) {
    return group_dev<bn_g1>(c, kGroupEq, d_a, d_b, n, nullptr, d_eq, stream);
}
int bn_g2_add_many_dev(bn_ctx* c, const bn_g2* d_a, const bn_g2* d_b, size_t n, bn_g2* d_out, void* stream) {
    return group_dev(c, kGroupAdd, d_a, d_b, n, d_out, nullptr, stream);
}
int bn_g2_sub_many_dev(bn_ctx* c, const bn_g2* d_a, const bn_g2* d_b, size_t n, bn_g2* d_out, void* stream) {
    return group_dev(c, kGroupSub, d_a, d_b, n, d_out, nullptr, stream);
}
int bn_g2_neg_many_dev(bn_ctx* c, const bn_g2* d_a, size_t n, bn_g2* d_out, void* stream) {
    return group_dev<bn_g2>(c, kGroupNeg, d_a, nullptr, n, d_out, nullptr, stream);
}
int bn_g2_normalize_many_dev(bn_ctx* c, const bn_g2* d_a, size_t n, bn_g2* d_out, void* stream) {
    return group_dev<bn_g2>(c, kGroupNormalize, d_a, nullptr, n, d_out, nullptr, stream);
}
int bn_g2_eq_many_dev(bn_ctx* c, const bn_g2* d_a, const bn_g2* d_b, size_t n, uint8_t* d_eq, void* stream) {
    return group_dev<bn_g2>(c, kGroupEq, d_a, d_b, n, nullptr, d_eq, stream);
}

}  // extern "C"
