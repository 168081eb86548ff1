// ds_check.hip -- GPU check and latency probe of the digit-sliced Fq12
// (csrc/fq12_ds.h) against the 16-lane functions of csrc/fq12_wide.h, one element
// per 384-thread block.  Not part of the product library; the product path is
// checked end to end by the pairing_batch parity tests.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I paritytech-bn_amd/csrc -o tools/ds_check tools/ds_check.hip
//   tools/ds_check [elements]
#define BN_FOLD_LDS 1
#define BN_WIDE_ARRS 5
#define BN_WIDE_THREADS 256
#include "fq.h"
#define BN_SPLIT 1
#include "fq12_ds.h"

#include <cstdio>
#include <cstdlib>
#include <vector>

using namespace bn;

enum { DSOP_CYC, DSOP_MUL, DSOP_MULC, DSOP_FROB1, DSOP_FROB2, DSOP_FROB3, DSOP_CONJ, DSOP_EXP, DSOP_FELAST, DSOP_COUNT };
static const char* kName[] = {"cyc", "mul", "mul_conj", "frob1", "frob2", "frob3", "conj", "exp_by_neg_z", "fe_last"};

__global__ void __launch_bounds__(kDsThreads) k_ds_check(const uint32_t* __restrict__ in, int op,
                                                         uint32_t* __restrict__ out, unsigned long long* cyc) {
    fold_table_init();
    ds_init();
    const int t = (int)threadIdx.x;
    const int l = t < 12 ? t : 10 + (t & 1);  // lanes 12..15 mirror e = 5
    Fq<2> a = widen<2>(fq_zero()), b = a;
    const uint32_t* e = in + (size_t)blockIdx.x * 2 * 12 * 9;
    if (t < 16) {
#pragma unroll
        for (int i = 0; i < 9; ++i) {
            a.v[i] = e[l * 9 + i];
            b.v[i] = e[(12 + l) * 9 + i];
        }
    }
    Fq<2> ref = a;
    if (t < 16) {
        switch (op) {
            case DSOP_CYC: ref = w12_cyc(a); break;
            case DSOP_MUL: ref = w12_mul(a, b); break;
            case DSOP_MULC: ref = w12_mul(a, w12_conj(b)); break;
            case DSOP_FROB1: ref = w12_frob<1>(a); break;
            case DSOP_FROB2: ref = w12_frob<2>(a); break;
            case DSOP_FROB3: ref = w12_frob<3>(a); break;
            case DSOP_CONJ: ref = w12_conj(a); break;
            case DSOP_EXP: ref = w12_exp_by_neg_z(a); break;
            default: ref = w12_fe_last(a); break;
        }
    }
    __syncthreads();
    const uint32_t da = ds_from_w12(a);
    const uint32_t db = ds_from_w12(b);
    __syncthreads();
    const unsigned long long t0 = clock64();
    uint32_t r;
    switch (op) {
        case DSOP_CYC: r = ds_cyc(da); break;
        case DSOP_MUL: r = ds_mul(da, db, false); break;
        case DSOP_MULC: r = ds_mul(da, db, true); break;
        case DSOP_FROB1: r = ds_frob<1>(da); break;
        case DSOP_FROB2: r = ds_frob<2>(da); break;
        case DSOP_FROB3: r = ds_frob<3>(da); break;
        case DSOP_CONJ: r = ds_conj(da); break;
        case DSOP_EXP: r = ds_exp_by_neg_z(da); break;
        default: r = ds_fe_last(da); break;
    }
    __syncthreads();
    const unsigned long long t1 = clock64();
    const Fq<2> got = ds_to_w12(r);
    if (t < 12) {
        const Fq<1> cr = fq_canonical(ref), cg = fq_canonical(got);
        uint32_t* o = out + ((size_t)blockIdx.x * 12 + t) * 18;
#pragma unroll
        for (int i = 0; i < 9; ++i) {
            o[i] = cr.v[i];
            o[9 + i] = cg.v[i];
        }
    }
    if (t == 0) cyc[blockIdx.x] = t1 - t0;
}

// latency probe: `iters` dependent DS squarings vs w12_cyc on group 0
__global__ void __launch_bounds__(kDsThreads) k_ds_time(const uint32_t* __restrict__ in, int iters, int which,
                                                        uint32_t* __restrict__ sink, unsigned long long* cyc) {
    fold_table_init();
    ds_init();
    const int t = (int)threadIdx.x;
    const int l = t < 12 ? t : 10 + (t & 1);
    Fq<2> a = widen<2>(fq_zero());
    if (t < 16)
        for (int i = 0; i < 9; ++i) a.v[i] = in[l * 9 + i];
    uint32_t da = ds_from_w12(a);
#if defined(BN_DS_STAMPS) && BN_DS_STAMPS
    if (threadIdx.x < 8) g_ds_stamp[threadIdx.x] = 0;
#endif
    __syncthreads();
    const unsigned long long t0 = clock64();
    if (which == 0) {
        for (int i = 0; i < iters; ++i) da = ds_cyc(da);
    } else if (which == 1) {
        for (int i = 0; i < iters; ++i) da = ds_mul(da, da, false);
    } else if (t < 16) {
        for (int i = 0; i < iters; ++i) a = which == 2 ? w12_cyc(a) : w12_mul(a, a);
    }
    __syncthreads();
    const unsigned long long t1 = clock64();
    sink[t] = da + a.v[0];
    if (t == 0) *cyc = t1 - t0;
#if defined(BN_DS_STAMPS) && BN_DS_STAMPS
    if (which == 0 && t < 8) cyc[1 + t] = g_ds_stamp[t];
#endif
}

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(2);                                                                 \
        }                                                                            \
    } while (0)

int main(int argc, char** argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 64;
    srand(12345);
    std::vector<uint32_t> h((size_t)n * 2 * 12 * 9);
    for (size_t i = 0; i < h.size(); i += 9) {
        for (int d = 0; d < 8; ++d) h[i + d] = (uint32_t)(((unsigned)rand() << 15) ^ (unsigned)rand()) & 0x1fffffffu;
        h[i + 8] = (uint32_t)rand() % 0x30644eu;  // below p's top digit: value < p
        if ((i / 9) % 7 == 3) {  // some maximal digits
            for (int d = 0; d < 8; ++d) h[i + d] = 0x1fffffffu;
            h[i + 8] = 0x30644du;
        }
    }
    uint32_t *d_in, *d_out, *d_sink;
    unsigned long long* d_cyc;
    CK(hipMalloc(&d_in, h.size() * 4));
    CK(hipMalloc(&d_out, (size_t)n * 12 * 18 * 4));
    CK(hipMalloc(&d_cyc, (size_t)(n < 16 ? 16 : n) * 8));
    CK(hipMalloc(&d_sink, kDsThreads * 4));
    CK(hipMemcpy(d_in, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    std::vector<uint32_t> o((size_t)n * 12 * 18);
    std::vector<unsigned long long> cy(n);
    int bad_total = 0;
    for (int op = 0; op < DSOP_COUNT; ++op) {
        const int nn = op >= DSOP_EXP ? (n < 8 ? n : 8) : n;
        hipLaunchKernelGGL(k_ds_check, dim3(nn), dim3(kDsThreads), 0, 0, d_in, op, d_out, d_cyc);
        CK(hipGetLastError());
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(o.data(), d_out, (size_t)nn * 12 * 18 * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(cy.data(), d_cyc, (size_t)nn * 8, hipMemcpyDeviceToHost));
        int bad = 0;
        for (int el = 0; el < nn; ++el)
            for (int c = 0; c < 12; ++c) {
                const uint32_t* p = &o[((size_t)el * 12 + c) * 18];
                for (int i = 0; i < 9; ++i)
                    if (p[i] != p[9 + i]) {
                        if (bad < 3)
                            printf("  %s el %d coord %d digit %d: ref %08x ds %08x\n", kName[op], el, c, i, p[i], p[9 + i]);
                        ++bad;
                        break;
                    }
            }
        printf("%-14s %s (%d elements, %d coordinate mismatches), %llu clocks\n", kName[op], bad ? "MISMATCH" : "ok", nn,
               bad, cy[0]);
        bad_total += bad;
    }
    const int iters = 200;
    const char* tn[] = {"ds_cyc", "ds_mul", "w12_cyc", "w12_mul"};
    for (int w = 0; w < 4; ++w) {
        unsigned long long c = 0;
        hipLaunchKernelGGL(k_ds_time, dim3(1), dim3(kDsThreads), 0, 0, d_in, iters, w, d_sink, d_cyc);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(&c, d_cyc, 8, hipMemcpyDeviceToHost));
        printf("latency %-8s %.0f clocks per op (%d dependent ops)\n", tn[w], (double)c / iters, iters);
#if defined(BN_DS_STAMPS) && BN_DS_STAMPS
        if (w == 0) {
            unsigned long long st[8];
            CK(hipMemcpy(st, d_cyc + 1, 64, hipMemcpyDeviceToHost));
            const char* ph[] = {"E write + barrier", "operand build", "product MADs", "REDC", "barrier 2", "combination", "fold"};
            for (int i = 0; i < 7; ++i) printf("  ds_cyc phase %-18s %6.0f clocks\n", ph[i], (double)st[i] / iters);
        }
#endif
    }
    printf(bad_total ? "DS CHECK FAILED\n" : "DS CHECK OK\n");
    return bad_total ? 1 : 0;
}
