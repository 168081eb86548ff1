// ubench2.hip -- per-instruction VALU cost on gfx950 + a prototype of the
// 9 x 29-bit-digit Montgomery multiplication (no per-product carry handling).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x)                                                                                      \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
            exit(1);                                                                               \
        }                                                                                          \
    } while (0)

// 8 independent 32-bit chains of one instruction form
#define BODY32(INSTR)                                                                                     \
    asm volatile(INSTR(0) INSTR(1) INSTR(2) INSTR(3) INSTR(4) INSTR(5) INSTR(6) INSTR(7)                  \
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)         \
                 : "v"(x), "v"(y))
#define K32(NAME, INSTR)                                                                                  \
    __global__ void NAME(uint32_t* out, uint32_t x, uint32_t y, int iters) {                              \
        uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,       \
                 a6 = a0 + 6, a7 = a0 + 7;                                                                \
        for (int i = 0; i < iters; ++i) BODY32(INSTR);                                                    \
        out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;               \
    }
#define I_ADD(n) "v_add_u32 %" #n ", %" #n ", %8\n\t"
#define I_AND(n) "v_and_b32 %" #n ", %" #n ", %8\n\t"
#define I_ALIGNBIT(n) "v_alignbit_b32 %" #n ", %" #n ", %8, 29\n\t"
#define I_BFE(n) "v_bfe_u32 %" #n ", %" #n ", 3, 29\n\t"
#define I_ADD3(n) "v_add3_u32 %" #n ", %" #n ", %8, %9\n\t"
#define I_MAD24(n) "v_mad_u32_u24 %" #n ", %" #n ", %8, %9\n\t"
#define I_MULHI24(n) "v_mul_hi_u32_u24 %" #n ", %" #n ", %8\n\t"
#define I_MULHI(n) "v_mul_hi_u32 %" #n ", %" #n ", %8\n\t"
#define I_MULLO(n) "v_mul_lo_u32 %" #n ", %" #n ", %8\n\t"
#define I_LSHR(n) "v_lshrrev_b32 %" #n ", 29, %" #n "\n\t"
#define I_CNDMASK(n) "v_cndmask_b32 %" #n ", %" #n ", %8, vcc\n\t"
#define I_XAD(n) "v_xad_u32 %" #n ", %" #n ", %8, %9\n\t"
#define I_LSHLADD(n) "v_lshl_add_u32 %" #n ", %" #n ", 3, %8\n\t"
K32(k_add, I_ADD)
K32(k_and, I_AND)
K32(k_alignbit, I_ALIGNBIT)
K32(k_bfe, I_BFE)
K32(k_add3, I_ADD3)
K32(k_mad24, I_MAD24)
K32(k_mulhi24, I_MULHI24)
K32(k_mulhi, I_MULHI)
K32(k_mullo, I_MULLO)
K32(k_lshr, I_LSHR)
K32(k_cndmask, I_CNDMASK)
K32(k_xad, I_XAD)
K32(k_lshladd, I_LSHLADD)

// 8 independent 64-bit chains
#define BODY64(INSTR)                                                                                     \
    asm volatile(INSTR(0) INSTR(1) INSTR(2) INSTR(3) INSTR(4) INSTR(5) INSTR(6) INSTR(7)                  \
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)         \
                 : "v"(x), "v"(y), "v"(z))
#define K64(NAME, INSTR)                                                                                  \
    __global__ void NAME(uint64_t* out, uint32_t x, uint32_t y, int iters) {                              \
        uint64_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,       \
                 a6 = a0 + 6, a7 = a0 + 7;                                                                \
        uint64_t z = ((uint64_t)y << 32) | x;                                                             \
        for (int i = 0; i < iters; ++i) BODY64(INSTR);                                                    \
        out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;               \
    }
#define I_MAD64(n) "v_mad_u64_u32 %" #n ", vcc, %8, %9, %" #n "\n\t"
#define I_MAD64_0(n) "v_mad_u64_u32 %" #n ", vcc, %8, %9, 0\n\t"
#define I_LSHR64(n) "v_lshrrev_b64 %" #n ", 29, %" #n "\n\t"
#define I_LSHLADD64(n) "v_lshl_add_u64 %" #n ", %" #n ", 0, %10\n\t"
#define I_MOV64(n) "v_mov_b64 %" #n ", %10\n\t"
K64(k_mad64, I_MAD64)
K64(k_mad64_0, I_MAD64_0)
K64(k_lshr64, I_LSHR64)
K64(k_lshladd64, I_LSHLADD64)
K64(k_mov64, I_MOV64)

// add with carry-out into independent SGPR pairs (4 chains: add_co then addc)
__global__ void k_addco(uint32_t* out, uint32_t x, uint32_t y, int iters) {
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, b0 = 1, b1 = 2, b2 = 3, b3 = 4;
    uint64_t c0, c1, c2, c3;
    for (int i = 0; i < iters; ++i)
        asm volatile(
            "v_add_co_u32_e64 %0, %8, %0, %12\n\t"
            "v_add_co_u32_e64 %1, %9, %1, %12\n\t"
            "v_add_co_u32_e64 %2, %10, %2, %12\n\t"
            "v_add_co_u32_e64 %3, %11, %3, %12\n\t"
            "v_addc_co_u32_e64 %4, %8, %4, %13, %8\n\t"
            "v_addc_co_u32_e64 %5, %9, %5, %13, %9\n\t"
            "v_addc_co_u32_e64 %6, %10, %6, %13, %10\n\t"
            "v_addc_co_u32_e64 %7, %11, %7, %13, %11\n\t"
            : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(b0), "+v"(b1), "+v"(b2), "+v"(b3), "=&s"(c0), "=&s"(c1),
              "=&s"(c2), "=&s"(c3)
            : "v"(x), "v"(y));
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ b0 ^ b1 ^ b2 ^ b3;
}

// ---------------------------------------------------------------- 29-bit-digit Montgomery
// p in 9 x 29-bit digits, R = 2^261, inv = -p^-1 mod 2^29
struct F9 {
    uint32_t v[9];
};
#define M29 0x1fffffffu
__device__ constexpr uint32_t kP29[9] = {0x187cfd47u, 0x010460b6u, 0x1c72a34fu, 0x02d522d0u, 0x1585d978u,
                                        0x02db40c0u, 0x00a6e141u, 0x0e5c2634u, 0x0030644eu};
#define INV29 0x04866389u
__device__ __forceinline__ F9 mul29(const F9& a, const F9& b) {
    uint32_t m[9];
    F9 r;
    uint64_t acc = 0;
#pragma unroll
    for (int k = 0; k < 17; ++k) {
        const int lo = k < 9 ? 0 : k - 8;
        const int hi = k < 9 ? k : 8;
#pragma unroll
        for (int i = lo; i <= hi; ++i) {
            acc += (uint64_t)a.v[i] * b.v[k - i];
            if (i < k) acc += (uint64_t)m[i] * kP29[k - i];
        }
        if (k < 9) {
            m[k] = ((uint32_t)acc * INV29) & M29;
            acc += (uint64_t)m[k] * kP29[0];
        } else {
            r.v[k - 9] = (uint32_t)acc & M29;
        }
        acc >>= 29;
    }
    r.v[8] = (uint32_t)acc;
    return r;
}
template <int CHAINS>
__global__ void k_mul29(F9* io, int iters) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    F9 y = io[i];
    F9 x[CHAINS];
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) {
        x[c] = y;
        x[c].v[0] ^= c;
    }
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int c = 0; c < CHAINS; ++c) x[c] = mul29(x[c], y);
    }
    F9 r = x[0];
#pragma unroll
    for (int c = 1; c < CHAINS; ++c)
#pragma unroll
        for (int j = 0; j < 9; ++j) r.v[j] += x[c].v[j];
    io[i] = r;
}
__global__ void k_mul29_check(const F9* a, const F9* b, F9* o, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) o[i] = mul29(a[i], b[i]);
}

template <typename F>
static float time_ms(F launch, int reps) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    launch();
    CK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < reps; ++r) {
        CK(hipEventRecord(e0));
        launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (ms < best) best = ms;
    }
    return best;
}

int main(int argc, char** argv) {
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    int cus = prop.multiProcessorCount;
    void* buf;
    CK(hipMalloc(&buf, (size_t)cus * 8 * 256 * 64));
    const int iters = 4096;
    struct {
        const char* name;
        void (*k32)(uint32_t*, uint32_t, uint32_t, int);
        void (*k64)(uint64_t*, uint32_t, uint32_t, int);
    } tab[] = {{"v_add_u32", k_add, 0},         {"v_and_b32", k_and, 0},         {"v_alignbit_b32", k_alignbit, 0},
               {"v_bfe_u32", k_bfe, 0},         {"v_add3_u32", k_add3, 0},       {"v_mad_u32_u24", k_mad24, 0},
               {"v_mul_hi_u32_u24", k_mulhi24, 0}, {"v_mul_hi_u32", k_mulhi, 0}, {"v_mul_lo_u32", k_mullo, 0},
               {"v_lshrrev_b32", k_lshr, 0},    {"v_cndmask_b32", k_cndmask, 0}, {"v_xad_u32", k_xad, 0},
               {"v_lshl_add_u32", k_lshladd, 0}, {"v_add_co+addc_e64(sgpr)", k_addco, 0},
               {"v_mad_u64_u32", 0, k_mad64},   {"v_mad_u64_u32(addend0)", 0, k_mad64_0},
               {"v_lshrrev_b64", 0, k_lshr64},  {"v_lshl_add_u64", 0, k_lshladd64}, {"v_mov_b64", 0, k_mov64}};
    for (int wps : {1, 2, 8}) {
        int blocks = cus * wps;
        double waves_per_simd_instr = (double)iters * 8;  // instructions per wave
        for (auto& t : tab) {
            float ms = time_ms(
                [&] {
                    if (t.k32)
                        t.k32<<<blocks, 256>>>((uint32_t*)buf, 3, 5, iters);
                    else
                        t.k64<<<blocks, 256>>>((uint64_t*)buf, 3, 5, iters);
                },
                3);
            // cycles per wave-instruction per SIMD at 2.4 GHz
            double cyc = ms * 1e-3 * 2.4e9 / (waves_per_simd_instr * wps);
            printf("{\"bench\": \"instr\", \"instr\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.4f, \"cycles_per_wave_instr\": %.2f}\n",
                   t.name, wps, ms, cyc);
        }
    }
    const int fiters = 256;
    for (int wps : {1, 2, 4}) {
        int blocks = cus * wps;
        double lanes = (double)blocks * 256;
        float ms = time_ms([&] { k_mul29<1><<<blocks, 256>>>((F9*)buf, fiters); }, 3);
        printf("{\"bench\": \"mul29\", \"chains\": 1, \"waves_per_simd\": %d, \"ms\": %.4f, \"Gmul_per_s\": %.2f}\n", wps, ms,
               lanes * fiters / (ms * 1e-3) / 1e9);
        ms = time_ms([&] { k_mul29<2><<<blocks, 256>>>((F9*)buf, fiters); }, 3);
        printf("{\"bench\": \"mul29\", \"chains\": 2, \"waves_per_simd\": %d, \"ms\": %.4f, \"Gmul_per_s\": %.2f}\n", wps, ms,
               lanes * fiters * 2 / (ms * 1e-3) / 1e9);
    }
    // correctness dump: a, b read from argv[1] (n x 9 u32 each), results to argv[2]
    if (argc > 2) {
        FILE* f = fopen(argv[1], "rb");
        int n;
        fread(&n, 4, 1, f);
        F9* h = (F9*)malloc(sizeof(F9) * n * 3);
        fread(h, sizeof(F9), 2 * n, f);
        fclose(f);
        F9* d;
        CK(hipMalloc(&d, sizeof(F9) * n * 3));
        CK(hipMemcpy(d, h, sizeof(F9) * 2 * n, hipMemcpyHostToDevice));
        k_mul29_check<<<(n + 255) / 256, 256>>>(d, d + n, d + 2 * n, n);
        CK(hipMemcpy(h + 2 * n, d + 2 * n, sizeof(F9) * n, hipMemcpyDeviceToHost));
        f = fopen(argv[2], "wb");
        fwrite(h + 2 * n, sizeof(F9), n, f);
        fclose(f);
        printf("{\"bench\": \"mul29_dump\", \"n\": %d}\n", n);
    }
    return 0;
}
