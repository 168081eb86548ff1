// kernels_latency_w2.hip -- k_pairing_latency_w2: the one-launch latency kernel
// (latency_kernel.h) built for TWO waves per SIMD, so that two
// blocks share a CU and 2,049-4,096 pairs run in one round of blocks instead of
// two.  Every kernel of this unit carries amdgpu_waves_per_eu(2, 2), so the
// wide-layout device functions it calls are compiled to the same 256-register
// budget (the one-wave build keeps its own copies in kernels_wide.hip), and the
// LDS shrinks to 77.8 KB per block: four operand arrays per group (squarings by
// w12_mul), a six-line ring per pair and a one-item channel in the two-group
// final exponentiation.  Values are the same residues as k_pairing_latency's.
#define BN_FOLD_LDS 1
#define BN_WIDE_ARRS 4
#define BN_LAT_RING 6
#define BN_DUO_RING 1
#define BN_LAT_KERNEL_NAME k_pairing_latency_w2
#define BN_LAT_KERNEL_ATTR __attribute__((amdgpu_waves_per_eu(2, 2)))
#include "fq.h"
#define BN_SPLIT 1
#include "fq12_wide.h"
#include "lines_wide.h"
#include "latency_kernel.h"

BN_EXPORT_FOLD_CHECK(latency_w2)
