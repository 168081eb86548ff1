#!/bin/bash
# Build an A/B variant of libbn254mi.so with extra compile flags into
# ab/lib_NAME.so (bench.py / tests load it with BN254MI_LIB=ab/lib_NAME.so).
# Usage: tools/build_variant.sh NAME "-DFLAG=1 ..."
set -e
NAME=$1; FLAGS=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
B=$ROOT/ab/build_$NAME
mkdir -p $B
SRCS="kernels_pairing kernels_fe kernels_group kernels_util kernels_codec kernels_gtpow kernels_wide kernels_latency_w2 kernels_reduce kernels_tail capi capi_multi"
for s in $SRCS; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function $FLAGS \
    -c -o $B/$s.o $ROOT/paritytech-bn_amd/csrc/$s.hip &
done
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $ROOT/ab/lib_$NAME.so $(for s in $SRCS; do echo $B/$s.o; done) -ldl
echo "built ab/lib_$NAME.so"
