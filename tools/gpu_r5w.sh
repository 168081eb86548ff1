#!/bin/bash
# round 5 session w: the sparse line product's six-product column sum as one asm chain
# (pairing.h BN_DOT6_ASM=1, ab/lib_dot6.so): parity on the variant, interleaved A/B, product PMC traffic
set -e
OUT=gpurun_out/r5w
mkdir -p $OUT
export TMPDIR=/tmp
BN254MI_LIB=ab/lib_dot6.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/dot6_tests.log 2>&1 || { tail -30 $OUT/dot6_tests.log; exit 1; }
tail -1 $OUT/dot6_tests.log
timeout -k 10 900 bash tools/gpu_ab.sh r5w_ab paritytech-bn_amd/libbn254mi.so ab/lib_dot6.so "pairing product"
for L in base dot6; do
  lib=paritytech-bn_amd/libbn254mi.so; [ $L = dot6 ] && lib=ab/lib_dot6.so
  BN254MI_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_prod_fetch_$L -o p -- python3 bench.py --workload product --steps 2 --warmup 1 --no-cpu-baseline > /dev/null 2> $OUT/pmc_prod_fetch_$L.err
  BN254MI_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_prod_write_$L -o p -- python3 bench.py --workload product --steps 2 --warmup 1 --no-cpu-baseline > /dev/null 2> $OUT/pmc_prod_write_$L.err
done
echo done
