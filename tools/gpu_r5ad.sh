#!/bin/bash
# round 5 session ad: jac_double with d carried normalized instead of folded (curve.h; ab/lib_dnorm.so = B)
# vs the r5ab build (A): G2 * Fr and config 3 parity + interleaved A/B
set -e
OUT=gpurun_out/r5ad
mkdir -p $OUT
export TMPDIR=/tmp
BN254MI_LIB=ab/lib_dnorm.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_group.py -m gpu -x -q --timeout 250 --timeout-method thread -k "g1_mul or g2_mul or config3 or group or kats" > $OUT/dnorm_tests.log 2>&1 || { tail -30 $OUT/dnorm_tests.log; exit 1; }
tail -1 $OUT/dnorm_tests.log
timeout -k 10 900 bash tools/gpu_ab.sh r5ad_ab paritytech-bn_amd/libbn254mi.so ab/lib_dnorm.so "g2mul g1mul"
