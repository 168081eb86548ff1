#!/bin/bash
# round 5 session s: G2 * Fr with two chains per lane pair (k_g2_mul2_split / _w):
# parity on the variant build, then interleaved A/B against the one-chain kernel
set -e
OUT=gpurun_out/r5s
mkdir -p $OUT
export TMPDIR=/tmp
BN254MI_LIB=ab/lib_g2m2.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "g2_mul" --timeout 200 --timeout-method thread > $OUT/g2m2_tests.log 2>&1 || { tail -30 $OUT/g2m2_tests.log; exit 1; }
grep -E "PASS|FAIL" $OUT/g2m2_tests.log | tail -8
timeout -k 10 600 bash tools/gpu_ab.sh r5s_ab paritytech-bn_amd/libbn254mi.so ab/lib_g2m2.so "g2mul"
