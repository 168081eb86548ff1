#!/bin/bash
# round 5 session g: P/Q of the fused Miller loop in LDS (BN_MILLER_LDS) A/B on config 2
set -e
OUT=gpurun_out/r5g
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "throughput or kat or config2 or full" > $OUT/tp_tests.log 2>&1 || { tail -30 $OUT/tp_tests.log; exit 1; }
tail -1 $OUT/tp_tests.log
timeout -k 10 600 bash tools/gpu_ab.sh r5g_ab paritytech-bn_amd/libbn254mi.so ab/lib_ml0.so "pairing"
timeout -k 10 600 bash tools/gpu_ab.sh r5g_ab2 paritytech-bn_amd/libbn254mi.so ab/lib_ml0.so "pairing"
