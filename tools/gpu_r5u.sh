#!/bin/bash
# round 5 session u: Granger-Scott square with t0/t2/t4/xi*t5 carried normalized instead of folded
# (tower.h BN_CYC_LAZY=1): parity subset on the variant build, then interleaved A/B
set -e
OUT=gpurun_out/r5u
mkdir -p $OUT
export TMPDIR=/tmp
BN254MI_LIB=ab/lib_cyclazy.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_codec.py tests/test_gpu_wide.py -m gpu -x -v --timeout 200 --timeout-method thread -k "fq12_ops or cyclotomic or reference_kats or throughput_path or large_batch or gt_pow or config5 or pairing_many" > $OUT/lazy_tests.log 2>&1 || { tail -30 $OUT/lazy_tests.log; exit 1; }
grep -cE "PASSED" $OUT/lazy_tests.log; tail -1 $OUT/lazy_tests.log
timeout -k 10 900 bash tools/gpu_ab.sh r5u_ab paritytech-bn_amd/libbn254mi.so ab/lib_cyclazy.so "pairing product gtpow"
