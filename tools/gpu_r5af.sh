#!/bin/bash
# round 5 session af: the product reduction's finishing level takes longer chains instead of one more
# launch (capi.hip BN_REDUCE_LAST=1, ab/lib_rlast.so = B) vs the r5ae build (A): parity + A/B + kernel trace
set -e
OUT=gpurun_out/r5af
mkdir -p $OUT
export TMPDIR=/tmp
BN254MI_LIB=ab/lib_rlast.so timeout -k 10 600 python -u -m pytest tests/test_gpu_wide.py tests/test_gpu_parity.py -m gpu -x -q --timeout 250 --timeout-method thread -k "product or batch or recombination or reduction or config5" > $OUT/rlast_tests.log 2>&1 || { tail -30 $OUT/rlast_tests.log; exit 1; }
tail -1 $OUT/rlast_tests.log
for r in 1 2 3; do
  for L in A B; do
    lib=paritytech-bn_amd/libbn254mi.so; [ $L = B ] && lib=ab/lib_rlast.so
    BN254MI_LIB=$lib timeout -k 10 120 python -u bench.py --workload product --steps 20 --warmup 3 --no-cpu-baseline > $OUT/p_${L}_$r.json 2> $OUT/p_${L}_$r.err
    python3 -c "import json; d=json.load(open('$OUT/p_${L}_$r.json')); print('product $L r$r', round(d['ms_per_step'],4))"
  done
done
BN254MI_LIB=ab/lib_rlast.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 bench.py --workload product --steps 5 --no-cpu-baseline > /dev/null 2> $OUT/prof.err
