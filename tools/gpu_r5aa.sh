#!/bin/bash
# round 5 session aa: the latency kernel's line product w12_mul_line as one asm chain
# (fq12_wide.h BN_W12_LINE_DOT6=1, ab/lib_wl6.so) vs the 17-column accumulator; parity, latency A/B
set -e
OUT=gpurun_out/r5aa
mkdir -p $OUT
export TMPDIR=/tmp
BN254MI_LIB=ab/lib_wl6.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_wide.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/wl6_tests.log 2>&1 || { tail -30 $OUT/wl6_tests.log; exit 1; }
tail -1 $OUT/wl6_tests.log
for r in 1 2; do
  for L in A B; do
    lib=paritytech-bn_amd/libbn254mi.so; [ $L = B ] && lib=ab/lib_wl6.so
    BN254MI_LIB=$lib timeout -k 10 200 python -u tools/latency.py --calls pairing_many_dev,pairing_batch --sizes 1,64,1024,2048,4096 --reps 7 > $OUT/lat_${L}_$r.jsonl 2> $OUT/lat_${L}_$r.err
    python3 -c "
import json
for l in open('$OUT/lat_${L}_$r.jsonl'):
    d=json.loads(l)
    if 'call' in d: print('$L r$r', d['call'], d['n'], round(d['ms'],4))
"
  done
done
