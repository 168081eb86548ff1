#!/bin/bash
# round 5 session e: segment-plan cost weights A/B on config 5 (+ product parity tests)
set -e
OUT=gpurun_out/r5e
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "product or batch or config5 or segmented" > $OUT/prod_tests.log 2>&1 || { tail -30 $OUT/prod_tests.log; exit 1; }
tail -1 $OUT/prod_tests.log
for r in 1 2; do
  for v in uniform 36,39 5338,4730 5338,5730 5338,6730 5338,8000; do
    if [ $v = uniform ]; then E="BN254MI_SEG_UNIFORM=1"; else E="BN254MI_SEG_W=$v"; fi
    env $E timeout -k 10 120 python -u bench.py --workload product --steps 15 --warmup 3 --no-cpu-baseline > $OUT/p_${v}_$r.json 2> $OUT/p_${v}_$r.err
    python3 -c "import json; d=json.load(open('$OUT/p_${v}_$r.json')); print('$v r$r', round(d['ms_per_step'],4))"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_product -o run -- python3 bench.py --workload product --steps 10 --no-cpu-baseline > /dev/null 2> $OUT/prof_product.err
