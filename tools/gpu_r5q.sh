#!/bin/bash
# round 5 session q: the two-lane products' register fences (fq2_split.h BN_FQ2_FENCE): 3 (inputs and
# results, the round-4 form) vs 1 (results) vs 0 (none); config 2, config 5, G2 * Fr, config 3
set -e
OUT=gpurun_out/r5q
mkdir -p $OUT
export TMPDIR=/tmp
for r in 1 2; do
  for v in 3 1 0; do
    case $v in 3) L=;; 1) L=ab/lib_fence1.so;; 0) L=ab/lib_fence0.so;; esac
    BN254MI_LIB=$L timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-config4-ref > $OUT/b_${v}_$r.json 2> $OUT/b_${v}_$r.err
    python3 -c "import json; d=json.load(open('$OUT/b_${v}_$r.json')); print('pairing fence=$v r$r', round(d['ms_per_step'],4), round(d['value']), round(d['roofline']['frac'],4))"
  done
done
for w in product g2mul g1mul; do
  for v in 3 0; do
    case $v in 3) L=;; 0) L=ab/lib_fence0.so;; esac
    BN254MI_LIB=$L timeout -k 10 200 python -u bench.py --workload $w --steps 10 --warmup 2 --no-cpu-baseline > $OUT/w_${w}_$v.json 2> $OUT/w_${w}_$v.err
    python3 -c "import json; d=json.load(open('$OUT/w_${w}_$v.json')); print('$w fence=$v', round(d['ms_per_step'],4), round(d['roofline']['frac'],4))"
  done
done
echo "== done"
