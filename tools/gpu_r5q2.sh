#!/bin/bash
# round 5 session q (part 2): BN_FQ2_FENCE 3 vs 0 on config 5, G2 * Fr, config 3
set -e
OUT=gpurun_out/r5q
mkdir -p $OUT
export TMPDIR=/tmp
for r in 1 2; do
for w in product g2mul g1mul; do
  for v in 3 0; do
    case $v in 3) L=;; 0) L=ab/lib_fence0.so;; esac
    BN254MI_LIB=$L timeout -k 10 200 python -u bench.py --workload $w --steps 10 --warmup 2 --no-cpu-baseline > $OUT/w_${w}_${v}_$r.json 2> $OUT/w_${w}_${v}_$r.err
    python3 -c "import json; d=json.load(open('$OUT/w_${w}_${v}_$r.json')); print('$w fence=$v r$r', round(d['ms_per_step'],4), round(d.get('roofline',{}).get('frac',0),4))"
  done
done
done
echo "== done"
