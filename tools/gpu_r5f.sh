#!/bin/bash
# round-5 session f (plan + reduce + asm + w12_cyc): GPU tests (with the failure-path test), the device
# fold-bound check over every unit, the bench line, the Fq2-product microbenchmark
set -e
OUT=gpurun_out/r5f
mkdir -p $OUT
export TMPDIR=/tmp
echo "== tests"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
echo "== fold check"
BN254MI_LIB=paritytech-bn_amd/libbn254mi_dbg.so timeout -k 10 300 python -u tools/fold_check.py 4096 > $OUT/fold_check.json 2> $OUT/fold_check.err || { tail -20 $OUT/fold_check.err; exit 1; }
cat $OUT/fold_check.json
echo "== bench"
timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
cut -c1-600 $OUT/bench.json

for w in product g1mul g2mul gtpow; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 10 --warmup 2 > $OUT/bench_$w.json 2> $OUT/bench_$w.err
  python3 -c "import json; d=json.load(open('$OUT/bench_$w.json')); print('$w', d['ms_per_step'], d['value'], d.get('roofline',{}).get('frac'))"
done
timeout -k 10 300 python -u tools/latency.py --calls pairing_many_dev,pairing_batch --sizes 1,64,2048,4096 > $OUT/latency.jsonl 2> $OUT/latency.err
cut -c1-200 $OUT/latency.jsonl

echo "== asm A/B: 7 (all) vs 1 (dot2 only) vs 6 (mul/sqr only)"
timeout -k 10 600 bash tools/gpu_ab.sh r5f_ab1 paritytech-bn_amd/libbn254mi.so ab/lib_d1.so "pairing product g2mul g1mul"
timeout -k 10 600 bash tools/gpu_ab.sh r5f_ab6 paritytech-bn_amd/libbn254mi.so ab/lib_d6.so "pairing product g2mul g1mul"
echo "== done"
