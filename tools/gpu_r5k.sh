#!/bin/bash
# round 5 session k: full GPU tests + fold check + config 5 / config 2 lines on the digit-sliced tail build
set -e
OUT=gpurun_out/r5k
mkdir -p $OUT
export TMPDIR=/tmp
echo "== tests"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
echo "== fold check"
BN254MI_LIB=paritytech-bn_amd/libbn254mi_dbg.so timeout -k 10 300 python -u tools/fold_check.py 4096 > $OUT/fold_check.json 2> $OUT/fold_check.err || { tail -20 $OUT/fold_check.err; exit 1; }
cat $OUT/fold_check.json
echo "== bench product"
timeout -k 10 300 python -u bench.py --workload product --steps 20 --warmup 3 > $OUT/bench_product.json 2> $OUT/bench_product.err
python3 -c "import json; d=json.load(open('$OUT/bench_product.json')); print('product', round(d['ms_per_step'],4), d['roofline']['frac'], d['cpu_baseline'].get('parity_sample_bit_exact', d['cpu_baseline'].get('bit_exact')))"
echo "== latency"
timeout -k 10 300 python -u tools/latency.py --calls pairing_batch --sizes 1,64,2048 > $OUT/lat.jsonl 2> $OUT/lat.err
cut -c1-110 $OUT/lat.jsonl
echo "== done"
