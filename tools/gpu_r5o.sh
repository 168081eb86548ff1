#!/bin/bash
# round 5 session o: full GPU tests, fold check, product / latency / config 2 lines on the S+M tail build
set -e
OUT=gpurun_out/r5o
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
python3 -c "import json; d=json.load(open('$OUT/bench_product.json')); print('product', round(d['ms_per_step'],4), round(d['roofline']['frac'],4), d['cpu_baseline'].get('parity_bit_exact'))"
echo "== latency"
timeout -k 10 300 python -u tools/latency.py --calls pairing_batch,pairing_many --sizes 1,64,2048 > $OUT/lat.jsonl 2> $OUT/lat.err
cut -c1-100 $OUT/lat.jsonl
echo "== bench config 2"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > $OUT/bench.json 2> $OUT/bench.err
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print('config2', round(d['value']), round(d['ms_per_step'],4), round(d['roofline']['frac'],4))"
echo "== done"
