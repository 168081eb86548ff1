#!/bin/bash
# round 5, session d: balanced segment plan (per-segment K) -- tests, config 5, trace
set -e
OUT=gpurun_out/r5d
mkdir -p $OUT
export TMPDIR=/tmp
echo "== tests"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
echo "== product"
for r in 1 2; do
timeout -k 10 300 python -u bench.py --workload product --steps 20 --warmup 3 > $OUT/bench_product_$r.json 2> $OUT/bench_product_$r.err
python3 -c "import json; d=json.load(open('$OUT/bench_product_$r.json')); print('product', d['ms_per_step'], d['roofline']['frac'], d.get('parity_bit_exact'))"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_product -o run -- python3 bench.py --workload product --steps 10 --no-cpu-baseline > /dev/null 2> $OUT/prof_product.err
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $OUT/pmc_prod_sq -o p -- python3 bench.py --workload product --steps 2 --warmup 1 --no-cpu-baseline > /dev/null 2> $OUT/pmc_prod_sq.err
echo "== done"
