#!/bin/bash
# round 5 session r: GPU tests + config 2 line on the no-fence build
set -e
OUT=gpurun_out/r5r
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > $OUT/bench.json 2> $OUT/bench.err
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print('config2', round(d['value']), round(d['ms_per_step'],4), round(d['roofline']['frac'],4), d['cpu_baseline'].get('parity_sample_bit_exact'))"
