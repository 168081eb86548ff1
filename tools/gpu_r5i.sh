#!/bin/bash
# round 5 session i (re-entry baseline of HEAD): GPU tests, config 2 and config 5 bench lines, kernel traces
set -e
OUT=gpurun_out/r5i
mkdir -p $OUT
export TMPDIR=/tmp
echo "== tests"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
echo "== bench config 2"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print('config2', round(d['value']), round(d['ms_per_step'],4), round(d['roofline']['frac'],4))"
echo "== bench config 5"
for r in 1 2; do
  timeout -k 10 120 python -u bench.py --workload product --steps 20 --warmup 3 --no-cpu-baseline > $OUT/p_$r.json 2> $OUT/p_$r.err
  python3 -c "import json; d=json.load(open('$OUT/p_$r.json')); print('product r$r', round(d['ms_per_step'],4))"
done
echo "== traces"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_pair -o run -- python3 bench.py --steps 10 --no-cpu-baseline > /dev/null 2> $OUT/prof_pair.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_product -o run -- python3 bench.py --workload product --steps 10 --no-cpu-baseline > /dev/null 2> $OUT/prof_product.err
echo "== done"
