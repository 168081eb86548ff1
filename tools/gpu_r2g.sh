#!/bin/bash
# wide-layout FE / device product reduction: tests, latency, config 5, config 2
set -e
OUT=gpurun_out/r2g
mkdir -p $OUT
export TMPDIR=/tmp
echo "== wide tests"; timeout -k 10 300 python -u -m pytest tests/test_gpu_wide.py -x -v --timeout 200 --timeout-method thread > $OUT/wide_tests.log 2>&1 || { tail -40 $OUT/wide_tests.log; exit 1; }
tail -3 $OUT/wide_tests.log
echo "== all gpu tests"; timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -3 $OUT/gpu_tests.log
echo "== latency"; timeout -k 10 300 python -u tools/latency.py --sizes 1,2,8,64,256,1024,4096,16384 > $OUT/latency.jsonl 2> $OUT/latency.err; cat $OUT/latency.jsonl
echo "== product"; timeout -k 10 300 python -u bench.py --workload product --steps 10 --warmup 2 > $OUT/product.json 2> $OUT/product.err; cat $OUT/product.json
echo "== product stats"; timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_product -o run -- python3 bench.py --workload product --steps 5 --warmup 1 > /dev/null 2> $OUT/prof_product.err
echo "== bench"; timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err; cat $OUT/bench.json
echo "== done"
