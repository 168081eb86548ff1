#!/bin/bash
# latency forms (column-parallel products) in the wide kernels
set -e
OUT=gpurun_out/r2n
mkdir -p $OUT
export TMPDIR=/tmp
echo "== wide ubench"; timeout -k 10 120 ./tools/wide_ubench > $OUT/wide_ubench.jsonl 2>&1; cat $OUT/wide_ubench.jsonl
echo "== tests"; timeout -k 10 500 python -u -m pytest tests/test_gpu_wide.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
echo "== latency"; timeout -k 10 300 python -u tools/latency.py --sizes 1,2,8,64,1024,4096,8192 > $OUT/latency.jsonl 2> $OUT/latency.err; cat $OUT/latency.jsonl
echo "== product"; timeout -k 10 300 python -u bench.py --workload product --steps 10 --warmup 2 > $OUT/product.json 2> $OUT/product.err; cat $OUT/product.json
echo "== done"
