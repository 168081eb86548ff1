#!/bin/bash
# round-5 first session: GPU tests (with the failure-path test), the device
# fold-bound check over every unit, the bench line, the Fq2-product microbenchmark
set -e
OUT=gpurun_out/r5a
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
echo "== dot2 ubench"
timeout -k 10 60 tools/dot2_ubench_c.bin > $OUT/dot2.jsonl
cat $OUT/dot2.jsonl
echo "== done"
