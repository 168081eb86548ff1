#!/bin/bash
# Host-buffer pipeline with the one-piece threshold: all GPU tests, the three-mode A/B, the bench line.
set -e
OUT=gpurun_out/${1:-r2al}
mkdir -p $OUT
echo "== tests"; timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1
tail -2 $OUT/gpu_tests.log
for r in 1 2; do
  for m in 0 2 1; do
    BN254MI_HOST_PIPELINE=$m timeout -k 10 240 python -u tools/host_e2e.py --sizes 65536,131072,262144,1048576 >> $OUT/e2e_ab.jsonl 2>> $OUT/e2e.err
  done
done
cat $OUT/e2e_ab.jsonl
echo "== bench"; timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
cat $OUT/bench.json
echo "== done"
