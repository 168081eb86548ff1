#!/bin/bash
# Host-buffer pipeline session: its GPU tests, the pageable/pinned A/B (interleaved), the bench line.
set -e
OUT=gpurun_out/${1:-r2ak}
mkdir -p $OUT
echo "== tests"; timeout -k 10 400 python -u -m pytest tests/test_gpu_host_pipeline.py tests/test_gpu_parity.py tests/test_gpu_concurrency.py -x -v --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
tail -2 $OUT/tests.log
for r in 1 2; do
  echo "== A/B round $r"
  BN254MI_HOST_PIPELINE=0 timeout -k 10 240 python -u tools/host_e2e.py --sizes 65536,262144,1048576 >> $OUT/e2e_ab.jsonl 2>> $OUT/e2e.err
  timeout -k 10 240 python -u tools/host_e2e.py --sizes 65536,262144,1048576 >> $OUT/e2e_ab.jsonl 2>> $OUT/e2e.err
done
cat $OUT/e2e_ab.jsonl
echo "== bench"; timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
cat $OUT/bench.json
echo "== done"
