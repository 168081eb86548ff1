#!/bin/bash
# A/B of the host pipeline's piece size (BN254MI_HOST_PIECE) on host-buffer bn_pairing_many.
set -e
OUT=gpurun_out/${1:-r2av}
mkdir -p $OUT
timeout -k 10 200 python -u -m pytest tests/test_gpu_host_pipeline.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
tail -1 $OUT/tests.log
for r in 1 2; do
  for pc in 65536 131072 262144; do
    echo "{\"host_piece\": $pc, \"round\": $r}" >> $OUT/piece_ab.jsonl
    BN254MI_HOST_PIECE=$pc timeout -k 10 240 python -u tools/host_e2e.py --sizes 262144,524288,1048576 >> $OUT/piece_ab.jsonl 2>> $OUT/e2e.err
  done
done
cat $OUT/piece_ab.jsonl
