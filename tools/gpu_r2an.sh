#!/bin/bash
# A/B of the start-time stagger (BN254MI_STAGGER) on the throughput kernels at 2^16 and 2^17 pairs.
# (The BN254MI_STAGGER switch was an A/B build that measured no gain and was removed)
set -e
OUT=gpurun_out/${1:-r2an}
mkdir -p $OUT
for r in 1 2; do
  for st in 0 0x004 0x010 0x104 0x204 0x208 0x202; do
    echo "{\"stagger\": \"$st\", \"round\": $r}" >> $OUT/stagger_ab.jsonl
    BN254MI_STAGGER=$st timeout -k 10 120 python -u tools/size_sweep.py --sizes 65536,131072 --reps 10 >> $OUT/stagger_ab.jsonl 2>> $OUT/stagger.err
  done
done
cat $OUT/stagger_ab.jsonl
