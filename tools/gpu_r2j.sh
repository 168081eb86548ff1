#!/bin/bash
# latency-path threshold sweep: pairing_many_dev with the wide path forced on / off
set -e
OUT=gpurun_out/r2j
mkdir -p $OUT
export TMPDIR=/tmp
for w in 0 1048576; do
  echo "== fe_wide_max $w"
  timeout -k 10 300 python -u tools/latency.py --calls pairing_many_dev --sizes 1,64,1024,2048,4096,8192,16384,32768,65536 --reps 5 --fe-wide-max $w > $OUT/sweep_$w.jsonl 2> $OUT/sweep_$w.err
  cat $OUT/sweep_$w.jsonl
done
echo "== done"
