#!/bin/bash
# Interleaved A/B of two library builds on small-batch latency (tools/latency.py) and config 5:
#   tools/gpu_ab_latency.sh TAG LIB_A LIB_B
set -e
TAG=$1; A=$2; B=$3
OUT=gpurun_out/$TAG
mkdir -p $OUT
for r in 1 2; do
  for L in A B; do
    lib=$A; [ $L = B ] && lib=$B
    BN254MI_LIB=$lib timeout -k 10 200 python -u tools/latency.py --calls pairing_many_dev,pairing_batch --sizes 1,64,4096 > $OUT/lat_${L}_$r.jsonl 2> $OUT/lat_${L}_$r.err
    python3 -c "
import json
for l in open('$OUT/lat_${L}_$r.jsonl'):
    d = json.loads(l)
    if 'call' in d: print('$L r$r', d['call'], d['n'], round(d['ms'], 4))"
    BN254MI_LIB=$lib timeout -k 10 120 python -u bench.py --workload product --steps 20 --warmup 3 --no-cpu-baseline > $OUT/product_${L}_$r.json 2> $OUT/product_${L}_$r.err
    python3 -c "import json; d=json.load(open('$OUT/product_${L}_$r.json')); print('$L r$r product', round(d['ms_per_step'],4))"
  done
done
