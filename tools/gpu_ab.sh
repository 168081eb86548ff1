#!/bin/bash
# Interleaved A/B of two library builds on configs 3 and 5 (and optionally config 2):
#   tools/gpu_ab.sh TAG LIB_A LIB_B [workloads]   (LIB_* = path of a libbn254mi.so build)
set -e
TAG=$1; A=$2; B=$3; W=${4:-"g1mul product"}
OUT=gpurun_out/$TAG
mkdir -p $OUT
for r in 1 2; do
  for w in $W; do
    for L in A B; do
      lib=$A; [ $L = B ] && lib=$B
      if [ $w = pairing ]; then args=""; else args="--workload $w"; fi
      BN254MI_LIB=$lib timeout -k 10 120 python -u bench.py $args --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-config4-ref > $OUT/${w}_${L}_$r.json 2> $OUT/${w}_${L}_$r.err
      python3 -c "import json; d=json.load(open('$OUT/${w}_${L}_$r.json')); print('$w $L r$r', round(d['ms_per_step'],4))"
    done
  done
done
