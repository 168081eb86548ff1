#!/bin/bash
# round 5 session h: k_horner_tree2 (FE squarer on a group pair) -- tests, fold check, A/B vs k_horner_tree
set -e
OUT=gpurun_out/r5h
mkdir -p $OUT
export TMPDIR=/tmp
echo "== tests"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
echo "== fold check"
BN254MI_LIB=paritytech-bn_amd/libbn254mi_dbg.so timeout -k 10 300 python -u tools/fold_check.py 4096 > $OUT/fold_check.json 2> $OUT/fold_check.err || { tail -20 $OUT/fold_check.err; exit 1; }
cat $OUT/fold_check.json
echo "== A/B tree2 (2) vs tree (1)"
for r in 1 2; do
  for v in 2 1; do
    BN254MI_HORNER_TREE=$v timeout -k 10 120 python -u bench.py --workload product --steps 20 --warmup 3 --no-cpu-baseline > $OUT/p_${v}_$r.json 2> $OUT/p_${v}_$r.err
    python3 -c "import json; d=json.load(open('$OUT/p_${v}_$r.json')); print('tree$v r$r', round(d['ms_per_step'],4))"
  done
done
for v in 2 1; do
  BN254MI_HORNER_TREE=$v timeout -k 10 300 python -u tools/latency.py --calls pairing_batch --sizes 1,64,2048 > $OUT/lat_$v.jsonl 2> $OUT/lat_$v.err
  echo "tree$v"; cut -c1-120 $OUT/lat_$v.jsonl
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_product -o run -- python3 bench.py --workload product --steps 10 --no-cpu-baseline > /dev/null 2> $OUT/prof_product.err
echo "== done"
