#!/bin/bash
# round 5 session j: the digit-sliced final exponentiation in the product tail (kernels_tail.hip BN_TAIL_DS)
set -e
OUT=gpurun_out/r5j
mkdir -p $OUT
export TMPDIR=/tmp
echo "== ds_check"
timeout -k 10 120 tools/ds_check 64 > $OUT/ds_check3.txt 2>&1 || { cat $OUT/ds_check3.txt; exit 1; }
tail -6 $OUT/ds_check3.txt
echo "== product parity"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "product or batch or config5 or miller_loop_batch or final" > $OUT/parity.log 2>&1 || { tail -40 $OUT/parity.log; exit 1; }
tail -1 $OUT/parity.log
echo "== A/B product: DS tail (1) vs w12 tail (0)"
for r in 1 2; do
  for v in 1 0; do
    if [ $v = 1 ]; then L=; else L=ab/lib_tailw12.so; fi
    BN254MI_LIB=$L timeout -k 10 120 python -u bench.py --workload product --steps 20 --warmup 3 --no-cpu-baseline > $OUT/p_${v}_$r.json 2> $OUT/p_${v}_$r.err
    python3 -c "import json; d=json.load(open('$OUT/p_${v}_$r.json')); print('tail_ds=$v r$r', round(d['ms_per_step'],4), d.get('parity_bit_exact', d.get('cpu_baseline',{}).get('parity_sample_bit_exact')))"
  done
done
for v in 1 0; do
  if [ $v = 1 ]; then L=; else L=ab/lib_tailw12.so; fi
  BN254MI_LIB=$L timeout -k 10 300 python -u tools/latency.py --calls pairing_batch --sizes 1,64,2048 > $OUT/lat_$v.jsonl 2> $OUT/lat_$v.err
  echo "tail_ds=$v"; cut -c1-150 $OUT/lat_$v.jsonl
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_product -o run -- python3 bench.py --workload product --steps 10 --no-cpu-baseline > /dev/null 2> $OUT/prof_product.err
echo "== done"
