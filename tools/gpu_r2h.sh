#!/bin/bash
# segmented product with one reduction launch per level; line-coefficient A/B
# (BN254MI_MILLER_FORM 0 = k_prepare + k_miller, 1 = fused, 2 = k_miller_seg S=1)
set -e
OUT=gpurun_out/r2h
mkdir -p $OUT
export TMPDIR=/tmp
echo "== all gpu tests"; timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
echo "== product"; timeout -k 10 300 python -u bench.py --workload product --steps 10 --warmup 2 > $OUT/product.json 2> $OUT/product.err; cat $OUT/product.json
echo "== product stats"; timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_product -o run -- python3 bench.py --workload product --steps 5 --warmup 1 > /dev/null 2> $OUT/prof_product.err
for form in 0 1 2 0 1 2; do
  echo "== bench miller form $form"
  BN254MI_MILLER_FORM=$form timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-e2e > $OUT/bench_form$form.json 2> $OUT/bench_form$form.err
  python3 -c "import json; d=json.load(open('$OUT/bench_form$form.json')); print($form, round(d['value']), d['roofline']['per_launch_ms'])" | tee -a $OUT/ab_forms.txt
done
echo "== fused correctness"; BN254MI_MILLER_FORM=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $OUT/fused_tests.log 2>&1 || { tail -30 $OUT/fused_tests.log; exit 1; }
tail -1 $OUT/fused_tests.log
echo "== seg1 correctness"; BN254MI_MILLER_FORM=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $OUT/seg1_tests.log 2>&1 || { tail -30 $OUT/seg1_tests.log; exit 1; }
tail -1 $OUT/seg1_tests.log
echo "== done"
