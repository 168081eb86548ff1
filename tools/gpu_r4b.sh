set -e
OUT=gpurun_out/r4b; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
for r in 1 2; do for S in 16 32; do
  BN254MI_BATCH_SEGS=$S timeout -k 10 120 python -u bench.py --workload product --steps 20 --warmup 3 --no-cpu-baseline > $OUT/product_S${S}_$r.json 2> $OUT/product_S${S}_$r.err
  python3 -c "import json; d=json.load(open('$OUT/product_S${S}_$r.json')); print('S=$S r$r', round(d['ms_per_step'],4), d.get('roofline',{}).get('per_step_ms'))"
done; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_product -o run -- python3 bench.py --workload product --steps 10 --no-cpu-baseline > /dev/null 2> $OUT/prof_product.err
BN254MI_LIB=exp/lib_mulstats.so timeout -k 10 120 python -u tools/mul_stats.py > $OUT/mul_stats.json 2> $OUT/mul_stats.err
cat $OUT/mul_stats.json
echo done
