#!/bin/bash
# round 5 session p: the first chunk with the Fq12 inversion spread over lane pairs (w12_fe_first_par)
set -e
OUT=gpurun_out/r5p
mkdir -p $OUT
export TMPDIR=/tmp
echo "== product parity"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_failure.py -m gpu -x -q --timeout 200 --timeout-method thread -k "product or batch or config5 or miller_loop_batch or final or capped" > $OUT/parity.log 2>&1 || { tail -40 $OUT/parity.log; exit 1; }
tail -1 $OUT/parity.log
echo "== A/B product: parallel first chunk (1) vs w12_fe_first (0) vs w12 tail (w)"
for r in 1 2 3; do
  for v in 1 0 w; do
    case $v in 1) L=;; 0) L=ab/lib_fe1seq.so;; w) L=ab/lib_tailw12.so;; esac
    BN254MI_LIB=$L timeout -k 10 120 python -u bench.py --workload product --steps 20 --warmup 3 --no-cpu-baseline > $OUT/p_${v}_$r.json 2> $OUT/p_${v}_$r.err
    python3 -c "import json; d=json.load(open('$OUT/p_${v}_$r.json')); print('form $v r$r', round(d['ms_per_step'],4))"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_product -o run -- python3 bench.py --workload product --steps 10 --no-cpu-baseline > /dev/null 2> $OUT/prof_product.err
echo "== done"
