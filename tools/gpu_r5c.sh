#!/bin/bash
# round 5, session c: the asm column-sum build -- GPU tests, bench lines, the
# product's kernel trace and SQ counters per kernel (k_prepare_wide's issue)
set -e
OUT=gpurun_out/r5c
mkdir -p $OUT
export TMPDIR=/tmp
Q="--no-cpu-baseline --no-e2e --no-config4-ref"
echo "== tests"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
echo "== bench"
timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
cut -c1-400 $OUT/bench.json
for w in product g1mul g2mul; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 10 --warmup 2 > $OUT/bench_$w.json 2> $OUT/bench_$w.err
  cut -c1-300 $OUT/bench_$w.json; echo
done
echo "== product trace + SQ counters"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_product -o run -- python3 bench.py --workload product --steps 10 --no-cpu-baseline > /dev/null 2> $OUT/prof_product.err
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $OUT/pmc_prod_sq -o p -- python3 bench.py --workload product --steps 2 --warmup 1 --no-cpu-baseline > /dev/null 2> $OUT/pmc_prod_sq.err
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU -d $OUT/pmc_prod_sq2 -o p -- python3 bench.py --workload product --steps 2 --warmup 1 --no-cpu-baseline > /dev/null 2> $OUT/pmc_prod_sq2.err
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_LDS -d $OUT/pmc_prod_sq3 -o p -- python3 bench.py --workload product --steps 2 --warmup 1 --no-cpu-baseline > /dev/null 2> $OUT/pmc_prod_sq3.err || echo "sq3 pass failed"
echo "== done"
