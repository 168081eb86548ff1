#!/bin/bash
# One GPU-box measurement session for round TAG: parity tests, the bench line,
# rocprofv3 kernel stats, the PMC passes (FETCH_SIZE / WRITE_SIZE / two SQ sets),
# the other BASELINE workloads and the latency sweep.  Each step is time-limited
# and the first failure ends the call.  Usage: tools/gpu_round.sh TAG
set -e
TAG=${1:-run}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
Q="--no-cpu-baseline --no-e2e --no-config4-ref"
echo "== tests"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
echo "== bench"
timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
cat $OUT/bench.json
echo "== config 4 in one process (bn_ctx_create_multi + bn_pairing_many_allgather_dev; RCCL world of the visible GPUs)"
timeout -k 10 300 python -u bench.py --form capi --gpus ${CAPI_GPUS:-1} --steps 3 --warmup 1 > $OUT/bench_capi.json 2> $OUT/bench_capi.err
head -c 400 $OUT/bench_capi.json; echo
echo "== kernel stats"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 bench.py $Q > $OUT/bench_prof.json 2> $OUT/prof.err
# per-kernel CSV with the steady-state columns (SteadyAverageNs: without the cold first launch; MedianNs)
python3 tools/rocpd_stats.py $(find $OUT/prof -name '*results.db' | head -1) > $OUT/kernel_stats.csv || true
echo "== pmc"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o p -- python3 bench.py --steps 2 --warmup 1 $Q > /dev/null 2> $OUT/pmc_fetch.err
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o p -- python3 bench.py --steps 2 --warmup 1 $Q > /dev/null 2> $OUT/pmc_write.err
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $OUT/pmc_sq -o p -- python3 bench.py --steps 2 --warmup 1 $Q > /dev/null 2> $OUT/pmc_sq.err
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU -d $OUT/pmc_sq2 -o p -- python3 bench.py --steps 2 --warmup 1 $Q > /dev/null 2> $OUT/pmc_sq2.err
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_prod_fetch -o p -- python3 bench.py --workload product --steps 2 --warmup 1 --no-cpu-baseline > /dev/null 2> $OUT/pmc_prod_fetch.err
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_prod_write -o p -- python3 bench.py --workload product --steps 2 --warmup 1 --no-cpu-baseline > /dev/null 2> $OUT/pmc_prod_write.err
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_g1_fetch -o p -- python3 bench.py --workload g1mul --steps 2 --warmup 1 --no-cpu-baseline > /dev/null 2> $OUT/pmc_g1_fetch.err
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_g1_write -o p -- python3 bench.py --workload g1mul --steps 2 --warmup 1 --no-cpu-baseline > /dev/null 2> $OUT/pmc_g1_write.err
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $OUT/pmc_g1_sq -o p -- python3 bench.py --workload g1mul --steps 2 --warmup 1 --no-cpu-baseline > /dev/null 2> $OUT/pmc_g1_sq.err
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $OUT/pmc_g2_sq -o p -- python3 bench.py --workload g2mul --steps 2 --warmup 1 --no-cpu-baseline > /dev/null 2> $OUT/pmc_g2_sq.err
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $OUT/pmc_prod_sq -o p -- python3 bench.py --workload product --steps 2 --warmup 1 --no-cpu-baseline > /dev/null 2> $OUT/pmc_prod_sq.err
# config 5 with the two-lane line producer (k_prepare, BN254MI_PREPARE_WIDE_MAX=0): its waves' VALU and lifetime
# (the chain a streamed two-lane producer would put in front of the segmented Miller loop)
BN254MI_PREPARE_WIDE_MAX=0 timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $OUT/pmc_prod2_sq -o p -- python3 bench.py --workload product --steps 2 --warmup 1 --no-cpu-baseline > /dev/null 2> $OUT/pmc_prod2_sq.err
if [ -f paritytech-bn_amd/libbn254mi_dbg.so ]; then
  echo "== fold check (libbn254mi_dbg.so: every fold site counts bound violations)"
  BN254MI_LIB=paritytech-bn_amd/libbn254mi_dbg.so timeout -k 10 300 python -u tools/fold_check.py 4096 > $OUT/fold_check.json 2> $OUT/fold_check.err || { tail -20 $OUT/fold_check.err; exit 1; }
  cat $OUT/fold_check.json
fi
echo "== workloads"
for w in g1mul g2mul product gtpow g2validate g2decompress; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 10 --warmup 2 > $OUT/bench_$w.json 2> $OUT/bench_$w.err
  head -c 300 $OUT/bench_$w.json; echo
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_product -o run -- python3 bench.py --workload product --steps 10 > /dev/null 2> $OUT/prof_product.err
python3 tools/rocpd_stats.py $(find $OUT/prof_product -name '*results.db' | head -1) > $OUT/product_kernel_stats.csv || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_g1mul -o run -- python3 bench.py --workload g1mul --steps 5 --cpu-sample 64 > /dev/null 2> $OUT/prof_g1mul.err
if [ -f exp/lib_mulstats.so ]; then
  echo "== G*Fr schedule counters (diagnostic build)"
  BN254MI_LIB=exp/lib_mulstats.so timeout -k 10 120 python -u tools/mul_stats.py > $OUT/mul_stats.json 2> $OUT/mul_stats.err
  cat $OUT/mul_stats.json
fi
echo "== latency"
timeout -k 10 300 python -u tools/latency.py --calls pairing_many_dev,pairing_many,pairing_batch --sizes 1,2,8,64,256,1024,2048,4096 > $OUT/latency.jsonl 2> $OUT/latency.err
head -3 $OUT/latency.jsonl
echo "== latency 2049-4096: one-launch two-wave build vs one-wave build (two rounds) vs segmented"
timeout -k 10 300 python -u tools/latency.py --calls pairing_many_dev,pairing_batch --sizes 2049,3072,4096 --latency-max 4096 > $OUT/latency_w2.jsonl 2> $OUT/latency_w2.err
BN254MI_LATENCY_W2=0 timeout -k 10 300 python -u tools/latency.py --calls pairing_many_dev --sizes 2049,4096 --latency-max 4096 > $OUT/latency_w1.jsonl 2> $OUT/latency_w1.err
grep -h '"n"' $OUT/latency_w2.jsonl $OUT/latency_w1.jsonl | cut -c1-120
echo "== done"
