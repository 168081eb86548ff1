#!/bin/bash
# One A/B session on a GPU box for a candidate build (replaces round 5's one-shot
# tools/gpu_r5*.sh scripts; git history keeps them):
#   tools/gpu_ab_session.sh TAG LIB_B [WORKLOADS] [PMC_WORKLOADS]
# 1. the -m gpu parity tests on LIB_B (BN254MI_LIB), first failure ends the call;
# 2. the interleaved A/B (tools/gpu_ab.sh) of the product library against LIB_B over
#    WORKLOADS (default "pairing product"; names as bench.py --workload, "pairing"
#    = config 2);
# 3. per library, PMC passes (FETCH_SIZE, WRITE_SIZE, the SQ set) of each workload in
#    PMC_WORKLOADS (default none), one rocprofv3 run per counter set.
# Set SKIP_TESTS=1 to skip step 1 (a variant already tested in an earlier call).
set -e
TAG=$1; B=$2; W=${3:-"pairing product"}; PW=${4:-""}
A=paritytech-bn_amd/libbn254mi.so
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
  BN254MI_LIB=$B timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/tests_B.log 2>&1 || { tail -30 $OUT/tests_B.log; exit 1; }
  tail -1 $OUT/tests_B.log
fi
timeout -k 10 1200 bash tools/gpu_ab.sh $TAG $A $B "$W"
for w in $PW; do
  if [ $w = pairing ]; then args="--no-e2e --no-config4-ref"; else args="--workload $w"; fi
  for L in A B; do
    lib=$A; [ $L = B ] && lib=$B
    for c in FETCH_SIZE WRITE_SIZE "SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
      n=$(echo $c | cut -d' ' -f1 | tr 'A-Z' 'a-z')
      BN254MI_LIB=$lib timeout -s KILL 180 rocprofv3 --pmc $c -d $OUT/pmc_${w}_${n}_$L -o p -- python3 bench.py $args --steps 2 --warmup 1 --no-cpu-baseline > /dev/null 2> $OUT/pmc_${w}_${n}_$L.err
    done
  done
done
echo "== done"
