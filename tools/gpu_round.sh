#!/bin/bash
# One GPU-box session: parity tests, bench line, rocprofv3 kernel stats and
# the three PMC passes (FETCH_SIZE / WRITE_SIZE / SQ), each step time-limited
# and chained so the first failure ends the call.  Usage: tools/gpu_round.sh TAG
set -e
TAG=${1:-run}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
echo "== tests"; timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1
tail -3 $OUT/gpu_tests.log
echo "== bench"; timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
cat $OUT/bench.json
echo "== stats"; timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 bench.py --no-cpu-baseline > $OUT/bench_prof.json 2> $OUT/prof.err
echo "== pmc"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o p -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > /dev/null 2> $OUT/pmc_fetch.err
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o p -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > /dev/null 2> $OUT/pmc_write.err
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $OUT/pmc_sq -o p -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > /dev/null 2> $OUT/pmc_sq.err
echo "== 8(f) workloads"
for w in g2validate g2decompress gtpow g1mul; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 5 --warmup 1 > $OUT/bench_$w.json 2> $OUT/bench_$w.err
  head -c 400 $OUT/bench_$w.json; echo
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_codec -o run -- python3 bench.py --workload g2validate --steps 3 --warmup 1 > /dev/null 2> $OUT/prof_codec.err
echo "== done"
