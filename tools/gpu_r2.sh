#!/bin/bash
# One GPU-box session of round 2: parity tests, bench line, rocprofv3 kernel
# stats; each GPU step under its own time limit, chained so the first failure
# ends the call.  Usage: tools/gpu_r2.sh TAG [pmc]
set -e
TAG=${1:-run}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
echo "== tests"; timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -3 $OUT/gpu_tests.log
echo "== smoke"; timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; tail -2 $OUT/smoke.log
echo "== bench"; timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
cat $OUT/bench.json
echo "== stats"; timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 bench.py --no-cpu-baseline --no-e2e > $OUT/bench_prof.json 2> $OUT/prof.err
if [ "$2" == "pmc" ]; then
echo "== pmc"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o p -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-e2e > /dev/null 2> $OUT/pmc_fetch.err
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o p -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-e2e > /dev/null 2> $OUT/pmc_write.err
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $OUT/pmc_sq -o p -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-e2e > /dev/null 2> $OUT/pmc_sq.err
fi
echo "== done"
