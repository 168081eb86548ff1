#!/bin/bash
# GPU session for the SURVEY 8(f) rows: parity tests, then one bench line per workload.
set -e
TAG=${1:-codec}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
echo "== tests"; timeout -k 10 600 python -u -m pytest tests/test_gpu_codec.py tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -3 $OUT/gpu_tests.log
for w in g2validate g2decompress gtpow; do
  echo "== $w"; timeout -k 10 300 python -u bench.py --workload $w --steps 5 --warmup 1 > $OUT/bench_$w.json 2> $OUT/bench_$w.err
  cat $OUT/bench_$w.json
done
