#!/bin/bash
# Final check of the host pipeline with 2^17 pieces: all GPU tests, smoke, host-buffer sweep, bench line.
set -e
OUT=gpurun_out/${1:-r2aw}
mkdir -p $OUT
echo "== tests"; timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1
tail -1 $OUT/gpu_tests.log
echo "== smoke"; timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; tail -1 $OUT/smoke.log
echo "== host e2e"; timeout -k 10 240 python -u tools/host_e2e.py --sizes 65536,131072,262144,524288,1048576 > $OUT/host_e2e.jsonl 2> $OUT/e2e.err; cat $OUT/host_e2e.jsonl
echo "== bench"; timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err; cat $OUT/bench.json
echo "== done"
