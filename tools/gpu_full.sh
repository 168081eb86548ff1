#!/bin/bash
# Full round check on one GPU box: -m gpu tests, smoke, bench (+ CPU baseline), rocprof
# kernel stats + PMC passes, latency sweep, config 5 (+ its kernel stats), Gt::pow.
# Usage: tools/gpu_full.sh TAG
set -e
TAG=${1:-full}
bash tools/gpu_r2.sh $TAG pmc
OUT=gpurun_out/$TAG
echo "== latency"; timeout -k 10 300 python -u tools/latency.py --sizes 1,2,8,64,256,1024,4096,8192,16384 > $OUT/latency.jsonl 2> $OUT/latency.err; cat $OUT/latency.jsonl
echo "== product"; timeout -k 10 300 python -u bench.py --workload product --steps 10 --warmup 2 > $OUT/product.json 2> $OUT/product.err; cat $OUT/product.json
echo "== product stats"; timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_product -o run -- python3 bench.py --workload product --steps 5 --warmup 1 > /dev/null 2> $OUT/prof_product.err
echo "== latency n=1 stats"; timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/prof_lat1 -o run -- python3 tools/latency.py --sizes 1 --reps 20 --calls pairing_many_dev > /dev/null 2> $OUT/prof_lat1.err
echo "== gtpow"; timeout -k 10 200 python -u bench.py --workload gtpow > $OUT/gtpow.json 2> $OUT/gtpow.err; cat $OUT/gtpow.json
echo "== all done"
