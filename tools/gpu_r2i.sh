#!/bin/bash
# full round check: tests, smoke, bench (+ CPU baseline), rocprof stats + PMC, latency, config 5
set -e
bash tools/gpu_r2.sh r2i pmc
OUT=gpurun_out/r2i
echo "== latency"; timeout -k 10 300 python -u tools/latency.py --sizes 1,2,8,64,256,1024,4096,8192,16384 > $OUT/latency.jsonl 2> $OUT/latency.err; cat $OUT/latency.jsonl
echo "== product"; timeout -k 10 300 python -u bench.py --workload product --steps 10 --warmup 2 > $OUT/product.json 2> $OUT/product.err; cat $OUT/product.json
echo "== product stats"; timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_product -o run -- python3 bench.py --workload product --steps 5 --warmup 1 > /dev/null 2> $OUT/prof_product.err
echo "== all done"
