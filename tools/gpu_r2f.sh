set -e
bash tools/gpu_r2.sh r2f
echo "== latency"; timeout -k 10 300 python -u tools/latency.py > gpurun_out/r2f/latency.jsonl 2> gpurun_out/r2f/latency.err; cat gpurun_out/r2f/latency.jsonl
echo "== product"; timeout -k 10 300 python -u bench.py --workload product --steps 5 --warmup 1 > gpurun_out/r2f/product.json 2> gpurun_out/r2f/product.err; cat gpurun_out/r2f/product.json
echo "== product stats"; timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2f/prof_product -o run -- python3 bench.py --workload product --steps 3 --warmup 1 > /dev/null 2> gpurun_out/r2f/prof_product.err
echo done
