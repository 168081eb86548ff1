set -e
mkdir -p gpurun_out/r5ac
for r in 1 2; do
  for L in A B; do
    if [ $L = B ]; then export BN254MI_PREPARE_WIDE_MAX=0; else unset BN254MI_PREPARE_WIDE_MAX; fi
    timeout -k 10 120 python -u bench.py --workload product --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r5ac/p_${L}_$r.json 2> gpurun_out/r5ac/p_${L}_$r.err
    python3 -c "import json; d=json.load(open('gpurun_out/r5ac/p_${L}_$r.json')); print('$L r$r', round(d['ms_per_step'],4))"
  done
done
unset BN254MI_PREPARE_WIDE_MAX
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r5ac/prof -o run -- python3 bench.py --workload product --steps 5 --no-cpu-baseline > /dev/null 2> gpurun_out/r5ac/prof.err
