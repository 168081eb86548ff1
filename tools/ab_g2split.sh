set -e
mkdir -p gpurun_out/r4m
BN254MI_G2_SPLIT=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "g2" > gpurun_out/r4m/tests.log 2>&1 || { tail -20 gpurun_out/r4m/tests.log; exit 1; }
tail -1 gpurun_out/r4m/tests.log
BN254MI_G2_SPLIT=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_wide.py tests/test_gpu_multi.py tests/test_gpu_concurrency.py > gpurun_out/r4m/tests2.log 2>&1 || { tail -20 gpurun_out/r4m/tests2.log; exit 1; }
tail -1 gpurun_out/r4m/tests2.log
for r in 1 2; do for S in 1 0; do
  BN254MI_G2_SPLIT=$S timeout -k 10 200 python -u bench.py --workload g2mul --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r4m/g2_S${S}_$r.json 2> gpurun_out/r4m/g2_S${S}_$r.err
  python3 -c "import json; d=json.load(open('gpurun_out/r4m/g2_S${S}_$r.json')); print('split=$S r$r', round(d['ms_per_step'],4), round(d['value']/1e6,3), 'M/s')"
done; done
BN254MI_G2_SPLIT=1 timeout -k 10 300 python -u bench.py --workload g2mul --steps 10 --warmup 2 > gpurun_out/r4m/g2_full.json 2> gpurun_out/r4m/g2_full.err
python3 -c "import json; d=json.load(open('gpurun_out/r4m/g2_full.json')); print(d['roofline']['frac'], d['cpu_baseline'])"
