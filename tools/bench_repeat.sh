set -e
mkdir -p gpurun_out/r4o
for r in 1 2 3 4 5; do
  timeout -k 10 200 python -u bench.py --no-e2e --no-config4-ref > gpurun_out/r4o/bench_$r.json 2> gpurun_out/r4o/bench_$r.err
  python3 -c "import json; d=json.load(open('gpurun_out/r4o/bench_$r.json')); r=d['roofline']; print('run $r', round(d['value']/1e6,4), 'M/s', round(d['ms_per_step'],4), 'ms/step', 'k_pairing_full', r['per_launch_ms'], 'frac', round(r['frac'],4), 'exact', d['cpu_baseline']['parity_sample_bit_exact'])"
done
