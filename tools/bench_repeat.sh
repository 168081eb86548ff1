# Repeat runs on ONE box: the spread of the bench lines the driver's single run is one
# sample of.  Usage (on the GPU box): bash tools/bench_repeat.sh TAG [RUNS]
set -e
TAG=${1:-repeat}
RUNS=${2:-5}
OUT=gpurun_out/$TAG
mkdir -p $OUT
for r in $(seq 1 $RUNS); do
  timeout -k 10 200 python -u bench.py --no-e2e --no-config4-ref --cpu-sample 2048 > $OUT/bench_$r.json 2> $OUT/bench_$r.err
  python3 -c "import json; d=json.loads([l for l in open('$OUT/bench_$r.json') if l.startswith('{')][-1]); r=d['roofline']; print('config 2 run $r', round(d['value']/1e6,4), 'M/s', round(d['ms_per_step'],4), 'ms/step', 'frac', round(r['frac'],4), 'exact', d['cpu_baseline']['parity_sample_bit_exact'])"
  timeout -k 10 200 python -u bench.py --workload product --steps 20 --warmup 3 > $OUT/product_$r.json 2> $OUT/product_$r.err
  python3 -c "import json; d=json.loads([l for l in open('$OUT/product_$r.json') if l.startswith('{')][-1]); print('config 5 run $r', round(d['ms_per_step'],4), 'ms', 'frac', round(d['roofline']['frac'],4), 'affine', round(d['affine_inputs']['ms_per_product'],4), 'exact', d['cpu_baseline']['parity_bit_exact'])"
done
