#!/bin/bash
# round 5 session z (evidence on the final build): smoke(), five config-2 bench runs on one box,
# the throughput kernel's launch-size sweep (config 4 runs 2^17 pairs per GPU at N = 8)
set -e
OUT=gpurun_out/r5z
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > $OUT/smoke.txt 2>&1 || { tail -20 $OUT/smoke.txt; exit 1; }
tail -1 $OUT/smoke.txt
for r in 1 2 3 4 5; do
  timeout -k 10 200 python -u bench.py --no-e2e --no-config4-ref > $OUT/bench_$r.json 2> $OUT/bench_$r.err
  python3 -c "import json; d=json.load(open('$OUT/bench_$r.json')); r=d['roofline']; print('run $r', round(d['value']/1e6,4), 'M/s', round(d['ms_per_step'],4), 'ms/step', 'k_pairing_full', r['per_launch_ms'], 'frac', round(r['frac'],4), 'exact', d['cpu_baseline']['parity_sample_bit_exact'])"
done
timeout -k 10 400 python -u tools/size_sweep.py > $OUT/size_sweep.jsonl 2> $OUT/size_sweep.err
cat $OUT/size_sweep.jsonl | cut -c1-200
