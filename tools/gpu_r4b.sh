#!/bin/bash
# Round-4 session b: the full round script (tests, bench lines, profiles, PMC, workloads, latency,
# G*Fr schedule counters), then config 5 with 16 against 32 segments, two interleaved rounds.
set -e
bash tools/gpu_round.sh r4b
OUT=gpurun_out/r4b
echo "== config 5: 16 vs 32 segments"
for r in 1 2; do for S in 16 32; do
  BN254MI_BATCH_SEGS=$S timeout -k 10 120 python -u bench.py --workload product --steps 20 --warmup 3 --no-cpu-baseline > $OUT/product_S${S}_$r.json 2> $OUT/product_S${S}_$r.err
  python3 -c "import json; d=json.load(open('$OUT/product_S${S}_$r.json')); print('S=$S r$r', round(d['ms_per_step'],4), d.get('roofline',{}).get('per_step_ms'))"
done; done
echo done
