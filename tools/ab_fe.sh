#!/bin/bash
# A/B timing of alternative builds of libbn254mi.so kept under exp/ (BN254MI_LIB
# selects the library); rounds interleave the variants.  Usage: tools/ab_fe.sh A D ...
mkdir -p gpurun_out/ab
for r in 1 2; do for v in "$@"; do
  BN254MI_LIB=exp/lib_$v.so timeout -k 5 120 python -u bench.py --no-cpu-baseline --steps 10 > gpurun_out/ab/$v$r.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/ab/$v$r.json'));print('$v$r', round(d['value']), d['roofline']['per_launch_ms'])"
done; done
