#!/bin/bash
# A/B of alternative libbn254mi.so builds (exp/lib_$v.so) on the SURVEY 8(f)
# workloads of bench.py; rounds interleave the variants.  Usage: tools/ab_workloads.sh A B ...
mkdir -p gpurun_out/abw
for r in 1 2; do for w in g1mul g2validate g2decompress gtpow; do for v in "$@"; do
  BN254MI_LIB=exp/lib_$v.so timeout -k 5 120 python -u bench.py --workload $w --no-cpu-baseline --steps 5 > gpurun_out/abw/$w.$v$r.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/abw/$w.$v$r.json'));print('$w $v$r', round(d['value']), d['ms_per_step'])"
done; done; done
