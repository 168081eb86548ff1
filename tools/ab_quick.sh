#!/bin/bash
# Config-2 per-kernel times of library variants exp/lib_<V>.so, ROUNDS interleaved
# rounds (default 4).  Usage: tools/ab_quick.sh OUTDIR ROUNDS A B ...
OUT=$1; R=$2; shift 2
mkdir -p $OUT
for r in $(seq 1 $R); do for v in "$@"; do
  BN254MI_LIB=exp/lib_$v.so timeout -k 5 120 python -u bench.py --no-cpu-baseline --no-e2e --steps 20 > $OUT/$v$r.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('$OUT/$v$r.json'));print('$v$r', round(d['value']), d['roofline']['per_launch_ms'])"
done; done
