#!/bin/bash
# A/B of alternative builds of libbn254mi.so kept under exp/lib_<V>.so (BN254MI_LIB
# selects the library): config 2 per-kernel times, config 5, Gt::pow and config 3, rounds
# interleaving the variants.  Usage: tools/ab_libs.sh OUTDIR A B ...
OUT=$1; shift
mkdir -p $OUT
for r in 1 2; do for v in "$@"; do
  BN254MI_LIB=exp/lib_$v.so timeout -k 5 120 python -u bench.py --no-cpu-baseline --no-e2e --steps 10 > $OUT/$v$r.json 2>/dev/null || exit 1
  BN254MI_LIB=exp/lib_$v.so timeout -k 5 120 python -u bench.py --workload product --steps 20 > $OUT/${v}${r}_product.json 2>/dev/null || exit 1
  BN254MI_LIB=exp/lib_$v.so timeout -k 5 120 python -u bench.py --workload gtpow --cpu-sample 64 > $OUT/${v}${r}_gtpow.json 2>/dev/null || exit 1
  BN254MI_LIB=exp/lib_$v.so timeout -k 5 120 python -u bench.py --workload g1mul --cpu-sample 64 > $OUT/${v}${r}_g1mul.json 2>/dev/null || exit 1
  python - <<EOF
import json
d = json.load(open("$OUT/$v$r.json")); p = json.load(open("$OUT/${v}${r}_product.json")); g = json.load(open("$OUT/${v}${r}_gtpow.json")); m = json.load(open("$OUT/${v}${r}_g1mul.json"))
print("$v$r", round(d["value"]), d["roofline"]["per_launch_ms"], "product_ms %.3f" % p["roofline"]["per_step_ms"],
      "gtpow_ms %.3f" % g["kernel"]["per_launch_ms"], "g1mul_ms %.3f" % m["ms_per_step"], flush=True)
EOF
done; done
