#!/bin/bash
# A/B of library variants exp/lib_<V>.so on config 2 (HBM-resident 2^16 pairs,
# per-kernel HIP-event times), ROUNDS interleaved rounds.  Optional WORKLOADS
# (space-separated bench.py --workload names) run after each config-2 line.
# Usage: tools/gpu_ab.sh OUTDIR ROUNDS V1 V2 ...
OUT=$1; ROUNDS=$2; shift 2
mkdir -p $OUT
for r in $(seq 1 $ROUNDS); do for v in "$@"; do
  BN254MI_LIB=exp/lib_$v.so timeout -k 5 150 python -u bench.py --no-cpu-baseline --no-e2e --steps 20 \
    > $OUT/$v$r.json 2> $OUT/$v$r.err || { echo "bench failed: $v$r"; tail -5 $OUT/$v$r.err; exit 1; }
  for w in $WORKLOADS; do
    BN254MI_LIB=exp/lib_$v.so timeout -k 5 150 python -u bench.py --workload $w --steps 10 --cpu-sample 64 \
      > $OUT/${v}${r}_$w.json 2>> $OUT/$v$r.err || { echo "bench $w failed: $v$r"; exit 1; }
  done
  python3 - <<PY
import json, os
d = json.load(open("$OUT/$v$r.json"))
extra = ""
for w in "$WORKLOADS".split():
    x = json.load(open("$OUT/${v}${r}_%s.json" % w))
    extra += " %s %.3f ms" % (w, x.get("roofline", {}).get("per_step_ms") or x.get("kernel", {}).get("per_launch_ms") or x["ms_per_step"])
print("$v$r", round(d["value"]), d["roofline"]["per_launch_ms"], extra, flush=True)
PY
done; done
