#!/usr/bin/env python3
"""Summarize rocprofv3 --pmc CSVs (separate FETCH_SIZE / WRITE_SIZE / SQ passes)
into profiles/pmc_summary.json (read by bench.py for roofline.traffic) and a
text table.  FETCH_SIZE / WRITE_SIZE are in KiB per dispatch.  Per
MI355X_MICROARCH.md §HBM, FETCH_SIZE reads half the bytes of 16-B/lane streaming
loads; this engine's loads are 4-B/lane dwords (uncalibrated), so the raw value
is reported and the caveat recorded."""
import collections
import csv
import json
import os
import sys

src, tag = sys.argv[1], sys.argv[2]  # e.g. gpurun_out r1
out_dir = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "profiles")
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for sub in ("pmc_fetch", "pmc_write", "pmc_sq"):
    path = os.path.join(src, sub, "p_counter_collection.csv")
    if not os.path.exists(path):
        continue
    for r in csv.DictReader(open(path)):
        agg[r["Kernel_Name"].split("(")[0].replace("bn::", "")][r["Counter_Name"]].append(float(r["Counter_Value"]))
summary = {}
lines = ["%-16s %14s %14s %14s %12s %10s" % ("kernel", "FETCH_bytes", "WRITE_bytes", "VALU/wave", "WAVE_CYC/w", "VALU/cyc")]
for k, v in sorted(agg.items()):
    if k.startswith("__amd"):
        continue
    m = {c: sum(x) / len(x) for c, x in v.items()}
    fetch = m.get("FETCH_SIZE", 0) * 1024
    write = m.get("WRITE_SIZE", 0) * 1024
    waves = m.get("SQ_WAVES", 0) or 1
    valu = m.get("SQ_INSTS_VALU", 0) / waves
    cyc = m.get("SQ_WAVE_CYCLES", 0) * 4 / waves  # quad-cycles
    summary[k] = {"hbm_bytes_per_launch": fetch + write, "fetch_bytes": fetch, "write_bytes": write,
                  "valu_insts_per_wave": valu, "wave_cycles": cyc,
                  "valu_per_cycle_per_wave": valu / cyc if cyc else None,
                  "note": "FETCH_SIZE/WRITE_SIZE raw (KiB*1024); dword loads uncalibrated (MI355X_MICROARCH §HBM)"}
    lines.append("%-16s %14.3e %14.3e %14.3e %12.3e %10.3f" % (k, fetch, write, valu, cyc, valu / cyc if cyc else 0))
json.dump(summary, open(os.path.join(out_dir, "pmc_summary.json"), "w"), indent=1)
open(os.path.join(out_dir, "%s_pmc.txt" % tag), "w").write("\n".join(lines) + "\n")
print("\n".join(lines))
