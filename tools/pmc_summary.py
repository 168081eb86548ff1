#!/usr/bin/env python3
"""Summarize one gpu_round.sh session (rocprofv3 sqlite output, ROCm 7.2).

    python tools/pmc_summary.py gpurun_out/TAG TAG

Reads  TAG/prof/run_results.db                    (--kernel-trace --stats pass)
       TAG/pmc_{fetch,write,sq}/p_results.db      (one --pmc pass each)
Writes profiles/TAG_kernel_stats.csv              (per-kernel launches, average / min / max ns)
       profiles/TAG_pmc.txt                       (per-kernel counter table)
       profiles/pmc_summary.json                  (bench.py reads roofline.traffic from it)

FETCH_SIZE / WRITE_SIZE are KiB per dispatch.  Per MI355X_MICROARCH.md §HBM,
FETCH_SIZE counts half the bytes of 16-B/lane streaming reads and must be
doubled; WRITE_SIZE is exact.  This engine's workspace accesses are 4-B/lane
coalesced dwords, which the guide leaves uncalibrated, so they are calibrated
here on k_fe_out, whose bytes are known exactly: per pairing it reads two
lane-strided Fq12 slots (2 x 432 B) plus one flag byte and writes one 384 B Gt
image.  The measured FETCH_SIZE / expected read bytes gives the read factor
(0.51 on gfx950, i.e. the same one-half), WRITE_SIZE / expected write bytes
checks the writes (1.00).  hbm_bytes_per_launch = FETCH / factor + WRITE.
"""
import collections
import csv
import glob
import json
import os
import sqlite3
import sys

src, tag = sys.argv[1], sys.argv[2]
out_dir = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "profiles")


def short(name):
    return name.split("(")[0].replace("bn::", "")


def one_db(pattern):
    hits = sorted(glob.glob(os.path.join(src, pattern)))
    return sqlite3.connect(hits[0]) if hits else None


# ---- kernel stats
db = one_db("prof/*results.db")
rows = []
if db is not None:
    per = collections.defaultdict(list)
    for name, dur in db.execute("select name, duration from kernels"):
        per[name].append(dur)
    with open(os.path.join(out_dir, "%s_kernel_stats.csv" % tag), "w", newline="") as fh:
        w = csv.writer(fh, quoting=csv.QUOTE_ALL)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
        tot = sum(sum(v) for v in per.values())
        for name, v in sorted(per.items(), key=lambda kv: -sum(kv[1])):
            w.writerow([name, len(v), sum(v), "%.1f" % (sum(v) / len(v)), "%.2f" % (100.0 * sum(v) / tot),
                        min(v), max(v)])
            rows.append((short(name), len(v), sum(v) / len(v)))
    for r in rows:
        print("%-28s %4d launches  avg %10.1f us" % (r[0], r[1], r[2] / 1e3))

# ---- PMC passes
agg = collections.defaultdict(lambda: collections.defaultdict(list))
prod = collections.defaultdict(lambda: collections.defaultdict(list))  # the config-5 product's kernels
for sub in ("pmc_prod_fetch", "pmc_prod_write", "pmc_prod_sq"):
    db = one_db(sub + "/*results.db")
    if db is None:
        continue
    for kname, cname, val in db.execute("select kernel_name, counter_name, value from counters_collection"):
        prod[short(kname)][cname].append(float(val))
for sub in ("pmc_fetch", "pmc_write", "pmc_sq", "pmc_sq2", "pmc_g1_fetch", "pmc_g1_write", "pmc_g1_sq", "pmc_g2_sq"):
    db = one_db(sub + "/*results.db")
    if db is None:
        continue
    # counters_collection holds one row per (dispatch, counter), already summed over instances
    for kname, cname, val in db.execute("select kernel_name, counter_name, value from counters_collection"):
        agg[short(kname)][cname].append(float(val))
# read calibration on k_fe_out (n pairings: 2 * 432 + 1 bytes read, 384 written)
cal = agg.get("k_fe_out", {})
read_factor, write_factor = None, None
factor_src = tag
prev = os.path.join(out_dir, "pmc_summary.json")
if cal.get("FETCH_SIZE") and cal.get("WRITE_SIZE"):
    n_cal = 65536  # bench.py's default batch (pairs per GPU)
    read_factor = (sum(cal["FETCH_SIZE"]) / len(cal["FETCH_SIZE"]) * 1024) / (n_cal * (2 * 432 + 1))
    write_factor = (sum(cal["WRITE_SIZE"]) / len(cal["WRITE_SIZE"]) * 1024) / (n_cal * 384)
    print("calibration on k_fe_out: FETCH_SIZE/expected reads = %.3f, WRITE_SIZE/expected writes = %.3f"
          % (read_factor, write_factor))
elif os.path.exists(prev):
    # the default build runs the whole pairing in k_pairing_full, so no k_fe_out to calibrate
    # on: keep the factor of the last session that had one (the same access pattern)
    for v in json.load(open(prev)).values():
        if v.get("read_factor"):
            read_factor, write_factor = v["read_factor"], v.get("write_factor")
            factor_src = v.get("read_factor_source", "an earlier session")
            break
    print("read factor %s from %s (no k_fe_out in this session)" % (read_factor, factor_src))
summary = {}
# SURVEY.md 8(d) generic Fq-mul counts per element of the bench's kernels, and how many
# elements one wave carries (the pairing path runs two lanes per pairing)
ALG_FQMUL = {"k_pairing_full": 19 + 2655 + 6045 + 8767, "k_pairing_fused": 19 + 2655 + 6045, "k_prepare": 19 + 2655, "k_miller": 6045, "k_fq12_vm": 8767,
             "k_g1_mul": 3800, "k_g1_mul2": 3800, "k_g2_mul": 9165, "k_g2_mul_split": 9165}
ELEMS_PER_WAVE = {"k_pairing_full": 32, "k_pairing_fused": 32, "k_prepare": 32, "k_miller": 32, "k_fq12_vm": 32, "k_fe_out": 32,
                  "k_g1_mul2": 128, "k_g2_mul_split": 32}
lines = ["%-16s %14s %14s %14s %12s %10s" % ("kernel", "FETCH_bytes", "WRITE_bytes", "VALU/wave", "WAVE_CYC/w",
                                                 "VALU/cyc")]
for k, v in sorted(agg.items()):
    if k.startswith("__amd"):
        continue
    m = {c: sum(x) / len(x) for c, x in v.items()}
    fetch = m.get("FETCH_SIZE", 0) * 1024
    write = m.get("WRITE_SIZE", 0) * 1024
    waves = m.get("SQ_WAVES", 0) or 1
    valu = m.get("SQ_INSTS_VALU", 0) / waves
    cyc = m.get("SQ_WAVE_CYCLES", 0) * 4 / waves  # quad-cycles -> cycles
    corr = (fetch / read_factor if read_factor else fetch) + write
    # VALU lane-operations per algorithmic MAD32 (SURVEY 8(d) Fq-mul count x 128):
    # wave-instructions x 64 lanes / elements per wave / algorithmic MADs per element
    alg = ALG_FQMUL.get(k)
    per_wave = ELEMS_PER_WAVE.get(k, 64)
    valu_per_mad = valu * 64 / per_wave / (alg * 128) if alg else None
    summary[k] = {"hbm_bytes_per_launch": corr, "fetch_bytes_raw": fetch, "write_bytes": write,
                  "read_factor": read_factor, "write_factor": write_factor, "read_factor_source": factor_src,
                  "valu_insts_per_wave": valu, "wave_cycles": cyc,
                  "valu_per_cycle_per_wave": valu / cyc if cyc else None,
                  "algorithmic_fqmul_per_element": alg, "elements_per_wave": per_wave,
                  "valu_lane_ops_per_algorithmic_mad": valu_per_mad,
                  "grbm_gui_active": m.get("GRBM_GUI_ACTIVE"),
                  # average wave lifetime as a fraction of the kernel (GRBM_GUI_ACTIVE sums the 8 XCDs):
                  # near 1 when the waves of a one-round launch finish together
                  "wave_life_frac": cyc / (m["GRBM_GUI_ACTIVE"] / 8) if m.get("GRBM_GUI_ACTIVE") else None,
                  # where a wave's cycles go (SQ_* in quad-cycles, per wave): issuing, waiting on
                  # s_waitcnt (memory / LDS), waiting on a dependency or a busy pipe
                  "cycles_per_wave": {c: m[c] * 4 / (m.get("SQ_WAVES") or waves)
                                      for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
                                                "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_MISC")
                                      if c in m},
                  "note": "FETCH_SIZE corrected by the read factor calibrated on k_fe_out (known bytes, session "
                          + factor_src + "), "
                          "WRITE_SIZE as counted (MI355X_MICROARCH §HBM); source %s" % tag}
    lines.append("%-16s %14.3e %14.3e %14.3e %12.3e %10.3f" % (k, fetch, write, valu, cyc, valu / cyc if cyc else 0))
if prod:
    # one product step = one launch of the last kernel (k_seg_tail since round 6, k_horner_tree2 in
    # round 5, k_horner_tree before); its traffic is every launch's bytes in the pass
    steps = (len(prod.get("k_seg_tail", {}).get("FETCH_SIZE", []))
             or len(prod.get("k_horner_tree2", {}).get("FETCH_SIZE", []))
             or len(prod.get("k_horner_tree", {}).get("FETCH_SIZE", [])) or 1)
    per_kernel = {}
    product_kernels = ("k_prepare_wide", "k_prepare", "k_miller_seg", "k_fq12_reduce_wide", "k_horner_tree",
                       "k_horner_tree2", "k_seg_fe1", "k_seg_tail", "k_horner_wide", "k_pairing_latency", "k_err_status")  # not the bench's input generation
    for k, v in prod.items():
        if k not in product_kernels:
            continue
        f = sum(v.get("FETCH_SIZE", [])) * 1024 / steps
        w = sum(v.get("WRITE_SIZE", [])) * 1024 / steps
        per_kernel[k] = {"fetch_bytes_raw": f, "write_bytes": w,
                         "hbm_bytes": (f / read_factor if read_factor else f) + w}
        if v.get("SQ_WAVES"):  # the product SQ pass: VALU instructions and cycles per wave
            waves = sum(v["SQ_WAVES"]) / len(v["SQ_WAVES"])
            per_kernel[k]["valu_insts_per_wave"] = sum(v.get("SQ_INSTS_VALU", [0])) / len(v["SQ_WAVES"]) / waves
            per_kernel[k]["wave_cycles"] = sum(v.get("SQ_WAVE_CYCLES", [0])) * 4 / len(v["SQ_WAVES"]) / waves
            per_kernel[k]["waves_per_launch"] = waves
    summary["product_step"] = {
        "hbm_bytes_per_step": sum(x["hbm_bytes"] for x in per_kernel.values()), "per_kernel": per_kernel,
        "steps_in_pass": steps, "read_factor": read_factor, "read_factor_source": factor_src,
        "note": "config 5 (bench.py --workload product): FETCH_SIZE (corrected by the read factor) + WRITE_SIZE of "
                "every kernel of one pairing_batch_dev call; source %s" % tag}
    print("product step: %.3e HBM bytes (%s)" % (summary["product_step"]["hbm_bytes_per_step"],
                                                ", ".join("%s %.2e" % (k, v["hbm_bytes"]) for k, v in per_kernel.items())))
if summary:
    if os.path.exists(prev):  # keep the entries of kernels this session did not profile
        old = json.load(open(prev))
        old.update(summary)
        summary = old
    json.dump(summary, open(os.path.join(out_dir, "pmc_summary.json"), "w"), indent=1)
    open(os.path.join(out_dir, "%s_pmc.txt" % tag), "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))
