#!/usr/bin/env python3
"""Per-kernel statistics (calls, total/avg/min/max ns, VGPR/AGPR, scratch) from a
rocprofv3 kernel-trace database (run_results.db), as CSV on stdout -- the same
columns as rocprofv3's kernel_stats.csv plus register counts, and the steady-state
figures: SteadyAverageNs (the mean without each kernel's first, cold launch) and
MedianNs, which are what a bench line's HIP-event time is comparable with
(the rocprof mean included the cold first launch).

    python tools/rocpd_stats.py gpurun_out/TAG/prof/run_results.db > profiles/TAG_kernel_stats.csv
"""
import csv
import sqlite3
import statistics
import sys


def main(path):
    con = sqlite3.connect(path)
    q = """select s.kernel_name, s.arch_vgpr_count, s.accum_vgpr_count, s.private_segment_size,
                  d.end - d.start, d.grid_size_x, d.workgroup_size_x
           from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id = s.id
           order by d.start"""
    agg = {}
    for name, vg, ag, scratch, dur, grid, wg in con.execute(q):
        a = agg.setdefault(name, {"calls": 0, "total": 0, "min": None, "max": 0, "vgpr": vg, "agpr": ag,
                                  "scratch": scratch, "grid": set(), "durs": []})
        a["durs"].append(dur)
        a["calls"] += 1
        a["total"] += dur
        a["min"] = dur if a["min"] is None else min(a["min"], dur)
        a["max"] = max(a["max"], dur)
        a["grid"].add(grid)
    tot = sum(a["total"] for a in agg.values()) or 1
    w = csv.writer(sys.stdout)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "arch_vgpr",
                "accum_vgpr", "scratch_bytes", "grid_sizes", "SteadyAverageNs", "MedianNs"])
    for name, a in sorted(agg.items(), key=lambda kv: -kv[1]["total"]):
        w.writerow([name, a["calls"], a["total"], round(a["total"] / a["calls"], 1), round(100.0 * a["total"] / tot, 2),
                    a["min"], a["max"], a["vgpr"], a["agpr"], a["scratch"], " ".join(str(g) for g in sorted(a["grid"])),
                    round(statistics.mean(a["durs"][1:] if len(a["durs"]) > 1 else a["durs"]), 1),
                    statistics.median(a["durs"])])


if __name__ == "__main__":
    main(sys.argv[1])
