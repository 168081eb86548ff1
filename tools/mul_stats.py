#!/usr/bin/env python3
"""Measured lane occupancy of G*Fr's ballot schedule.

Runs config 3's launch (2^18 G1 * Fr, random scalars) on the diagnostic build
exp/lib_mulstats.so (tools/build_variant.sh mulstats -DBN_MUL_STATS=1) and reads
the counters of curve.h BN_MUL_STAT: additions and doublings the waves ran, the
lanes each served, and the unfinished lanes per iteration.  Prints one JSON line:
per wave the iterations of each kind, their Fq-mul weight (doubling 7, addition
14 with the base's z^2, z^3 computed once), the weight a lane needs on average
(its own chain) and the lane occupancy served / (iterations x 64).

    BN254MI_LIB=exp/lib_mulstats.so python tools/mul_stats.py [--n 262144]
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "paritytech-bn_amd"))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 18)
    args = ap.parse_args()
    import torch

    from substrate_bn import Context, _native, synth
    n = args.n
    dev = torch.device("cuda", 0)
    ctx = Context(0)
    L = _native.load()
    fn = L.bn_dbg_mul_stats
    fn.argtypes, fn.restype = [ctypes.c_void_p], ctypes.c_int
    g1 = torch.from_numpy(np.tile(synth.g1_one_image().view(np.int64), (n, 1))).to(dev)
    k = synth.fr_images(n, 6)
    kd = torch.from_numpy(k.view(np.int64)).to(dev)
    out = torch.empty((n, 12), dtype=torch.int64, device=dev)
    torch.cuda.synchronize(dev)
    st = np.zeros(5, np.uint64)
    fn(st.ctypes.data)  # clear
    ctx.g1_mul_many_dev(g1.data_ptr(), kd.data_ptr(), n, out.data_ptr())
    torch.cuda.synchronize(dev)
    ctx.dev_status()
    fn(st.ctypes.data)
    adds, dbls, lane_adds, lane_dbls, live = (int(x) for x in st)
    # k_g1_mul2 (two chains per lane, capi.hip g1_mul_launch) from 2^18 rows on;
    # its addition recomputes the base's z^2, z^3 (16 Fq-mul, the bases sit in LDS)
    chains = 2 if (n + 1) // 2 >= 256 * 512 else 1
    add_w = 16 if chains == 2 else 14
    waves = ((n + chains - 1) // chains + 63) // 64
    weight_wave = (add_w * adds + 7 * dbls) / waves
    weight_lane = (14 * lane_adds + 7 * lane_dbls) / n
    print(json.dumps({
        "n": n, "waves": waves, "add_iterations_per_wave": adds / waves, "dbl_iterations_per_wave": dbls / waves,
        "adds_per_lane": lane_adds / n, "dbls_per_lane": lane_dbls / n,
        "fqmul_weight_per_wave": weight_wave, "fqmul_weight_per_lane_needed": weight_lane,
        "chains_per_lane": chains, "addition_weight": add_w,
        "schedule_overhead": weight_wave / (chains * weight_lane),
        "occupancy_of_iterations": (lane_adds + lane_dbls) / (64.0 * (adds + dbls)),
        "occupancy_of_unfinished_lanes": (lane_adds + lane_dbls) / max(live, 1),
        "what": "ballot schedule of curve.h jac_mul / jac_mul2 on config 3's launch: per wave the additions "
                "(addition_weight Fq-mul) and doublings (7) run, against the weight the wave's chains need "
                "(their additions at 14, the base's z^2, z^3 computed once)"}), flush=True)


if __name__ == "__main__":
    main()
