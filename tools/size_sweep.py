#!/usr/bin/env python3
"""Per-kernel device time of the throughput path (k_pairing_fused, k_fq12_vm,
k_fe_out; HIP events on the launch stream via bn_set_phase_timing) per 2^16
pairings, for launches of --sizes pairs (HBM-resident inputs): how much of a
2^16-pair launch (config 2: one wave per SIMD slot) is fixed per-launch cost.
Prints one JSON line per size.
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "paritytech-bn_amd"))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="16384,32768,65536,98304,131072,196608,262144")
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    import torch

    from substrate_bn import Context, synth

    dev = torch.device("cuda", 0)
    ctx = Context(0)
    ctx.set_fe_wide_max(0)  # every size on the throughput path
    sizes = [int(s) for s in args.sizes.split(",")]
    nmax = max(sizes)
    s, t = synth.dataset_scalars(0, nmax)
    g1 = torch.from_numpy(np.tile(synth.g1_one_image().view(np.int64), (nmax, 1))).to(dev)
    g2 = torch.from_numpy(np.tile(synth.g2_one_image().view(np.int64), (nmax, 1))).to(dev)
    P = torch.empty((nmax, 12), dtype=torch.int64, device=dev)
    Q = torch.empty((nmax, 24), dtype=torch.int64, device=dev)
    sd = torch.from_numpy(s.view(np.int64)).to(dev)
    td = torch.from_numpy(t.view(np.int64)).to(dev)
    stream = torch.cuda.Stream(dev)
    sh = stream.cuda_stream
    ctx.g1_mul_many_dev(g1.data_ptr(), sd.data_ptr(), nmax, P.data_ptr(), sh)
    ctx.g2_mul_many_dev(g2.data_ptr(), td.data_ptr(), nmax, Q.data_ptr(), sh)
    out = torch.empty((nmax, 48), dtype=torch.int64, device=dev)
    ctx.reserve(nmax)
    torch.cuda.synchronize(dev)
    for n in sizes:
        ctx.pairing_many_dev(P.data_ptr(), Q.data_ptr(), n, out.data_ptr(), sh)
        torch.cuda.synchronize(dev)
        ctx.set_phase_timing(True)
        ctx.phase_times()
        for _ in range(args.reps):
            ctx.pairing_many_dev(P.data_ptr(), Q.data_ptr(), n, out.data_ptr(), sh)
        ms, launches = ctx.phase_times()
        ctx.set_phase_timing(False)
        per = [m / launches for m in ms]
        scale = 65536.0 / n
        print(json.dumps({"n": n, "launch_sets": launches, "ms_per_launch": {"miller": per[1] + per[0], "fe": per[2],
                                                                             "fe_out": per[3]},
                          "ms_per_65536": {"miller": (per[0] + per[1]) * scale, "fe": per[2] * scale,
                                           "total": sum(per) * scale}}), flush=True)


if __name__ == "__main__":
    main()
