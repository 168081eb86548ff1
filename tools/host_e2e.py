#!/usr/bin/env python3
"""End-to-end bn_pairing_many on host buffers (H2D + kernels + D2H) against the
HBM-resident bn_pairing_many_dev on the same inputs, for each n in --sizes:
median wall time of --reps calls after a warm call of the same size, and a
bit-exact comparison of the host result with the device result.  Run once with
BN254MI_HOST_PIPELINE=0 (pageable hipMemcpyAsync of the caller's buffers), 2
(pinned double-buffered pipeline at every size) and 1 (the default: the
pipeline above one piece) for the A/B in DESIGN.md §8.
Prints one JSON line per n.
"""
import argparse
import json
import os
import statistics
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "paritytech-bn_amd"))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="65536,262144")
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    import torch

    from substrate_bn import Context, synth

    dev = torch.device("cuda", 0)
    ctx = Context(0)
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
    torch.cuda.synchronize(dev)
    p = P.cpu().numpy().view(np.uint64)
    q = Q.cpu().numpy().view(np.uint64)
    out = torch.empty((nmax, 48), dtype=torch.int64, device=dev)
    pipe = int(os.environ.get("BN254MI_HOST_PIPELINE", "1"))
    for n in sizes:
        ctx.pairing_many_dev(P.data_ptr(), Q.data_ptr(), n, out.data_ptr(), sh)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(args.reps):
            ctx.pairing_many_dev(P.data_ptr(), Q.data_ptr(), n, out.data_ptr(), sh)
        torch.cuda.synchronize(dev)
        dt_dev = (time.perf_counter() - t0) / args.reps
        ref = out[:n].cpu().numpy().view(np.uint64)
        r = ctx.pairing_many(p[:n], q[:n])  # warm: workspace, staging, pinned buffers
        ok = bool(np.array_equal(r, ref))
        ts = []
        for _ in range(args.reps):
            t0 = time.perf_counter()
            r = ctx.pairing_many(p[:n], q[:n])
            ts.append(time.perf_counter() - t0)
        ok = ok and bool(np.array_equal(r, ref))
        dt = statistics.median(ts)
        print(json.dumps({"n": n, "host_pipeline": pipe, "host_ms": dt * 1e3, "host_pairings_per_s": n / dt,
                          "dev_ms": dt_dev * 1e3, "dev_pairings_per_s": n / dt_dev, "bit_exact_vs_dev": ok}),
              flush=True)
        if not ok:
            sys.exit(1)


if __name__ == "__main__":
    main()
