#!/usr/bin/env python3
"""Small-batch latency of the pairing path through the C ABI.

For n in --sizes: median wall time of
  pairing_many   (host buffers: H2D + kernels + D2H, bn_pairing_many)
  pairing_batch  (host buffers, bn_pairing_batch: Miller product + one FE)
  pairing_many_dev (HBM-resident inputs, bn_pairing_many_dev + stream sync)
and the CPU oracle's single-thread time per pairing for comparison.
Prints one JSON line per (call, n).
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


def med(fn, reps):
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return statistics.median(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="1,2,4,8,16,64,256,1024,4096")
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--calls", default="pairing_many,pairing_batch,pairing_many_dev")
    ap.add_argument("--fe-wide-max", type=int, default=None,
                    help="batches up to this size take the latency path (bn_set_fe_wide_max)")
    ap.add_argument("--latency-max", type=int, default=None,
                    help="latency-path batches up to this size run k_pairing_latency (bn_set_latency_max)")
    ap.add_argument("--warm-ms", type=float, default=100.0,
                    help="repeat each call this long before timing it (the GPU clock ramps up under load)")
    args = ap.parse_args()
    import torch

    from substrate_bn import Context, synth
    from oracle import oracle as O

    dev = torch.device("cuda", 0)
    ctx = Context(0)
    if args.fe_wide_max is not None:
        ctx.set_fe_wide_max(args.fe_wide_max)
    if args.latency_max is not None:
        ctx.set_latency_max(args.latency_max)
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
    ctx.reserve(nmax)
    # CPU single-thread reference cost per pairing
    m = 16
    t0 = time.perf_counter()
    ref = O.pairing_many(p[:m], q[:m], 1)
    cpu1 = (time.perf_counter() - t0) / m
    print(json.dumps({"cpu_oracle_ms_per_pairing_1thread": cpu1 * 1e3}), flush=True)
    assert np.array_equal(ctx.pairing_many(p[:m], q[:m]), ref)
    for call in args.calls.split(","):
        for n in sizes:
            if call == "pairing_many":
                fn = lambda: ctx.pairing_many(p[:n], q[:n])  # noqa: E731
            elif call == "pairing_batch":
                fn = lambda: ctx.pairing_batch(p[:n], q[:n])  # noqa: E731
            else:
                def fn():
                    ctx.pairing_many_dev(P.data_ptr(), Q.data_ptr(), n, out.data_ptr(), sh)
                    stream.synchronize()
            t_end = time.perf_counter() + args.warm_ms * 1e-3
            fn()
            while time.perf_counter() < t_end:
                fn()
            dt = med(fn, args.reps)
            print(json.dumps({"call": call, "n": n, "ms": dt * 1e3, "per_item_us": dt / n * 1e6,
                              "cpu_1thread_ms": cpu1 * n * 1e3, "fe_wide_max": args.fe_wide_max,
                              "latency_max": args.latency_max}), flush=True)


if __name__ == "__main__":
    main()
