#!/usr/bin/env python3
"""bench.py -- BN254 pairings/sec on MI355X (BASELINE.json metric, config 2 at N=1).

One step = one pass of the hot path over one batch: `pairs` independent
optimal-ate pairings e(P_i, Q_i) per GPU (default 2^16 = BASELINE config 2),
inputs resident in HBM, through the engine's C ABI (bn_pairing_many_dev:
to_affine + G2 line precomputation, Miller loop, final exponentiation).  With
N > 1 GPUs each rank runs its own 2^16 pairs (weak scaling, no data-path
collective) and the step ends with one RCCL all-gather of every rank's Gt
results over xGMI (BASELINE config 4's exchange), so every rank holds all
N x 2^16 results.

Synthetic inputs: P_i = s_i * G1::one(), Q_i = t_i * G2::one() with s_i, t_i
uniform in [1, r) from a seeded SplitMix64 (seed 1 + rank), computed by the
engine's own scalar-multiplication kernels and kept in Jacobian form (z != 1),
exactly the reference's `G * Fr` output images.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--pairs n]
    torchrun --nproc-per-node N bench.py --gpus N ...
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "paritytech-bn_amd"))
sys.path.insert(0, ROOT)

# Algorithmic work per pairing in generic Fq Montgomery products (SURVEY.md §8(d),
# Appendix B: reference formulas with x(-1) and x xi folded into adds, inversions
# excluded), per kernel phase of bn_pairing_many_dev.
# k_fq12_vm: the reference's 8767 less what the width-4 signed-window chains for u
# save per exp_by_neg_z (16 Fq12 products instead of 27, one extra cyclotomic
# square of 18): the work counted is the work the kernel does.
FQMUL_PER_PAIRING = {"k_prepare": 19 + 2655, "k_miller": 6045, "k_fq12_vm": 8767 - 3 * (11 * 54 - 18), "k_fe_out": 0}
MAD32_PER_FQMUL = 128  # one 8x32-bit CIOS product: 64 (a*b) + 64 (m*p) v_mad_u64_u32
# gfx950 integer-VALU peak for v_mad_u64_u32: 4 cycles per wave64 instruction (measured,
# tools/ubench.hip) = 256 CU x 4 SIMD x 16 lanes/clk x 2.4 GHz.  ubench sustains 34.7 T/s.
PEAK_MAD32_PER_S = 256 * 4 * 16 * 2.4e9
PHASES = ["k_prepare", "k_miller", "k_fq12_vm", "k_fe_out"]


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def fr_images(n, seed, lo=1):
    from substrate_bn import synth  # product-side input sampling; oracle/ is only the checker
    return synth.fr_images(n, seed, lo)


def device_points(ctx, n, seed_g1, seed_g2, dev, sh):
    """P_i = s_i * G1::one(), Q_i = t_i * G2::one() on the engine's own scalar-mul kernels."""
    import torch
    from substrate_bn import synth
    P = torch.empty((n, 12), dtype=torch.int64, device=dev)
    Q = torch.empty((n, 24), dtype=torch.int64, device=dev)
    if seed_g1 is not None:
        g1 = torch.from_numpy(np.tile(synth.g1_one_image().view(np.int64), (n, 1))).to(dev)
        s_img = torch.from_numpy(fr_images(n, seed_g1).view(np.int64)).to(dev)
        ctx.g1_mul_many_dev(g1.data_ptr(), s_img.data_ptr(), n, P.data_ptr(), sh)
    if seed_g2 is not None:
        g2 = torch.from_numpy(np.tile(synth.g2_one_image().view(np.int64), (n, 1))).to(dev)
        t_img = torch.from_numpy(fr_images(n, seed_g2).view(np.int64)).to(dev)
        ctx.g2_mul_many_dev(g2.data_ptr(), t_img.data_ptr(), n, Q.data_ptr(), sh)
    torch.cuda.synchronize(dev)
    return P, Q


def cpu_baseline(p_host, q_host, gpu_out, threads):
    """Oracle (C restatement of the reference CPU path) on a bounded sample."""
    from oracle import oracle as O
    n = p_host.shape[0]
    O.pairing_many(p_host[:16], q_host[:16], threads)  # warm
    t0 = time.perf_counter()
    ref = O.pairing_many(p_host, q_host, threads)
    dt = time.perf_counter() - t0
    return {"value": n / dt, "unit": "pairings/s", "cores": threads, "kind": "port",
            "sample": "%d pairings of the bench's own inputs, oracle/bn_oracle.c (C restatement of substrate-bn "
                      "0.6.0: u128-digit Montgomery, binary-EEA inverse, same formulas), %d threads, %.2f s wall"
                      % (n, threads, dt),
            "parity_sample_bit_exact": bool(np.array_equal(ref, gpu_out))}


def pmc_traffic(kernel):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC summary, if any."""
    path = os.path.join(ROOT, "profiles", "pmc_summary.json")
    try:
        with open(path) as fh:
            d = json.load(fh)
        return d.get(kernel, {}).get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        return None


def other_workload(args, local_rank):
    """BASELINE config 3 (batched G1 * Fr) and config 5 (pairing product), 1 GPU."""
    import torch

    from substrate_bn import Context

    dev = torch.device("cuda", local_rank)
    ctx = Context(local_rank)
    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream
    res = {"n_gpus": 1, "steps": args.steps, "warmup": args.warmup, "higher_is_better": True, "scaling": "weak",
           "vs_baseline": None, "dtype": "u32 (9x29-bit Montgomery digits, integer only)", "data": "synthetic"}
    if args.workload == "g1mul":
        n = args.pairs if args.pairs != (1 << 16) else (1 << 18)
        P, _ = device_points(ctx, n, 5, None, dev, sh)  # random Jacobian bases
        k2 = torch.from_numpy(fr_images(n, 6).view(np.int64)).to(dev)
        out = torch.empty_like(P)
        step = lambda: ctx.g1_mul_many_dev(P.data_ptr(), k2.data_ptr(), n, out.data_ptr(), sh)  # noqa: E731
        unit = "G1 scalar muls/s"
        res["config"] = {"workload": "BASELINE config 3: batched Fr x G1 (reference double-and-add chain, "
                                     "bit-exact Jacobian output)", "muls": n}
    else:
        n = args.pairs if args.pairs != (1 << 16) else (1 << 14)
        Pd, Qd = device_points(ctx, n, 21, 22, dev, sh)
        p, q = Pd.cpu().numpy().view(np.uint64), Qd.cpu().numpy().view(np.uint64)
        step = lambda: ctx.pairing_batch(p, q)  # noqa: E731
        unit = "pairing-product terms/s"
        res["config"] = {"workload": "BASELINE config 5: one pairing_batch over 2^14 terms (per-term Miller "
                                     "values, product tree, one final exponentiation; host buffers incl. PCIe)",
                         "terms": n}
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    res.update({"metric": unit, "value": n * args.steps / el, "unit": unit, "ms_per_step": el / args.steps * 1e3})
    from oracle import oracle as O  # the checker (cpu_baseline leg)
    if args.workload == "g1mul":
        m = min(args.cpu_sample or 2048, n)
        threads = min(16, os.cpu_count() or 1)
        ph, kh, oh = (t[:m].cpu().numpy().view(np.uint64) for t in (P, k2, out))
        t0 = time.perf_counter()
        ref = O.g1_mul(ph, kh, threads)
        dt = time.perf_counter() - t0
        res["cpu_baseline"] = {"value": m / dt, "unit": unit, "cores": threads, "kind": "port",
                               "sample": "%d G1*Fr of the bench inputs, oracle, %d threads" % (m, threads),
                               "parity_sample_bit_exact": bool(np.array_equal(ref, oh))}
    else:
        res["parity_bit_exact"] = bool(np.array_equal(ctx.pairing_batch(p, q), O.pairing_batch(p[:n], q[:n])))
    print(json.dumps(res), flush=True)


def codec_workload(args, local_rank):
    """SURVEY 8(f) rows on 2^16 elements, inputs resident in HBM, device-pointer C ABI on torch's stream."""
    import torch

    from substrate_bn import Context, synth

    dev = torch.device("cuda", local_rank)
    ctx = Context(local_rank)
    stream = torch.cuda.Stream(dev)  # a real stream: handle 0 would mean the context's own stream
    sh = stream.cuda_stream
    n = args.pairs
    threads = min(16, os.cpu_count() or 1)
    t0 = time.perf_counter()
    if args.workload in ("g2validate", "g2decompress"):
        _, Qd = device_points(ctx, n, None, 61, dev, sh)  # n distinct points of the order-r subgroup
        aff = synth.g2_jacobian_to_affine(Qd.cpu().numpy().view(np.uint64))
        del Qd
        out = torch.empty((n, 24), dtype=torch.int64, device=dev)
        st = torch.empty(n, dtype=torch.uint8, device=dev)
        if args.workload == "g2validate":
            x = torch.from_numpy(np.ascontiguousarray(aff[:, :8]).view(np.int64)).to(dev)
            y = torch.from_numpy(np.ascontiguousarray(aff[:, 8:]).view(np.int64)).to(dev)
            step = lambda: ctx.g2_affine_new_many_dev(x.data_ptr(), y.data_ptr(), n, out.data_ptr(),  # noqa: E731
                                                      st.data_ptr(), sh)
            unit, kname = "G2 validations/s", "k_g2_affine_new"
            wl = "AffineG2::new on 2^16 affine points (curve equation + order check [r]P == 0), mod.rs:95-113"
            ref_fn = lambda m: O.g2_affine_new(aff[:m, :8], aff[:m, 8:], threads)  # noqa: E731
        else:
            rec = synth.compress_g2(aff)
            b = torch.from_numpy(rec).to(dev)
            step = lambda: ctx.g2_from_compressed_many_dev(b.data_ptr(), n, out.data_ptr(), st.data_ptr(), sh)  # noqa
            unit, kname = "G2 decompressions/s", "k_g2_from_compressed"
            wl = "G2::from_compressed on 2^16 65-byte records (Fq2 sqrt + order check), lib.rs:506-526"
            ref_fn = lambda m: O.g2_from_compressed(rec[:m], threads)  # noqa: E731
    else:
        Pd, Qd = device_points(ctx, 1024, 71, 73, dev, sh)
        gd = torch.empty((1024, 48), dtype=torch.int64, device=dev)
        ctx.pairing_many_dev(Pd.data_ptr(), Qd.data_ptr(), 1024, gd.data_ptr(), sh)
        torch.cuda.synchronize(dev)
        g = gd.cpu().numpy().view(np.uint64)
        a = torch.from_numpy(np.ascontiguousarray(np.tile(g, (n // 1024, 1))).view(np.int64)).to(dev)
        k = fr_images(n, 72, lo=0)
        kt = torch.from_numpy(np.ascontiguousarray(k).view(np.int64)).to(dev)
        out = torch.empty((n, 48), dtype=torch.int64, device=dev)
        st = None
        step = lambda: ctx.gt_pow_many_dev(a.data_ptr(), kt.data_ptr(), n, out.data_ptr(), sh)  # noqa: E731
        unit, kname = "Gt pows/s", "k_gt_pow"
        wl = "Gt::pow(Fr) on 2^16 (Gt, uniform Fr) pairs (1024 distinct pairing outputs tiled), lib.rs:592-594"
        a_h = np.ascontiguousarray(np.tile(g, (n // 1024, 1)))
        ref_fn = lambda m: (O.gt_pow(a_h[:m], k[:m]), None)  # noqa: E731
    log("inputs ready in %.1f s" % (time.perf_counter() - t0))
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(stream)
    for _ in range(args.steps):
        step()
    e1.record(stream)
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    kms = e0.elapsed_time(e1) / args.steps
    res = {"metric": unit, "value": n * args.steps / el, "unit": unit, "n_gpus": 1, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": el / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
           "vs_baseline": None, "dtype": "u32 (9x29-bit Montgomery digits, integer only)", "data": "synthetic",
           "config": {"workload": wl, "elements": n},
           "kernel": {"name": kname, "per_launch_ms": kms}}
    from oracle import oracle as O  # the checker (cpu_baseline leg)
    m = min(args.cpu_sample or 2048, n)
    g_out = out[:m].cpu().numpy().view(np.uint64)
    t0 = time.perf_counter()
    ref, rst = ref_fn(m)
    dt = time.perf_counter() - t0
    same = np.array_equal(ref, g_out) and (rst is None or np.array_equal(rst, st[:m].cpu().numpy()))
    res["cpu_baseline"] = {"value": m / dt, "unit": unit, "cores": threads, "kind": "port",
                           "sample": "%d elements of the bench inputs, oracle, %d threads" % (m, threads),
                           "parity_sample_bit_exact": bool(same)}
    print(json.dumps(res), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--pairs", type=int, default=1 << 16, help="pairings per GPU per step")
    ap.add_argument("--cpu-sample", type=int, default=None,
                    help="oracle sample size (default: 16384 pairings, 2048 for the 8(f) workloads; ~10-30 s of CPU-thread work)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--workload", default="pairing",
                    choices=["pairing", "g1mul", "product", "g2validate", "g2decompress", "gtpow"],
                    help="pairing: config 2 (default); g1mul: config 3 (2^18 G1*Fr); product: config 5 "
                         "(2^14-term pairing_batch); SURVEY 8(f): g2validate (AffineG2::new incl. the order "
                         "check), g2decompress (G2::from_compressed), gtpow (Gt::pow(Fr)), 2^16 each")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    else:
        torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)

    from substrate_bn import Context

    if args.workload in ("g2validate", "g2decompress", "gtpow"):
        return codec_workload(args, local_rank)
    if args.workload != "pairing":
        return other_workload(args, local_rank)

    n = args.pairs
    ctx = Context(local_rank)
    ctx.reserve(n)
    # One real (non-default) stream for the engine's kernels, torch's copies and the
    # RCCL all-gather, so the collective is ordered after the pairings it gathers
    # (handle 0 would send the kernels to the context's own non-blocking stream).
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    sh = stream.cuda_stream

    # ---- synthetic inputs in HBM (engine kernels; Jacobian images)
    P, Q = device_points(ctx, n, 1 + rank, 1001 + rank, dev, sh)
    out = torch.empty((n, 48), dtype=torch.int64, device=dev)
    gathered = torch.empty((world * n, 48), dtype=torch.int64, device=dev) if world > 1 else None
    torch.cuda.synchronize(dev)

    def step():
        ctx.pairing_many_dev(P.data_ptr(), Q.data_ptr(), n, out.data_ptr(), sh)
        if world > 1:
            dist.all_gather_into_tensor(gathered, out)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    ctx.phase_times()  # discard

    ctx.set_phase_timing(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    ctx.set_phase_timing(False)
    phase_ms, launches = ctx.phase_times()

    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    total = n * world * args.steps
    value = total / elapsed
    # dominant kernel: largest share of device time
    per_launch_ms = {PHASES[k]: phase_ms[k] / max(launches, 1) for k in range(4)}
    dom = max(per_launch_ms, key=per_launch_ms.get)
    mad_per_launch = FQMUL_PER_PAIRING[dom] * MAD32_PER_FQMUL * n
    achieved = mad_per_launch / (per_launch_ms[dom] * 1e-3)
    roofline = {"bound": "valu", "achieved": achieved / 1e12, "peak": PEAK_MAD32_PER_S / 1e12,
                "unit": "TMAD32/s (v_mad_u64_u32, algorithmic)", "frac": achieved / PEAK_MAD32_PER_S,
                "traffic": pmc_traffic(dom), "kernel": dom,
                "per_launch_ms": {k: round(v, 4) for k, v in per_launch_ms.items()},
                "whole_pairing_frac": value / world * sum(FQMUL_PER_PAIRING.values()) * MAD32_PER_FQMUL
                / PEAK_MAD32_PER_S}

    res = {
        "metric": "BN254 pairings/sec (batched) at 1/2/4/8 MI355X; bit-exact vs CPU ref",
        "value": value, "unit": "pairings/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "u32 (9x29-bit Montgomery digits, integer only)",
        "data": "synthetic: P_i = s_i*G1::one(), Q_i = t_i*G2::one(), s,t uniform in [1,r), SplitMix64 seed 1+rank",
        "config": {"workload": "BASELINE config 2: 2^16 independent pairings e(P_i,Q_i) per GPU"
                               + (" + RCCL all-gather of Gt (config 4 exchange)" if world > 1 else ""),
                   "pairs_per_gpu": n, "parallelism": "dp%d" % world, "inputs": "HBM-resident Jacobian images",
                   "hbm_io_bytes_per_pairing": 96 + 192 + 384},
        "roofline": roofline,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        m = min(args.cpu_sample or 16384, n)
        threads = min(16, os.cpu_count() or 1)
        p_h = P[:m].cpu().numpy().view(np.uint64)
        q_h = Q[:m].cpu().numpy().view(np.uint64)
        o_h = out[:m].cpu().numpy().view(np.uint64)
        res["cpu_baseline"] = cpu_baseline(p_h, q_h, o_h, threads)
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
