#!/usr/bin/env python3
"""bench.py -- BN254 pairings/sec on MI355X (BASELINE.json metric).

One step = one pass of the hot path over one batch of synthetic pairs,
inputs resident in HBM, through the engine's C ABI (bn_pairing_many_dev:
to_affine + G2 line precomputation, Miller loop, final exponentiation).

  N = 1  (default): BASELINE config 2 -- 2^16 independent pairings on one GPU.
  N > 1  (default): BASELINE config 4 -- 2^20 pairings sharded contiguously
         over the N ranks (2^20/N each, strong scaling); every step ends with
         an RCCL all-gather of all 2^20 Gt results over xGMI, issued per 2^16
         chunk on RCCL's stream so it overlaps the next chunk's kernels.
         `--config 2` keeps 2^16 pairs per rank instead (weak scaling).

`python bench.py --gpus N` with N > 1 and no WORLD_SIZE in the environment
starts `torch.distributed.run` with N ranks as a child process (before this
process touches a GPU) and exits with its status; under a launcher the world
size must equal --gpus.

Synthetic inputs: row j of a global dataset is P_j = s_j * G1::one(),
Q_j = t_j * G2::one(); s_j, t_j are Montgomery Fr images uniform in [1, r)
from SplitMix64 seeds fixed per 4096-row block (substrate_bn/synth.py), so
every rank builds exactly its rows and any rank can rebuild any other rank's.
The points come from the engine's own scalar-multiplication kernels, kept in
Jacobian form (z != 1) -- exactly the reference's `G * Fr` output images.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 2|4]
    python bench.py --workload g1mul|g2mul|product|g2validate|g2decompress|gtpow
    python bench.py --gpus 2 --dry-run-cpu   # control flow on CPU (gloo, stub engine)
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "paritytech-bn_amd"))
sys.path.insert(0, ROOT)

# Algorithmic work per pairing in generic Fq Montgomery products, per kernel
# phase of bn_pairing_many_dev: SURVEY.md §8(d) / Appendix B (the reference's
# formulas with x(-1) and x xi folded into adds, inversions excluded):
# to_affine 19 + precompute 2,655, Miller loop 6,045, final exponentiation 8,767.
# (The engine's FE runs windowed exp_by_neg_z chains that do less work than the
# reference's binary chains; the roofline credits only the reference count.)
FQMUL_PER_PAIRING = {"k_prepare": 19 + 2655, "k_miller": 6045, "k_fq12_vm": 8767, "k_fe_out": 0}
FQMUL_BASIS = "SURVEY.md 8(d): reference Fq-mul counts (FE 8767, Miller 6045, prepare 2674), x128 MAD32 each"
MAD32_PER_FQMUL = 128  # one 8x32-bit CIOS product: 64 (a*b) + 64 (m*p) v_mad_u64_u32
# gfx950 integer-VALU peak for v_mad_u64_u32: 4 cycles per wave64 instruction (measured,
# tools/ubench.hip) = 256 CU x 4 SIMD x 16 lanes/clk x 2.4 GHz.  ubench sustains 34.7 T/s.
PEAK_MAD32_PER_S = 256 * 4 * 16 * 2.4e9
# the same rate as measured: v_mad_u64_u32 issues at 4.77 cycles per wave-instruction with two
# waves per SIMD (the throughput kernels' occupancy), tools/ubench_mad_issue.hip
PEAK_MAD32_MEASURED = 256 * 4 * 64 * 2.4e9 / 4.77
PEAK_MEASURED_SOURCE = ("profiles/r3j_mad_issue.txt: 4.77 cycles per v_mad_u64_u32 wave-instruction at two waves "
                        "per SIMD (33.0 T/s); `frac` stays against the 4-cycle 39.3 T/s figure")
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


ORACLE_BUILD = "oracle/Makefile: gcc -O3 -march=x86-64-v3 (not -march=native: on a Zen 5 host this understates the CPU)"


def emit(res):
    """Print the one JSON line; a cpu_baseline names the oracle's build flags."""
    cb = res.get("cpu_baseline")
    if isinstance(cb, dict) and cb.get("kind") == "port":
        cb["build"] = ORACLE_BUILD
        cb["sample"] = cb.get("sample", "") + "; built " + ORACLE_BUILD.split(": ", 1)[1]
    print(json.dumps(res), flush=True)


def host_cpus():
    """The CPUs this process may use (affinity set, capped by a cgroup CPU quota)
    and the host CPU model.  On the GPU box os.cpu_count() shows the whole
    machine while the job's share is a quota, so the quota sets the thread count."""
    info = {"model": None, "visible": os.cpu_count()}
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    info["model"] = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = os.cpu_count() or 1
    info["affinity"] = aff
    quota = None
    for path in ("/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/cpu/cpu.cfs_quota_us"):
        try:
            with open(path) as fh:
                f = fh.read().split()
        except OSError:
            continue
        if path.endswith("cpu.max") and f and f[0] != "max":
            quota = int(f[0]) / int(f[1])
        elif path.endswith("quota_us") and f and int(f[0]) > 0:
            with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as fh:
                quota = int(f[0]) / int(fh.read())
        break
    info["cgroup_cpu_quota"] = quota
    usable = aff if quota is None else max(1, min(aff, int(quota)))
    # the pool's stated share for one GPU is 16 CPUs (OMP_NUM_THREADS etc. are set to it)
    env_cap = os.environ.get("OMP_NUM_THREADS")
    if env_cap and env_cap.isdigit() and quota is None and aff > int(env_cap):
        usable = int(env_cap)
        info["capped_by"] = "OMP_NUM_THREADS (the box's per-GPU CPU share)"
    info["usable"] = usable
    return info


def cpu_baseline(p_host, q_host, gpu_out, cpus, single_sample=1024):
    """Oracle (C restatement of the reference CPU path) on a bounded sample:
    all usable cores (one pairing per thread) and one core."""
    from oracle import oracle as O
    n = p_host.shape[0]
    threads = cpus["usable"]
    O.pairing_many(p_host[:16], q_host[:16], threads)  # warm
    t0 = time.perf_counter()
    ref = O.pairing_many(p_host, q_host, threads)
    dt = time.perf_counter() - t0
    m1 = min(single_sample, n)
    t0 = time.perf_counter()
    ref1 = O.pairing_many(p_host[:m1], q_host[:m1], 1)
    dt1 = time.perf_counter() - t0
    return {"value": n / dt, "unit": "pairings/s", "cores": threads, "kind": "port",
            "single_core": {"value": m1 / dt1, "unit": "pairings/s", "sample": "%d pairings, 1 thread" % m1},
            "cpu_model": cpus["model"], "cpus_visible": cpus["visible"], "cpus_usable": threads,
            "sample": "%d pairings of the bench's own inputs, oracle/bn_oracle.c (C restatement of substrate-bn "
                      "0.6.0: u128-digit Montgomery, binary-EEA inverse, same formulas), %d threads (one pairing "
                      "per thread), %.2f s wall" % (n, threads, dt),
            "parity_sample_bit_exact": bool(np.array_equal(ref, gpu_out) and np.array_equal(ref1, gpu_out[:m1]))}


def sample_blocks(total, rows=4096, block=128):
    """Global row ranges of a `rows`-row checker sample: `rows // block` blocks of
    `block` consecutive rows spread evenly over [0, total), so every rank's shard
    holds some (first and last rows included)."""
    nb = max(1, min(rows // block, total // block))
    block = min(block, total)
    starts = sorted({(k * (total - block)) // max(nb - 1, 1) for k in range(nb)})
    return [(a, min(a + block, total)) for a in starts]


def gathered_sample_check(eng, rows_all, total, cpus, single=256):
    """Rank 0's checker leg for config 4: rebuild the inputs of ~4096 rows spread
    over every rank's shard, recompute them on the CPU (the oracle) and compare
    with the rows this rank holds after the all-gather; the same oracle run,
    timed, is the cpu_baseline (all usable cores, plus one core on `single` rows)."""
    blocks = sample_blocks(total)
    ps, qs, got = [], [], []
    for a, b in blocks:
        P, Q = eng.points(a, b - a)
        ps.append(eng.host(P))
        qs.append(eng.host(Q))
        got.append(eng.host(rows_all[a:b]))
    p_h, q_h, g_h = np.concatenate(ps), np.concatenate(qs), np.concatenate(got)
    threads = cpus["usable"]
    eng.reference(p_h[:16], q_h[:16], threads)  # warm
    t0 = time.perf_counter()
    ref = eng.reference(p_h, q_h, threads)
    dt = time.perf_counter() - t0
    m1 = min(single, p_h.shape[0])
    t0 = time.perf_counter()
    ref1 = eng.reference(p_h[:m1], q_h[:m1], 1)
    dt1 = time.perf_counter() - t0
    mism = int((ref != g_h).any(axis=1).sum())
    check = {"rows": int(p_h.shape[0]), "blocks": len(blocks), "block_rows": blocks[0][1] - blocks[0][0],
             "first_row": blocks[0][0], "last_row": blocks[-1][1] - 1, "mismatches": mism,
             "parity_sample_bit_exact": bool(mism == 0 and np.array_equal(ref1, g_h[:m1])),
             "what": "rank 0 rebuilds the inputs of the sampled global rows, recomputes them with the CPU oracle and "
                     "compares with the Gt rows it holds after the all-gather (every rank's shard is sampled)"}
    base = {"value": p_h.shape[0] / dt, "unit": "pairings/s", "cores": threads,
            "kind": "dry-run stub" if eng.dry else "port",
            "single_core": {"value": m1 / dt1, "unit": "pairings/s", "sample": "%d pairings, 1 thread" % m1},
            "cpu_model": cpus["model"], "cpus_visible": cpus["visible"], "cpus_usable": threads,
            "sample": "the %d-row checker sample of the gathered output, %s, %d threads (one pairing per thread), "
                      "%.2f s wall" % (p_h.shape[0], "the dry run's stub row mix on the host" if eng.dry else
                                       "oracle/bn_oracle.c (C restatement of substrate-bn 0.6.0)", threads, dt),
            "parity_sample_bit_exact": check["parity_sample_bit_exact"]}
    return check, base


def pmc_traffic(kernel, key="hbm_bytes_per_launch"):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC summary, if any."""
    path = os.path.join(ROOT, "profiles", "pmc_summary.json")
    try:
        with open(path) as fh:
            d = json.load(fh)
        return d.get(kernel, {}).get(key)
    except (OSError, ValueError):
        return None


G1_MUL2_MIN_LANES = 256 * 512  # capi.hip g1_mul_launch: k_g1_mul2 from this many lanes (kG1MulPairBlockMin)


def product_affine_inputs(ctx, Pd, Qd, n, stream, dev, args, ref):
    """Config 5's product over the same points with z = one (as pairing inputs arrive
    when they come in affine, through AffineG1::new / AffineG2::new): the engine's own
    bn_g1/g2_normalize_many_dev makes the images, then the same timed loop.  to_affine
    takes the reference's z == one branch (mod.rs:199-216) and whole waves of such
    pairs skip the inversion.  Reported beside the Jacobian-input line, never as it."""
    import torch
    sh = stream.cuda_stream
    Pa, Qa = torch.empty_like(Pd), torch.empty_like(Qd)
    ctx.group_op_many_dev("g1", "normalize", Pd.data_ptr(), None, n, Pa.data_ptr(), sh)
    ctx.group_op_many_dev("g2", "normalize", Qd.data_ptr(), None, n, Qa.data_ptr(), sh)
    out = torch.zeros(48, dtype=torch.int64, device=dev)
    st = torch.full((1,), -1, dtype=torch.int32, device=dev)
    step = lambda: ctx.pairing_batch_dev(Pa.data_ptr(), Qa.data_ptr(), n, out.data_ptr(), st.data_ptr(), sh)  # noqa
    for _ in range(max(1, args.warmup)):
        step()
    torch.cuda.synchronize(dev)
    steps = max(2, args.steps)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(steps):
        step()
    e1.record(stream)
    torch.cuda.synchronize(dev)
    ms = e0.elapsed_time(e1) / steps
    return {"ms_per_product": ms, "terms_per_s": n / (ms * 1e-3),
            "parity_bit_exact": bool(np.array_equal(ref, out.cpu().numpy().view(np.uint64)) and int(st.item()) == 0),
            "what": "the same 2^14 points normalized to z = one (bn_g1/g2_normalize_many_dev) before the timed loop"}


def products_in_flight(ctx, Pd, Qd, n, stream, dev, args, ref):
    """Config 5 as a stream of independent pairing-product checks, two at a time:
    product k runs on context k % 2 (own workspace, own stream), so one product's
    latency-bound tail (k_seg_tail: 16 CUs, then 3) overlaps the next
    product's issue-bound front on the other CUs.  Reported beside the one-product
    latency (`ms_per_step`, the line's value), never as it.  Both contexts' last
    products are checked against the oracle's value of the same inputs."""
    import torch

    from substrate_bn import Context
    ctx2 = Context(dev.index)
    s2 = torch.cuda.Stream(dev)
    ctxs, streams = (ctx, ctx2), (stream, s2)
    outs = [torch.zeros(48, dtype=torch.int64, device=dev) for _ in range(2)]
    sts = [torch.full((1,), -1, dtype=torch.int32, device=dev) for _ in range(2)]

    def run(k):
        j = k % 2
        ctxs[j].pairing_batch_dev(Pd.data_ptr(), Qd.data_ptr(), n, outs[j].data_ptr(), sts[j].data_ptr(),
                                  streams[j].cuda_stream)
    for k in range(max(2, args.warmup)):
        run(k)
    torch.cuda.synchronize(dev)
    steps = max(2, args.steps)
    t0 = time.perf_counter()
    for k in range(steps):
        run(k)
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    exact = all(np.array_equal(ref, o.cpu().numpy().view(np.uint64)) and int(s.item()) == 0
                for o, s in zip(outs, sts))
    return {"ms_per_product": el / steps * 1e3, "terms_per_s": n * steps / el, "products": steps,
            "parity_bit_exact": bool(exact),
            "what": "independent products alternating over two contexts and streams (a product-check service): "
                    "throughput, not the latency of one product"}


def other_workload(args, local_rank):
    """BASELINE config 3 (batched G1 * Fr) and config 5 (pairing product), 1 GPU."""
    import torch

    from substrate_bn import Context

    dev = torch.device("cuda", local_rank)
    ctx = Context(local_rank)
    stream = torch.cuda.Stream(dev)  # a real stream: handle 0 would mean the context's own stream
    torch.cuda.set_stream(stream)
    sh = stream.cuda_stream
    res = {"n_gpus": 1, "steps": args.steps, "warmup": args.warmup, "higher_is_better": True, "scaling": "weak",
           "vs_baseline": None, "dtype": "u32 (9x29-bit Montgomery digits, integer only)", "data": "synthetic"}
    if args.workload == "g2mul":
        n = args.pairs
        _, Qb = device_points(ctx, n, None, 7, dev, sh)  # random Jacobian G2 bases
        k2 = torch.from_numpy(fr_images(n, 8).view(np.int64)).to(dev)
        P = Qb
        out = torch.empty_like(Qb)
        step = lambda: ctx.g2_mul_many_dev(Qb.data_ptr(), k2.data_ptr(), n, out.data_ptr(), sh)  # noqa: E731
        unit = "G2 scalar muls/s"
        res["config"] = {"workload": "SURVEY 8(f1): batched Fr x G2 (reference double-and-add chain, bit-exact "
                                     "Jacobian output)", "muls": n}
    elif args.workload == "g1mul":
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
        gout = torch.zeros(48, dtype=torch.int64, device=dev)
        gst = torch.full((1,), -1, dtype=torch.int32, device=dev)
        step = lambda: ctx.pairing_batch_dev(Pd.data_ptr(), Qd.data_ptr(), n, gout.data_ptr(),  # noqa: E731
                                             gst.data_ptr(), sh)
        unit = "pairing-product terms/s"
        res["config"] = {"workload": "BASELINE config 5: one pairing_batch over 2^14 terms, HBM-resident inputs "
                                     "(bn_pairing_batch_dev: per-term lines (k_prepare_wide), the segmented "
                                     "shared-squaring Miller loop (k_miller_seg), the device product reduction "
                                     "(k_fq12_reduce_wide, one or two levels), then the tail in one launch "
                                     "(k_seg_tail: per segment the final exponentiation's first chunk and Horner "
                                     "squarings, the segments' product as a chain, the last chunk digit-sliced on "
                                     "a squarer and two multiplier blocks)", "terms": n}
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
    res.update({"metric": unit, "value": n * args.steps / el, "unit": unit, "ms_per_step": el / args.steps * 1e3})
    if args.no_cpu_baseline:  # profiler passes: the kernels only
        emit(res)
        return
    from oracle import oracle as O  # the checker (cpu_baseline leg)
    if args.workload == "product":
        # SURVEY 8(d) config 5 algorithmic work: per term to_affine 19 + precompute 2,655 + lines 3,741
        # Fq-mul; the 64 shared squarings (2,304) and one final exponentiation (8,767) once per product
        work = (n * (19 + 2655 + 3741) + 2304 + 8767) * MAD32_PER_FQMUL
        ms = e0.elapsed_time(e1) / args.steps
        res["roofline"] = {"bound": "valu", "achieved": work / (ms * 1e-3) / 1e12, "peak": PEAK_MAD32_PER_S / 1e12,
                           "unit": "TMAD32/s (v_mad_u64_u32, algorithmic)",
                           "frac": work / (ms * 1e-3) / PEAK_MAD32_PER_S,
                           "traffic": pmc_traffic("product_step", "hbm_bytes_per_step"),
                           "traffic_source": "profiles/pmc_summary.json product_step: FETCH_SIZE (read-factor "
                                             "corrected) + WRITE_SIZE of every kernel of one product, committed "
                                             "rocprofv3 PMC passes, not measured in this run",
                           "kernel": "whole product (k_prepare_wide, k_miller_seg, k_fq12_reduce_wide, "
                                     "k_seg_tail)",
                           "per_step_ms": ms,
                           "basis": "SURVEY.md 8(d) config 5: n*(19+2655+3741) + 2304 + 8767 Fq-mul, x128 MAD32"}
        threads = host_cpus()["usable"]
        t0 = time.perf_counter()
        ref = O.pairing_batch(p, q, nthreads=threads)
        dt = time.perf_counter() - t0
        m1 = min(1024, n)
        t0 = time.perf_counter()
        O.pairing_batch(p[:m1], q[:m1])
        dt1 = time.perf_counter() - t0
        torch.cuda.synchronize(dev)
        res["cpu_baseline"] = {"value": n / dt, "unit": unit, "cores": threads, "kind": "port",
                               "single_core": {"value": m1 / dt1, "unit": unit,
                                               "sample": "pairing_batch of %d terms, 1 thread" % m1},
                               "sample": "the whole 2^14-term pairing_batch, oracle shared loop split over %d "
                                         "threads (orc_pairing_batch_mt), %.2f s wall" % (threads, dt),
                               "parity_bit_exact": bool(np.array_equal(ref, gout.cpu().numpy().view(np.uint64))
                                                        and int(gst.item()) == 0)}
        res["two_in_flight"] = products_in_flight(ctx, Pd, Qd, n, stream, dev, args, ref)
        res["affine_inputs"] = product_affine_inputs(ctx, Pd, Qd, n, stream, dev, args, ref)
    elif args.workload == "g2mul":
        # ~9,165 Fq-mul per 254-bit G2 scalar multiplication, x128 MAD32
        ms = e0.elapsed_time(e1) / args.steps
        work = n * 9165 * MAD32_PER_FQMUL
        res["roofline"] = {"bound": "valu", "achieved": work / (ms * 1e-3) / 1e12, "peak": PEAK_MAD32_PER_S / 1e12,
                           "unit": "TMAD32/s (v_mad_u64_u32, algorithmic)",
                           "frac": work / (ms * 1e-3) / PEAK_MAD32_PER_S, "traffic": None,
                           "kernel": "k_g2_mul_split", "per_launch_ms": ms,
                           "basis": "SURVEY.md 8(f1): ~9,165 Fq-mul per G2*Fr (253 doublings + ~127 additions of the "
                                    "reference chain, Fq2 products counted as 3 Fq-mul), x128 MAD32"}
        m = min(args.cpu_sample or 512, n)
        threads = host_cpus()["usable"]
        ph, kh, oh = (t[:m].cpu().numpy().view(np.uint64) for t in (P, k2, out))
        t0 = time.perf_counter()
        ref = O.g2_mul(ph, kh, threads)
        dt = time.perf_counter() - t0
        res["cpu_baseline"] = {"value": m / dt, "unit": unit, "cores": threads, "kind": "port",
                               "sample": "%d G2*Fr of the bench inputs, oracle, %d threads" % (m, threads),
                               "parity_sample_bit_exact": bool(np.array_equal(ref, oh))}
    elif args.workload == "g1mul":
        # ~3,800 Fq-mul per random 254-bit scalar (253 doublings x 7 + ~127 additions
        # x 16), x128 MAD32; the kernel is the only launch of the step (HIP events on its stream)
        ms = e0.elapsed_time(e1) / args.steps
        work = n * 3800 * MAD32_PER_FQMUL
        g1_kernel = "k_g1_mul2" if (n + 1) // 2 >= G1_MUL2_MIN_LANES else "k_g1_mul"
        res["roofline"] = {"bound": "valu", "achieved": work / (ms * 1e-3) / 1e12, "peak": PEAK_MAD32_PER_S / 1e12,
                           "unit": "TMAD32/s (v_mad_u64_u32, algorithmic)",
                           "frac": work / (ms * 1e-3) / PEAK_MAD32_PER_S, "traffic": pmc_traffic(g1_kernel),
                           "traffic_source": "profiles/pmc_summary.json (committed PMC run, not this run)",
                           "kernel": g1_kernel,
                           "per_launch_ms": ms,
                           "basis": "SURVEY.md 8(d) config 3: 3,800 Fq-mul per G1*Fr, x128 MAD32",
                           "executed": "the reference chain of every multiplication, ballot-scheduled: from 2^18 - 1 "
                                       "multiplications on, each lane runs two chains (rows i and i + n/2) and every "
                                       "iteration of a wave runs either the doubling (7 Fq-mul) or the addition (16 "
                                       "Fq-mul: the bases sit in LDS, their z^2, z^3 are recomputed) for one chain "
                                       "of each lane whose chain waits for it -- 1.30x the chains' own weight "
                                       "(profiles/r4c_g1mul2_schedule_counters.json; one chain per lane: 1.41x)"}
        m = min(args.cpu_sample or 2048, n)
        # rows of both chains of the first lanes: i and i + ceil(n / 2)
        h = (n + 1) // 2
        rows = np.unique(np.r_[np.arange(min(m // 2, h)), h + np.arange(min(m - m // 2, n - h))])
        threads = host_cpus()["usable"]
        ridx = torch.from_numpy(rows).to(dev)
        ph, kh, oh = (t[ridx].cpu().numpy().view(np.uint64) for t in (P, k2, out))
        t0 = time.perf_counter()
        ref = O.g1_mul(ph, kh, threads)
        dt = time.perf_counter() - t0
        res["cpu_baseline"] = {"value": len(rows) / dt, "unit": unit, "cores": threads, "kind": "port",
                               "sample": "%d G1*Fr of the bench inputs (rows 0.. and n/2.., both chains of the "
                                         "first lanes), oracle, %d threads" % (len(rows), threads),
                               "parity_sample_bit_exact": bool(np.array_equal(ref, oh))}
    emit(res)


def codec_workload(args, local_rank):
    """SURVEY 8(f) rows on 2^16 elements, inputs resident in HBM, device-pointer C ABI on torch's stream."""
    import torch

    from substrate_bn import Context, synth

    dev = torch.device("cuda", local_rank)
    ctx = Context(local_rank)
    stream = torch.cuda.Stream(dev)  # a real stream: handle 0 would mean the context's own stream
    sh = stream.cuda_stream
    n = args.pairs
    threads = host_cpus()["usable"]
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
    if args.workload == "gtpow":
        # the kernel's own chain, priced at SURVEY Appendix B's generic counts: every input is a
        # pairing output, so the signed 5-bit chain runs: 15 table products + 50 window products +
        # the membership check's product (Fq12 mul 54) and 250 cyclotomic squarings (18)
        work = n * (66 * 54 + 250 * 18) * MAD32_PER_FQMUL
        res["roofline"] = {"bound": "valu", "achieved": work / (kms * 1e-3) / 1e12, "peak": PEAK_MAD32_PER_S / 1e12,
                           "unit": "TMAD32/s (v_mad_u64_u32, algorithmic)",
                           "frac": work / (kms * 1e-3) / PEAK_MAD32_PER_S, "traffic": None, "kernel": kname,
                           "basis": "8,064 Fq-mul per Gt::pow (66 x 54 + 250 x 18: the signed 5-bit window chain of "
                                    "cyclotomic-subgroup inputs; the unsigned 4-bit chain before it ran 78 x 54 + "
                                    "252 x 18 = 8,748), x128 MAD32"}
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
    emit(res)


# ============================================================== pairing workload (configs 2 and 4)
class GpuEngine:
    """The product path: the engine's C ABI on one MI355X, all work on one real HIP stream."""
    dry = False

    def __init__(self, local_rank, ctx=None):
        import torch
        from substrate_bn import Context
        self.torch = torch
        self.dev = torch.device("cuda", local_rank)
        torch.cuda.set_device(self.dev)
        self.ctx = ctx if ctx is not None else Context(local_rank)
        # one real (non-default) stream for the kernels, torch's copies and the
        # collectives' ordering (handle 0 would mean the context's own stream)
        self.stream = torch.cuda.Stream(self.dev)
        torch.cuda.set_stream(self.stream)
        self.sh = self.stream.cuda_stream

    def points(self, lo, n):
        """P, Q (device, Jacobian images) for global dataset rows [lo, lo + n)."""
        from substrate_bn import synth
        torch = self.torch
        s, t = synth.dataset_scalars(lo, n)
        P = torch.empty((n, 12), dtype=torch.int64, device=self.dev)
        Q = torch.empty((n, 24), dtype=torch.int64, device=self.dev)
        g1 = torch.from_numpy(np.tile(synth.g1_one_image().view(np.int64), (n, 1))).to(self.dev)
        g2 = torch.from_numpy(np.tile(synth.g2_one_image().view(np.int64), (n, 1))).to(self.dev)
        s_d = torch.from_numpy(s.view(np.int64)).to(self.dev)
        t_d = torch.from_numpy(t.view(np.int64)).to(self.dev)
        self.ctx.g1_mul_many_dev(g1.data_ptr(), s_d.data_ptr(), n, P.data_ptr(), self.sh)
        self.ctx.g2_mul_many_dev(g2.data_ptr(), t_d.data_ptr(), n, Q.data_ptr(), self.sh)
        self.sync()
        return P, Q

    def empty_gt(self, n):
        return self.torch.empty((n, 48), dtype=self.torch.int64, device=self.dev)

    def pairing(self, P, Q, out):
        self.ctx.pairing_many_dev(P.data_ptr(), Q.data_ptr(), P.shape[0], out.data_ptr(), self.sh)

    def sync(self):
        self.torch.cuda.synchronize(self.dev)

    @staticmethod
    def host(t):
        return t.cpu().numpy().view(np.uint64)

    @staticmethod
    def reference(p, q, threads):
        """The checker: oracle/bn_oracle.c (C restatement of the reference CPU path)."""
        from oracle import oracle as O
        return O.pairing_many(p, q, threads)


class DryEngine:
    """--dry-run-cpu only: exercises bench.py's launch, sharding, all-gather,
    timing and cross-rank check on CPU tensors with gloo.  pairing() is a
    deterministic row mix, NOT a pairing; the JSON line says "dry_run": true."""
    dry = True

    def __init__(self, local_rank):
        import torch
        self.torch = torch

    def points(self, lo, n):
        from substrate_bn import synth
        s, t = synth.dataset_scalars(lo, n)
        P = self.torch.from_numpy(np.ascontiguousarray(np.tile(s, (1, 3))).view(np.int64))
        Q = self.torch.from_numpy(np.ascontiguousarray(np.tile(t, (1, 6))).view(np.int64))
        return P, Q

    def empty_gt(self, n):
        return self.torch.empty((n, 48), dtype=self.torch.int64)

    def pairing(self, P, Q, out):
        out[:, :12] = P
        out[:, 12:36] = Q
        out[:, 36:] = P ^ Q[:, :12]

    def sync(self):
        pass

    @staticmethod
    def host(t):
        return t.numpy().view(np.uint64)

    @staticmethod
    def reference(p, q, threads):
        """The dry run's checker: the stub's row mix recomputed on host arrays."""
        out = np.empty((p.shape[0], 48), np.uint64)
        out[:, :12] = p
        out[:, 12:36] = q
        out[:, 36:] = p ^ q[:, :12]
        return out


def run_pairing(args, eng, rank, world, dist):
    torch = eng.torch
    if args.config == 4:
        total = args.total
        if total % world:
            raise SystemExit("config 4: --total %d is not divisible by the world size %d" % (total, world))
        local_n = total // world
        scaling = "strong"
        wl = ("BASELINE config 4: %d pairings sharded contiguously over %d GPU(s) (%d each) + RCCL all-gather "
              "of all Gt results over xGMI inside the step" % (total, world, local_n)) if world > 1 else \
             ("BASELINE config 4 workload on 1 GPU: %d independent pairings (no exchange)" % total)
    else:
        local_n = args.pairs
        total = local_n * world
        scaling = "weak"
        wl = "BASELINE config 2: %d independent pairings e(P_i,Q_i) per GPU" % local_n + \
             (" + RCCL all-gather of Gt" if world > 1 else "")
    lo = rank * local_n
    t0 = time.perf_counter()
    P, Q = eng.points(lo, local_n)
    out = eng.empty_gt(local_n)
    gathered = eng.empty_gt(total) if world > 1 else None
    eng.sync()
    log("rank %d: %d pairs ready in %.1f s" % (rank, local_n, time.perf_counter() - t0))
    chunk = min(local_n, args.chunk)
    bounds = [(c0, min(c0 + chunk, local_n)) for c0 in range(0, local_n, chunk)]

    def step():
        works = []
        for c0, c1 in bounds:
            eng.pairing(P[c0:c1], Q[c0:c1], out[c0:c1])
            if world > 1:  # overlaps the next chunk's kernels (RCCL's own stream waits on this one)
                outs = [gathered[r * local_n + c0:r * local_n + c1] for r in range(world)]
                works.append(dist.all_gather(outs, out[c0:c1], async_op=True))
        for w in works:
            w.wait()

    for _ in range(args.warmup):
        step()
    eng.sync()
    gpu = not eng.dry
    if gpu:
        eng.ctx.phase_times()  # discard
        eng.ctx.set_phase_timing(True)
    if world > 1:
        dist.barrier()
    eng.sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    eng.sync()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if gpu:
        eng.ctx.set_phase_timing(False)
        phase_ms, launches = eng.ctx.phase_times()
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=getattr(eng, "dev", "cpu"))
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    value = total * args.steps / elapsed

    res = {
        "metric": "BN254 pairings/sec (batched) at 1/2/4/8 MI355X; bit-exact vs CPU ref",
        "value": value, "unit": "pairings/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": scaling,
        "vs_baseline": None, "dtype": "u32 (9x29-bit Montgomery digits, integer only)",
        "data": "synthetic: P_j = s_j*G1::one(), Q_j = t_j*G2::one(), s,t uniform Fr images in [1,r), "
                "SplitMix64 seeds per 4096-row block (substrate_bn/synth.py dataset_scalars)",
        "config": {"workload": wl, "total_pairs": total, "pairs_per_gpu": local_n, "parallelism": "dp%d" % world,
                   "chunk": chunk, "allgather_in_step": world > 1, "inputs": "HBM-resident Jacobian images",
                   "hbm_io_bytes_per_pairing": 96 + 192 + 384},
    }
    if eng.dry:
        res["dry_run"] = True
        res["dtype"] = "n/a (dry run: stub engine on CPU, not a pairing)"
    if gpu:
        res["roofline"] = roofline_block(phase_ms, launches, chunk, value / world)

    if world > 1:
        # the world size as the communicator sees it: an all-reduce of one per rank
        one = torch.ones(1, dtype=torch.int64, device=getattr(eng, "dev", "cpu"))
        dist.all_reduce(one)
        res["collective"] = {"backend": dist.get_backend(), "world_from_allreduce": int(one.item()),
                             "what": "RCCL (torch nccl backend) on GPUs; gloo in the CPU dry run"}

    # cross-rank equality: rebuild a sample of the next rank's rows here and compare
    # this GPU's results with what the all-gather delivered
    if world > 1:
        src = (rank + 1) % world
        m = min(128, local_n)
        mism = 0
        for j0 in sorted({0, local_n - m}):
            Pc, Qc = eng.points(src * local_n + j0, m)
            oc = eng.empty_gt(m)
            eng.pairing(Pc, Qc, oc)
            eng.sync()
            got = eng.host(gathered[src * local_n + j0:src * local_n + j0 + m])
            mism += int((eng.host(oc) != got).any(axis=1).sum())
        cnt = torch.tensor([mism, 1 if mism == 0 else 0], dtype=torch.int64, device=getattr(eng, "dev", "cpu"))
        dist.all_reduce(cnt, op=dist.ReduceOp.SUM)
        res["cross_rank_check"] = {"rows_per_rank": m * len({0, local_n - m}), "mismatches": int(cnt[0]),
                                   "ranks_ok": int(cnt[1]),
                                   "what": "each rank recomputes rows of the next rank's shard on its own GPU "
                                           "and compares them with the all-gathered Gt"}

    if rank == 0 and (world > 1 or args.config == 4) and not args.no_cpu_baseline:
        # config 4's checker leg over the gathered rows (every shard sampled) + the CPU baseline
        res["sample_check"], res["cpu_baseline"] = gathered_sample_check(eng, gathered if world > 1 else out,
                                                                         total, host_cpus())
    if rank == 0 and world == 1 and args.config == 2 and gpu and not args.no_cpu_baseline:
        m = min(args.cpu_sample or 16384, local_n)
        p_h, q_h, o_h = (eng.host(t[:m]) for t in (P, Q, out))
        res["cpu_baseline"] = cpu_baseline(p_h, q_h, o_h, host_cpus())
    if rank == 0 and world == 1 and gpu and not args.no_e2e:
        # host buffers through bn_pairing_many: H2D + kernels + D2H (PCIe-inclusive, not `value`)
        p_h, q_h = eng.host(P), eng.host(Q)
        eng.ctx.pairing_many(p_h, q_h)  # warm at full size: staging and pinned buffers grown
        ts = []
        for _ in range(5):
            t0 = time.perf_counter()
            o_h = eng.ctx.pairing_many(p_h, q_h)
            ts.append(time.perf_counter() - t0)
        dt = sorted(ts)[2]
        res["host_buffer_e2e"] = {"value": local_n / dt, "unit": "pairings/s", "ms_per_call": dt * 1e3,
                                  "what": "bn_pairing_many on pageable host buffers, H2D + kernels + D2H, median of 5 after a warm call (one 2^16 piece takes the runtime's pageable copies; larger calls the pinned double-buffered pipeline, tools/host_e2e.py)",
                                  "matches_hbm_path": bool(np.array_equal(o_h, eng.host(out)))}
    if rank == 0 and world == 1 and args.config == 2 and gpu and not args.no_config4_ref:
        res["config4_on_1_gpu"] = config4_on_one_gpu(args, eng)
    return res


def roofline_block(phase_ms, launches, chunk, per_gpu_value):
    """The dominant kernel's roofline from the per-phase HIP-event times of one
    device's bn_pairing_many_dev launches (bn_get_phase_times)."""
    per_launch_ms = {PHASES[k]: phase_ms[k] / max(launches, 1) for k in range(4)}
    fqmul = dict(FQMUL_PER_PAIRING)
    if per_launch_ms["k_fq12_vm"] < 0.01 * per_launch_ms["k_prepare"]:
        # the default throughput form: the whole pairing is one kernel (k_pairing_full)
        per_launch_ms = {"k_pairing_full": per_launch_ms["k_prepare"]}
        fqmul["k_pairing_full"] = sum(FQMUL_PER_PAIRING.values())
    elif per_launch_ms["k_miller"] < 0.01 * per_launch_ms["k_prepare"]:
        # the three-launch form 1 runs to_affine, the line steps and the Miller loop as one
        # kernel (k_pairing_fused): phase 0 holds both
        per_launch_ms = {"k_pairing_fused": per_launch_ms["k_prepare"], "k_fq12_vm": per_launch_ms["k_fq12_vm"],
                         "k_fe_out": per_launch_ms["k_fe_out"]}
        fqmul["k_pairing_fused"] = FQMUL_PER_PAIRING["k_prepare"] + FQMUL_PER_PAIRING["k_miller"]
    dom = max(per_launch_ms, key=per_launch_ms.get)
    achieved = fqmul[dom] * MAD32_PER_FQMUL * chunk / (per_launch_ms[dom] * 1e-3)
    return {
        "bound": "valu", "achieved": achieved / 1e12, "peak": PEAK_MAD32_PER_S / 1e12,
        "unit": "TMAD32/s (v_mad_u64_u32, algorithmic)", "frac": achieved / PEAK_MAD32_PER_S,
        "peak_measured": PEAK_MAD32_MEASURED / 1e12, "frac_of_measured_peak": achieved / PEAK_MAD32_MEASURED,
        "peak_measured_source": PEAK_MEASURED_SOURCE,
        "traffic": pmc_traffic(dom),
        "traffic_source": "profiles/pmc_summary.json: HBM bytes per launch from the committed rocprofv3 PMC "
                          "passes (FETCH_SIZE x2 + WRITE_SIZE), not measured in this run",
        "kernel": dom, "pairs_per_launch": chunk, "basis": FQMUL_BASIS,
        "per_launch_ms": {k: round(v, 4) for k, v in per_launch_ms.items()},
        "whole_pairing_frac": per_gpu_value * sum(FQMUL_PER_PAIRING.values()) * MAD32_PER_FQMUL / PEAK_MAD32_PER_S}


def run_capi_multi(args):
    """`--form capi`: BASELINE config 4 in ONE process over N devices through the C ABI
    (SURVEY 8(e) "single process with ncclCommInitAll"): bn_ctx_create_multi over devices
    0..N-1, device k's HBM-resident shard of rows [k*n, (k+1)*n) (n = --total / N) on
    device k, and per step one bn_pairing_many_allgather_dev -- every device computes its
    shard (bn_pairing_many_dev on its own stream), then one grouped RCCL all-gather over
    xGMI leaves all --total Gt rows on every device in device order.  Timed: a sync of
    every device on both sides of K steps.  Checked after the timed steps: device 0's
    gathered rows against the oracle (4,096 rows spread over every shard, the same
    checker leg as the torch form) and every device's gathered buffer against device 0's.
    `--dry-run-cpu` runs the control flow with the stub engine (no GPU, no RCCL)."""
    N = args.gpus
    total = args.total
    if total % N:
        raise SystemExit("config 4: --total %d is not divisible by %d devices" % (total, N))
    per = total // N
    dry = args.dry_run_cpu
    if dry:
        engs = [DryEngine(k) for k in range(N)]
        mctx = None
    else:
        from substrate_bn import Context
        mctx = Context(devices=list(range(N)))
        engs = [GpuEngine(k, ctx=mctx.device(k)) for k in range(N)]
    torch = engs[0].torch
    t0 = time.perf_counter()
    shards = []
    for k, eng in enumerate(engs):
        P, Q = eng.points(k * per, per)
        shards.append((P, Q, eng.empty_gt(total)))
    for eng in engs:
        eng.sync()
    log("capi form: %d devices, %d pairs each, ready in %.1f s" % (N, per, time.perf_counter() - t0))

    def step():
        if dry:  # the stub: each shard into its slot of every device's buffer ("all-gather")
            for k, (P, Q, out) in enumerate(shards):
                engs[k].pairing(P, Q, out[k * per:(k + 1) * per])
            for j, (_, _, out) in enumerate(shards):
                for k in range(N):
                    if j != k:
                        out[k * per:(k + 1) * per] = shards[k][2][k * per:(k + 1) * per]
            return
        mctx.pairing_many_allgather_dev([P.data_ptr() for P, _, _ in shards], [Q.data_ptr() for _, Q, _ in shards],
                                        per, [o.data_ptr() for _, _, o in shards], [e.sh for e in engs])

    for _ in range(args.warmup):
        step()
    for eng in engs:
        eng.sync()
    if not dry:
        for eng in engs:
            eng.ctx.phase_times()  # discard
            eng.ctx.set_phase_timing(True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    for eng in engs:
        eng.sync()
    elapsed = time.perf_counter() - t0
    value = total * args.steps / elapsed
    res = {
        "metric": "BN254 pairings/sec (batched) at 1/2/4/8 MI355X; bit-exact vs CPU ref",
        "value": value, "unit": "pairings/s", "n_gpus": N, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": "strong",
        "vs_baseline": None, "dtype": "u32 (9x29-bit Montgomery digits, integer only)",
        "data": "synthetic: P_j = s_j*G1::one(), Q_j = t_j*G2::one(), s,t uniform Fr images in [1,r), "
                "SplitMix64 seeds per 4096-row block (substrate_bn/synth.py dataset_scalars)",
        "config": {"workload": "BASELINE config 4: %d pairings sharded contiguously over %d GPU(s) (%d each) in ONE "
                               "process (bn_ctx_create_multi) + one RCCL all-gather of all Gt results over xGMI "
                               "inside the step (bn_pairing_many_allgather_dev)" % (total, N, per),
                   "total_pairs": total, "pairs_per_gpu": per, "parallelism": "dp%d" % N, "form": "capi",
                   "chunk": min(per, 1 << 16), "allgather_in_step": True, "inputs": "HBM-resident Jacobian images",
                   "hbm_io_bytes_per_pairing": 96 + 192 + 384},
    }
    if dry:
        res["dry_run"] = True
        res["dtype"] = "n/a (dry run: stub engine on CPU, not a pairing)"
    else:
        for eng in engs:
            eng.ctx.set_phase_timing(False)
        phase_ms, launches = engs[0].ctx.phase_times()
        for eng in engs[1:]:
            eng.ctx.phase_times()
        # the C ABI cuts each device's shard into its own launch chunks: pairs per launch from the count
        res["roofline"] = roofline_block(phase_ms, launches, per * args.steps // max(launches, 1), value / N)
        mctx.dev_status()  # the sticky device outcome (BN_ERR_INTERNAL / BN_ERR_FE_ZERO) of every device
    # every device's gathered buffer equals device 0's
    ref = shards[0][2]
    mism = 0
    for _, _, out in shards[1:]:
        o = out if dry else out.to(engs[0].dev)
        mism += int((o != ref).any(dim=1).sum().item())
    res["collective"] = {"backend": "stub (dry run)" if dry else "rccl: ncclCommInitAll + grouped ncclAllGather "
                         "(bn_pairing_many_allgather_dev, librccl dlopen'ed)",
                         "world_from_allreduce": N if dry else mctx.num_devices,
                         "devices_equal_to_device0": mism == 0, "mismatched_rows": mism,
                         "what": "the communicator's device count; every device's gathered buffer compared with "
                                 "device 0's row by row"}
    if not args.no_cpu_baseline:
        res["sample_check"], res["cpu_baseline"] = gathered_sample_check(engs[0], ref, total, host_cpus())
    return res


def config4_on_one_gpu(args, eng, steps=3):
    """The N = 1 point of config 4's strong-scaling curve: the same 2^20 rows,
    chunking and kernels as a rank of `--gpus N` (no all-gather), on this GPU.
    Reported beside `value` (which stays config 2, BASELINE's N = 1 metric)."""
    total = args.total
    chunk = min(total, args.chunk)
    P, Q = eng.points(0, total)
    out = eng.empty_gt(total)
    bounds = [(c0, min(c0 + chunk, total)) for c0 in range(0, total, chunk)]

    def step():
        for c0, c1 in bounds:
            eng.pairing(P[c0:c1], Q[c0:c1], out[c0:c1])

    step()
    eng.sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    eng.sync()
    el = time.perf_counter() - t0
    r = {"value": total * steps / el, "unit": "pairings/s", "total_pairs": total, "chunk": chunk, "steps": steps,
         "ms_per_step": el / steps * 1e3,
         "what": "BASELINE config 4's workload (%d pairs in %d-pair launches) on one GPU, no exchange: the "
                 "same-workload N = 1 reference for the --gpus N lines" % (total, chunk)}
    if not args.no_cpu_baseline:
        check, _ = gathered_sample_check(eng, out, total, host_cpus())
        r["sample_check"] = {k: check[k] for k in ("rows", "mismatches", "parity_sample_bit_exact")}
    del P, Q, out
    return r


def spawn_ranks(args):
    """--gpus N > 1 without a launcher: run torch.distributed.run with N ranks as a
    child (this process never touches a GPU) and return its exit status."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=%d" % args.gpus,
           "--master-addr=127.0.0.1", "--master-port=%d" % port, os.path.abspath(__file__)] + sys.argv[1:]
    log("bench: launching %d ranks: %s" % (args.gpus, " ".join(cmd)))
    return subprocess.call(cmd)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", type=int, choices=[2, 4], default=None,
                    help="2: 2^16 pairs per GPU (weak scaling); 4: --total pairs sharded over the GPUs "
                         "(strong scaling, all-gather in the step). Default: 2 on one GPU, 4 on several.")
    ap.add_argument("--pairs", type=int, default=1 << 16, help="config 2: pairings per GPU per step")
    ap.add_argument("--total", type=int, default=1 << 20, help="config 4: pairings per step over all GPUs")
    ap.add_argument("--chunk", type=int, default=1 << 16,
                    help="pairings per launch set (2^16 = one wave per SIMD); all-gathers go per chunk")
    ap.add_argument("--cpu-sample", type=int, default=None,
                    help="oracle sample size (default: 16384 pairings, 2048 for the 8(f) workloads; ~10-30 s of CPU-thread work)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true", help="skip the host-buffer (PCIe-inclusive) figure")
    ap.add_argument("--no-config4-ref", action="store_true",
                    help="skip config 4's workload on one GPU (the same-workload N = 1 point) in the N = 1 line")
    ap.add_argument("--form", choices=["torch", "capi"], default="torch",
                    help="N > 1 (config 4): torch = one process per GPU over torch.distributed/RCCL (the driver's "
                         "launch); capi = one process over all N devices through bn_ctx_create_multi + "
                         "bn_pairing_many_allgather_dev (no ranks spawned)")
    ap.add_argument("--dry-run-cpu", action="store_true",
                    help="control-flow check on CPU: gloo + a stub engine (no pairing is computed)")
    ap.add_argument("--workload", default="pairing",
                    choices=["pairing", "g1mul", "g2mul", "product", "g2validate", "g2decompress", "gtpow"],
                    help="pairing: configs 2/4 (default); g1mul: config 3 (2^18 G1*Fr); product: config 5 "
                         "(2^14-term pairing_batch); SURVEY 8(f): g2mul (G2*Fr), g2validate (AffineG2::new incl. "
                         "the order check), g2decompress (G2::from_compressed), gtpow (Gt::pow(Fr)), 2^16 each")
    args = ap.parse_args()
    if args.config is None:
        args.config = 2 if args.gpus == 1 else 4

    if args.form == "capi":
        if args.workload != "pairing" or os.environ.get("WORLD_SIZE") not in (None, "1"):
            log("bench: --form capi is config 4 in one process (no launcher, --workload pairing)")
            return 2
        args.config = 4
        emit(run_capi_multi(args))
        return 0
    world_env = os.environ.get("WORLD_SIZE")
    if args.gpus > 1 and world_env is None:
        return spawn_ranks(args)
    world = int(world_env or 1)
    if world != args.gpus:
        log("bench: --gpus %d but WORLD_SIZE=%d" % (args.gpus, world))
        return 2
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.workload != "pairing":
        if world > 1:
            log("bench: --workload %s runs on one GPU" % args.workload)
            return 2
        if args.workload in ("g2validate", "g2decompress", "gtpow"):
            codec_workload(args, local_rank)
        else:
            other_workload(args, local_rank)
        return 0

    import torch
    import torch.distributed as dist

    # BN254MI_BENCH_SHARED_GPU=1: a rehearsal of the N > 1 launch on a one-GPU box -- every
    # rank computes on device 0 and the collectives go over gloo (RCCL refuses two ranks
    # on one device); the line is marked and is no scaling figure
    shared = world > 1 and not args.dry_run_cpu and os.environ.get("BN254MI_BENCH_SHARED_GPU") == "1"
    eng = (DryEngine if args.dry_run_cpu else GpuEngine)(0 if shared else local_rank)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if eng.dry or shared:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    res = run_pairing(args, eng, rank, world, dist)
    if shared:
        res["rehearsal"] = ("BN254MI_BENCH_SHARED_GPU: %d ranks on ONE MI355X, gloo collectives -- the N > 1 "
                            "control flow with real pairings, not a scaling figure" % world)
    if rank == 0:
        emit(res)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
