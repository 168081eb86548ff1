#!/usr/bin/env python3
"""Device-side fold-bound check (diagnostic; not a parity test).

Loads libbn254mi_dbg.so (`make -C paritytech-bn_amd dbg`: every fold counts
the lanes whose top-digit quotient estimate q exceeds the static bound of its
input, fq.h BN_DEVICE_CHECKS), drives every kernel family over seeded inputs (the one-launch latency kernels at
n pairs -- the two-wave build above 2,048 -- a 4n-term segmented product, the
throughput kernel k_pairing_full over 16n pairs, the segmented latency path and
the wide final exponentiation) and prints the per-translation-unit violation counters as one JSON line.
All counters 0 means no fold saw a value above the bound its type claims, so
no LDS table index went past its 161 entries.

    BN254MI_LIB=paritytech-bn_amd/libbn254mi_dbg.so python tools/fold_check.py [n]
"""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "paritytech-bn_amd"))
os.environ.setdefault("BN254MI_LIB", os.path.join(ROOT, "paritytech-bn_amd", "libbn254mi_dbg.so"))

from substrate_bn import _native, synth  # noqa: E402

TUS = ["pairing", "fe", "wide", "latency_w2", "group", "gtpow", "codec", "util", "reduce", "tail"]  # every unit (Makefile dbg)


def counters(L):
    out = {}
    for t in TUS:
        fn = getattr(L, "bn_dbg_fold_bad_" + t)
        fn.restype = ctypes.c_uint
        out[t] = int(fn())
    return out


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    L = _native.load()
    ctx = _native.Context(0)
    before = counters(L)
    g1 = np.tile(synth.g1_one_image(), (n, 1))
    g2 = np.tile(synth.g2_one_image(), (n, 1))
    p = ctx.g1_mul_many(g1, synth.fr_images(n, 1))
    q = ctx.g2_mul_many(g2, synth.fr_images(n, 2))
    gt = ctx.pairing_many(p, q)
    ctx.pairing_batch(p[:1024], q[:1024])
    ctx.pairing_batch(np.tile(p, (4, 1)), np.tile(q, (4, 1)))  # segmented product (2^14 terms at n = 4096)
    ctx.miller_loop_batch(q[:3000], p[:3000])
    ctx.miller_loop_many(p[:256], q[:256])
    # the throughput path (k_pairing_full, config 2's kernel) over 16 n pairs (2^16 at n = 4096)
    tp = _native.Context(0)
    tp.set_fe_wide_max(0)
    tp.pairing_many(np.tile(p, (16, 1)), np.tile(q, (16, 1)))
    # the segmented latency path (k_prepare_wide + k_miller_seg + k_horner_wide) and k_fe_wide
    seg = _native.Context(0)
    seg.set_latency_max(0)
    seg.pairing_many(p[:2048], q[:2048])
    seg.final_exponentiation_many(seg.miller_loop_many(p[:64], q[:64]))
    ctx.gt_pow_many(gt, synth.fr_images(n, 3, lo=0))
    for op in ("mul", "sqr", "inv", "cyc_sqr", "exp_by_neg_z", "frob1", "frob2", "frob3"):
        ctx.fq12_op_many(op, gt[:256], gt[256:512] if op == "mul" else None)
    aff = synth.g2_jacobian_to_affine(q[:512])
    ctx.g2_affine_new_many(aff[:, :8], aff[:, 8:])
    ctx.g2_from_compressed_many(synth.compress_g2(aff))
    after = counters(L)
    res = {"check": "device fold bound (q <= static bound) on every fold, BN_DEVICE_CHECKS build",
           "n": n, "violations": {t: after[t] - before[t] for t in TUS}}
    res["ok"] = all(v == 0 for v in res["violations"].values())
    print(json.dumps(res), flush=True)
    return 0 if res["ok"] else 1


if __name__ == "__main__":
    sys.exit(main())
