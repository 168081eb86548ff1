"""Child process of tests/test_gpu_failure.py (not collected by pytest).

Runs with BN254MI_LIB = paritytech-bn_amd/libbn254mi_cap0.so: the product library
with the capped LDS hand-off waits of the latency kernels and the two-group
final exponentiation built at spin cap 0 (fq12_wide.h BN_SPIN_CAP), so that the
first wait of each runs out.  Prints one JSON line with what every entry point
returned; the test asserts on it.  The oracle is the checker only.  With
libbn254mi_chanfail.so or libbn254mi_latem.so (the product's tail with dropped
channel stores / a late multiplier block) it runs the segmented product only.
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "paritytech-bn_amd"))

from oracle import oracle as O  # noqa: E402
from substrate_bn import _native  # noqa: E402


def code_of(fn):
    """BN_OK or the BnError code of fn(), plus its value when it returned."""
    try:
        return _native.BN_OK, fn()
    except _native.BnError as e:
        return e.code, None


def tail_probe(kind):
    """libbn254mi_chanfail.so / libbn254mi_latem.so: only the product's tail differs
    from the product build (paritytech-bn_amd/Makefile), so only the segmented
    pairing_batch (4,224 terms) is run: its tail is k_seg_tail (one launch, the
    segment chain and two multiplier blocks), or k_seg_fe1 + k_horner_tree2 with
    BN254MI_TAIL_FUSED=0.  kind "main": the product library itself (FAILURE_PROBE_TAIL=1)."""
    ctx = _native.Context(0)
    p, q, _, _ = O.random_pairs(24, seed=43, nthreads=8)
    reps = 4224 // 24
    P4, Q4 = np.tile(p, (reps, 1)), np.tile(q, (reps, 1))
    res = {"kind": kind}
    for k in range(2):  # the second call is timed warm
        t0 = time.perf_counter()
        res["code"], v = code_of(lambda: ctx.pairing_batch(P4, Q4))
        res["seconds_%d" % k] = time.perf_counter() - t0
    res["value_returned"] = v is not None
    if v is not None:
        res["bit_exact"] = bool(np.array_equal(v, O.pairing_batch(P4, Q4)))
    print(json.dumps(res), flush=True)


def main():
    import torch
    for kind in ("chanfail", "latem"):
        if _native.LIB_PATH.endswith("libbn254mi_%s.so" % kind):
            return tail_probe(kind)
    if os.environ.get("FAILURE_PROBE_TAIL") == "1":
        return tail_probe("main")
    assert _native.LIB_PATH.endswith("libbn254mi_cap0.so"), _native.LIB_PATH
    ctx = _native.Context(0)
    n = 24
    p, q, _, _ = O.random_pairs(n, seed=41, nthreads=8)
    res = {}
    # host-buffer forms: the latency kernel (n <= latency_max) -> BN_ERR_INTERNAL, no output
    res["pairing_many"], v = code_of(lambda: ctx.pairing_many(p, q))
    res["pairing_many_value_returned"] = v is not None
    res["pairing_batch"], v = code_of(lambda: ctx.pairing_batch(p, q))
    res["pairing_batch_value_returned"] = v is not None
    res["miller_loop_batch"], _ = code_of(lambda: ctx.miller_loop_batch(q, p))
    # past the one-launch threshold: the segmented product, whose only capped waits are the
    # tail's squarer <-> multiplier channel (fq12_ds.h ds_chan_ld, k_horner_tree2 on two blocks)
    reps = 4224 // n
    P4, Q4 = np.tile(p, (reps, 1)), np.tile(q, (reps, 1))
    t0 = time.perf_counter()
    res["pairing_batch_segmented"], v = code_of(lambda: ctx.pairing_batch(P4, Q4))
    res["pairing_batch_segmented_s"] = time.perf_counter() - t0
    res["pairing_batch_segmented_value_returned"] = v is not None
    # the two-group final exponentiation of k_fe_wide (its S <-> M channel waits)
    _, mv = O.miller_loop_batch(q[:1], p[:1])
    f = np.tile(mv.reshape(1, 48), (4, 1))
    res["final_exponentiation_many"], _ = code_of(lambda: ctx.final_exponentiation_many(f))
    # device forms: the status-less bn_pairing_many_dev reports through bn_dev_status
    dev = torch.device("cuda", 0)
    P = torch.from_numpy(p.view(np.int64)).to(dev)
    Q = torch.from_numpy(q.view(np.int64)).to(dev)
    out = torch.zeros((n, 48), dtype=torch.int64, device=dev)
    torch.cuda.synchronize(dev)
    res["pairing_many_dev_call"], _ = code_of(lambda: ctx.pairing_many_dev(P.data_ptr(), Q.data_ptr(), n, out.data_ptr()))
    res["dev_status_after"], _ = code_of(lambda: ctx.dev_status())
    res["dev_status_cleared"], _ = code_of(lambda: ctx.dev_status())  # the sticky word was cleared
    # bn_pairing_batch_dev with its device status word
    st = torch.full((1,), -1, dtype=torch.int32, device=dev)
    gt = torch.zeros((1, 48), dtype=torch.int64, device=dev)
    res["pairing_batch_dev_call"], _ = code_of(
        lambda: ctx.pairing_batch_dev(P.data_ptr(), Q.data_ptr(), n, gt.data_ptr(), st.data_ptr()))
    torch.cuda.synchronize(dev)
    res["pairing_batch_dev_status"] = int(st.cpu().item())
    # the throughput path has no capped waits: the same library must still be right there
    ctx.set_latency_max(0)
    ctx.set_fe_wide_max(0)
    code, v = code_of(lambda: ctx.pairing_many(p, q))
    res["throughput_path"] = code
    res["throughput_path_bit_exact"] = bool(v is not None and np.array_equal(v, O.pairing_many(p, q, 8)))
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
