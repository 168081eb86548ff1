"""The C ABI's threading contract (include/bn254mi.h): one context may be used
from several host threads -- each call holds the context for its whole
duration -- and _dev calls enqueued on different streams run in call order on
the shared workspace.  The reference is reentrant from any thread
(lib.rs:303-305, Group: Send + Sync); results must not depend on interleaving.
Expected values come from the oracle, computed before the threads start."""
import threading

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu
NT = 16


@pytest.fixture(scope="module")
def data():
    p, q, _, _ = O.random_pairs(192, seed=4242, nthreads=NT)
    ks, K = O.random_scalars(192, seed=4243, lo=0)
    return {"p": p, "q": q, "K": K, "gt": O.pairing_many(p, q, NT), "g1k": O.g1_mul(p, K, NT),
            "prod": O.pairing_batch(p[:40], q[:40])}


def test_two_threads_one_context(data):
    from substrate_bn import Context
    ctx = Context(0)
    errors = []

    def pairing_worker():
        try:
            for m in (7, 192, 33, 129, 64):  # staging buffer regrows between calls
                got = ctx.pairing_many(data["p"][:m], data["q"][:m])
                if not np.array_equal(got, data["gt"][:m]):
                    errors.append("pairing_many(%d) mismatch" % m)
        except Exception as e:  # noqa: BLE001 -- reported below
            errors.append(repr(e))

    def mixed_worker():
        try:
            for _ in range(3):
                if not np.array_equal(ctx.g1_mul_many(data["p"], data["K"]), data["g1k"]):
                    errors.append("g1_mul_many mismatch")
                if not np.array_equal(ctx.pairing_batch(data["p"][:40], data["q"][:40]), data["prod"]):
                    errors.append("pairing_batch mismatch")
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))

    ts = [threading.Thread(target=pairing_worker), threading.Thread(target=mixed_worker)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=100)
    assert not any(t.is_alive() for t in ts), "worker hung"
    assert not errors, errors


def test_dev_calls_on_two_streams_share_the_workspace(data):
    import torch
    from substrate_bn import Context
    ctx = Context(0)
    dev = torch.device("cuda", 0)
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    P = torch.from_numpy(data["p"].view(np.int64)).to(dev)
    Q = torch.from_numpy(data["q"].view(np.int64)).to(dev)
    torch.cuda.synchronize(dev)
    o1 = torch.zeros((96, 48), dtype=torch.int64, device=dev)
    o2 = torch.zeros((96, 48), dtype=torch.int64, device=dev)
    # back to back, no host synchronization: both use the context's coefficient and slot buffers
    ctx.pairing_many_dev(P[:96].data_ptr(), Q[:96].data_ptr(), 96, o1.data_ptr(), s1.cuda_stream)
    ctx.pairing_many_dev(P[96:].data_ptr(), Q[96:].data_ptr(), 96, o2.data_ptr(), s2.cuda_stream)
    ctx.pairing_many_dev(P[:96].data_ptr(), Q[:96].data_ptr(), 96, o1.data_ptr(), s1.cuda_stream)
    torch.cuda.synchronize(dev)
    assert np.array_equal(o1.cpu().numpy().view(np.uint64), data["gt"][:96])
    assert np.array_equal(o2.cpu().numpy().view(np.uint64), data["gt"][96:])
