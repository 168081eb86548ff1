"""World-size-2 and -8 gloo tests of the multi-GPU path (substrate_bn/parallel.py) on
CPU: sharding, the variable-length all-gather of Gt results, and the
rank-ordered partial-product exchange of pairing_batch.  The per-shard compute
is injected (the oracle stands in for the GPU engine here; it is only the
checker, and the GPU path is exercised by the -m gpu tests)."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def worker(rank, world, port, n, qout):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "paritytech-bn_amd")]
    import torch.distributed as dist

    from oracle import oracle as O
    from substrate_bn import parallel

    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    p, q, _, _ = O.random_pairs(n, seed=31, nthreads=2)
    if n > 2:
        p[2] = 0
        p[2, 4:8] = O.canon_to_mont_array([1])  # a zero point, skipped by pairing_batch
    many = parallel.pairing_many_distributed(p, q, compute=lambda a, b: O.pairing_many(a, b, 2))
    import torch

    def into(a, b, out):  # the device-resident form's per-shard compute, here on CPU tensors
        res = O.pairing_many(a.numpy().view(np.uint64), b.numpy().view(np.uint64), 2)
        out.copy_(torch.from_numpy(res.view(np.int64)))
    many_dev = parallel.pairing_many_distributed_dev(torch.from_numpy(p.view(np.int64)),
                                                     torch.from_numpy(q.view(np.int64)), compute=into)
    assert np.array_equal(many_dev.numpy().view(np.uint64), many)
    mp_fn = lambda a, b: O.miller_loop_batch(b, a)[1]  # noqa: E731
    mul = lambda a, b: O.binary("orc_fq12_mul", a, b, 48, 48, 48)[0]  # noqa: E731
    def fe(f):
        out, rcs = O.final_exponentiation(f)
        return out, [rc == 0 for rc in rcs]
    try:
        prod = parallel.pairing_batch_distributed(p, q, miller_product=mp_fn, fq12_mul=mul, final_exp=fe)
    except Exception as e:  # report instead of hanging the parent
        qout.put((rank, None, repr(e)))
        raise
    qout.put((rank, many, prod))
    dist.destroy_process_group()


@pytest.mark.parametrize("world,n", [(2, 7), (2, 2), (8, 13), (8, 5)])
def test_world_sharding_and_gather(world, n):
    """World 8 is config 4's rank count: 13 pairs give shards of
    one and two, 5 pairs leave three ranks with an empty shard."""
    from oracle import oracle as O
    ctx = mp.get_context("spawn")
    qout = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=worker, args=(r, world, port, n, qout)) for r in range(world)]
    for pr in procs:
        pr.start()
    res = {}
    for _ in range(world):
        rank, many, prod = qout.get(timeout=120)
        assert many is not None, prod
        res[rank] = (many, prod)
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    p, q, _, _ = O.random_pairs(n, seed=31, nthreads=2)
    if n > 2:
        p[2] = 0
        p[2, 4:8] = O.canon_to_mont_array([1])
    want_many = O.pairing_many(p, q, 2)
    want_prod = O.pairing_batch(p, q)
    for r in range(world):
        assert np.array_equal(res[r][0], want_many)
        assert np.array_equal(res[r][1], want_prod)


def test_shard_bounds_cover():
    sys.path[:0] = [os.path.join(ROOT, "paritytech-bn_amd")]
    from substrate_bn.parallel import shard_bounds
    for n in (0, 1, 7, 65536, 1 << 20):
        for world in (1, 2, 3, 8):
            spans = [shard_bounds(n, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[r][1] == spans[r + 1][0] for r in range(world - 1))
