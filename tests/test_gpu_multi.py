"""Multi-device context of the C ABI (bn_ctx_create_multi) on the
one-GPU box: a context over devices [0, 0] runs two sub-contexts on the same
MI355X, which exercises the contiguous sharding, the concurrent per-device
threads and the partial-product combination exactly as on 8 devices; the RCCL
all-gather form runs as a world of one (ncclCommInitAll over [0]).  Results
must equal the single-device engine and the oracle bit for bit."""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu
NT = 16


@pytest.fixture(scope="module")
def data():
    p, q, _, _ = O.random_pairs(101, seed=909, nthreads=NT)
    z = p.copy()
    z[5] = 0
    z[5, 4:8] = O.canon_to_mont_array([1])  # a zero point: one for pairing, skipped by pairing_batch
    return {"p": p, "q": q, "pz": z, "gt": O.pairing_many(z, q, NT), "prod": O.pairing_batch(z, q)}


@pytest.fixture(scope="module")
def mctx():
    from substrate_bn import Context
    return Context(devices=[0, 0])


def test_multi_context_shards_host_calls(mctx, data):
    assert mctx.num_devices == 2
    assert np.array_equal(mctx.pairing_many(data["pz"], data["q"]), data["gt"])
    assert np.array_equal(mctx.pairing_batch(data["pz"], data["q"]), data["prod"])
    ks, K = O.random_scalars(101, seed=910, lo=0)
    assert np.array_equal(mctx.g1_mul_many(data["p"], K), O.g1_mul(data["p"], K, NT))
    ml = mctx.miller_loop_many(data["p"][:9], data["q"][:9])
    out, ok = mctx.final_exponentiation_many(ml)
    assert ok.all() and np.array_equal(out, O.pairing_many(data["p"][:9], data["q"][:9], NT))
    # miller_loop_batch: product of the per-device partials equals the oracle's shared loop
    _, want = O.miller_loop_batch(data["q"][:33], data["p"][:33])
    assert np.array_equal(mctx.miller_loop_batch(data["q"][:33], data["p"][:33]), want)
    # fewer elements than devices: an empty shard
    assert np.array_equal(mctx.pairing_many(data["p"][:1], data["q"][:1]), O.pairing_many(data["p"][:1], data["q"][:1]))


def test_multi_context_refuses_single_device_calls(mctx, data):
    from substrate_bn import BnError
    with pytest.raises(BnError):
        mctx.gt_pow_many(data["gt"][:2], np.zeros((2, 4), np.uint64))


def test_allgather_dev_world_of_one(data):
    import torch
    from substrate_bn import Context
    ctx = Context(devices=[0])
    dev = torch.device("cuda", 0)
    P = torch.from_numpy(data["pz"].view(np.int64)).to(dev)
    Q = torch.from_numpy(data["q"].view(np.int64)).to(dev)
    out = torch.zeros((101, 48), dtype=torch.int64, device=dev)
    s = torch.cuda.Stream(dev)
    ctx.pairing_many_allgather_dev([P.data_ptr()], [Q.data_ptr()], 101, [out.data_ptr()], [s.cuda_stream])
    torch.cuda.synchronize(dev)
    assert np.array_equal(out.cpu().numpy().view(np.uint64), data["gt"])


def test_torch_distributed_forms_world_of_one(data):
    """substrate_bn/parallel.py on the engine (no injected compute) under the nccl
    backend (RCCL) as a world of one: the device-resident all-gather form and the
    rank-ordered pairing_batch exchange equal the oracle bit for bit."""
    import socket

    import torch
    import torch.distributed as dist
    from substrate_bn import parallel
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % port, rank=0, world_size=1, device_id=dev)
    try:
        P = torch.from_numpy(data["pz"].view(np.int64)).to(dev)
        Q = torch.from_numpy(data["q"].view(np.int64)).to(dev)
        got = parallel.pairing_many_distributed_dev(P, Q)
        torch.cuda.synchronize(dev)
        assert np.array_equal(got.cpu().numpy().view(np.uint64), data["gt"])
        st = torch.cuda.Stream(dev)
        got2 = parallel.pairing_many_distributed_dev(P, Q, stream=st)
        torch.cuda.synchronize(dev)
        assert np.array_equal(got2.cpu().numpy().view(np.uint64), data["gt"])
        # non-contiguous inputs (column views of wider tensors): the shard copies
        # are made on torch's stream before the engine stream waits for it
        wideP = torch.zeros((101, 20), dtype=torch.int64, device=dev)
        wideP[:, 3:15] = P
        wideQ = torch.zeros((101, 30), dtype=torch.int64, device=dev)
        wideQ[:, 5:29] = Q
        got3 = parallel.pairing_many_distributed_dev(wideP[:, 3:15], wideQ[:, 5:29], stream=st)
        torch.cuda.synchronize(dev)
        assert np.array_equal(got3.cpu().numpy().view(np.uint64), data["gt"])
        assert np.array_equal(parallel.pairing_batch_distributed(data["pz"], data["q"]), data["prod"])
        assert np.array_equal(parallel.pairing_many_distributed(data["pz"], data["q"]), data["gt"])
    finally:
        dist.destroy_process_group()


def _device_count():
    import torch
    return torch.cuda.device_count()  # does not initialize the GPU runtime on this image


needs_two = pytest.mark.skipif(_device_count() < 2, reason="needs two or more visible MI355X")


@needs_two
def test_multi_context_distinct_devices(data):
    """bn_ctx_create_multi over every visible device: the sharded host calls and the
    per-device products combined in device order equal the oracle bit for bit."""
    from substrate_bn import Context
    nd = _device_count()
    ctx = Context(devices=list(range(nd)))
    assert ctx.num_devices == nd
    assert np.array_equal(ctx.pairing_many(data["pz"], data["q"]), data["gt"])
    assert np.array_equal(ctx.pairing_batch(data["pz"], data["q"]), data["prod"])
    _, want = O.miller_loop_batch(data["q"][:33], data["p"][:33])
    assert np.array_equal(ctx.miller_loop_batch(data["q"][:33], data["p"][:33]), want)
    ks, K = O.random_scalars(101, seed=911, lo=0)
    assert np.array_equal(ctx.g1_mul_many(data["p"], K), O.g1_mul(data["p"], K, NT))


@needs_two
def test_allgather_dev_distinct_devices(data):
    """BASELINE config 4's C-ABI form on real devices: device k computes its HBM-resident
    shard, one RCCL all-gather (ncclCommInitAll + grouped ncclAllGather) leaves every
    device holding all rows in device order -- each device's buffer equals the oracle."""
    import torch
    from substrate_bn import Context
    nd = min(_device_count(), 4)
    per = 101 // nd
    n = per * nd
    ctx = Context(devices=list(range(nd)))
    ins, outs, streams = [], [], []
    for k in range(nd):
        dev = torch.device("cuda", k)
        P = torch.from_numpy(np.ascontiguousarray(data["pz"][k * per:(k + 1) * per]).view(np.int64)).to(dev)
        Q = torch.from_numpy(np.ascontiguousarray(data["q"][k * per:(k + 1) * per]).view(np.int64)).to(dev)
        ins.append((P, Q))
        outs.append(torch.zeros((n, 48), dtype=torch.int64, device=dev))
        streams.append(torch.cuda.Stream(dev))
        torch.cuda.synchronize(dev)
    ctx.pairing_many_allgather_dev([P.data_ptr() for P, _ in ins], [Q.data_ptr() for _, Q in ins], per,
                                   [o.data_ptr() for o in outs], [s.cuda_stream for s in streams])
    for k in range(nd):
        torch.cuda.synchronize(torch.device("cuda", k))
    ctx.dev_status()
    for k in range(nd):
        assert np.array_equal(outs[k].cpu().numpy().view(np.uint64), data["gt"][:n]), "device %d" % k


def _ranks_worker(rank, world, port, n, qout):
    """One rank of the torch.distributed form with the ENGINE as its compute (no
    injected hook): every rank's context on device 0, the collective over gloo
    (RCCL refuses two ranks on one device)."""
    import os
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "paritytech-bn_amd")]
    try:
        import torch.distributed as dist

        from oracle import oracle as O
        from substrate_bn import parallel
        dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
        p, q, _, _ = O.random_pairs(n, seed=912, nthreads=2)
        p[3] = 0
        p[3, 4:8] = O.canon_to_mont_array([1])  # a zero point: one for pairing, skipped by pairing_batch
        many = parallel.pairing_many_distributed(p, q)
        prod = parallel.pairing_batch_distributed(p, q)
        dist.destroy_process_group()
        qout.put((rank, many, prod))
    except Exception as e:  # report instead of hanging the parent
        qout.put((rank, None, repr(e)))
        raise


@pytest.mark.parametrize("world,n", [(4, 4099), (8, 5)])
def test_torch_distributed_ranks_on_one_gpu(world, n):
    """config 4's control flow with the engine as each rank's compute: `world` rank
    processes (one context each, all on the one MI355X of this box), contiguous shards,
    the Gt rows gathered in rank order and pairing_batch's partials multiplied in rank
    order.  n = 5 at world 8 leaves three ranks with an empty shard.  Every rank's
    results equal the oracle bit for bit."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    qout = ctx.Queue()
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = [ctx.Process(target=_ranks_worker, args=(r, world, port, n, qout)) for r in range(world)]
    for pr in procs:
        pr.start()
    res = {}
    try:
        for _ in range(world):
            rank, many, prod = qout.get(timeout=150)
            assert many is not None, prod
            res[rank] = (many, prod)
    finally:
        for pr in procs:
            pr.join(timeout=60)
            if pr.exitcode is None:
                pr.kill()
    assert all(pr.exitcode == 0 for pr in procs)
    p, q, _, _ = O.random_pairs(n, seed=912, nthreads=NT)
    p[3] = 0
    p[3, 4:8] = O.canon_to_mont_array([1])
    want_many = O.pairing_many(p, q, NT)
    want_prod = O.pairing_batch(p, q)
    for r in range(world):
        assert np.array_equal(res[r][0], want_many), "rank %d" % r
        assert np.array_equal(res[r][1], want_prod), "rank %d" % r


def test_bench_driver_launch_two_ranks_on_one_gpu():
    """The driver's own N > 1 command (torch.distributed.run --nproc-per-node 2 ...
    bench.py --gpus 2) with BN254MI_BENCH_SHARED_GPU=1: both ranks on device 0 over
    gloo.  Config 4's sharding, the in-step all-gather, the max-over-ranks timing and
    both checks (cross-rank recompute, oracle sample of the gathered rows) run with
    real pairings."""
    import json
    import os
    import socket
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, BN254MI_BENCH_SHARED_GPU="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--total", "16384", "--chunk", "4096", "--cpu-sample", "256", "--no-e2e"]
    r = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["scaling"] == "strong" and "rehearsal" in line
    assert line["collective"]["world_from_allreduce"] == 2
    assert line["cross_rank_check"]["mismatches"] == 0 and line["cross_rank_check"]["ranks_ok"] == 2
    assert line["sample_check"]["parity_sample_bit_exact"] is True
