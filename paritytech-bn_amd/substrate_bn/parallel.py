"""Multi-GPU batching over torch.distributed (one process per GPU; backend
"nccl" is RCCL over xGMI on ROCm).

SURVEY.md §8(e): independent pairings shard with no data-path exchange, so
each rank takes a contiguous slice [k*n/G, (k+1)*n/G) of the batch; the only
collective is one all-gather of the Gt results (BASELINE config 4).  For a
pairing *product* (pairing_batch) each rank reduces its slice to one Miller
value, the 384-byte partials are all-gathered, multiplied in rank order on
every rank (so every rank holds the identical Gt) and finally exponentiated.
The product is exact: Fq12 multiplication is commutative and the reference's
shared-squaring loop equals the product of per-pair Miller values.

`compute` hooks exist so the world_size-2 gloo tests can run the sharding and
collectives on CPU; in production they default to the GPU engine.
"""
import numpy as np
import torch
import torch.distributed as dist


def shard_bounds(n, rank, world):
    """Contiguous shard of rank `rank`."""
    return n * rank // world, n * (rank + 1) // world


def _gather_rows(local, world, max_rows, device):
    """All-gather variable-length (rows, 48) uint64 blocks; returns the list per rank."""
    rows = local.shape[0]
    buf = torch.zeros((max_rows, local.shape[1]), dtype=torch.int64, device=device)
    if rows:
        buf[:rows] = torch.from_numpy(np.ascontiguousarray(local).view(np.int64)).to(device)
    out = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(out, buf)
    return [o.cpu().numpy().view(np.uint64) for o in out]


def pairing_many_distributed(p, q, compute=None, device=None):
    """out[i] = pairing(p[i], q[i]) for the whole batch, on every rank."""
    world, rank = dist.get_world_size(), dist.get_rank()
    n = p.shape[0]
    lo, hi = shard_bounds(n, rank, world)
    if compute is None:
        from . import context
        compute = context().pairing_many
    local = compute(p[lo:hi], q[lo:hi]) if hi > lo else np.zeros((0, 48), np.uint64)
    max_rows = max(shard_bounds(n, r, world)[1] - shard_bounds(n, r, world)[0] for r in range(world))
    parts = _gather_rows(local, world, max_rows, device or _default_device())
    return np.concatenate([parts[r][: shard_bounds(n, r, world)[1] - shard_bounds(n, r, world)[0]]
                           for r in range(world)], axis=0)


def pairing_many_distributed_dev(P, Q, compute=None, stream=None):
    """Device-resident form (BASELINE config 4 as a library call): P (n, 12) and
    Q (n, 24) int64 tensors holding the reference images, the same on every rank
    (or at least this rank's shard); each rank pairs its contiguous shard into a
    buffer on its own device and one all_gather_into_tensor (RCCL over xGMI with
    the nccl backend) returns all n results, (n, 48) int64, on every rank -- no
    host round trip.  `compute(P_shard, Q_shard, out)` fills `out`; by default
    the engine's bn_pairing_many_dev on `stream` (a torch.cuda.Stream, or the
    context's own stream), and torch's current stream -- where the collective
    is issued -- waits for it."""
    world, rank = dist.get_world_size(), dist.get_rank()
    n = P.shape[0]
    lo, hi = shard_bounds(n, rank, world)
    max_rows = max(shard_bounds(n, r, world)[1] - shard_bounds(n, r, world)[0] for r in range(world))
    # every buffer the engine reads or writes is made on torch's current stream
    # first (the contiguous copies of a non-contiguous P or Q included), and only
    # then does the engine stream wait for that stream
    buf = torch.zeros((max_rows, 48), dtype=torch.int64, device=P.device)
    ps = P[lo:hi].contiguous() if hi > lo else None
    qs = Q[lo:hi].contiguous() if hi > lo else None
    engine_stream = None
    if compute is None:
        from . import context
        ctx = context()
        engine_stream = stream if stream is not None else torch.cuda.ExternalStream(ctx.stream, device=P.device)
        engine_stream.wait_stream(torch.cuda.current_stream(P.device))  # inputs and buf are ready
        for t in (buf, ps, qs):  # the caching allocator must not reuse them before the engine is done
            if t is not None:
                t.record_stream(engine_stream)

        def compute(a, b, out):
            ctx.pairing_many_dev(a.data_ptr(), b.data_ptr(), a.shape[0], out.data_ptr(), engine_stream.cuda_stream)
    if hi > lo:
        compute(ps, qs, buf[:hi - lo])
    if engine_stream is not None:
        torch.cuda.current_stream(P.device).wait_stream(engine_stream)
    gathered = torch.empty((world * max_rows, 48), dtype=torch.int64, device=P.device)
    dist.all_gather_into_tensor(gathered, buf)
    if max_rows * world == n:
        return gathered
    return torch.cat([gathered[r * max_rows:r * max_rows + shard_bounds(n, r, world)[1]
                               - shard_bounds(n, r, world)[0]] for r in range(world)])


def pairing_batch_distributed(p, q, miller_product=None, fq12_mul=None, final_exp=None, device=None):
    """pairing_batch over the whole batch (mod.rs:904-926), identical Gt on every rank."""
    world, rank = dist.get_world_size(), dist.get_rank()
    n = p.shape[0]
    lo, hi = shard_bounds(n, rank, world)
    if miller_product is None:
        from . import context
        ctx = context()
        miller_product = lambda a, b: ctx.miller_loop_batch(b, a) if a.shape[0] else None  # noqa: E731
        fq12_mul = lambda a, b: ctx.fq12_op_many("mul", a, b)[0]  # noqa: E731
        final_exp = lambda f: ctx.final_exponentiation_many(f)  # noqa: E731
    # zero points are skipped (mod.rs:911-920): drop them before the product
    # (zero iff z == 0: G1 z is words 8..11, G2 z words 16..23)
    ps, qs = p[lo:hi], q[lo:hi]
    keep = ps[:, 8:12].any(axis=1) & qs[:, 16:24].any(axis=1)
    ps, qs = ps[keep], qs[keep]
    local = miller_product(ps, qs) if ps.shape[0] else None
    flag = np.zeros((1, 48), np.uint64)
    if local is not None:
        flag[0] = local
    have = np.array([[1 if local is not None else 0] + [0] * 47], dtype=np.uint64)
    parts = _gather_rows(np.concatenate([flag, have]), world, 2, device or _default_device())
    acc = None
    for r in range(world):  # fixed rank order: every rank computes the same product
        if parts[r][1, 0]:
            acc = parts[r][0] if acc is None else fq12_mul(acc, parts[r][0])
    if acc is None:  # nothing left: Fq12::one() (mod.rs:922-924)
        one = np.zeros(48, np.uint64)
        one[:4] = [0xd35d438dc58f0d9d, 0x0a78eb28f5c70b3d, 0x666ea36f7879462c, 0x0e0a77c19a07df2f]
        return one
    out, ok = final_exp(acc.reshape(1, 48))
    if not ok[0]:
        raise RuntimeError("miller loop cannot produce zero")
    return out[0]


def _default_device():
    if dist.get_backend() == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")
