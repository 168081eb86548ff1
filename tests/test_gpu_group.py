"""The group law at the C ABI (bn_{g1,g2}_{add,sub,neg,normalize,eq}_many and their
_dev forms; lib.rs:388-423, 539-574, groups/mod.rs:169-216, 294-358) against the
oracle, bit for bit on the Jacobian images: random points with z != 1, zero
operands (both shortcuts of mod.rs:298-304), P + P and P + (the same point in
another Jacobian scaling) -- the doubling branch, mod.rs:315-316 --, P + (-P),
ragged sizes, and the device-pointer forms."""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu
NT = 16


def _zero(width):
    z = np.zeros(width, np.uint64)
    one = O.canon_to_mont_array([1]).reshape(4)
    z[width // 3:width // 3 + 4] = one  # (0, 1, 0): y = one (c0 of y for G2)
    return z


@pytest.fixture(scope="module")
def ctx():
    from substrate_bn import Context
    return Context(0)


@pytest.fixture(scope="module")
def pts():
    p, q, _, _ = O.random_pairs(257, seed=4242, nthreads=NT)
    p2, q2, _, _ = O.random_pairs(257, seed=4343, nthreads=NT)
    return {"g1": (p, p2), "g2": (q, q2)}


ORACLE = {
    "g1": {"add": O.g1_add, "sub": O.g1_sub, "neg": O.g1_neg, "normalize": O.g1_normalize, "eq": O.g1_eq},
    "g2": {"add": O.g2_add, "sub": O.g2_sub, "neg": O.g2_neg, "normalize": O.g2_normalize, "eq": O.g2_eq},
}
WIDTH = {"g1": 12, "g2": 24}


def _edge_operands(group, a, b):
    """a, b with the reference's special cases planted in the first rows."""
    a, b = a.copy(), b.copy()
    w = WIDTH[group]
    z = _zero(w)
    a[0], b[0] = z, b[0]            # zero + P -> P (mod.rs:298-300)
    a[1], b[1] = a[1], z            # P + zero -> P (mod.rs:302-304)
    a[2], b[2] = z, z               # zero + zero
    b[3] = a[3]                     # P + P: the doubling branch, same image
    b[4] = ORACLE[group]["normalize"](a[4:5])[0]  # P + P in another scaling: doubling branch
    b[5] = ORACLE[group]["neg"](a[5:6])[0]        # P + (-P): h = 0, s2 - s1 != 0 -> z3 = 0
    b[6] = ORACLE[group]["normalize"](ORACLE[group]["neg"](a[6:7]))[0]  # -P, another scaling
    return a, b


@pytest.mark.parametrize("group", ["g1", "g2"])
@pytest.mark.parametrize("op", ["add", "sub", "neg", "normalize", "eq"])
def test_group_law_host(ctx, pts, group, op):
    a, b = _edge_operands(group, *pts[group])
    for n in (1, 7, 257):
        got = ctx.group_op_many(group, op, a[:n], b[:n])
        if op == "eq":
            want = np.array(ORACLE[group]["eq"](a[:n], b[:n]), np.uint8)
        elif op in ("neg", "normalize"):
            want = ORACLE[group][op](a[:n])
        else:
            want = ORACLE[group][op](a[:n], b[:n])
        assert np.array_equal(got, want), (group, op, n)


@pytest.mark.parametrize("group", ["g1", "g2"])
def test_group_law_identities(ctx, pts, group):
    """Equalities the reference's law must satisfy: P == normalize(P), P - P is zero
    (z = 0), -(-P) == P, P + Q == Q + P, (P + Q) - Q == P (projective eq)."""
    a, b = pts[group]
    w = WIDTH[group]
    n = a.shape[0]
    norm = ctx.group_op_many(group, "normalize", a)
    assert ctx.group_op_many(group, "eq", a, norm).all()
    zero_z = ctx.group_op_many(group, "sub", a, a)[:, 2 * w // 3:]
    assert not zero_z.any()
    assert ctx.group_op_many(group, "eq", ctx.group_op_many(group, "neg", ctx.group_op_many(group, "neg", a)), a).all()
    s1 = ctx.group_op_many(group, "add", a, b)
    assert ctx.group_op_many(group, "eq", s1, ctx.group_op_many(group, "add", b, a)).all()
    assert ctx.group_op_many(group, "eq", ctx.group_op_many(group, "sub", s1, b), a).all()
    assert not ctx.group_op_many(group, "eq", a, ctx.group_op_many(group, "neg", a)).any()
    assert n == 257


@pytest.mark.parametrize("group", ["g1", "g2"])
def test_group_law_dev(ctx, pts, group):
    import torch
    dev = torch.device("cuda", 0)
    a, b = _edge_operands(group, *pts[group])
    n, w = a.shape
    da = torch.from_numpy(a.view(np.int64)).to(dev)
    db = torch.from_numpy(b.view(np.int64)).to(dev)
    s = torch.cuda.Stream(dev)
    for op in ("add", "sub", "neg", "normalize"):
        out = torch.zeros((n, w), dtype=torch.int64, device=dev)
        torch.cuda.synchronize(dev)  # s is not ordered after torch's stream
        ctx.group_op_many_dev(group, op, da.data_ptr(), db.data_ptr(), n, out.data_ptr(), s.cuda_stream)
        torch.cuda.synchronize(dev)
        want = ORACLE[group][op](a) if op in ("neg", "normalize") else ORACLE[group][op](a, b)
        assert np.array_equal(out.cpu().numpy().view(np.uint64), want), op
    # in place (out aliases a): each lane reads its element before it writes it
    inplace = da.clone()
    torch.cuda.synchronize(dev)
    ctx.group_op_many_dev(group, "normalize", inplace.data_ptr(), 0, n, inplace.data_ptr(), s.cuda_stream)
    torch.cuda.synchronize(dev)
    assert np.array_equal(inplace.cpu().numpy().view(np.uint64), ORACLE[group]["normalize"](a))
    eq = torch.full((n,), 7, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize(dev)
    ctx.group_op_many_dev(group, "eq", da.data_ptr(), db.data_ptr(), n, eq.data_ptr(), s.cuda_stream)
    torch.cuda.synchronize(dev)
    assert np.array_equal(eq.cpu().numpy(), np.array(ORACLE[group]["eq"](a, b), np.uint8))


def test_group_law_python_mirror(ctx):
    """G1/G2 operators of the Python mirror (lib.rs's Add/Sub/Neg/normalize/PartialEq)."""
    import substrate_bn as bn
    g = bn.G1.one()
    three = g * bn.Fr.from_int(3)
    assert (g + g + g) == three and (three - g - g) == g and -(-g) == g and (g - g).is_zero()
    t = bn.G2.one() * bn.Fr.from_int(5)
    u = bn.G2(t.img.copy())
    u.normalize()
    assert u == t and not u.same_image(t) and u.z() == bn.Fq2(np.concatenate([O.canon_to_mont_array([1]).reshape(4),
                                                                                 np.zeros(4, np.uint64)]))
    z = bn.G1.zero()
    z2 = bn.G1(z.img.copy())
    z2.normalize()
    assert z2.same_image(z)  # normalize leaves zero unchanged (to_affine is None)


def test_dev_status_clean(ctx):
    """bn_dev_status after status-less _dev calls that succeed: BN_OK."""
    import torch
    dev = torch.device("cuda", 0)
    p, q, _, _ = O.random_pairs(3, seed=5, nthreads=NT)
    P = torch.from_numpy(p.view(np.int64)).to(dev)
    Q = torch.from_numpy(q.view(np.int64)).to(dev)
    out = torch.zeros((3, 48), dtype=torch.int64, device=dev)
    torch.cuda.synchronize(dev)  # the context's own stream is not ordered after torch's
    ctx.pairing_many_dev(P.data_ptr(), Q.data_ptr(), 3, out.data_ptr())
    ctx.dev_status()
    assert np.array_equal(out.cpu().numpy().view(np.uint64), O.pairing_many(p, q, NT))
