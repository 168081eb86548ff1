"""The latency path (16-lane groups, kernels_wide.hip) against the oracle:
final exponentiation on both layouts, the device product reduction behind
pairing_batch / miller_loop_batch (mod.rs:609-640, 904-926), their
device-pointer forms, and BASELINE config 5 (a 2^14-term pairing product).
Runs on the GPU box: python -m pytest tests -m gpu."""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu
NT = 16


@pytest.fixture(scope="module")
def ctx():
    from substrate_bn import Context
    return Context(0)


@pytest.fixture(scope="module")
def pairs():
    p, q, _, _ = O.random_pairs(512, seed=2024, nthreads=NT)
    return p, q


def _dev(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to("cuda:0")


def test_final_exp_both_layouts(ctx, pairs):
    """The same Miller values through the 16-lane FE and the two-lane step
    machine: identical, and equal to the oracle; zero -> None on both."""
    p, q = pairs
    f = ctx.miller_loop_many(p[:40], q[:40])
    f = np.concatenate([f, np.zeros((1, 48), np.uint64), O.canon_to_mont_array([1] + [0] * 11)[None, :]])
    want = O.final_exponentiation(f)[0]
    try:
        ctx.set_fe_wide_max(1 << 20)
        wide, ok_w = ctx.final_exponentiation_many(f)
        ctx.set_fe_wide_max(0)
        vm, ok_v = ctx.final_exponentiation_many(f)
    finally:
        ctx.set_fe_wide_max(8192)
    assert np.array_equal(wide, vm) and np.array_equal(ok_w, ok_v)
    assert list(ok_w) == [1] * 40 + [0, 1]
    assert np.array_equal(wide, want)


@pytest.mark.parametrize("n", [1, 2, 17, 31, 32, 33, 100, 1025])
def test_pairing_many_small_batches_wide(ctx, pairs, n):
    """pairing_many below the wide threshold (FE on 16-lane groups), partial
    groups and blocks, a zero point included."""
    p, q = pairs
    reps = (n + 511) // 512
    p2, q2 = np.tile(p, (reps, 1))[:n].copy(), np.tile(q, (reps, 1))[:n].copy()
    for z in (2, 514):  # G1::zero() in both copies of row 2
        if z < n and n > 3:
            p2[z] = 0
            p2[z, 4:8] = O.canon_to_mont_array([1])
    got = ctx.pairing_many(p2, q2)
    u = min(n, 512)
    assert np.array_equal(got[:u], O.pairing_many(p2[:u], q2[:u], NT))
    if n > 512:
        assert np.array_equal(got[512:], got[:n - 512])


@pytest.mark.parametrize("n", [2, 31, 32, 33, 64, 1023, 1025])
def test_pairing_batch_reduction_sizes(ctx, pairs, n):
    """Device product reduction (32 factors per block, several levels) for sizes
    around the block and level boundaries."""
    p, q = pairs
    reps = (n + 511) // 512
    p2, q2 = np.tile(p, (reps, 1))[:n], np.tile(q, (reps, 1))[:n]
    assert np.array_equal(ctx.pairing_batch(p2, q2), O.pairing_batch(p2, q2, nthreads=NT))
    rc, want = O.miller_loop_batch(q2, p2)
    assert rc == 0 and np.array_equal(ctx.miller_loop_batch(q2, p2), want)


def test_batch_dev_forms(ctx, pairs):
    """bn_pairing_batch_dev / bn_miller_loop_batch_dev on HBM-resident inputs,
    device status word included."""
    import torch
    p, q = pairs
    n = 77
    P, Q = _dev(p[:n]), _dev(q[:n])
    out = torch.zeros(48, dtype=torch.int64, device="cuda:0")
    st = torch.full((1,), -1, dtype=torch.int32, device="cuda:0")
    ctx.pairing_batch_dev(P.data_ptr(), Q.data_ptr(), n, out.data_ptr(), st.data_ptr())
    torch.cuda.synchronize()
    assert int(st.item()) == 0
    assert np.array_equal(out.cpu().numpy().view(np.uint64), O.pairing_batch(p[:n], q[:n], nthreads=NT))
    ctx.miller_loop_batch_dev(Q.data_ptr(), P.data_ptr(), n, out.data_ptr(), st.data_ptr())
    torch.cuda.synchronize()
    assert int(st.item()) == 0
    assert np.array_equal(out.cpu().numpy().view(np.uint64), O.miller_loop_batch(q[:n], p[:n])[1])
    # a zero point: ToAffineConversion for miller_loop_batch (lib.rs:629-630), skipped by pairing_batch
    p2 = p[:n].copy()
    p2[5] = 0
    p2[5, 4:8] = O.canon_to_mont_array([1])
    P2 = _dev(p2)
    ctx.miller_loop_batch_dev(Q.data_ptr(), P2.data_ptr(), n, out.data_ptr(), st.data_ptr())
    torch.cuda.synchronize()
    assert int(st.item()) == 2  # BN_ERR_TO_AFFINE
    ctx.pairing_batch_dev(P2.data_ptr(), Q.data_ptr(), n, out.data_ptr(), st.data_ptr())
    torch.cuda.synchronize()
    assert int(st.item()) == 0
    assert np.array_equal(out.cpu().numpy().view(np.uint64), O.pairing_batch(p2, q[:n], nthreads=NT))
    # empty batch -> Gt::one() (mod.rs:922-924)
    ctx.pairing_batch_dev(P.data_ptr(), Q.data_ptr(), 0, out.data_ptr(), st.data_ptr())
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy().view(np.uint64), O.canon_to_mont_array([1] + [0] * 11))


def test_config5_product_2_14(ctx):
    """BASELINE config 5: one pairing_batch over 2^14 random terms (HBM-resident
    inputs through the device-pointer form), bit-exact against the oracle's
    pairing_batch (shared loop split over threads, tests/test_oracle.py)."""
    import torch
    n = 1 << 14
    p, q, _, _ = O.random_pairs(n, seed=514, nthreads=NT)
    P, Q = _dev(p), _dev(q)
    out = torch.zeros(48, dtype=torch.int64, device="cuda:0")
    st = torch.full((1,), -1, dtype=torch.int32, device="cuda:0")
    ctx.pairing_batch_dev(P.data_ptr(), Q.data_ptr(), n, out.data_ptr(), st.data_ptr())
    torch.cuda.synchronize()
    assert int(st.item()) == 0
    assert np.array_equal(out.cpu().numpy().view(np.uint64), O.pairing_batch(p, q, nthreads=NT))


def test_product_ragged_reduction_chains(ctx):
    """A 12,345-term pairing_batch and miller_loop_batch: K = 2 pairs per lane pair,
    6,173 segment values per set, so the first reduction level runs chains of
    G = 16 factors per group with a ragged last block (capi.hip product_wide), the
    second a single block; bit-exact against the oracle."""
    n = 12345
    p, q, _, _ = O.random_pairs(n, seed=12345, nthreads=NT)
    assert np.array_equal(ctx.pairing_batch(p, q), O.pairing_batch(p, q, nthreads=NT))
    rc, want = O.miller_loop_batch(q[:4099], p[:4099])
    assert rc == 0 and np.array_equal(ctx.miller_loop_batch(q[:4099], p[:4099]), want)


def test_product_across_chunks_is_one(ctx):
    """2^18 + 2 terms (two chunks of the reduction): pairs (s_i G1, t_i G2) and
    ((r - s_i) G1, t_i G2), so the product is e(G1, G2)^(r t) = Gt::one() --
    a size-independent check of the multi-chunk reduction."""
    import torch
    from substrate_bn import synth
    half = (1 << 17) + 1
    s, t = synth.dataset_scalars(0, half)
    # Montgomery image of r - s is r - image(s) (images are canonical, nonzero)
    neg = O.ints_to_array([O.R - v for v in O.array_to_ints(s)]).reshape(half, 4)
    k1 = _dev(np.concatenate([s, neg]))
    k2 = _dev(np.concatenate([t, t]))
    n = 2 * half
    g1 = _dev(np.tile(synth.g1_one_image(), (n, 1)))
    g2 = _dev(np.tile(synth.g2_one_image(), (n, 1)))
    P = torch.empty((n, 12), dtype=torch.int64, device="cuda:0")
    Q = torch.empty((n, 24), dtype=torch.int64, device="cuda:0")
    ctx.g1_mul_many_dev(g1.data_ptr(), k1.data_ptr(), n, P.data_ptr())
    ctx.g2_mul_many_dev(g2.data_ptr(), k2.data_ptr(), n, Q.data_ptr())
    torch.cuda.synchronize()
    out = torch.zeros(48, dtype=torch.int64, device="cuda:0")
    st = torch.full((1,), -1, dtype=torch.int32, device="cuda:0")
    ctx.pairing_batch_dev(P.data_ptr(), Q.data_ptr(), n, out.data_ptr(), st.data_ptr())
    torch.cuda.synchronize()
    assert int(st.item()) == 0
    assert np.array_equal(out.cpu().numpy().view(np.uint64), O.canon_to_mont_array([1] + [0] * 11))


@pytest.mark.parametrize("tree", ["1", "0"])
def test_segmented_product_recombination(ctx, tree, monkeypatch):
    """Products above the one-launch size (4,500 terms: prepare + 16 segments of
    the shared-squaring loop + reduction) through both recombination kernels:
    k_horner_tree (the segments' squarings side by side, then a product tree;
    default) and k_horner_wide (Horner's rule on one group, BN254MI_HORNER_TREE=0)
    -- pairing_batch and miller_loop_batch (no final exponentiation) bit-exact
    against the oracle (mod.rs:609-640, 904-926)."""
    monkeypatch.setenv("BN254MI_HORNER_TREE", tree)
    n = 4500
    p, q, _, _ = O.random_pairs(n, seed=77, nthreads=NT)
    p[4400] = 0  # a zero point: skipped by pairing_batch (outside the miller_loop_batch slice)
    p[4400, 4:8] = O.canon_to_mont_array([1])
    assert np.array_equal(ctx.pairing_batch(p, q), O.pairing_batch(p, q, nthreads=NT))
    rc, want = O.miller_loop_batch(q[:4200], p[:4200])
    assert rc == 0 and np.array_equal(ctx.miller_loop_batch(q[:4200], p[:4200]), want)
