"""Parity of the MI355X kernels (through the C ABI) with the CPU restatement
oracle of substrate-bn 0.6.0, bit-exact, plus the reference's known answers.
Runs on the GPU box: python -m pytest tests -m gpu."""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu
NT = 16  # oracle threads on the GPU box's host share


@pytest.fixture(scope="module")
def ctx():
    from substrate_bn import Context
    return Context(0)


@pytest.fixture(scope="module")
def ctx_tp():
    """A context whose every pairing_many batch takes the THROUGHPUT path
    (k_pairing_full, the kernel bench.py's `value` measures): the latency-path
    threshold is 0."""
    from substrate_bn import Context
    c = Context(0)
    c.set_fe_wide_max(0)
    return c


@pytest.fixture(scope="module")
def ctx_seg():
    """A context whose small pairing_many batches take the segmented latency path
    (k_prepare_wide + k_miller_seg + k_horner_wide) instead of the one-launch
    k_pairing_latency."""
    from substrate_bn import Context
    c = Context(0)
    c.set_latency_max(0)
    return c


@pytest.fixture(scope="module")
def pairs():
    p, q, s, t = O.random_pairs(256, seed=1234, nthreads=NT)
    return p, q


def rnd_fq12(n, seed):
    g = O.SplitMix64(seed)
    return O.canon_to_mont_array([g.below(O.P) for _ in range(12 * n)]).reshape(n, 48)


def test_fq12_ops(ctx):
    a, b = rnd_fq12(64, 1), rnd_fq12(64, 2)
    assert np.array_equal(ctx.fq12_op_many("mul", a, b), O.binary("orc_fq12_mul", a, b, 48, 48, 48))
    assert np.array_equal(ctx.fq12_op_many("sqr", a), O.unary("orc_fq12_squared", a, 48)[0])
    assert np.array_equal(ctx.fq12_op_many("inv", a), O.unary("orc_fq12_inverse", a, 48)[0])
    assert np.array_equal(ctx.fq12_op_many("cyc_sqr", a), O.unary("orc_fq12_cyclotomic_squared", a, 48)[0])
    assert np.array_equal(ctx.fq12_op_many("exp_by_neg_z", a[:16]), O.unary("orc_fq12_exp_by_neg_z", a[:16], 48)[0])
    for pw in (1, 2, 3):
        want = np.zeros_like(a)
        for k in range(a.shape[0]):
            O.lib().orc_fq12_frobenius_map(O._p(a[k]), pw, O._p(want[k]))
        assert np.array_equal(ctx.fq12_op_many("frob%d" % pw, a), want)


def test_cyclotomic_exp_kat(ctx, kats):
    t = kats["test_cyclotomic_exp"]  # src/fields/mod.rs:230-344
    got = ctx.fq12_op_many("exp_by_neg_z", O.canon_to_mont_array([int(x) for x in t["orig"]]))
    assert O.mont_array_to_canon(got[0]) == [int(x) for x in t["expected"]]


def test_g1_mul(ctx, pairs):
    p, _ = pairs
    ks, K = O.random_scalars(256, seed=77, lo=0)
    assert np.array_equal(ctx.g1_mul_many(p, K), O.g1_mul(p, K, NT))
    # edges: zero point, scalars 0, 1, r-1, 2^254-ish
    z = np.zeros(12, np.uint64)
    z[4:8] = O.canon_to_mont_array([1])
    edge_p = np.stack([z, p[0], p[1], p[2], p[3]])
    edge_k = O.canon_to_mont_array([5, 0, 1, O.R - 1, (1 << 253) + 12345], O.FR).reshape(5, 4)
    assert np.array_equal(ctx.g1_mul_many(edge_p, edge_k), O.g1_mul(edge_p, edge_k))


def test_g2_mul(ctx, pairs):
    _, q = pairs
    ks, K = O.random_scalars(64, seed=78)
    assert np.array_equal(ctx.g2_mul_many(q[:64], K), O.g2_mul(q[:64], K, NT))


def test_reference_kats(ctx, kats):
    t = kats["test_reduced_pairing"]  # src/groups/mod.rs:929-999
    p = O.g1_mul(O.g1_one(), O.canon_to_mont_array([int(t["g1_scalar"])], O.FR))
    q = O.g2_mul(O.g2_one(), O.canon_to_mont_array([int(t["g2_scalar"])], O.FR))
    gt = ctx.pairing_many(p, q)
    assert O.mont_array_to_canon(gt[0]) == [int(x) for x in t["gt"]]
    m = kats["test_miller_loop"]  # src/groups/mod.rs:643-691
    f = ctx.miller_loop_many(p, q)
    assert O.mont_array_to_canon(f[0]) == [int(x) for x in m["f"]]
    f2 = ctx.miller_loop_batch(q, p)
    assert np.array_equal(f2, f[0])


def test_config1(ctx):
    """e(G1::one(), G2::one()) == oracle (BASELINE config 1)."""
    assert np.array_equal(ctx.pairing_many(O.g1_one(), O.g2_one()), O.pairing_many(O.g1_one(), O.g2_one()))


def test_pairing_many(ctx, pairs):
    p, q = pairs
    assert np.array_equal(ctx.pairing_many(p, q), O.pairing_many(p, q, NT))


def test_miller_and_final_exp(ctx, pairs):
    p, q = pairs
    f = ctx.miller_loop_many(p[:64], q[:64])
    want_f = np.stack([O.miller_loop_batch(q[k], p[k])[1] for k in range(64)])
    assert np.array_equal(f, want_f)
    fe, ok = ctx.final_exponentiation_many(f)
    assert ok.all() and np.array_equal(fe, O.pairing_many(p[:64], q[:64], NT))
    # f == 0 -> None (fq12.rs:63-72)
    fe0, ok0 = ctx.final_exponentiation_many(np.zeros((2, 48), np.uint64))
    assert not ok0.any() and not fe0.any()


def test_zero_points(ctx, pairs):
    """pairing() of a zero point is Fq12::one() (mod.rs:896)."""
    p, q = pairs
    p2, q2 = p[:4].copy(), q[:4].copy()
    one = O.canon_to_mont_array([1])
    p2[1] = 0
    p2[1, 4:8] = one                 # G1::zero()
    q2[2] = 0
    q2[2, 8:12] = one                # G2::zero(): y = (1, 0)
    assert np.array_equal(ctx.pairing_many(p2, q2), O.pairing_many(p2, q2))


@pytest.mark.parametrize("n", [1, 63, 65, 129, 255])
def test_pairing_many_ragged(ctx, pairs, n):
    """Batch sizes that leave a partial wave / workgroup, with zero points in the tail lanes."""
    p, q = pairs
    p2, q2 = p[:n].copy(), q[:n].copy()
    one = O.canon_to_mont_array([1])
    p2[n - 1] = 0
    p2[n - 1, 4:8] = one             # G1::zero() in the last lane
    if n > 2:
        q2[n - 2] = 0
        q2[n - 2, 8:12] = one        # G2::zero() in the lane before it
    assert np.array_equal(ctx.pairing_many(p2, q2), O.pairing_many(p2, q2, NT))
    assert np.array_equal(ctx.pairing_batch(p2, q2), O.pairing_batch(p2, q2))


@pytest.mark.parametrize("n", [0, 1, 5, 64])
def test_pairing_batch(ctx, pairs, n):
    p, q = pairs
    p2, q2 = p[:n].copy(), q[:n].copy()
    if n >= 5:
        p2[3] = 0
        p2[3, 4:8] = O.canon_to_mont_array([1])   # skipped pair
    assert np.array_equal(ctx.pairing_batch(p2, q2), O.pairing_batch(p2, q2))


def test_miller_loop_batch(ctx, pairs):
    from substrate_bn import BnError
    p, q = pairs
    rc, want = O.miller_loop_batch(q[:33], p[:33])
    assert rc == 0 and np.array_equal(ctx.miller_loop_batch(q[:33], p[:33]), want)
    p2 = p[:3].copy()
    p2[1] = 0
    with pytest.raises(BnError):
        ctx.miller_loop_batch(q[:3], p2)


def test_rust_api_mirror(ctx):
    """The substrate_bn mirror reads like the reference's own tests."""
    import substrate_bn as bn
    s = bn.Fr.from_int(0x1234567)
    a = bn.pairing(bn.G1.one() * s, bn.G2.one())
    b = bn.pairing(bn.G1.one(), bn.G2.one() * s)
    assert a == b and a != bn.Gt.one()
    assert bn.pairing(bn.G1.zero(), bn.G2.one()) == bn.Gt.one()
    assert bn.pairing_batch([]) == bn.Gt.one()
    with pytest.raises(bn.CurveError):
        bn.miller_loop_batch([(bn.G2.one(), bn.G1.zero())])
    assert bn.miller_loop_batch([(bn.G2.one(), bn.G1.one())]).final_exponentiation() == \
        bn.pairing(bn.G1.one(), bn.G2.one())


def test_large_batch_parity_and_bilinearity(ctx):
    """4096 pairings bit-exact vs the oracle, then the size-independent checks at
    2^16 (BASELINE config 2): bilinearity e(sP, Q) == e(P, sQ) on every lane."""
    p, q, _, _ = O.random_pairs(4096, seed=4096, nthreads=NT)
    got = ctx.pairing_many(p, q)
    assert np.array_equal(got, O.pairing_many(p, q, NT))
    n = 1 << 16
    s_vals, S = O.random_scalars(n, seed=7)
    base1 = np.tile(O.g1_one(), (n, 1))
    base2 = np.tile(O.g2_one(), (n, 1))
    P = ctx.g1_mul_many(base1, S)
    Q = ctx.g2_mul_many(base2, np.roll(S, 1, axis=0))
    sP = ctx.g1_mul_many(P, np.roll(S, 2, axis=0))
    sQ = ctx.g2_mul_many(Q, np.roll(S, 2, axis=0))
    e1 = ctx.pairing_many(sP, Q)
    e2 = ctx.pairing_many(P, sQ)
    assert np.array_equal(e1, e2)
    # spot-check a sample of lanes against the oracle
    idx = np.random.default_rng(0).choice(n, 256, replace=False)
    assert np.array_equal(e1[idx], O.pairing_many(sP[idx], Q[idx], NT))


def test_config2_full_size_every_row(ctx_tp):
    """BASELINE config 2 at its full size on the kernel bench.py measures
    (k_pairing_full): 2^16 random pairs with random Jacobian z (not one), every
    Gt image bit-exact against the oracle (~7 s of 16 host threads)."""
    n = 1 << 16
    _, S = O.random_scalars(n, seed=2020, lo=1)
    P = ctx_tp.g1_mul_many(np.tile(O.g1_one(), (n, 1)), S)
    Q = ctx_tp.g2_mul_many(np.tile(O.g2_one(), (n, 1)), np.roll(S, 5, axis=0))
    got = ctx_tp.pairing_many(P, Q)
    assert np.array_equal(got, O.pairing_many(P, Q, NT))


def test_prepared_g2_on_gpu(ctx, kats, pairs):
    """All 87 line coefficients computed on the GPU (bn_g2_precompute_many):
    the reference's test_prepared_g2 vector (src/groups/mod.rs:780-892) and 64
    random points against the oracle's G2Precomp, bit for bit; a zero point is
    ToAffineConversion."""
    from substrate_bn import BnError
    t = kats["test_prepared_g2"]
    q = O.g2_mul(O.g2_one(), O.canon_to_mont_array([int(t["g2_scalar"])], O.FR))
    c = ctx.g2_precompute_many(q)
    assert c.shape == (1, 87, 24)
    assert O.mont_array_to_canon(c.reshape(-1)) == [int(x) for row in t["coeffs"] for x in row]
    _, qs = pairs
    got = ctx.g2_precompute_many(qs[:64])
    for k in range(64):
        qa, rc = O.g2_to_affine(qs[k])
        assert rc == [0] and np.array_equal(got[k], O.g2_precompute(qa[0])), k
    z = qs[:2].copy()
    z[1] = 0
    z[1, 8:12] = O.canon_to_mont_array([1])   # G2::zero()
    with pytest.raises(BnError):
        ctx.g2_precompute_many(z)


def test_config3_g1_mul_full_size(ctx):
    """BASELINE config 3 at its full size: 2^18 G1 * Fr on random Jacobian bases and
    uniform scalars, every lane bit-exact (raw Jacobian image) against the oracle."""
    n = 1 << 18
    _, S = O.random_scalars(n, seed=333, lo=0)
    base = ctx.g1_mul_many(np.tile(O.g1_one(), (n, 1)), np.roll(S, 7, axis=0))  # random Jacobian bases (z != 1)
    got = ctx.g1_mul_many(base, S)
    assert np.array_equal(got, O.g1_mul(base, S, NT))


def test_g1_mul_two_chain_odd_tail(ctx):
    """The two-chains-per-lane kernel (k_g1_mul2, lane i runs rows i and i + h,
    h = ceil(n / 2)) at an odd size: the last lane has one chain.  Zero bases, zero
    scalars, k = 1 and k = r - 1 planted in both halves; rows around 0, h and the
    tail checked against the oracle."""
    n = (1 << 18) + 3
    h = (n + 1) // 2
    _, S = O.random_scalars(n, seed=444, lo=0)
    base = ctx.g1_mul_many(np.tile(O.g1_one(), (n, 1)), np.roll(S, 11, axis=0))
    one = O.canon_to_mont_array([1]).reshape(4)
    for row in (1, h + 1, n - 1):
        base[row] = 0
        base[row, 4:8] = one                          # G1::zero()
    S[[2, h + 2, n - 2]] = 0
    S[[3, h + 3]] = O.canon_to_mont_array([1], O.FR).reshape(4)
    S[[4, h + 4]] = O.canon_to_mont_array([O.R - 1], O.FR).reshape(4)
    got = ctx.g1_mul_many(base, S)
    rows = np.r_[0:64, h - 64:h + 64, n - 64:n]
    assert np.array_equal(got[rows], O.g1_mul(base[rows], S[rows], NT))


@pytest.mark.parametrize("n", [(1 << 16) + 1, (1 << 17) + 3])
def test_g2_mul_two_chain_odd_tail(ctx, n):
    """G2 * Fr at odd sizes past 2^16 (k_g2_mul_split; written for the two-chains-per-pair
    kernels of profiles/r5s_ab_g2_mul2.txt, which ran pair i on rows i and i + h).  Zero
    bases, zero scalars, k = 1 and k = r - 1 planted in both halves; rows around 0,
    h = ceil(n / 2) and the tail checked against the oracle on the raw Jacobian image."""
    h = (n + 1) // 2
    _, S = O.random_scalars(n, seed=555 + n % 7, lo=0)
    base = ctx.g2_mul_many(np.tile(O.g2_one(), (n, 1)), np.roll(S, 13, axis=0))  # z != 1
    one = O.canon_to_mont_array([1]).reshape(4)
    for row in (1, h + 1, n - 1):
        base[row] = 0
        base[row, 8:12] = one                         # G2::zero(): y = (1, 0)
    S[[2, h + 2, n - 2]] = 0
    S[[3, h + 3]] = O.canon_to_mont_array([1], O.FR).reshape(4)
    S[[4, h + 4]] = O.canon_to_mont_array([O.R - 1], O.FR).reshape(4)
    got = ctx.g2_mul_many(base, S)
    rows = np.r_[0:48, h - 48:h + 48, n - 48:n]
    assert np.array_equal(got[rows], O.g2_mul(base[rows], S[rows], NT))


# ---- the throughput path (the kernels `value` measures) on the edge cases, vs the oracle
def test_throughput_path_pairing_many(ctx_tp, pairs):
    p, q = pairs
    assert np.array_equal(ctx_tp.pairing_many(p, q), O.pairing_many(p, q, NT))


def test_throughput_path_zero_points(ctx_tp, pairs):
    """pairing() of a zero point is Fq12::one() (mod.rs:896), on k_pairing_full (a.skip)."""
    p, q = pairs
    p2, q2 = p[:4].copy(), q[:4].copy()
    one = O.canon_to_mont_array([1])
    p2[1] = 0
    p2[1, 4:8] = one                 # G1::zero()
    q2[2] = 0
    q2[2, 8:12] = one                # G2::zero(): y = (1, 0)
    assert np.array_equal(ctx_tp.pairing_many(p2, q2), O.pairing_many(p2, q2))


@pytest.mark.parametrize("n", [1, 63, 65, 129, 255, 257, 511, 513])
def test_throughput_path_ragged(ctx_tp, pairs, n):
    """Sizes that leave partial waves and partial 512-thread blocks of the
    balanced kernels, with zero points in the tail lanes (src/groups/mod.rs:894-902)."""
    p, q = pairs
    reps = (n + p.shape[0] - 1) // p.shape[0]
    p2, q2 = np.tile(p, (reps, 1))[:n].copy(), np.tile(q, (reps, 1))[:n].copy()
    one = O.canon_to_mont_array([1])
    p2[n - 1] = 0
    p2[n - 1, 4:8] = one             # G1::zero() in the last lane
    if n > 2:
        q2[n - 2] = 0
        q2[n - 2, 8:12] = one        # G2::zero() in the lane before it
    assert np.array_equal(ctx_tp.pairing_many(p2, q2), O.pairing_many(p2, q2, NT))


@pytest.mark.parametrize("form", [0, 1, 2])
def test_throughput_path_other_forms(pairs, form, monkeypatch):
    """The A/B forms of the throughput path (BN254MI_MILLER_FORM):
    0 = k_prepare + k_miller, 1 = k_pairing_fused, 2 = k_prepare + k_miller_seg (one
    segment), each followed by k_fq12_vm + k_fe_out -- the same Gt as k_pairing_full,
    zero points included."""
    from substrate_bn import Context
    monkeypatch.setenv("BN254MI_MILLER_FORM", str(form))
    c = Context(0)
    c.set_fe_wide_max(0)
    p, q = pairs
    p2, q2 = np.concatenate([p, p[:44]]), np.concatenate([q, q[:44]])  # 300 pairs
    one = O.canon_to_mont_array([1])
    p2[7] = 0
    p2[7, 4:8] = one
    q2[299] = 0
    q2[299, 8:12] = one
    assert np.array_equal(c.pairing_many(p2, q2), O.pairing_many(p2, q2, NT))


def test_throughput_path_4096_and_final_exp(ctx_tp):
    """4096 random pairings through the throughput kernels bit-exact against the
    oracle; the step-machine final exponentiation alone on their Miller values,
    a zero value included (fq12.rs:63-72 returns None)."""
    p, q, _, _ = O.random_pairs(4096, seed=4097, nthreads=NT)
    want = O.pairing_many(p, q, NT)
    assert np.array_equal(ctx_tp.pairing_many(p, q), want)
    f = ctx_tp.miller_loop_many(p[:300], q[:300])
    f[7] = 0
    fe, ok = ctx_tp.final_exponentiation_many(f)
    assert ok[7] == 0 and not fe[7].any()
    keep = np.ones(300, bool)
    keep[7] = False
    assert ok[keep].all() and np.array_equal(fe[keep], want[:300][keep])


@pytest.mark.parametrize("n", [1, 7, 8, 9, 63, 255])
def test_latency_paths_ragged(ctx, ctx_seg, pairs, n):
    """Both latency-path forms -- the one-launch k_pairing_latency (ctx: 8 pairs
    per block, partial blocks, idle producer slots) and the segmented kernels
    (ctx_seg) -- against the oracle, zero points in the tail lanes."""
    p, q = pairs
    p2, q2 = p[:n].copy(), q[:n].copy()
    one = O.canon_to_mont_array([1])
    p2[n - 1] = 0
    p2[n - 1, 4:8] = one
    if n > 2:
        q2[n - 2] = 0
        q2[n - 2, 8:12] = one
    want = O.pairing_many(p2, q2, NT)
    assert np.array_equal(ctx.pairing_many(p2, q2), want)
    assert np.array_equal(ctx_seg.pairing_many(p2, q2), want)


def test_latency_kernel_1024(ctx, pairs):
    """1024 pairs (the default k_pairing_latency threshold: 128 blocks) bit-exact."""
    p, q, _, _ = O.random_pairs(1024, seed=1025, nthreads=NT)
    assert np.array_equal(ctx.pairing_many(p, q), O.pairing_many(p, q, NT))


@pytest.fixture(scope="module")
def ctx_w2():
    """A context whose one-launch latency path reaches 4,096 pairs: above 2,048 it
    runs the two-wave build k_pairing_latency_w2 (kernels_latency_w2.hip)."""
    from substrate_bn import Context
    c = Context(0)
    c.set_latency_max(4096)
    return c


@pytest.mark.parametrize("n", [2049, 3001, 4096])
def test_latency_kernel_two_wave_build(ctx_w2, n):
    """k_pairing_latency_w2 (two blocks per CU: six-line ring, one-item FE channel,
    squarings by w12_mul) bit-exact against the oracle, with zero points on both
    sides and a partial last block; pairing_batch and miller_loop_batch take the
    same kernel for their Miller values (f_out mode)."""
    p, q, _, _ = O.random_pairs(n, seed=7000 + n, nthreads=NT)
    one = O.canon_to_mont_array([1])
    p[n - 1] = 0
    p[n - 1, 4:8] = one
    q[5] = 0
    q[5, 8:12] = one
    want = O.pairing_many(p, q, NT)
    assert np.array_equal(ctx_w2.pairing_many(p, q), want)
    if n == 3001:
        assert np.array_equal(ctx_w2.pairing_batch(p, q), O.pairing_batch(p, q))
        _, mlb = O.miller_loop_batch(q[6:n - 1], p[6:n - 1])  # rows without a zero point
        assert np.array_equal(ctx_w2.miller_loop_batch(q[6:n - 1], p[6:n - 1]), mlb)
