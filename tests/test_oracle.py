"""Pin the CPU restatement oracle against the reference's own known-answer
vectors (tests/golden/reference_kats.json, extracted from /root/reference by
tests/golden/extract_reference_kats.py) and against the reference's property
tests (src/fields/tests.rs, src/groups/tests.rs, src/groups/mod.rs:1002-1124)."""
import numpy as np
import pytest

from oracle import oracle as O


def I(xs):
    return [int(x) for x in xs]


def test_str_minus_one(kats):
    """src/fields/mod.rs:68-81: -1 in Fr and Fq."""
    for field, key in ((O.FR, "fr_minus_one"), (O.FQ, "fq_minus_one")):
        one = O.canon_to_mont_array([1], field)
        neg, _ = O.unary("orc_fe_neg", one, 4, field)
        assert O.mont_array_to_canon(neg, field) == [int(kats["test_str"][key])]


def test_prepared_g2(kats):
    """src/groups/mod.rs:780-892: affine s2*G2 and all 87 line coefficients."""
    t = kats["test_prepared_g2"]
    q = O.g2_mul(O.g2_one(), O.canon_to_mont_array([int(t["g2_scalar"])], O.FR))
    qa, rc = O.g2_to_affine(q)
    assert rc == [0]
    assert O.mont_array_to_canon(qa[0]) == I(t["q_affine"]["x"] + t["q_affine"]["y"])
    c = O.g2_precompute(qa[0])
    assert c.shape == (87, 24)
    assert O.mont_array_to_canon(c.reshape(-1)) == [int(x) for row in t["coeffs"] for x in row]


def _g1g2(t):
    p = O.g1_mul(O.g1_one(), O.canon_to_mont_array([int(t["g1_scalar"])], O.FR))
    q = O.g2_mul(O.g2_one(), O.canon_to_mont_array([int(t["g2_scalar"])], O.FR))
    return p, q


def test_miller_loop(kats):
    """src/groups/mod.rs:643-691."""
    t = kats["test_miller_loop"]
    p, q = _g1g2(t)
    pa, _ = O.g1_to_affine(p)
    qa, _ = O.g2_to_affine(q)
    f = O.miller_loop(O.g2_precompute(qa[0]), pa[0, :4], pa[0, 4:])
    assert O.mont_array_to_canon(f) == I(t["f"])
    # miller_loop_batch of one pair is the same value (lib.rs:625-633)
    rc, fb = O.miller_loop_batch(q, p)
    assert rc == 0 and np.array_equal(fb, f)


def test_reduced_pairing(kats):
    """src/groups/mod.rs:929-999."""
    t = kats["test_reduced_pairing"]
    p, q = _g1g2(t)
    gt = O.pairing_many(p, q)
    assert O.mont_array_to_canon(gt[0]) == I(t["gt"])
    # final_exponentiation(miller_loop) == pairing
    rc, f = O.miller_loop_batch(q, p)
    fe, rcs = O.final_exponentiation(f)
    assert rcs == [0] and np.array_equal(fe[0], gt[0])


def test_fq12_test_vector(kats):
    """src/fields/mod.rs:94-227."""
    t = kats["fq12_test_vector"]
    start = O.canon_to_mont_array(I(t["start"]))
    nxt = start.copy()
    for _ in range(100):
        nxt = O.binary("orc_fq12_mul", nxt, start, 48, 48, 48)[0]
    cpy = nxt.copy()
    for _ in range(10):
        nxt = O.unary("orc_fq12_squared", nxt, 48)[0][0]
    for _ in range(10):
        nxt = O.binary("orc_fq12_add", nxt, start, 48, 48, 48)[0]
        nxt = O.binary("orc_fq12_sub", nxt, cpy, 48, 48, 48)[0]
        nxt = O.unary("orc_fq12_neg", nxt, 48)[0][0]
    nxt = O.unary("orc_fq12_squared", nxt, 48)[0][0]
    assert O.mont_array_to_canon(nxt) == I(t["finally"])


def test_cyclotomic_exp(kats):
    """src/fields/mod.rs:230-344."""
    t = kats["test_cyclotomic_exp"]
    e, _ = O.unary("orc_fq12_exp_by_neg_z", O.canon_to_mont_array(I(t["orig"])), 48)
    assert O.mont_array_to_canon(e[0]) == I(t["expected"])


def test_config1_one_pairing():
    """BASELINE config 1: e(G1::one(), G2::one()) -- the derived KAT of SURVEY.md §8(c)."""
    want = [17264119758069723980713015158403419364912226240334615592005620718956030922389,
            1300711225518851207585954685848229181392358478699795190245709208408267917898,
            8894217292938489450175280157304813535227569267786222825147475294561798790624,
            1829859855596098509359522796979920150769875799037311140071969971193843357227,
            4968700049505451466697923764727215585075098085662966862137174841375779106779,
            12814315002058128940449527172080950701976819591738376253772993495204862218736,
            4233474252585134102088637248223601499779641130562251948384759786370563844606,
            9420544134055737381096389798327244442442230840902787283326002357297404128074,
            13457906610892676317612909831857663099224588803620954529514857102808143524905,
            5122435115068592725432309312491733755581898052459744089947319066829791570839,
            8891987925005301465158626530377582234132838601606565363865129986128301774627,
            440796048150724096437130979851431985500142692666486515369083499585648077975]
    gt = O.pairing_many(O.g1_one(), O.g2_one())
    assert O.mont_array_to_canon(gt[0]) == want


def test_field_trials_small():
    """Restated subset of field_trials (src/fields/tests.rs:110-130) for Fq and Fr."""
    g = O.SplitMix64(103245)
    for field, m in ((O.FQ, O.P), (O.FR, O.R)):
        for _ in range(50):
            a, b, c = (g.below(m) for _ in range(3))
            A, B, C = (O.canon_to_mont_array([x], field) for x in (a, b, c))
            ab = O.binary("orc_fe_mul", A, B, 4, 4, 4, field)
            assert O.mont_array_to_canon(ab, field) == [a * b % m]
            s = O.binary("orc_fe_add", A, C, 4, 4, 4, field)
            assert O.mont_array_to_canon(s, field) == [(a + c) % m]
            d = O.binary("orc_fe_sub", A, C, 4, 4, 4, field)
            assert O.mont_array_to_canon(d, field) == [(a - c) % m]
            if a:
                inv, rc = O.unary("orc_fe_inverse", A, 4, field)
                assert rc == [0] and O.mont_array_to_canon(inv, field) == [pow(a, -1, m)]
        zero = O.canon_to_mont_array([0], field)
        _, rc = O.unary("orc_fe_inverse", zero, 4, field)
        assert rc == [1]


def test_bilinearity():
    """src/groups/mod.rs:1088-1124 (own seed; StdRng is not reproducible here)."""
    p, q, _, _ = O.random_pairs(3, seed=7)
    s_vals, s = O.random_scalars(3, seed=11)
    sp = O.g1_mul(p, s)
    sq = O.g2_mul(q, s)
    b = O.pairing_many(sp, q)
    c = O.pairing_many(p, sq)
    assert np.array_equal(b, c)
    a = O.pairing_many(p, q)
    for k in range(3):
        apow = O.binary("orc_fq12_pow", a[k], O.ints_to_array([s_vals[k]]), 48, 4, 48)
        assert np.array_equal(apow[0], b[k])


def test_pairing_batch_semantics():
    """pairing_batch (mod.rs:904-926): empty -> one, zero points skipped, equals Π e(P_i,Q_i)."""
    one = O.pairing_many(np.zeros((1, 12), np.uint64), np.zeros((1, 24), np.uint64))[0]
    gt_one = O.canon_to_mont_array([1] + [0] * 11)
    assert np.array_equal(one, gt_one)          # zero point -> Fq12::one() (mod.rs:896)
    assert np.array_equal(O.pairing_batch(np.zeros((0, 12), np.uint64), np.zeros((0, 24), np.uint64)), gt_one)
    p, q, _, _ = O.random_pairs(4, seed=3)
    prod = O.pairing_many(p, q)
    acc = prod[0]
    for k in range(1, 4):
        acc = O.binary("orc_fq12_mul", acc, prod[k], 48, 48, 48)[0]
    assert np.array_equal(O.pairing_batch(p, q), acc)
    # a zero G1 in the middle is skipped
    p2 = p.copy()
    p2[1] = 0
    p2[1, 4:8] = O.canon_to_mont_array([1])     # G1::zero() = (0, 1, 0)
    acc2 = O.binary("orc_fq12_mul", O.binary("orc_fq12_mul", prod[0], prod[2], 48, 48, 48)[0], prod[3], 48, 48, 48)[0]
    assert np.array_equal(O.pairing_batch(p2, q), acc2)
    # miller_loop_batch refuses a zero point (lib.rs:629-630)
    rc, _ = O.miller_loop_batch(q, p2)
    assert rc == 1


def test_pairing_batch_threads_match_shared_loop():
    """The threaded pairing_batch (the CPU baseline of config 5) splits the shared
    loop (mod.rs:609-640) into per-thread slices whose values are multiplied in
    order: the same Gt as the single shared loop, zero pairs and empty slices included."""
    p, q, _, _ = O.random_pairs(9, seed=41)
    p[4] = 0
    p[4, 4:8] = O.canon_to_mont_array([1])      # G1::zero() inside one slice
    ref = O.pairing_batch(p, q)
    for t in (1, 2, 3, 4, 9, 16):
        assert np.array_equal(O.pairing_batch(p, q, nthreads=t), ref), t
    # a slice with nothing but zero points, and all pairs skipped -> Gt::one()
    pz = p.copy()
    pz[:5] = 0
    pz[:5, 4:8] = O.canon_to_mont_array([1])
    assert np.array_equal(O.pairing_batch(pz, q, nthreads=3), O.pairing_batch(pz, q))
    gt_one = O.canon_to_mont_array([1] + [0] * 11)
    pz[:] = 0
    pz[:, 4:8] = O.canon_to_mont_array([1])
    assert np.array_equal(O.pairing_batch(pz, q, nthreads=4), gt_one)


def test_oracle_group_law_identities():
    """The oracle's group-law helpers (checkers of tests/test_gpu_group.py) agree with
    each other: P - P has z = 0, normalize keeps the point and sets z = one,
    -(-P) is P's image, (P + Q) - Q == P projectively."""
    p, q, _, _ = O.random_pairs(4, seed=77, nthreads=4)
    for a, w, add, sub, neg, norm, eq in ((p, 12, O.g1_add, O.g1_sub, O.g1_neg, O.g1_normalize, O.g1_eq),
                                          (q, 24, O.g2_add, O.g2_sub, O.g2_neg, O.g2_normalize, O.g2_eq)):
        b = a[::-1].copy()
        assert not sub(a, a)[:, 2 * w // 3:].any()
        na = norm(a)
        assert all(eq(a, na)) and not np.array_equal(na, a)
        assert np.array_equal(na[:, 2 * w // 3:2 * w // 3 + 4], np.tile(O.canon_to_mont_array([1]).reshape(4), (4, 1)))
        assert np.array_equal(neg(neg(a)), a)
        assert all(eq(sub(add(a, b), b), a))
