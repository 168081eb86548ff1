"""The engine's kernel formulas (paritytech-bn_amd/csrc/*.h), compiled for the
host, against the oracle -- bit-exact.  CPU-only; the same headers compile
into the gfx950 kernels that tests/test_gpu_*.py check on the MI355X."""
import numpy as np
import pytest

from oracle import oracle as O
from tests.native import hostemul as H


@pytest.fixture(scope="module")
def rnd():
    g = O.SplitMix64(2024)
    return lambda n, m=O.P: [g.below(m) for _ in range(n)]


def fe(vals):
    return O.canon_to_mont_array(vals)


def test_fq_ops(rnd):
    a, b = rnd(40), rnd(40)
    A, B = fe(a).reshape(-1, 4), fe(b).reshape(-1, 4)
    for k in range(40):
        assert O.mont_array_to_canon(H.call("he_fq_mul", A[k], B[k], out_words=8)) == [a[k] * b[k] % O.P]
        assert O.mont_array_to_canon(H.call("he_fq_add", A[k], B[k], out_words=8)) == [(a[k] + b[k]) % O.P]
        assert O.mont_array_to_canon(H.call("he_fq_sub", A[k], B[k], out_words=8)) == [(a[k] - b[k]) % O.P]
        assert O.mont_array_to_canon(H.call("he_fq_neg", A[k], out_words=8)) == [(-a[k]) % O.P]
    # edge values
    for v in (0, 1, O.P - 1, O.P - 2, 2 ** 253, 2 ** 254 % O.P):
        X = fe([v])
        assert O.mont_array_to_canon(H.call("he_fq_mul", X, X, out_words=8)) == [v * v % O.P]
        assert O.mont_array_to_canon(H.call("he_fq_neg", X, out_words=8)) == [(-v) % O.P]
        if v:
            assert O.mont_array_to_canon(H.call("he_fq_inv", X, out_words=8)) == [pow(v, -1, O.P)]


def test_fq_inv_binary_gcd_sweep(rnd):
    # fq_inv is the 19-round binary GCD (tower.h fq_inv_bgcd): random values,
    # small values, powers of two, values next to p and to 2^254, 1 and p - 1;
    # the host build aborts if a round count ever falls short (BN_HOST_CHECKS)
    g = O.SplitMix64(77)
    vals = rnd(600) + list(range(1, 40)) + [1 << k for k in range(254)] + [O.P - 1 - k for k in range(40)]
    vals += [(1 << 253) + g.below(1 << 64) for _ in range(40)] + [O.P // 3, O.P // 2, (O.P + 1) // 2]
    X = fe(vals).reshape(-1, 4)
    for k, v in enumerate(vals):
        assert O.mont_array_to_canon(H.call("he_fq_inv", X[k], out_words=8)) == [pow(v, -1, O.P)], v
    assert O.mont_array_to_canon(H.call("he_fq_inv", fe([0]), out_words=8)) == [0]  # as the Fermat chain


def test_fq_fold_value(rnd):
    # fold(64x + x - x + 20p-ish) == 64x + ... : compare with the exact residue
    for v in rnd(30) + [0, O.P - 1]:
        got = O.mont_array_to_canon(H.call("he_fq_fold", fe([v]), out_words=8))
        assert got == [(64 * v + v - v) % O.P]


def test_fq_is_zero(rnd):
    """fq_is_zero / fq_eq (fold, then compare with 0, p, 2p) on multiples of p with
    lazy digits and on plain values, including 0 and p - 1."""
    vals = rnd(20) + [0, 1, O.P - 1]
    for k, v in enumerate(vals):
        w = vals[(k + 1) % len(vals)] if k % 3 else v
        bits = int(H.call("he_fq_zero_checks", fe([v]), fe([w]), out_words=2)[0])
        want = 0b1 | 0b10 | 0b100 | ((v == 0) << 3) | ((v == w) << 4) | (1 << 5) | (1 << 6) | ((v == w) << 7) | (1 << 8)
        assert bits == want, (v, w, bin(bits), bin(want))


def test_tower_vs_oracle(rnd):
    for _ in range(6):
        a = fe(rnd(12))
        b = fe(rnd(12))
        assert np.array_equal(H.call("he_fq12_mul", a, b, out_words=96), O.binary("orc_fq12_mul", a, b, 48, 48, 48)[0])
        assert np.array_equal(H.call("he_fq12_sqr", a, out_words=96), O.unary("orc_fq12_squared", a, 48)[0][0])
        assert np.array_equal(H.call("he_fq12_inv", a, out_words=96), O.unary("orc_fq12_inverse", a, 48)[0][0])
        assert np.array_equal(H.call("he_fq12_cyc_sqr", a, out_words=96),
                              O.unary("orc_fq12_cyclotomic_squared", a, 48)[0][0])
        for pw in (1, 2, 3):
            assert np.array_equal(H.call("he_fq12_frob", a, out_words=96, ints=(pw,)), _frob(a, pw))
        e = [fe(rnd(2)) for _ in range(3)]
        want = np.zeros(48, np.uint64)
        L = O.lib()
        L.orc_fq12_mul_by_024(O._p(a), O._p(e[0]), O._p(e[1]), O._p(e[2]), O._p(want))
        assert np.array_equal(H.call("he_fq12_mul_by_024", a, e[0], e[1], e[2], out_words=96), want)
        x = fe(rnd(2))
        assert np.array_equal(H.call("he_fq2_inv", x, out_words=16), O.unary("orc_fq2_inverse", x, 8)[0][0])
        assert np.array_equal(H.call("he_fq2_sqr", x, out_words=16), O.unary("orc_fq2_squared", x, 8)[0][0])


def test_gt_pow_formulas():
    # k_gt_pow's window chain on a pairing output (cyclotomic squarings) and a
    # (non-cyclotomic) Miller value (generic squarings)
    p, q, _, _ = O.random_pairs(2, seed=61)
    a = np.concatenate([O.pairing_many(p[:1], q[:1]), O.miller_loop_batch(q[1:2], p[1:2])[1][None]])
    vals, k = O.random_scalars(2, 62, lo=0)
    # with runs of ones and alternating bits: Booth digits 0 with a carry (six ones), -1, +-16
    for scal in (vals[0], 0, 1, O.R - 1, (1 << 250) - 1, (1 << 253) - 1, int("01" * 126, 2), int("10000" * 50, 2)):
        K = O.canon_to_mont_array([scal], O.FR).reshape(1, 4)
        words = np.frombuffer(int(scal).to_bytes(32, "little"), np.uint64).copy()
        for j in range(2):
            got, cyc = H.call("he_gt_pow", a[j], words, out_words=96, ret=True)
            assert cyc == (j == 0)  # the pairing output takes the cyclotomic chain, the Miller value not
            assert np.array_equal(got, O.gt_pow(a[j:j + 1], K)[0])


def _frob(a, pw):
    out = np.zeros(48, np.uint64)
    O.lib().orc_fq12_frobenius_map(O._p(np.ascontiguousarray(a)), pw, O._p(out))
    return out


def test_cyclotomic_exp_kat(kats):
    t = kats["test_cyclotomic_exp"]
    got = H.call("he_fq12_exp_by_neg_z", O.canon_to_mont_array([int(x) for x in t["orig"]]), out_words=96)
    assert O.mont_array_to_canon(got) == [int(x) for x in t["expected"]]


def test_prepared_g2_and_miller_kat(kats):
    t = kats["test_prepared_g2"]
    qa = O.canon_to_mont_array([int(x) for x in t["q_affine"]["x"] + t["q_affine"]["y"]])
    coeffs = H.call("he_g2_precompute", qa, out_words=87 * 48)
    assert O.mont_array_to_canon(coeffs) == [int(x) for row in t["coeffs"] for x in row]
    m = kats["test_miller_loop"]
    p = O.g1_mul(O.g1_one(), O.canon_to_mont_array([int(m["g1_scalar"])], O.FR))
    pa, _ = O.g1_to_affine(p)
    f = H.call("he_miller_loop", coeffs, pa[0, :4], pa[0, 4:], out_words=96)
    assert O.mont_array_to_canon(f) == [int(x) for x in m["f"]]
    # final exponentiation of that Miller value == test_reduced_pairing
    gt = H.call("he_final_exp", f, out_words=96)
    assert O.mont_array_to_canon(gt) == [int(x) for x in kats["test_reduced_pairing"]["gt"]]


def test_group_mul_vs_oracle():
    p, q, s, t = O.random_pairs(3, seed=99)
    ks, K = O.random_scalars(3, seed=5)
    for i in range(3):
        kc = O.ints_to_array([ks[i]])
        g1 = H.call("he_g1_mul", p[i], kc, out_words=24)
        assert np.array_equal(g1, O.g1_mul(p[i], K[i])[0])
        g2 = H.call("he_g2_mul", q[i], kc, out_words=48)
        assert np.array_equal(g2, O.g2_mul(q[i], K[i])[0])
    # zero point and zero scalar
    z = np.zeros(12, np.uint64)
    z[4:8] = O.canon_to_mont_array([1])
    kc = O.ints_to_array([12345])
    assert np.array_equal(H.call("he_g1_mul", z, kc, out_words=24), O.g1_mul(z, O.canon_to_mont_array([12345], O.FR))[0])
    assert np.array_equal(H.call("he_g1_mul", p[0], O.ints_to_array([0]), out_words=24),
                          O.g1_mul(p[0], O.canon_to_mont_array([0], O.FR))[0])
