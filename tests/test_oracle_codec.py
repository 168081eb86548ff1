"""The oracle's encodings, validation, square roots and decompression
 pinned to the reference's own known answers:
sqrt_fq (fp.rs:289-296), sqrt_fq2 (fq2.rs:235-258), g1_from_compressed /
g2_from_compressed (lib.rs:681-743), testing_divrem (arith.rs:588-666),
from_slice / to_big_endian (arith.rs:561-586), test_rsquared (fp.rs:267-287).
CPU only."""
import json
import os

import numpy as np
import pytest

from oracle import oracle as O

KATS = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "reference_kats.json")))
P, R = O.P, O.R


def be(x, n=32):
    return np.frombuffer(int(x).to_bytes(n, "big"), dtype=np.uint8).copy()


def mont(vals, field=O.FQ):
    return O.canon_to_mont_array([int(v) for v in vals], field)


def canon(arr, field=O.FQ):
    return O.mont_array_to_canon(arr, field)


def test_u256_big_endian_kats():
    k = KATS["u256_one_big_endian"]
    b = bytes.fromhex(k["bytes"])
    # Fr::to_big_endian writes the raw image: raw 1 -> ...01
    assert bytes(O.fr_to_big_endian(np.array([1, 0, 0, 0], np.uint64))[0]) == b
    # Fq::from_slice(00..01) is the Montgomery image of 1; to_big_endian gives it back
    out, st = O.fq_from_slice(np.frombuffer(b, np.uint8))
    assert st[0] == O.OK and canon(out) == [1]
    assert bytes(O.fq_to_big_endian(out)[0]) == b


def test_divrem_kats():
    k = KATS["testing_divrem"]
    assert int(k["modulo"]) == P
    for c in k["cases"]:
        q, r, some = O.u512_divrem(be(int(c["a"]), 64))
        assert r == int(c["r"])
        if c["q"] is None:
            assert not some
        else:
            assert some and q == int(c["q"])


def test_fq_from_slice_rejects_and_roundtrips():
    rng = np.random.default_rng(1)
    vals = [0, 1, P - 1, P, P + 1, (1 << 256) - 1] + [int.from_bytes(rng.bytes(32), "big") for _ in range(64)]
    out, st = O.fq_from_slice(np.stack([be(v) for v in vals]))
    for v, o, s in zip(vals, out, st):
        if v >= P:
            assert s == O.FIELD_NOT_MEMBER
        else:
            assert s == O.OK and canon(o) == [v]
            assert int.from_bytes(bytes(O.fq_to_big_endian(o)[0]), "big") == v


def test_fq2_from_slice():
    rng = np.random.default_rng(2)
    vals = [0, P, P * P - 1, P * P, (1 << 512) - 1] + [int.from_bytes(rng.bytes(64), "big") >> 4 for _ in range(64)]
    out, st = O.fq2_from_slice(np.stack([be(v, 64) for v in vals]))
    for v, o, s in zip(vals, out, st):
        if v >= P * P:
            assert s == O.FIELD_NOT_MEMBER
        else:
            assert s == O.OK and canon(o) == [v % P, v // P]  # c1 * q + c0


def test_fr_from_slice_reduces_and_raw_to_big_endian():
    rng = np.random.default_rng(3)
    vals = [0, 1, R - 1, R, (1 << 256) - 1] + [int.from_bytes(rng.bytes(32), "big") for _ in range(32)]
    out = O.fr_from_slice(np.stack([be(v) for v in vals]))
    assert canon(out, O.FR) == [v % R for v in vals]  # new_mul_factor reduces mod r
    raw = O.fr_to_big_endian(out)
    assert [int.from_bytes(bytes(r), "big") for r in raw] == O.array_to_ints(out)  # raw Montgomery


def test_sqrt_kats():
    k = KATS["sqrt_fq"]
    root, ok = O.fq_sqrt(mont([k["square"]]))
    assert ok[0] and canon(root) == [int(k["root"])]
    k = KATS["sqrt_fq2"]
    root, ok = O.fq2_sqrt(mont(k["square"]))
    assert ok[0] and canon(root) == [int(x) for x in k["root"]]
    root, ok = O.fq2_sqrt(mont([P - 1, 0]))
    assert ok[0] and canon(root) == [0, 1]  # sqrt(-1) == i
    _, ok = O.fq2_sqrt(mont(k["no_root"]))
    assert not ok[0]


def test_sqrt_properties():
    rng = np.random.default_rng(4)
    xs = [0] + [int.from_bytes(rng.bytes(32), "big") % P for _ in range(40)]
    root, ok = O.fq_sqrt(mont(xs))
    for x, r, good in zip(xs, canon(root), ok):
        if good:
            assert r * r % P == x
        else:
            assert pow(x, (P - 1) // 2, P) == P - 1


def test_g1_from_compressed_kat_and_errors():
    k = KATS["g1_from_compressed"]
    b = bytes.fromhex(k["bytes"])
    out, st = O.g1_from_compressed_one(b)
    assert st == O.OK
    assert canon(out) == [int(k["x"]), int(k["y"]), 1]
    assert O.g1_from_compressed_one(b[:-1])[1] == O.CURVE_INVALID_ENCODING
    assert O.g1_from_compressed_one(bytes([4]) + b[1:])[1] == O.CURVE_INVALID_ENCODING
    assert O.g1_from_compressed_one(bytes([2]) + P.to_bytes(32, "big"))[1] == O.FIELD_NOT_MEMBER
    # the other sign gives the negated y
    out3, st3 = O.g1_from_compressed_one(bytes([3]) + b[1:])
    assert st3 == O.OK and canon(out3)[1] == P - int(k["y"])


def test_g2_from_compressed_kat_and_errors():
    k = KATS["g2_from_compressed"]
    out, st = O.g2_from_compressed_one(bytes.fromhex(k["bytes_0a"]))
    assert st == O.OK
    assert canon(out) == [int(v) for v in k["x"] + k["y"]] + [1, 0]
    out_b, st_b = O.g2_from_compressed_one(bytes.fromhex(k["bytes_0b_negated"]))
    neg = np.zeros(24, np.uint64)
    O.lib().orc_g2_neg(O._p(out_b), O._p(neg))
    assert st_b == O.OK and canon(neg) == [int(v) for v in k["x"] + k["y"]] + [1, 0]
    assert O.g2_from_compressed_one(bytes.fromhex(k["bytes_0c_invalid"]))[1] == O.CURVE_INVALID_ENCODING
    assert O.g2_from_compressed_one(bytes.fromhex(k["bytes_0a"])[:-1])[1] == O.CURVE_INVALID_ENCODING


def random_twist_points(n, seed):
    """(x, y) on E'(Fq2) but (almost surely) outside the order-r subgroup."""
    rng = np.random.default_rng(seed)
    xs, ys = [], []
    # b' of the twist from the generator: y^2 - x^3 (groups/mod.rs:452-467)
    g = O.g2_one()
    gy2 = O.binary("orc_fq2_mul", g[8:16], g[8:16], 8, 8, 8)
    gx3 = O.binary("orc_fq2_mul", O.binary("orc_fq2_mul", g[:8], g[:8], 8, 8, 8), g[:8], 8, 8, 8)
    b = [(u - v) % P for u, v in zip(canon(gy2), canon(gx3))]
    while len(xs) < n:
        x = mont([int.from_bytes(rng.bytes(32), "big") % P for _ in range(2)])
        x3 = O.binary("orc_fq2_mul", O.binary("orc_fq2_mul", x, x, 8, 8, 8), x, 8, 8, 8)
        rhs = [(u + v) % P for u, v in zip(canon(x3), b)]
        y, ok = O.fq2_sqrt(mont(rhs))
        if ok[0]:
            xs.append(x.reshape(8))
            ys.append(y.reshape(8))
    return np.stack(xs), np.stack(ys)


def test_affine_new_subgroup_and_curve_checks():
    # subgroup points: k * G2::one() to affine
    _, t = O.random_scalars(4, 77)
    q = O.g2_mul(O.g2_one(), t)
    aff, _ = O.g2_to_affine(q)
    out, st = O.g2_affine_new(aff[:, :8], aff[:, 8:])
    assert list(st) == [O.OK] * 4
    assert np.array_equal(out[:, :16], aff) and canon(out[0, 16:24]) == [1, 0]
    # on the twist, outside the subgroup
    x, y = random_twist_points(3, 5)
    _, st = O.g2_affine_new(x, y)
    assert list(st) == [O.GROUP_NOT_IN_SUBGROUP] * 3
    # off the curve
    y_bad = y.copy()
    y_bad[:, 0] ^= 1
    _, st = O.g2_affine_new(x, y_bad)
    assert list(st) == [O.GROUP_NOT_ON_CURVE] * 3
    # G1: on-curve check only (check_order false)
    p = O.g1_mul(O.g1_one(), t)
    a1, _ = O.g1_to_affine(p)
    out, st = O.g1_affine_new(a1[:, :4], a1[:, 4:])
    assert list(st) == [O.OK] * 4
    out, st = O.g1_affine_new(a1[:, 4:], a1[:, :4])
    assert list(st) == [O.GROUP_NOT_ON_CURVE] * 4


def test_gt_pow_matches_repeated_products():
    p, q, _, _ = O.random_pairs(2, seed=3)
    g = O.pairing_many(p, q)
    k = O.canon_to_mont_array([5, R - 1], O.FR).reshape(2, 4)
    out = O.gt_pow(g, k)
    g5 = g[0]
    for _ in range(4):
        g5 = O.binary("orc_fq12_mul", g5, g[0], 48, 48, 48)[0]
    assert np.array_equal(out[0], g5)
    # g^(r-1) * g == 1 for a pairing output (order r)
    one = O.binary("orc_fq12_mul", out[1], g[1], 48, 48, 48)[0]
    assert canon(one) == [1] + [0] * 11


def test_psi_identity_behind_the_g2_order_check():
    """codec.h decides [r]P == 0 as [t](psi(P) - P) == psi^2(P) - P; the identity
    (psi^2 - t psi + p = 0 on the whole twist) is checked with plain integers."""
    import runpy
    runpy.run_path(os.path.join(os.path.dirname(__file__), "..", "tools", "psi_check.py"), run_name="psi_check")
