"""codec.h (the device encodings / sqrt / validation / decompression code)
compiled for the host, checked bit for bit against the oracle and the
reference KATs on CPU."""
import ctypes
import json
import os

import numpy as np
import pytest

from oracle import oracle as O
from tests.native import hostemul
from tests.test_oracle_codec import KATS, be, canon, mont, random_twist_points

P, R = O.P, O.R


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def he(name, inp, out_words):
    fn = getattr(hostemul.lib(), name)
    fn.restype = ctypes.c_int
    inp = np.ascontiguousarray(inp)
    out = np.zeros(out_words, dtype=np.uint32)
    rc = fn(_p(inp), _p(out))
    return out.view(np.uint64), rc


def test_fq_from_slice_and_to_be():
    rng = np.random.default_rng(11)
    vals = [0, 1, P - 1, P, (1 << 256) - 1] + [int.from_bytes(rng.bytes(32), "big") for _ in range(24)]
    for v in vals:
        ref, st = O.fq_from_slice(be(v))
        got, rc = he("he_fq_from_slice", be(v), 8)
        assert rc == st[0]
        if rc == O.OK:
            assert np.array_equal(got, ref[0])
            b = np.zeros(32, np.uint8)
            fn = hostemul.lib().he_fq_to_be
            fn(_p(np.ascontiguousarray(ref[0]).view(np.uint32)), _p(b))
            assert np.array_equal(b, O.fq_to_big_endian(ref)[0])


def test_fq2_from_slice_and_divrem_kats():
    rng = np.random.default_rng(12)
    vals = [int(c["a"]) for c in KATS["testing_divrem"]["cases"]]
    vals += [0, P * P - 1, P * P, (1 << 512) - 1] + [int.from_bytes(rng.bytes(64), "big") >> 5 for _ in range(24)]
    for v in vals:
        ref, st = O.fq2_from_slice(be(v, 64))
        got, rc = he("he_fq2_from_slice", be(v, 64), 16)
        assert rc == st[0], v
        if rc == O.OK:
            assert np.array_equal(got, ref[0]), v


def test_fr_from_slice():
    rng = np.random.default_rng(13)
    vals = [0, 1, R - 1, R, (1 << 256) - 1] + [int.from_bytes(rng.bytes(32), "big") for _ in range(24)]
    for v in vals:
        got, _ = he("he_fr_from_slice", be(v), 8)
        assert np.array_equal(got, O.fr_from_slice(be(v))[0]), v


def test_sqrt_kats_and_random():
    k = KATS["sqrt_fq"]
    got, some = he("he_fq_sqrt", mont([k["square"]]).view(np.uint32), 8)
    assert some and canon(got) == [int(k["root"])]
    k = KATS["sqrt_fq2"]
    got, some = he("he_fq2_sqrt", mont(k["square"]).view(np.uint32), 16)
    assert some and canon(got) == [int(x) for x in k["root"]]
    got, some = he("he_fq2_sqrt", mont([P - 1, 0]).view(np.uint32), 16)
    assert some and canon(got) == [0, 1]
    _, some = he("he_fq2_sqrt", mont(k["no_root"]).view(np.uint32), 16)
    assert not some
    rng = np.random.default_rng(14)
    for _ in range(6):
        a = mont([int.from_bytes(rng.bytes(32), "big") % P for _ in range(2)])
        ref, ok = O.fq2_sqrt(a)
        got, some = he("he_fq2_sqrt", a.view(np.uint32), 16)
        assert bool(some) == bool(ok[0])
        if some:
            assert np.array_equal(got, ref[0])
        ref, ok = O.fq_sqrt(a[:4])
        got, some = he("he_fq_sqrt", a[:4].view(np.uint32), 8)
        assert bool(some) == bool(ok[0])
        if some:
            assert np.array_equal(got, ref[0])


def test_g2_affine_new_vs_oracle():
    _, t = O.random_scalars(2, 91)
    aff, _ = O.g2_to_affine(O.g2_mul(O.g2_one(), t))
    x, y = random_twist_points(2, 17)
    y_bad = y.copy()
    y_bad[:, 0] ^= 1
    xs = np.concatenate([aff[:, :8], x, x])
    ys = np.concatenate([aff[:, 8:], y, y_bad])
    ref, st = O.g2_affine_new(xs, ys)
    assert list(st) == [0, 0, 7, 7, 6, 6]
    for k in range(xs.shape[0]):
        got, rc = he("he_g2_affine_new", np.concatenate([xs[k], ys[k]]).view(np.uint32), 48)
        assert rc == st[k]
        if rc == O.OK:
            assert np.array_equal(got, ref[k])


def test_decompression_kats_and_errors():
    k = KATS["g1_from_compressed"]
    b = bytes.fromhex(k["bytes"])
    cases1 = [b, bytes([3]) + b[1:], bytes([4]) + b[1:], bytes([2]) + P.to_bytes(32, "big"),
              bytes([2]) + (5).to_bytes(32, "big")]
    for c in cases1:
        ref, st = O.g1_from_compressed_one(c)
        got, rc = he("he_g1_from_compressed", np.frombuffer(c, np.uint8), 24)
        assert rc == st, c.hex()
        if rc == O.OK:
            assert np.array_equal(got, ref)
    k = KATS["g2_from_compressed"]
    cases2 = [bytes.fromhex(k[n]) for n in ("bytes_0a", "bytes_0b_negated", "bytes_0c_invalid")]
    cases2.append(bytes([10]) + (P * P).to_bytes(64, "big"))
    for c in cases2:
        ref, st = O.g2_from_compressed_one(c)
        got, rc = he("he_g2_from_compressed", np.frombuffer(c, np.uint8), 48)
        assert rc == st, c.hex()
        if rc == O.OK:
            assert np.array_equal(got, ref)
