"""GPU parity of SURVEY §8(f) rows 1-4 through the C ABI: encodings, square
roots, AffineG::new validation (incl. the G2 order check), decompression and
Gt::pow, bit-exact (images and per-element status) against the oracle, plus the
reference's known answers.  Runs on the GPU box: python -m pytest tests -m gpu."""
import numpy as np
import pytest

from oracle import oracle as O
from tests.codec_util import be, canon, compress_g1, compress_g2, random_twist_points, subgroup_affine

pytestmark = pytest.mark.gpu
NT = 16
P, R = O.P, O.R


@pytest.fixture(scope="module")
def ctx():
    from substrate_bn import Context
    return Context(0)


def test_field_encodings(ctx):
    rng = np.random.default_rng(5)
    vals = [0, 1, P - 1, P, P + 1, (1 << 256) - 1] + [int.from_bytes(rng.bytes(32), "big") for _ in range(2000)]
    vals += [int.from_bytes(rng.bytes(32), "big") % P for _ in range(2000)]
    b = np.stack([be(v) for v in vals])
    out, st = ctx.fq_from_slice_many(b)
    ref, rst = O.fq_from_slice(b)
    assert np.array_equal(st, rst) and np.array_equal(out, ref)
    ok = st == 0
    assert np.array_equal(ctx.fq_to_big_endian_many(out[ok]), O.fq_to_big_endian(ref[ok]))
    assert np.array_equal(ctx.fr_from_slice_many(b), O.fr_from_slice(b))
    fr = O.fr_from_slice(b)
    assert np.array_equal(ctx.fr_to_big_endian_many(fr), O.fr_to_big_endian(fr))
    # Fq2 / U512 divrem, including the reference's own divrem cases
    v2 = [0, P, P * P - 1, P * P, P * P + 1, (1 << 512) - 1]
    v2 += [int.from_bytes(rng.bytes(64), "big") >> 5 for _ in range(2000)]
    b2 = np.stack([be(v, 64) for v in v2])
    out2, st2 = ctx.fq2_from_slice_many(b2)
    ref2, rst2 = O.fq2_from_slice(b2)
    assert np.array_equal(st2, rst2) and np.array_equal(out2, ref2)


def test_divrem_kats(ctx, kats):
    for c in kats["testing_divrem"]["cases"]:
        out, st = ctx.fq2_from_slice_many(be(int(c["a"]), 64))
        if c["q"] is None:
            assert st[0] == O.FIELD_NOT_MEMBER
        else:
            assert st[0] == 0 and canon(out[0]) == [int(c["r"]), int(c["q"])]


def test_sqrt(ctx, kats):
    k = kats["sqrt_fq"]
    out, ok = ctx.fq_sqrt_many(O.canon_to_mont_array([int(k["square"])]))
    assert ok[0] and canon(out[0]) == [int(k["root"])]
    k = kats["sqrt_fq2"]
    out, ok = ctx.fq2_sqrt_many(O.canon_to_mont_array([int(x) for x in k["square"]]))
    assert ok[0] and canon(out[0]) == [int(x) for x in k["root"]]
    out, ok = ctx.fq2_sqrt_many(O.canon_to_mont_array([P - 1, 0]))
    assert ok[0] and canon(out[0]) == [0, 1]
    _, ok = ctx.fq2_sqrt_many(O.canon_to_mont_array([int(x) for x in k["no_root"]]))
    assert not ok[0]
    g = O.SplitMix64(9)
    a = O.canon_to_mont_array([0] + [g.below(P) for _ in range(1023)]).reshape(-1, 4)
    out, ok = ctx.fq_sqrt_many(a)
    ref, rok = O.fq_sqrt(a)
    assert np.array_equal(ok.astype(bool), rok) and np.array_equal(out[rok], ref[rok])
    a2 = a.reshape(-1, 8)
    out, ok = ctx.fq2_sqrt_many(a2)
    ref, rok = O.fq2_sqrt(a2)
    assert np.array_equal(ok.astype(bool), rok) and np.array_equal(out[rok], ref[rok])


def test_affine_new(ctx):
    g2aff, g1aff = subgroup_affine(64, 31, NT)
    tx, ty = random_twist_points(16, 32)
    ty_bad = ty.copy()
    ty_bad[:, 0] ^= 2
    x = np.concatenate([g2aff[:, :8], tx, tx])
    y = np.concatenate([g2aff[:, 8:], ty, ty_bad])
    out, st = ctx.g2_affine_new_many(x, y)
    ref, rst = O.g2_affine_new(x, y, NT)
    assert list(rst[:64]) == [0] * 64 and list(rst[64:80]) == [7] * 16 and list(rst[80:]) == [6] * 16
    assert np.array_equal(st, rst) and np.array_equal(out, ref)
    out, st = ctx.g1_affine_new_many(g1aff[:, :4], g1aff[:, 4:])
    ref, rst = O.g1_affine_new(g1aff[:, :4], g1aff[:, 4:])
    assert list(st) == [0] * 64 and np.array_equal(out, ref)
    _, st = ctx.g1_affine_new_many(g1aff[:, 4:], g1aff[:, :4])
    assert list(st) == [O.GROUP_NOT_ON_CURVE] * 64


def test_decompression_kats(ctx, kats):
    k = kats["g1_from_compressed"]
    out, st = ctx.g1_from_compressed_many(np.frombuffer(bytes.fromhex(k["bytes"]), np.uint8))
    assert st[0] == 0 and canon(out[0]) == [int(k["x"]), int(k["y"]), 1]
    k = kats["g2_from_compressed"]
    recs = np.stack([np.frombuffer(bytes.fromhex(k[n]), np.uint8)
                     for n in ("bytes_0a", "bytes_0b_negated", "bytes_0c_invalid")])
    out, st = ctx.g2_from_compressed_many(recs)
    assert list(st) == [0, 0, O.CURVE_INVALID_ENCODING]
    assert canon(out[0]) == [int(v) for v in k["x"] + k["y"]] + [1, 0]
    ref, rst = O.g2_from_compressed(recs)
    assert np.array_equal(out, ref) and np.array_equal(st, rst)


def test_decompression_random_and_invalid(ctx):
    g2aff, g1aff = subgroup_affine(512, 41, NT)
    c1 = compress_g1(g1aff)
    c2 = compress_g2(g2aff)
    # invalid variants: bad sign byte, x >= p (G1) / x >= p^2 (G2), random x (no root or not in the subgroup)
    rng = np.random.default_rng(42)
    bad1 = c1[:64].copy()
    bad1[:16, 0] = 4
    bad1[16:32, 1:] = be(P)
    bad1[32:, 1:] = np.stack([be(int.from_bytes(rng.bytes(32), "big") % P) for _ in range(32)])
    bad2 = c2[:64].copy()
    bad2[:16, 0] = 12
    bad2[16:32, 1:] = be(P * P, 64)
    bad2[32:, 1:] = np.stack([be(int.from_bytes(rng.bytes(64), "big") % (P * P), 64) for _ in range(32)])
    a1 = np.concatenate([c1, bad1])
    a2 = np.concatenate([c2, bad2])
    out, st = ctx.g1_from_compressed_many(a1)
    ref, rst = O.g1_from_compressed(a1, NT)
    assert list(rst[:512]) == [0] * 512
    assert np.array_equal(st, rst) and np.array_equal(out, ref)
    assert np.array_equal(out[:512, :8], g1aff)
    out, st = ctx.g2_from_compressed_many(a2)
    ref, rst = O.g2_from_compressed(a2, NT)
    assert list(rst[:512]) == [0] * 512 and set(rst[576 - 32:]) <= {O.CURVE_NOT_MEMBER}
    assert np.array_equal(st, rst) and np.array_equal(out, ref)
    assert np.array_equal(out[:512, :16], g2aff)


def test_gt_pow(ctx):
    p, q, _, _ = O.random_pairs(64, seed=51, nthreads=NT)
    g = O.pairing_many(p, q, NT)
    # non-cyclotomic inputs: Miller values (a Gt may hold a miller_loop_batch output)
    ml = np.stack([O.miller_loop_batch(q[k:k + 1], p[k:k + 1])[1] for k in range(8)])
    a = np.concatenate([g, ml])
    vals, k = O.random_scalars(a.shape[0], 52, lo=0)
    k[0] = O.canon_to_mont_array([0], O.FR)
    k[1] = O.canon_to_mont_array([1], O.FR)
    k[2] = O.canon_to_mont_array([R - 1], O.FR)
    # runs of ones and alternating bits (the signed 5-bit windows' carries and +-16 digits)
    k[3:7] = O.canon_to_mont_array([(1 << 250) - 1, (1 << 253) - 1, int("01" * 126, 2), int("10000" * 50, 2)],
                                   O.FR).reshape(4, 4)
    out = ctx.gt_pow_many(a, k)
    assert np.array_equal(out, O.gt_pow(a, k))
    # waves holding only pairing outputs take the cyclotomic squarings, the rest the
    # generic ones: a Miller value and a zero element inside an otherwise cyclotomic wave
    b = np.concatenate([g[:10], ml[:1], g[10:40], np.zeros((1, 48), np.uint64), g[40:], ml[1:]])
    kb = np.concatenate([k, k[:1]])
    out = ctx.gt_pow_many(b, kb)
    assert np.array_equal(out, O.gt_pow(b, kb))


def test_rust_api_mirror_codec(kats):
    import substrate_bn as bn
    k = kats["g1_from_compressed"]
    g = bn.G1.from_compressed(bytes.fromhex(k["bytes"]))
    assert g.x().into_int() == int(k["x"]) and g.y().into_int() == int(k["y"])
    with pytest.raises(bn.CurveError):
        bn.G2.from_compressed(bytes.fromhex(kats["g2_from_compressed"]["bytes_0c_invalid"]))
    with pytest.raises(bn.FieldError):
        bn.Fq.from_slice(P.to_bytes(32, "big"))
    assert bn.Fq.from_slice((5).to_bytes(32, "big")).to_big_endian() == (5).to_bytes(32, "big")
    assert bn.Fr.from_slice(R.to_bytes(32, "big")) == bn.Fr.zero()
    tx, ty = random_twist_points(1, 77)
    with pytest.raises(bn.GroupError):
        bn.AffineG2.new(bn.Fq2(tx[0]), bn.Fq2(ty[0]))
    gt = bn.pairing(bn.G1.one(), bn.G2.one())
    assert gt.pow(bn.Fr.from_int(3)) == gt * gt * gt
