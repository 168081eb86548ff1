"""Test helpers for SURVEY §8(f) rows (encodings / validation / decompression):
compressed encodings of known points and seeded invalid inputs, built from the
oracle (test infrastructure)."""
import numpy as np

from oracle import oracle as O

P = O.P


def canon(arr):
    return O.mont_array_to_canon(arr)


def be(x, n=32):
    return np.frombuffer(int(x).to_bytes(n, "big"), dtype=np.uint8).copy()


def compress_g1(aff):
    """affine (n, 8) images -> (n, 33) G1::from_compressed records (lib.rs:359-375)."""
    out = []
    for row in aff:
        x, y = canon(row[:4])[0], canon(row[4:])[0]
        out.append(np.concatenate([[2 if y % 2 == 0 else 3], be(x)]))
    return np.stack(out).astype(np.uint8)


def compress_g2(aff):
    """affine (n, 16) images -> (n, 65) G2::from_compressed records (lib.rs:506-526)."""
    out = []
    for row in aff:
        x0, x1, y0, y1 = canon(row)
        yn0, yn1 = (-y0) % P, (-y1) % P
        larger = (y1, y0) > (yn1, yn0)
        out.append(np.concatenate([[11 if larger else 10], be(x1 * P + x0, 64)]))
    return np.stack(out).astype(np.uint8)


def random_twist_points(n, seed):
    """(x, y) images on E'(Fq2) but (almost surely) outside the order-r subgroup."""
    rng = np.random.default_rng(seed)
    g = O.g2_one()
    mul = lambda a, b: O.binary("orc_fq2_mul", a, b, 8, 8, 8)  # noqa: E731
    b = [(u - v) % P for u, v in zip(canon(mul(g[8:16], g[8:16])), canon(mul(mul(g[:8], g[:8]), g[:8])))]
    xs, ys = [], []
    while len(xs) < n:
        x = O.canon_to_mont_array([int.from_bytes(rng.bytes(32), "big") % P for _ in range(2)])
        rhs = [(u + v) % P for u, v in zip(canon(mul(mul(x, x), x)), b)]
        y, ok = O.fq2_sqrt(O.canon_to_mont_array(rhs))
        if ok[0]:
            xs.append(x.reshape(8))
            ys.append(y.reshape(8))
    return np.stack(xs), np.stack(ys)


def subgroup_affine(n, seed, nthreads=8):
    """n affine G2 points k * G2::one() as (n, 16) images, and n affine G1 points (n, 8)."""
    _, t = O.random_scalars(n, seed)
    g2aff, _ = O.g2_to_affine(O.g2_mul(O.g2_one(), t, nthreads))
    g1aff, _ = O.g1_to_affine(O.g1_mul(O.g1_one(), t, nthreads))
    return g2aff, g1aff
