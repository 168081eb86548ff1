"""Synthetic benchmark inputs, generated without the test oracle.

bench.py draws its scalars here (SplitMix64, the same stream and rejection rule
as the tests' helper, so a seed names the same data everywhere). It builds
points with the engine's own scalar-multiplication kernels and converts them
on the host with plain Python integers.  oracle/ stays the checker only.
"""
import numpy as np

from . import P, R_ORDER, G1, G2

_RM = 1 << 256
_M64 = 0xFFFFFFFFFFFFFFFF


class SplitMix64:
    def __init__(self, seed):
        self.s = seed & _M64

    def next(self):
        self.s = (self.s + 0x9E3779B97F4A7C15) & _M64
        z = self.s
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & _M64
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & _M64
        return z ^ (z >> 31)

    def below(self, m):
        """uniform in [0, m): 256-bit draws masked to m's bit length, rejected when >= m."""
        bits = m.bit_length()
        while True:
            v = 0
            for i in range(4):
                v |= self.next() << (64 * i)
            v &= (1 << bits) - 1
            if v < m:
                return v


def _limbs(vals):
    out = np.zeros((len(vals), 4), np.uint64)
    for i, v in enumerate(vals):
        for j in range(4):
            out[i, j] = (v >> (64 * j)) & _M64
    return out


def _ints(arr):
    a = np.asarray(arr, np.uint64).reshape(-1, 4)
    return [int(a[i, 0]) | int(a[i, 1]) << 64 | int(a[i, 2]) << 128 | int(a[i, 3]) << 192 for i in range(a.shape[0])]


def fr_images(n, seed, lo=1):
    """n scalars uniform in [lo, r) as Montgomery Fr images (n, 4) uint64."""
    g = SplitMix64(seed)
    vals = []
    for _ in range(n):
        v = g.below(R_ORDER)
        while v < lo:
            v = g.below(R_ORDER)
        vals.append(v)
    return _limbs([v * _RM % R_ORDER for v in vals])


def g1_one_image():
    return G1.one().img.reshape(12).copy()


def g2_one_image():
    return G2.one().img.reshape(24).copy()


def g2_jacobian_to_affine(img):
    """(n, 24) Jacobian G2 images (z != 0) -> (n, 16) affine images x.c0, x.c1, y.c0, y.c1
    (to_affine, mod.rs:199-216: x / z^2, y / z^3)."""
    w = _ints(img)
    inv_rm = pow(_RM, -1, P)
    out = []
    for i in range(len(w) // 6):
        x0, x1, y0, y1, z0, z1 = (v * inv_rm % P for v in w[6 * i:6 * i + 6])
        ni = pow((z0 * z0 + z1 * z1) % P, -1, P)  # Fq2 = Fq[u]/(u^2 + 1)
        a0, a1 = z0 * ni % P, -z1 * ni % P  # 1/z
        b0, b1 = (a0 * a0 - a1 * a1) % P, 2 * a0 * a1 % P  # 1/z^2
        c0, c1 = (b0 * a0 - b1 * a1) % P, (b0 * a1 + b1 * a0) % P  # 1/z^3
        out += [(x0 * b0 - x1 * b1) % P, (x0 * b1 + x1 * b0) % P, (y0 * c0 - y1 * c1) % P, (y0 * c1 + y1 * c0) % P]
    return _limbs([v * _RM % P for v in out]).reshape(-1, 16)


def compress_g2(aff):
    """(n, 16) affine G2 images -> (n, 65) G2::from_compressed records (lib.rs:506-526):
    11 when y is the larger root (compared as the U512 c1 * p + c0), else 10; then x as
    the 64-byte big-endian U512 c1 * p + c0."""
    w = _ints(aff)
    inv_rm = pow(_RM, -1, P)
    rec = np.zeros((len(w) // 4, 65), np.uint8)
    for i in range(len(w) // 4):
        x0, x1, y0, y1 = (v * inv_rm % P for v in w[4 * i:4 * i + 4])
        larger = y1 * P + y0 > ((-y1) % P) * P + (-y0) % P
        rec[i, 0] = 11 if larger else 10
        rec[i, 1:] = np.frombuffer((x1 * P + x0).to_bytes(64, "big"), np.uint8)
    return rec


# ---------------------------------------------------------------- the bench dataset
# bench.py's pairs are indexed globally, so any rank (and any world size) can
# build exactly the rows it owns: block b (kBlockRows rows) draws its G1 and G2
# scalars from SplitMix64 seeds DATASET_SEED + 2b and DATASET_SEED + 2b + 1.
# The scalars are drawn directly as Montgomery Fr images uniform in [1, r)
# (the image of a uniform scalar is uniform), fully vectorized.
DATASET_SEED = 1_000_000
BLOCK_ROWS = 4096
_GAMMA = np.uint64(0x9E3779B97F4A7C15)
_R_LIMBS = [(R_ORDER >> (64 * i)) & _M64 for i in range(4)]


def _splitmix_draws(seed, first, count):
    """draws first+1 .. first+count of SplitMix64(seed) (the same stream as SplitMix64.next)."""
    k = np.arange(first + 1, first + count + 1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = np.uint64(seed & _M64) + k * _GAMMA
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def fr_images_raw(n, seed, lo=1):
    """n Montgomery Fr images uniform in [lo, r), vectorized: candidate j takes draws
    4j+1..4j+4 as little-endian limbs masked to r's 254 bits and is kept when < r
    (SplitMix64.below's rule) and >= lo."""
    top_mask = np.uint64((1 << (R_ORDER.bit_length() - 192)) - 1)
    out, have, first = [], 0, 0
    while have < n:
        m = int((n - have) * 1.4) + 64
        d = _splitmix_draws(seed, first, 4 * m).reshape(m, 4)
        first += 4 * m
        d[:, 3] &= top_mask
        lt = np.zeros(m, bool)
        eq = np.ones(m, bool)
        for i in (3, 2, 1, 0):  # lexicographic compare with r from the top limb
            li = np.uint64(_R_LIMBS[i])
            lt |= eq & (d[:, i] < li)
            eq &= d[:, i] == li
        ok = lt
        if lo:
            nz = (d[:, 0] >= np.uint64(lo)) | (d[:, 1] != 0) | (d[:, 2] != 0) | (d[:, 3] != 0)
            ok &= nz
        sel = d[ok]
        out.append(sel[:n - have])
        have += min(len(sel), n - have)
    return np.ascontiguousarray(np.concatenate(out)[:n])


def dataset_scalars(lo, n):
    """(s, t) scalar images of global rows [lo, lo + n) of the bench dataset."""
    s, t = [], []
    b0, b1 = lo // BLOCK_ROWS, (lo + n + BLOCK_ROWS - 1) // BLOCK_ROWS
    for b in range(b0, b1):
        s.append(fr_images_raw(BLOCK_ROWS, DATASET_SEED + 2 * b))
        t.append(fr_images_raw(BLOCK_ROWS, DATASET_SEED + 2 * b + 1))
    off = lo - b0 * BLOCK_ROWS
    return np.concatenate(s)[off:off + n], np.concatenate(t)[off:off + n]
