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
