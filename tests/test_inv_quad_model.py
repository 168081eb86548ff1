"""The binary-GCD inversion split over a quad of lanes (paritytech-bn_amd/csrc/tower.h
fq_inv_quad), restated in Python lane by lane: lane r of a quad keeps a (r = 0), b (1),
u (2) or v (3) as nine 29-bit digits, runs the 29 steps on the approximations of lanes
0 and 1, and applies ONE linear update per round -- (own * c + partner * e + K p) / 2^29
with K = 0 on the exact lanes and k + 3 * 2^29 on the Montgomery lanes, the exact sign
fix reaching the Montgomery lanes as 6p - r -- then the fold estimate in float32.  Each
round's invariants are asserted (the exact lanes stay in [0, p] and fold with q = 0, the
Montgomery lanes in [0, 6p]); the result is checked against the modular inverse in the
engine's Montgomery form (R = 2^261).  The GPU path is checked bit for bit through every
pairing test that runs k_prepare_wide, the latency kernel or k_seg_tail."""
import random

import numpy as np

P = 0x30644e72e131a029b85045b68181585d97816a916871ca8d3c208c16d87cfd47
M29 = (1 << 29) - 1
R = 1 << 261
MASK64 = (1 << 64) - 1
FOLD_C = np.float32(3.1531629e-07)  # fq.h fq_fold's estimate constant


def digits(x):
    return [(x >> (29 * i)) & M29 for i in range(8)] + [x >> (29 * 8)]


def value(d):
    return sum(d[i] << (29 * i) for i in range(8)) + (d[8] << (29 * 8))


P29 = digits(P)
P6 = digits(6 * P)
PINV29 = (-pow(P, -1, 1 << 29)) % (1 << 29)


def s32(x):
    x &= 0xffffffff
    return x - (1 << 32) if x >> 31 else x


def sx64(x):
    return x - (1 << 64) if x >> 63 else x


def inv_quad(y):
    """fq_inv_quad on the plain integer y (= x*R mod p): returns x^-1 * R mod p"""
    own = [digits(y), digits(P), digits(1), digits(0)]  # lanes a, b, u, v
    for _ in range(19):
        lens = []
        for r in range(4):
            ln = 0
            for d in range(9):
                if own[r][d]:
                    ln = 29 * d + 32 - (32 - (own[r][d] | 1).bit_length())
            lens.append(ln)
        aps = []
        for r in range(4):
            n = max(lens[r], lens[r ^ 1], 60)  # quad_perm [1,0,3,2]
            s = n - 31
            dd, off = s // 29, s - 29 * (s // 29)
            w0 = w1 = w2 = 0
            for d in range(1, 9):
                if dd == d:
                    w0 = own[r][d]
                    w1 = own[r][d + 1] if d + 1 < 9 else 0
                    w2 = own[r][d + 2] if d + 2 < 9 else 0
            wv = (w0 | (w1 << 29) | (w2 << 58)) & MASK64
            aps.append(own[r][0] | (((wv >> off) & 0x7fffffff) << 29))
        ab, bb = aps[0], aps[1]  # quad_perm [0,0,0,0] and [1,1,1,1]
        pa, pb = 1, 1 << 32
        for _ in range(29):
            odd = ab & 1
            sw = odd and ab < bb
            ta, tb, tp, tq = (bb, ab, pb, pa) if sw else (ab, bb, pa, pb)
            ab = ((ta - (tb if odd else 0)) & MASK64) >> 1
            pa = (tp - (tq if odd else 0)) & MASK64
            bb, pb = tb, (tq << 1) & MASK64
        f0, f1 = s32(pa), s32(pb)
        g0 = s32(sx64((pa - (f0 & MASK64)) & MASK64) >> 32)
        g1 = s32(sx64((pb - (f1 & MASK64)) & MASK64) >> 32)
        rs, ms = [], []
        for r in range(4):
            c, e = (g1, f1) if r & 1 else (f0, g0)
            part = own[r ^ 1]
            t = [s32(own[r][i]) * c + s32(part[i]) * e for i in range(9)]
            K = (((t[0] * PINV29) & M29) + (3 << 29)) if r >= 2 else 0
            t = [t[i] + K * P29[i] for i in range(9)]
            assert t[0] & M29 == 0
            out, cr = [0] * 9, t[0] >> 29
            for i in range(1, 9):
                sm = t[i] + cr
                out[i - 1], cr = sm & M29, sm >> 29
            out[8] = cr & 0xffffffff
            rs.append(out)
            ms.append(0xffffffff if s32(out[8]) < 0 else 0)
        new = []
        for r in range(4):
            m = ms[r & 1]  # quad_perm [0,1,0,1]
            mont = 0xffffffff if r >= 2 else 0
            z, cn = [0] * 9, 0
            for i in range(8):
                v = s32(((rs[r][i] ^ m) - m) & 0xffffffff) + (P6[i] & m & mont) + cn
                z[i], cn = v & M29, v >> 29
            z[8] = (s32(((rs[r][8] ^ m) - m) & 0xffffffff) + (P6[8] & m & mont) + cn) & 0xffffffff
            val = value(z)
            q = int(np.float32(z[8]) * FOLD_C)
            if r < 2:
                assert 0 <= val <= P and q == 0
            else:
                assert 0 <= val <= 6 * P and q <= 6
            new.append(digits(val - q * P))
        own = new
    if y:
        assert value(own[1]) == 1  # b ends at gcd = 1
    v = value(own[3])
    return v * pow(2, 783, P) * pow(R, -1, P) % P  # fq_mul(v, R^3 mod p)


def test_quad_inversion_model():
    rng = random.Random(20261018)
    cases = [1, 2, P - 1, P - 2, (1 << 253) % P, (1 << 254) % P] + [rng.randrange(1, P) for _ in range(300)]
    for y in cases:
        assert inv_quad(y) == R * R * pow(y, -1, P) % P
    assert inv_quad(0) == 0  # as fq_inv_bgcd: y = 0 keeps v = 0
