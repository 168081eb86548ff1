#!/usr/bin/env python3
"""Checks, with plain Python integers, the identity behind the G2 order check of
codec.h: the twisted Frobenius psi (the reference's mul_by_q) satisfies
psi^2 - t psi + p = 0 on random points of E'(Fq2), so [r]P == 0 exactly when
[t](psi(P) - P) == psi^2(P) - P.  Run: python tools/psi_check.py"""
# numeric check of psi^2 - t psi + p = 0 on random points of the BN254 twist E'(Fq2), and of
# [r]P == 0  <=>  [t](psi(P) - P) == psi^2(P) - P
import random
P = 0x30644E72E131A029B85045B68181585D97816A916871CA8D3C208C16D87CFD47
R = 0x30644E72E131A029B85045B68181585D2833E84879B9709143E1F593F0000001
U = 4965661367192848881
T = 6 * U * U + 1
assert P + 1 - T == R, "trace"
RINV = pow(1 << 256, -1, P)
def u64s(a, b, c, d): return a | (b << 64) | (c << 128) | (d << 192)
def canon(x): return x * RINV % P
# twist_mul_by_q_x / _y (groups/mod.rs:531-564), reference Montgomery images
CX = (canon(u64s(13075984984163199792, 3782902503040509012, 8791150885551868305, 1825854335138010348)),
      canon(u64s(7963664994991228759, 12257807996192067905, 13179524609921305146, 2767831111890561987)))
CY = (canon(u64s(16482010305593259561, 13488546290961988299, 3578621962720924518, 2681173117283399901)),
      canon(u64s(11661927080404088775, 553939530661941723, 7860678177968807019, 3208568454732775116)))
B2 = (canon(u64s(0x3bf938e377b802a8, 0x020b1b273633535d, 0x26b7edf049755260, 0x2514c6324384a86d)),
      canon(u64s(0x38e7ecccd1dcff67, 0x65f0b37d93ce0d3e, 0xd749d0dd22ac00aa, 0x0141b9ce4a688d4d)))
def add(a, b): return ((a[0] + b[0]) % P, (a[1] + b[1]) % P)
def sub(a, b): return ((a[0] - b[0]) % P, (a[1] - b[1]) % P)
def mul(a, b): return ((a[0] * b[0] - a[1] * b[1]) % P, (a[0] * b[1] + a[1] * b[0]) % P)
def inv(a):
    n = pow((a[0] * a[0] + a[1] * a[1]) % P, P - 2, P)
    return (a[0] * n % P, (-a[1]) * n % P)
def conj(a): return (a[0], (-a[1]) % P)
def sqrt2(a):  # brute: (a^((p^2+7)/16)...) -- use generic Tonelli-free method for p = 3 mod 4 over Fq2
    # Algorithm 9 (as the reference): returns a root or None
    def pw(x, e):
        r = (1, 0)
        while e:
            if e & 1: r = mul(r, x)
            x = mul(x, x); e >>= 1
        return r
    a1 = pw(a, (P - 3) // 4); alpha = mul(a1, mul(a1, a)); a0 = mul(conj(alpha), alpha)
    if a0 == (P - 1, 0): return None
    if alpha == (P - 1, 0): return mul((0, 1), mul(a1, a))
    b = pw(add(alpha, (1, 0)), (P - 1) // 2)
    return mul(b, mul(a1, a))
O = None
def ec_add(p1, p2):
    if p1 is O: return p2
    if p2 is O: return p1
    if p1[0] == p2[0]:
        if add(p1[1], p2[1]) == (0, 0): return O
        l = mul(mul((3, 0), mul(p1[0], p1[0])), inv(add(p1[1], p1[1])))
    else:
        l = mul(sub(p2[1], p1[1]), inv(sub(p2[0], p1[0])))
    x3 = sub(sub(mul(l, l), p1[0]), p2[0])
    return (x3, sub(mul(l, sub(p1[0], x3)), p1[1]))
def neg(p1): return O if p1 is O else (p1[0], ((-p1[1][0]) % P, (-p1[1][1]) % P))
def smul(k, p1):
    r = O
    for bit in bin(k)[2:]:
        r = ec_add(r, r)
        if bit == '1': r = ec_add(r, p1)
    return r
def psi(p1): return O if p1 is O else (mul(CX, conj(p1[0])), mul(CY, conj(p1[1])))
rng = random.Random(5)
pts = []
while len(pts) < 6:
    x = (rng.randrange(P), rng.randrange(P))
    y = sqrt2(add(mul(mul(x, x), x), B2))
    if y is not None:
        assert mul(y, y) == add(mul(mul(x, x), x), B2)
        pts.append((x, y))
# G2 generator (mod.rs:418-450)
G = ((10857046999023057135944570762232829481370756359578518086990519993285655852781,
      11559732032986387107991004021392285783925812861821192530917403151452391805634),
     (8495653923123431417604973247489272438418190587263600148770280649306958101930,
      4082367875863433681332203403145435568316851327593401208105741076214120093531))
pts += [G, smul(12345, G)]
for i, p1 in enumerate(pts):
    lhs = ec_add(ec_add(smul(T, psi(p1)), neg(psi(psi(p1)))), O)  # [t]psi(P) - psi^2(P) should be [p]P
    assert lhs == smul(P, p1), "char poly fails at %d" % i
    in_g2 = smul(R, p1) is O
    test = smul(T, ec_add(psi(p1), neg(p1))) == ec_add(psi(psi(p1)), neg(p1))
    print(i, "in G2:", in_g2, "identity test:", test)
    assert in_g2 == test
print("ok")
