#!/usr/bin/env python3
"""Lane-level model of the digit-sliced Fq12 arithmetic of csrc/fq12_ds.h.

One Fq coordinate per slot of lanes (the device: 21 lanes, three slots per wave;
the model: 32, a superset); 26-bit digits, ten per value, Montgomery R = 2^260.
Product columns live at lanes 0..18 (lane j: column j); values
(digits) at lanes 10..19 ("digit k at lane 10 + k"), the top digit (lane 19) a
signed sink that takes every carry out of the lanes below it.  Carries move one
lane up per DPP wave_shr:1 (shr1 here: lane j gets lane j - 1, lane 0 gets 0).
The model applies the device's steps lane by lane and checks every bound the
device code relies on (64-bit columns, 32-bit operands, signed ranges) with
asserts, and the values against big-integer arithmetic.  Design aid and test of
the algebra only; the device code is checked against fq12_wide.h on the GPU by
tools/ds_check.hip (tests/test_gpu_ds.py); tests/test_ds_model.py runs this model.

    python tools/ds_model.py [trials]
"""
import random
import struct
import sys

P = 21888242871839275222246405745257275088696311157297823662689037894645226208583
DIG, ND, W, B = 26, 10, 32, 10  # digit bits, digits, slot lanes, lane of digit 0
TOP = B + ND - 1                 # lane of the top digit (the sink)
M = (1 << DIG) - 1
R = 1 << (DIG * ND)
PINV = (-pow(P, -1, R)) % R
PD = [(P >> (DIG * k)) & M for k in range(ND)]
PID = [(PINV >> (DIG * k)) & M for k in range(ND)]
FOLD_C = struct.unpack("f", struct.pack("f", (2 ** 234 / P) * (1 - 2 ** -18)))[0]


def f32(x):
    return struct.unpack("f", struct.pack("f", x))[0]


def chk(v, lo, hi, what):
    for j, d in enumerate(v):
        assert lo <= d < hi, (what, j, d)


def i64(v):
    chk(v, -(1 << 63), 1 << 63, "i64")


def i32(v):
    chk(v, -(1 << 31), 1 << 31, "i32")


def u32(v):
    chk(v, 0, 1 << 32, "u32")


def shr1(v):
    return [0] + v[:-1]


def val_at(v, base):
    """value of digits at lanes base.. (digit k at lane base + k); lanes below base must be 0"""
    assert all(d == 0 for d in v[:base]), v
    return sum(d << (DIG * (j - base)) for j, d in enumerate(v) if j >= base)


def val_cols(v):
    return sum(d << (DIG * j) for j, d in enumerate(v))


def split64(c, sink=None):
    """c = c0 + c1 2^26 + c2 2^52 per lane (c0, c1 unsigned 26-bit, c2 signed); d_j = c0_j + c1_(j-1) + c2_(j-2).
    sink: that lane keeps its whole value, the lane below it hands its c2 over as c1 (both land in the sink)"""
    i64(c)
    c0 = [x & M for x in c]
    c1 = [(x >> DIG) & M for x in c]
    c2 = [x >> (2 * DIG) for x in c]
    if sink is not None:
        c0[sink], c1[sink], c2[sink] = c[sink], 0, 0
        c1[sink - 1] = c[sink - 1] >> DIG  # signed, whole
        c2[sink - 1] = 0
    d = [a + b + e for a, b, e in zip(c0, shr1(c1), shr1(shr1(c2)))]
    return d


def split32(d, sink=None):
    i32(d)
    lo = [x & M for x in d]
    hi = [x >> DIG for x in d]
    if sink is not None:
        lo[sink], hi[sink] = d[sink], 0
    r = [a + b for a, b in zip(lo, shr1(hi))]
    i32(r)
    return r


def digits(x):
    """value x >= 0 as a slot vector at lanes B.. (the top digit takes the rest)"""
    v = [0] * W
    for k in range(ND):
        v[B + k] = (x >> (DIG * k)) & M
    v[TOP] = x >> (DIG * (ND - 1))
    return v


def spread(K):
    """K*p at lanes B..TOP with digits 0..8 raised by 2^26 (the next digit pays)"""
    s = digits(K * P)
    for k in range(ND - 1):
        s[B + k] += 1 << DIG
        s[B + k + 1] -= 1
    assert val_at(s, B) == K * P and min(s) >= 0
    return s


def window_product(u, v):
    """lane j: sum_i u_(B+i) * v_(B+j-i) (u, v digits at lanes B..TOP)"""
    out = [0] * W
    for j in range(W):
        s = 0
        for i in range(ND):
            if 0 <= j - i < ND:
                s += u[B + i] * v[B + j - i]
        out[j] = s
    return out


def redc(T):
    """signed 64-bit columns (lanes 0..18) -> signed int32 digits at lanes B..TOP (TOP a wrapped sink) of T / R,
    value in (-3p, T/R + 3p).  One split for m; the low part's quotient from the split digits (32-bit)."""
    i64(T)
    tv = val_cols(T)
    d = split64(T)                                 # lanes 0..20
    i32(d)
    assert val_cols(d) == tv
    m = [sum(d[i] * PID[j - i] for i in range(j + 1)) if j < ND else 0 for j in range(W)]
    i64(m)
    m = split64(m)
    m = [x if j < ND else 0 for j, x in enumerate(m)]   # mod R
    i32(m)
    assert (val_cols(m) * P + val_cols(d)) % R == 0
    s = [d[j] + sum(m[i] * PD[j - i] for i in range(ND) if 0 <= j - i < ND) for j in range(W)]
    i64(s)
    total = val_cols(s)
    # lane 20 joins the sink (lane 19), then one split with the sink
    assert all(x == 0 for x in s[21:])
    s2 = list(s)
    s2[TOP] += s2[TOP + 1] << DIG
    s2[TOP + 1] = 0
    r = split64(s2, sink=TOP)
    assert val_cols(r) == total and all(x == 0 for x in r[TOP + 1:])
    i32(r[:TOP])
    # q = (low part of r) / R exactly, from lanes 7, 8, 9 in 32-bit arithmetic
    a = [x >> DIG for x in r]
    b = [x + y for x, y in zip(r, shr1(a))]
    c = [x >> DIG for x in b]
    t = [x + y for x, y in zip(r, shr1(c))]
    q = [(x + 2) >> DIG for x in t]
    i32(t[:ND])
    low = sum(r[j] << (DIG * j) for j in range(ND))
    assert low == q[ND - 1] * R, (low / R, q[ND - 1])
    o = [x if j >= B else 0 for j, x in enumerate(r)]
    o = [x + y if j == B else x for j, x, y in zip(range(W), o, shr1(q))]
    i32(o)
    assert val_at(o, B) == total // R
    assert (val_at(o, B) - tv * pow(R, -1, P)) % P == 0
    return o


def fold(y, digits_in=False):
    """signed int64 per lane (lanes B..TOP; TOP may be large) -> non-negative digits, 0..8 <= 2^26 + 2, value in [0, 5p)"""
    i64(y)
    v0 = val_at(y, B)
    d = split64(y, sink=TOP) if not digits_in else list(y)
    i64(d)
    X = f32(float(d[TOP]))
    q = int((f32(X * FOLD_C)) // 1)
    z = [d[j] - q * PD[j - B] if B <= j <= TOP else d[j] for j in range(W)]
    i64(z)
    z = split64(z, sink=TOP)
    i32(z)
    z = split32(z, sink=TOP)
    chk(z[B:TOP], -1, (1 << DIG) + 2, "fold z")
    S = spread(3)
    r = [a + b for a, b in zip(z, S)]
    chk(r, 0, 1 << 31, "fold r")
    r = split32(r, sink=TOP)
    chk(r[B:TOP], 0, (1 << DIG) + 3, "fold out")
    chk(r[TOP:TOP + 1], 0, 1 << 23, "fold top")
    assert all(x == 0 for x in r[:B] + r[TOP + 1:])
    assert (val_at(r, B) - v0) % P == 0 and 0 <= val_at(r, B) < 5 * P, val_at(r, B) / P
    return r


def rand_e():
    return fold(digits(random.randrange(0, 60 * P)))


def xi_c(y0, y1, c):
    """(xi * y).c per digit, non-negative: c = 0: 9 y0 - y1 + S(8), c = 1: 9 y1 + y0"""
    if c == 0:
        S = spread(8)
        r = [9 * a - b + s for a, b, s in zip(y0, y1, S)]
    else:
        r = [9 * b + a for a, b in zip(y0, y1)]
    u32(r)
    return r


def cyc(z):
    """Granger-Scott squaring (fq12.rs:198-247 as fq12_wide.h w12_cyc) of coordinates z[cid], cid = 2e + c"""
    prods = {}
    for cid in range(12):
        e, c = cid >> 1, cid & 1
        hi = e >= 3
        k = e - 3 if hi else e
        x0, x1, y0, y1 = z[2 * k], z[2 * k + 1], z[2 * k + 6], z[2 * k + 7]
        if hi:
            u0 = [a + b for a, b in zip(x0, y0)]
            u1 = [a + b for a, b in zip(x1, y1)]
            v0 = [a + b for a, b in zip(xi_c(y0, y1, 0), x0)]
            v1 = [a + b for a, b in zip(xi_c(y0, y1, 1), x1)]
        else:
            u0, u1, v0, v1 = x0, x1, y0, y1
        for a in (u0, u1, v0, v1):
            u32(a)
        vo, vp = (v0, v1) if c == 0 else (v1, v0)
        a1 = window_product(u0, vo)
        a2 = window_product(u1, vp)
        chk(a1 + a2, 0, 1 << 63, "columns")
        T = [x - y if c == 0 else x + y for x, y in zip(a1, a2)]
        prods[cid] = redc(T)
    out = []
    for cid in range(12):
        e, c = cid >> 1, cid & 1
        a = z[cid]
        ka = e >> 1

        def xi_p(p0, p1):
            return [9 * x - y for x, y in zip(p0, p1)] if c == 0 else [9 * y + x for x, y in zip(p0, p1)]
        if e % 2 == 0:
            t = [u - v - w for u, v, w in zip(prods[2 * (ka + 3) + c], prods[2 * ka + c], xi_p(prods[2 * ka], prods[2 * ka + 1]))]
            y = [3 * tt - 2 * aa for tt, aa in zip(t, a)]
        else:
            px = xi_p(prods[4], prods[5]) if e == 1 else prods[(e - 3) + c]
            y = [6 * x + 2 * aa for x, aa in zip(px, a)]
        out.append(fold(y))
    return out


def mul(a, b):
    """a * b (fq12.rs:319-327) on the w-basis: out_e = sum_i a'_i b_(e-i mod 6), a'_i = xi a_i when i > e"""
    out = []
    for cid in range(12):
        e, c = cid >> 1, cid & 1
        pos = [0] * W
        neg = [0] * W
        for i in range(6):
            wrap = i > e
            j = e - i + 6 if wrap else e - i
            x0, x1 = a[2 * i], a[2 * i + 1]
            if wrap:
                x0, x1 = xi_c(a[2 * i], a[2 * i + 1], 0), xi_c(a[2 * i], a[2 * i + 1], 1)
            y0, y1 = b[2 * j], b[2 * j + 1]
            if c == 0:  # x0 y0 - x1 y1
                pos = [p + q for p, q in zip(pos, window_product(x0, y0))]
                neg = [p + q for p, q in zip(neg, window_product(x1, y1))]
            else:       # x0 y1 + x1 y0
                pos = [p + q for p, q in zip(pos, window_product(x0, y1))]
                pos = [p + q for p, q in zip(pos, window_product(x1, y0))]
        chk(pos + neg, 0, 1 << 63, "mul columns")
        T = [p - q for p, q in zip(pos, neg)]
        out.append(fold(redc(T), digits_in=True))
    return out


def ref_vals(z):
    return [val_at(x, B) % P for x in z]


def cyc_ref(v):
    Ri = pow(R, -1, P)

    def m2(a, b):
        return ((a[0] * b[0] - a[1] * b[1]) * Ri % P, (a[0] * b[1] + a[1] * b[0]) * Ri % P)

    def xi(a):
        return ((9 * a[0] - a[1]) % P, (9 * a[1] + a[0]) % P)
    co = [(v[2 * e], v[2 * e + 1]) for e in range(6)]
    t = []
    for k in range(3):
        x, y = co[k], co[k + 3]
        tmp = m2(x, y)
        s = ((x[0] + y[0]) % P, (x[1] + y[1]) % P)
        q = m2(s, tuple((a + b) % P for a, b in zip(xi(y), x)))
        t.append((tuple((a - b - c) % P for a, b, c in zip(q, tmp, xi(tmp))), tuple(2 * a % P for a in tmp)))
    (t0, t1), (t2, t3), (t4, t5) = t
    z0, z1, z2, z3, z4, z5 = co
    res = [tuple((3 * a - 2 * b) % P for a, b in zip(t0, z0)),
           tuple((3 * a + 2 * b) % P for a, b in zip(xi(t5), z1)),
           tuple((3 * a - 2 * b) % P for a, b in zip(t2, z2)),
           tuple((3 * a + 2 * b) % P for a, b in zip(t1, z3)),
           tuple((3 * a - 2 * b) % P for a, b in zip(t4, z4)),
           tuple((3 * a + 2 * b) % P for a, b in zip(t3, z5))]
    return [c for e in range(6) for c in res[e]]


def mul_ref(va, vb):
    Ri = pow(R, -1, P)
    out = []
    for e in range(6):
        for c in range(2):
            s = 0
            for i in range(6):
                j = (e - i) % 6
                x = (va[2 * i], va[2 * i + 1])
                if i > e:
                    x = ((9 * x[0] - x[1]) % P, (9 * x[1] + x[0]) % P)
                y = (vb[2 * j], vb[2 * j + 1])
                s += (x[0] * y[0] - x[1] * y[1]) if c == 0 else (x[0] * y[1] + x[1] * y[0])
            out.append(s * Ri % P)
    return out


def main(trials):
    random.seed(1)
    for t in range(trials):
        z = [rand_e() for _ in range(12)]
        assert ref_vals(cyc(z)) == cyc_ref(ref_vals(z)), t
        w = [rand_e() for _ in range(12)]
        assert ref_vals(mul(z, w)) == mul_ref(ref_vals(z), ref_vals(w)), t
        x = z
        for _ in range(3):  # chains stay bounded
            x = cyc(x)
    print("ds_model: %d trials ok (cyc, mul, chains)" % trials)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 100)
