"""ctypes wrapper around oracle/liboracle_bn.so -- the CPU restatement of
substrate-bn 0.6.0 (see bn_oracle.h).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, never by the product package.

Data layout everywhere: numpy uint64 arrays in the reference memory image
(canonical Montgomery residues, 4 little-endian u64 limbs per Fq/Fr):
  G1 (n, 12) = x,y,z   G2 (n, 24) = x.c0,x.c1,y.c0,...   Gt/Fq12 (n, 48)
  Fq12 flatten order c0.c0.c0, c0.c0.c1, c0.c1.c0, ... (index 6i+2j+k).
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle_bn.so")

# Appendix A of SURVEY.md / src/fields/fp.rs:166-222
P = 0x30644E72E131A029B85045B68181585D97816A916871CA8D3C208C16D87CFD47
R = 0x30644E72E131A029B85045B68181585D2833E84879B9709143E1F593F0000001
RMONT = 1 << 256
U_PARAM = 4965661367192848881

FQ, FR = 0, 1
_MOD = {FQ: P, FR: R}


def to_mont(x, field=FQ):
    return (x % _MOD[field]) * RMONT % _MOD[field]


def from_mont(x, field=FQ):
    m = _MOD[field]
    return x * pow(RMONT, -1, m) % m


def int_to_limbs(x):
    return [(x >> (64 * i)) & 0xFFFFFFFFFFFFFFFF for i in range(4)]


def limbs_to_int(limbs):
    return sum(int(l) << (64 * i) for i, l in enumerate(limbs))


def ints_to_array(vals):
    """list of canonical-Montgomery ints -> flat uint64 array."""
    out = []
    for v in vals:
        out.extend(int_to_limbs(v))
    return np.array(out, dtype=np.uint64)


def array_to_ints(arr):
    a = np.asarray(arr, dtype=np.uint64).reshape(-1, 4)
    return [limbs_to_int(r) for r in a]


def canon_to_mont_array(vals, field=FQ):
    """canonical integers -> Montgomery memory image (what Fq::new / from_str give)."""
    return ints_to_array([to_mont(int(v), field) for v in vals])


def mont_array_to_canon(arr, field=FQ):
    return [from_mont(v, field) for v in array_to_ints(arr)]


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        vp, sz, i = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
        sigs = {
            "orc_fe_from_canonical": ([i, vp, vp], None),
            "orc_fe_to_canonical": ([i, vp, vp], None),
            "orc_fe_add": ([i, vp, vp, vp], None),
            "orc_fe_sub": ([i, vp, vp, vp], None),
            "orc_fe_mul": ([i, vp, vp, vp], None),
            "orc_fe_neg": ([i, vp, vp], None),
            "orc_fe_inverse": ([i, vp, vp], i),
            "orc_fq2_mul": ([vp, vp, vp], None),
            "orc_fq2_squared": ([vp, vp], None),
            "orc_fq2_inverse": ([vp, vp], i),
            "orc_fq6_mul": ([vp, vp, vp], None),
            "orc_fq6_squared": ([vp, vp], None),
            "orc_fq6_inverse": ([vp, vp], i),
            "orc_fq12_mul": ([vp, vp, vp], None),
            "orc_fq12_squared": ([vp, vp], None),
            "orc_fq12_add": ([vp, vp, vp], None),
            "orc_fq12_sub": ([vp, vp, vp], None),
            "orc_fq12_neg": ([vp, vp], None),
            "orc_fq12_inverse": ([vp, vp], i),
            "orc_fq12_frobenius_map": ([vp, i, vp], None),
            "orc_fq12_cyclotomic_squared": ([vp, vp], None),
            "orc_fq12_exp_by_neg_z": ([vp, vp], None),
            "orc_fq12_mul_by_024": ([vp, vp, vp, vp, vp], None),
            "orc_fq12_pow": ([vp, vp, vp], None),
            "orc_final_exponentiation": ([vp, vp], i),
            "orc_g1_one": ([vp], None),
            "orc_g2_one": ([vp], None),
            "orc_g1_add": ([vp, vp, vp], None),
            "orc_g1_double": ([vp, vp], None),
            "orc_g1_neg": ([vp, vp], None),
            "orc_g1_mul": ([vp, vp, vp], None),
            "orc_g1_eq": ([vp, vp], i),
            "orc_g1_to_affine": ([vp, vp, vp], i),
            "orc_g2_add": ([vp, vp, vp], None),
            "orc_g2_double": ([vp, vp], None),
            "orc_g2_neg": ([vp, vp], None),
            "orc_g2_mul": ([vp, vp, vp], None),
            "orc_g2_eq": ([vp, vp], i),
            "orc_g2_to_affine": ([vp, vp], i),
            "orc_g1_on_curve_affine": ([vp, vp], i),
            "orc_g2_precompute": ([vp, vp], None),
            "orc_miller_loop": ([vp, vp, vp, vp], None),
            "orc_pairing": ([vp, vp, vp], None),
            "orc_pairing_batch": ([vp, vp, sz, vp], None),
            "orc_miller_loop_batch": ([vp, vp, sz, vp], i),
            "orc_pairing_many": ([vp, vp, sz, vp, i], None),
            "orc_pairing_batch_mt": ([vp, vp, sz, vp, i], None),
            "orc_g1_mul_many": ([vp, vp, sz, vp, i], None),
            "orc_g2_mul_many": ([vp, vp, sz, vp, i], None),
            "orc_fq_from_slice": ([vp, vp], i),
            "orc_fq_to_big_endian": ([vp, vp], None),
            "orc_fq2_from_slice": ([vp, vp], i),
            "orc_fr_from_slice": ([vp, vp], None),
            "orc_fr_to_big_endian": ([vp, vp], None),
            "orc_u512_divrem": ([vp, vp, vp], i),
            "orc_fq_sqrt": ([vp, vp], i),
            "orc_fq2_sqrt": ([vp, vp], i),
            "orc_g1_affine_new": ([vp, vp, vp], i),
            "orc_g2_affine_new": ([vp, vp, vp], i),
            "orc_g1_from_compressed": ([vp, sz, vp], i),
            "orc_g2_from_compressed": ([vp, sz, vp], i),
            "orc_gt_pow": ([vp, vp, vp], None),
            "orc_decode_many": ([i, vp, sz, vp, vp, i], None),
        }
        for name, (args, res) in sigs.items():
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = res
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _u64(a, width):
    a = np.ascontiguousarray(a, dtype=np.uint64)
    assert a.size % width == 0, (a.shape, width)
    return a.reshape(-1, width)


# ---------------------------------------------------------------- scalars/elements
def fe_from_canonical(vals, field=FQ):
    return canon_to_mont_array(vals, field)


def unary(name, a, width, *extra):
    a = _u64(a, width)
    out = np.zeros_like(a)
    fn = getattr(lib(), name)
    rcs = []
    for k in range(a.shape[0]):
        rc = fn(*extra, _p(a[k]), _p(out[k])) if extra else fn(_p(a[k]), _p(out[k]))
        rcs.append(rc)
    return out, rcs


def binary(name, a, b, wa, wb, wo, *extra):
    a, b = _u64(a, wa), _u64(b, wb)
    n = max(a.shape[0], b.shape[0])
    out = np.zeros((n, wo), dtype=np.uint64)
    fn = getattr(lib(), name)
    for k in range(n):
        ak, bk = a[k % a.shape[0]], b[k % b.shape[0]]
        if extra:
            fn(*extra, _p(ak), _p(bk), _p(out[k]))
        else:
            fn(_p(ak), _p(bk), _p(out[k]))
    return out


def g1_one():
    out = np.zeros(12, dtype=np.uint64)
    lib().orc_g1_one(_p(out))
    return out


def g2_one():
    out = np.zeros(24, dtype=np.uint64)
    lib().orc_g2_one(_p(out))
    return out


def g1_mul(p, k, nthreads=1):
    p, k = _u64(p, 12), _u64(k, 4)
    n = max(p.shape[0], k.shape[0])
    if p.shape[0] != n:
        p = np.ascontiguousarray(np.broadcast_to(p, (n, 12)))
    if k.shape[0] != n:
        k = np.ascontiguousarray(np.broadcast_to(k, (n, 4)))
    out = np.zeros((n, 12), dtype=np.uint64)
    lib().orc_g1_mul_many(_p(p), _p(k), n, _p(out), nthreads)
    return out


def g2_mul(p, k, nthreads=1):
    p, k = _u64(p, 24), _u64(k, 4)
    n = max(p.shape[0], k.shape[0])
    if p.shape[0] != n:
        p = np.ascontiguousarray(np.broadcast_to(p, (n, 24)))
    if k.shape[0] != n:
        k = np.ascontiguousarray(np.broadcast_to(k, (n, 4)))
    out = np.zeros((n, 24), dtype=np.uint64)
    lib().orc_g2_mul_many(_p(p), _p(k), n, _p(out), nthreads)
    return out


def pairing_many(p, q, nthreads=1):
    p, q = _u64(p, 12), _u64(q, 24)
    n = p.shape[0]
    out = np.zeros((n, 48), dtype=np.uint64)
    lib().orc_pairing_many(_p(p), _p(q), n, _p(out), nthreads)
    return out


def pairing_batch(p, q, nthreads=None):
    """pairing_batch (mod.rs:904-926); nthreads splits the shared loop over
    threads (orc_pairing_batch_mt, the same result)."""
    p, q = _u64(p, 12), _u64(q, 24)
    out = np.zeros(48, dtype=np.uint64)
    if nthreads is None:
        lib().orc_pairing_batch(_p(p), _p(q), p.shape[0], _p(out))
    else:
        lib().orc_pairing_batch_mt(_p(p), _p(q), p.shape[0], _p(out), nthreads)
    return out


def miller_loop_batch(q, p):
    q, p = _u64(q, 24), _u64(p, 12)
    out = np.zeros(48, dtype=np.uint64)
    rc = lib().orc_miller_loop_batch(_p(q), _p(p), q.shape[0], _p(out))
    return rc, out


def final_exponentiation(f):
    f = _u64(f, 48)
    out = np.zeros_like(f)
    rcs = [lib().orc_final_exponentiation(_p(f[k]), _p(out[k])) for k in range(f.shape[0])]
    return out, rcs


def g2_precompute(q_affine):
    q = np.ascontiguousarray(q_affine, dtype=np.uint64).reshape(16)
    out = np.zeros((87, 24), dtype=np.uint64)
    lib().orc_g2_precompute(_p(q), _p(out))
    return out


def miller_loop(coeffs, px, py):
    c = np.ascontiguousarray(coeffs, dtype=np.uint64).reshape(87 * 24)
    px = np.ascontiguousarray(px, dtype=np.uint64).reshape(4)
    py = np.ascontiguousarray(py, dtype=np.uint64).reshape(4)
    out = np.zeros(48, dtype=np.uint64)
    lib().orc_miller_loop(_p(c), _p(px), _p(py), _p(out))
    return out


def g1_to_affine(p):
    p = _u64(p, 12)
    out = np.zeros((p.shape[0], 8), dtype=np.uint64)
    rcs = []
    for k in range(p.shape[0]):
        rcs.append(lib().orc_g1_to_affine(_p(p[k]), _p(out[k, :4]), _p(out[k, 4:])))
    return out, rcs


def g2_to_affine(q):
    q = _u64(q, 24)
    out = np.zeros((q.shape[0], 16), dtype=np.uint64)
    rcs = [lib().orc_g2_to_affine(_p(q[k]), _p(out[k])) for k in range(q.shape[0])]
    return out, rcs


def g1_add(a, b):  # mod.rs:294-334
    return binary("orc_g1_add", a, b, 12, 12, 12)


def g2_add(a, b):
    return binary("orc_g2_add", a, b, 24, 24, 24)


def g1_neg(a):  # mod.rs:336-350
    return unary("orc_g1_neg", a, 12)[0]


def g2_neg(a):
    return unary("orc_g2_neg", a, 24)[0]


def g1_sub(a, b):  # mod.rs:352-358: a + (-b)
    return g1_add(a, g1_neg(b))


def g2_sub(a, b):
    return g2_add(a, g2_neg(b))


def g1_normalize(a):
    """Group::normalize (lib.rs:391-398): to_affine then to_jacobian; zero unchanged."""
    a = _u64(a, 12)
    aff, rcs = g1_to_affine(a)
    out = a.copy()
    one = canon_to_mont_array([1]).reshape(4)
    for k, rc in enumerate(rcs):
        if rc == 0:
            out[k] = np.concatenate([aff[k], one])
    return out


def g2_normalize(a):
    a = _u64(a, 24)
    aff, rcs = g2_to_affine(a)
    out = a.copy()
    one = np.concatenate([canon_to_mont_array([1]).reshape(4), np.zeros(4, np.uint64)])
    for k, rc in enumerate(rcs):
        if rc == 0:
            out[k] = np.concatenate([aff[k], one])
    return out


def g1_eq(a, b):
    a, b = _u64(a, 12), _u64(b, 12)
    return [bool(lib().orc_g1_eq(_p(a[k]), _p(b[k]))) for k in range(a.shape[0])]


def g2_eq(a, b):
    a, b = _u64(a, 24), _u64(b, 24)
    return [bool(lib().orc_g2_eq(_p(a[k]), _p(b[k]))) for k in range(a.shape[0])]


# ---------------------------------------------------------------- encodings
# per-element status codes (bn_oracle.h ORC_*, == bn_elem_status of include/bn254mi.h)
OK, FIELD_INVALID_SLICE_LENGTH, FIELD_INVALID_U512, FIELD_NOT_MEMBER = 0, 1, 2, 3
CURVE_INVALID_ENCODING, CURVE_NOT_MEMBER, GROUP_NOT_ON_CURVE, GROUP_NOT_IN_SUBGROUP = 4, 5, 6, 7


def _u8(a, width):
    a = np.ascontiguousarray(a, dtype=np.uint8)
    assert a.size % width == 0, (a.shape, width)
    return a.reshape(-1, width)


def _rows(fn, inp, win, wout, dtype_out=np.uint64, has_status=True):
    """apply fn(in_row, out_row) -> status to every row."""
    out = np.zeros((inp.shape[0], wout), dtype=dtype_out)
    st = np.zeros(inp.shape[0], dtype=np.uint8)
    for k in range(inp.shape[0]):
        rc = fn(_p(inp[k]), _p(out[k]))
        if has_status:
            st[k] = rc
    return out, st


def fq_from_slice(be):
    return _rows(lib().orc_fq_from_slice, _u8(be, 32), 32, 4)


def fq_to_big_endian(a):
    return _rows(lib().orc_fq_to_big_endian, _u64(a, 4), 4, 32, np.uint8, False)[0]


def fq2_from_slice(be):
    return _rows(lib().orc_fq2_from_slice, _u8(be, 64), 64, 8)


def fr_from_slice(be):
    return _rows(lib().orc_fr_from_slice, _u8(be, 32), 32, 4, has_status=False)[0]


def fr_to_big_endian(a):
    return _rows(lib().orc_fr_to_big_endian, _u64(a, 4), 4, 32, np.uint8, False)[0]


def u512_divrem(be64):
    """(q, r, q_is_some) of U512::divrem by the Fq modulus, plain integers."""
    b = _u8(be64, 64)[0]
    q = np.zeros(4, dtype=np.uint64)
    r = np.zeros(4, dtype=np.uint64)
    some = lib().orc_u512_divrem(_p(b), _p(q), _p(r))
    return limbs_to_int(q), limbs_to_int(r), bool(some)


def fq_sqrt(a):
    out, st = _rows(lib().orc_fq_sqrt, _u64(a, 4), 4, 4)
    return out, st == 0


def fq2_sqrt(a):
    out, st = _rows(lib().orc_fq2_sqrt, _u64(a, 8), 8, 8)
    return out, st == 0


def g1_affine_new(x, y):
    x, y = _u64(x, 4), _u64(y, 4)
    out = np.zeros((x.shape[0], 12), dtype=np.uint64)
    st = np.array([lib().orc_g1_affine_new(_p(x[k]), _p(y[k]), _p(out[k])) for k in range(x.shape[0])], np.uint8)
    return out, st


def g2_affine_new(x, y, nthreads=1):
    x, y = _u64(x, 8), _u64(y, 8)
    xy = np.ascontiguousarray(np.concatenate([x, y], axis=1))
    n = x.shape[0]
    out = np.zeros((n, 24), dtype=np.uint64)
    st = np.zeros(n, dtype=np.uint8)
    lib().orc_decode_many(2, _p(xy), n, _p(out), _p(st), nthreads)
    return out, st


def g1_from_compressed(b, nthreads=1):
    b = _u8(b, 33)
    n = b.shape[0]
    out = np.zeros((n, 12), dtype=np.uint64)
    st = np.zeros(n, dtype=np.uint8)
    lib().orc_decode_many(0, _p(b), n, _p(out), _p(st), nthreads)
    return out, st


def g2_from_compressed(b, nthreads=1):
    b = _u8(b, 65)
    n = b.shape[0]
    out = np.zeros((n, 24), dtype=np.uint64)
    st = np.zeros(n, dtype=np.uint8)
    lib().orc_decode_many(1, _p(b), n, _p(out), _p(st), nthreads)
    return out, st


def g1_from_compressed_one(b):
    """G1::from_compressed on one slice of any length (length errors included)."""
    buf = np.frombuffer(bytes(b) + b"\0", dtype=np.uint8).copy()
    out = np.zeros(12, dtype=np.uint64)
    st = lib().orc_g1_from_compressed(_p(buf), len(b), _p(out))
    return out, st


def g2_from_compressed_one(b):
    buf = np.frombuffer(bytes(b) + b"\0", dtype=np.uint8).copy()
    out = np.zeros(24, dtype=np.uint64)
    st = lib().orc_g2_from_compressed(_p(buf), len(b), _p(out))
    return out, st


def gt_pow(a, k):
    return binary("orc_gt_pow", a, k, 48, 4, 48)


# ---------------------------------------------------------------- seeded inputs
class SplitMix64:
    """Deterministic host PRNG for synthetic inputs (stated seed per run)."""

    def __init__(self, seed):
        self.s = seed & 0xFFFFFFFFFFFFFFFF

    def next(self):
        self.s = (self.s + 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF
        z = self.s
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
        return z ^ (z >> 31)

    def below(self, m):
        """uniform in [0, m) by rejection on 256-bit draws masked to m's bit length."""
        bits = m.bit_length()
        while True:
            v = 0
            for i in range(4):
                v |= self.next() << (64 * i)
            v &= (1 << bits) - 1
            if v < m:
                return v


def random_scalars(n, seed, lo=1):
    """n Fr scalars uniform in [lo, r), as Montgomery Fr images (n, 4)."""
    g = SplitMix64(seed)
    vals = []
    for _ in range(n):
        v = g.below(R)
        while v < lo:
            v = g.below(R)
        vals.append(v)
    return vals, canon_to_mont_array(vals, FR).reshape(n, 4)


def random_pairs(n, seed, nthreads=8):
    """P_i = s_i * G1::one(), Q_i = t_i * G2::one(), Jacobian (z != 1), SURVEY.md §8(d)."""
    s_vals, s = random_scalars(n, seed)
    t_vals, t = random_scalars(n, seed ^ 0x5DEECE66D)
    p = g1_mul(g1_one(), s, nthreads)
    q = g2_mul(g2_one(), t, nthreads)
    return p, q, s, t
