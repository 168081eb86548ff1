"""substrate_bn -- Python mirror of the substrate-bn 0.6.0 pairing API
(risc0/paritytech-bn src/lib.rs) over the MI355X engine's C ABI.

Same names and argument meaning as the Rust crate for the batched hot path:

    pairing(p: G1, q: G2) -> Gt                        lib.rs:611-613
    pairing_batch([(G1, G2), ...]) -> Gt               lib.rs:615-623
    miller_loop_batch([(G2, G1), ...]) -> Gt           lib.rs:625-633 (raises CurveError)
    Gt.final_exponentiation() -> Gt | None             lib.rs:598-600
    G1 * Fr, G2 * Fr                                   lib.rs:425-431, 575-581
    Gt * Gt                                            lib.rs:603-609

and the wire formats and validation around it:

    Fq.from_slice / to_big_endian / sqrt               lib.rs:154-183
    Fq2.from_slice / sqrt                              lib.rs:238-267
    Fr.from_slice / to_big_endian                      lib.rs:45-55
    AffineG1.new, AffineG2.new (curve + order check)   lib.rs:413-415, 549-551
    G1.from_compressed, G2.from_compressed             lib.rs:359-375, 506-526
    Gt.pow(Fr)                                         lib.rs:592-594

plus the batched forms the reference lacks (pairing_many, g1_mul_many) that
the engine exists for.  Values keep the reference's memory images (canonical
Montgomery, little-endian u64 limbs), so a Gt compares equal exactly when the
reference's derived PartialEq would.  Every computation runs on the GPU; there
is no CPU fallback.
"""
import os

import numpy as np

from . import _native
from ._native import BnError, Context  # noqa: F401

P = 0x30644E72E131A029B85045B68181585D97816A916871CA8D3C208C16D87CFD47
R_ORDER = 0x30644E72E131A029B85045B68181585D2833E84879B9709143E1F593F0000001
_RM = 1 << 256


class FieldError(Exception):
    """lib.rs:99-104: InvalidSliceLength, InvalidU512Encoding, NotMember (args[0])."""


class CurveError(Exception):
    """lib.rs:106-116: InvalidEncoding, NotMember, Field(FieldError), ToAffineConversion (args[0])."""


class GroupError(Exception):
    """groups/mod.rs:89-92: NotOnCurve, NotInSubgroup (args[0])."""


_FIELD = {1: "InvalidSliceLength", 2: "InvalidU512Encoding", 3: "NotMember"}


def _curve_error(st):
    if st in _FIELD:
        return CurveError("Field", FieldError(_FIELD[st]))
    return CurveError({4: "InvalidEncoding", 5: "NotMember"}[st])


_ctx = None


def context():
    """Process-wide engine context on LOCAL_RANK's device (torch.distributed style)."""
    global _ctx
    if _ctx is None:
        _ctx = Context(int(os.environ.get("LOCAL_RANK", "0")))
    return _ctx


def _limbs(x):
    return np.array([(x >> (64 * i)) & 0xFFFFFFFFFFFFFFFF for i in range(4)], dtype=np.uint64)


def _int(l):
    return sum(int(v) << (64 * i) for i, v in enumerate(l))


class Fr:
    """Scalar in Montgomery form mod r (fields::Fr, fp.rs:166-193)."""
    __slots__ = ("img",)

    def __init__(self, img):
        self.img = np.ascontiguousarray(img, dtype=np.uint64).reshape(4)

    @classmethod
    def from_int(cls, v):
        return cls(_limbs((v % R_ORDER) * _RM % R_ORDER))

    @classmethod
    def from_str(cls, s):
        """fp.rs:23-43: ASCII decimal digits only (char::to_digit(10)), reduced mod r;
        the empty string is zero; any other character gives None."""
        if not all(c in "0123456789" for c in s):
            return None
        return cls.from_int(int(s, 10) if s else 0)

    @classmethod
    def one(cls):
        return cls.from_int(1)

    @classmethod
    def zero(cls):
        return cls.from_int(0)

    def into_int(self):
        return _int(self.img) * pow(_RM, -1, R_ORDER) % R_ORDER

    def __neg__(self):
        return Fr.from_int(-self.into_int())

    @classmethod
    def from_slice(cls, b):  # lib.rs:45-49: new_mul_factor reduces mod r
        if len(b) != 32:
            raise FieldError("InvalidSliceLength")
        return cls(context().fr_from_slice_many(np.frombuffer(bytes(b), np.uint8))[0])

    def to_big_endian(self):  # lib.rs:50-55: the raw Montgomery image
        return bytes(context().fr_to_big_endian_many(self.img)[0])

    def __eq__(self, o):
        return isinstance(o, Fr) and np.array_equal(self.img, o.img)


class Fq:
    """Base-field element in Montgomery form (fields::Fq, fp.rs:195-222)."""
    __slots__ = ("img",)

    def __init__(self, img):
        self.img = np.ascontiguousarray(img, dtype=np.uint64).reshape(4)

    @classmethod
    def from_int(cls, v):
        return cls(_limbs((v % P) * _RM % P))

    @classmethod
    def from_slice(cls, b):  # lib.rs:154-159
        if len(b) != 32:
            raise FieldError("InvalidSliceLength")
        out, st = context().fq_from_slice_many(np.frombuffer(bytes(b), np.uint8))
        if st[0]:
            raise FieldError(_FIELD[int(st[0])])
        return cls(out[0])

    def to_big_endian(self):  # lib.rs:160-170
        return bytes(context().fq_to_big_endian_many(self.img)[0])

    def sqrt(self):  # fp.rs:245-260
        out, ok = context().fq_sqrt_many(self.img)
        return Fq(out[0]) if ok[0] else None

    def into_int(self):
        return _int(self.img) * pow(_RM, -1, P) % P

    def __eq__(self, o):
        return isinstance(o, Fq) and np.array_equal(self.img, o.img)


class Fq2:
    """c0 + c1 u (fields::Fq2, fq2.rs); img = c0 limbs then c1 limbs."""
    __slots__ = ("img",)

    def __init__(self, img):
        self.img = np.ascontiguousarray(img, dtype=np.uint64).reshape(8)

    @classmethod
    def new(cls, a, b):  # lib.rs:238-240
        return cls(np.concatenate([a.img, b.img]))

    @classmethod
    def from_slice(cls, b):  # lib.rs:260-267
        if len(b) != 64:
            raise FieldError("InvalidU512Encoding")
        out, st = context().fq2_from_slice_many(np.frombuffer(bytes(b), np.uint8))
        if st[0]:
            raise FieldError(_FIELD[int(st[0])])
        return cls(out[0])

    def real(self):
        return Fq(self.img[:4])

    def imaginary(self):
        return Fq(self.img[4:])

    def sqrt(self):  # fq2.rs:208-224
        out, ok = context().fq2_sqrt_many(self.img)
        return Fq2(out[0]) if ok[0] else None

    def __eq__(self, o):
        return isinstance(o, Fq2) and np.array_equal(self.img, o.img)


class _Point:
    WIDTH = 0
    __slots__ = ("img",)

    def __init__(self, img):
        self.img = np.ascontiguousarray(img, dtype=np.uint64).reshape(self.WIDTH)

    def is_zero(self):  # mod.rs:246-248: z == 0
        z = self.img[2 * self.WIDTH // 3:]
        return not z.any()

    def same_image(self, o):
        return type(o) is type(self) and np.array_equal(self.img, o.img)

    # the group law on the engine (bn_{g1,g2}_*_many, lib.rs:388-423, 539-574)
    def _op(self, op, o=None):
        return context().group_op_many(self.GROUP, op, self.img, None if o is None else o.img)

    def __add__(self, o):  # mod.rs:294-334
        return type(self)(self._op("add", o)[0])

    def __sub__(self, o):  # mod.rs:352-358
        return type(self)(self._op("sub", o)[0])

    def __neg__(self):  # mod.rs:336-350
        return type(self)(self._op("neg")[0])

    def normalize(self):  # lib.rs:391-398 (in place, as the reference's &mut self)
        self.img = self._op("normalize")[0]

    def __eq__(self, o):  # PartialEq: projective equality, mod.rs:169-195
        return type(o) is type(self) and bool(self._op("eq", o)[0])

    def __ne__(self, o):
        return not self == o

    __hash__ = None


_MONT_ONE = _limbs(_RM % P)


class G1(_Point):
    """Jacobian G1 point (groups::G1, mod.rs:45-50, 371-402)."""
    WIDTH = 12
    GROUP = "g1"

    @classmethod
    def one(cls):  # mod.rs:381-392: (1, 2, 1)
        return cls(np.concatenate([_MONT_ONE, _limbs(2 * _RM % P), _MONT_ONE]))

    @classmethod
    def zero(cls):  # (0, 1, 0), mod.rs:230-236
        return cls(np.concatenate([np.zeros(4, np.uint64), _MONT_ONE, np.zeros(4, np.uint64)]))

    def __mul__(self, k):
        return G1(context().g1_mul_many(self.img, k.img)[0])

    @classmethod
    def from_compressed(cls, b):  # lib.rs:359-375
        if len(b) != 33:
            raise CurveError("InvalidEncoding")
        out, st = context().g1_from_compressed_many(np.frombuffer(bytes(b), np.uint8))
        if st[0]:
            raise _curve_error(int(st[0]))
        return cls(out[0])

    def x(self):
        return Fq(self.img[0:4])

    def y(self):
        return Fq(self.img[4:8])

    def z(self):
        return Fq(self.img[8:12])


class G2(_Point):
    """Jacobian G2 point over Fq2 (groups::G2, mod.rs:408-472)."""
    WIDTH = 24
    GROUP = "g2"
    _X = (10857046999023057135944570762232829481370756359578518086990519993285655852781,
          11559732032986387107991004021392285783925812861821192530917403151452391805634)
    _Y = (8495653923123431417604973247489272438418190587263600148770280649306958101930,
          4082367875863433681332203403145435568316851327593401208105741076214120093531)

    @classmethod
    def one(cls):  # mod.rs:418-450 (EIP-197 generator), z = 1
        c = [cls._X[0], cls._X[1], cls._Y[0], cls._Y[1], 1, 0]
        return cls(np.concatenate([_limbs(v * _RM % P) for v in c]))

    @classmethod
    def zero(cls):
        z = np.zeros(4, np.uint64)
        return cls(np.concatenate([z, z, _MONT_ONE, z, z, z]))

    def __mul__(self, k):
        return G2(context().g2_mul_many(self.img, k.img)[0])

    @classmethod
    def from_compressed(cls, b):  # lib.rs:506-526
        if len(b) != 65:
            raise CurveError("InvalidEncoding")
        out, st = context().g2_from_compressed_many(np.frombuffer(bytes(b), np.uint8))
        if st[0]:
            raise _curve_error(int(st[0]))
        return cls(out[0])

    def x(self):
        return Fq2(self.img[0:8])

    def y(self):
        return Fq2(self.img[8:16])

    def z(self):
        return Fq2(self.img[16:24])


class AffineG1:
    """lib.rs:397-433; new() validates (mod.rs:95-113, G1: curve equation only)."""

    @staticmethod
    def new(x, y):
        out, st = context().g1_affine_new_many(x.img, y.img)
        if st[0]:
            raise GroupError({6: "NotOnCurve", 7: "NotInSubgroup"}[int(st[0])])
        return G1(out[0])  # From<AffineG1> for G1 (to_jacobian)


class AffineG2:
    """lib.rs:533-571; new() validates the curve equation and the order (mod.rs:95-113)."""

    @staticmethod
    def new(x, y):
        out, st = context().g2_affine_new_many(x.img, y.img)
        if st[0]:
            raise GroupError({6: "NotOnCurve", 7: "NotInSubgroup"}[int(st[0])])
        return G2(out[0])


class Gt:
    """Target group element (Gt(Fq12), lib.rs:584-609)."""
    __slots__ = ("img",)

    def __init__(self, img):
        self.img = np.ascontiguousarray(img, dtype=np.uint64).reshape(48)

    @classmethod
    def one(cls):
        img = np.zeros(48, np.uint64)
        img[:4] = _MONT_ONE
        return cls(img)

    def __mul__(self, o):
        return Gt(context().fq12_op_many("mul", self.img, o.img)[0])

    def pow(self, k):  # lib.rs:592-594
        return Gt(context().gt_pow_many(self.img, k.img)[0])

    def final_exponentiation(self):
        out, ok = context().final_exponentiation_many(self.img)
        return Gt(out[0]) if ok[0] else None

    def __eq__(self, o):
        return isinstance(o, Gt) and np.array_equal(self.img, o.img)

    def __ne__(self, o):
        return not self.__eq__(o)

    def __repr__(self):
        return "Gt(%s)" % ", ".join("%x" % _int(self.img[4 * k:4 * k + 4]) for k in range(12))


def pairing(p, q):
    return Gt(context().pairing_many(p.img, q.img)[0])


def pairing_batch(pairs):
    pairs = list(pairs)
    p = np.stack([a.img for a, _ in pairs]) if pairs else np.zeros((0, 12), np.uint64)
    q = np.stack([b.img for _, b in pairs]) if pairs else np.zeros((0, 24), np.uint64)
    return Gt(context().pairing_batch(p, q))


def miller_loop_batch(pairs):
    pairs = list(pairs)
    q = np.stack([a.img for a, _ in pairs]) if pairs else np.zeros((0, 24), np.uint64)
    p = np.stack([b.img for _, b in pairs]) if pairs else np.zeros((0, 12), np.uint64)
    try:
        return Gt(context().miller_loop_batch(q, p))
    except BnError as e:
        if e.code == _native.BN_ERR_TO_AFFINE:
            raise CurveError("ToAffineConversion") from None
        raise


# ---- batched forms (numpy arrays of memory images)
def pairing_many(p, q):
    return context().pairing_many(p, q)


def g1_mul_many(p, k):
    return context().g1_mul_many(p, k)


def g2_mul_many(p, k):
    return context().g2_mul_many(p, k)


def g2_affine_new_many(x, y):
    """(G2 images, bn_elem_status) for arrays of affine (x, y): AffineG2::new batched."""
    return context().g2_affine_new_many(x, y)


def g1_from_compressed_many(b33):
    return context().g1_from_compressed_many(b33)


def g2_from_compressed_many(b65):
    return context().g2_from_compressed_many(b65)


def gt_pow_many(a, k):
    return context().gt_pow_many(a, k)
