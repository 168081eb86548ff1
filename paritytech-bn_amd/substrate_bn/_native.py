"""ctypes binding of libbn254mi.so (include/bn254mi.h).

The product path: every call runs the HIP kernels on an MI355X.  There is no
CPU fallback -- if the library or a GPU is missing the calls raise.
Arrays are numpy uint64 in the reference memory image:
  G1 (n, 12), G2 (n, 24), Gt (n, 48), Fr (n, 4).
"""
import ctypes
import os

import numpy as np

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("BN254MI_LIB") or os.path.join(PKG_DIR, "libbn254mi.so")  # override: A/B builds

BN_OK = 0
BN_ERR_INVALID_ARGUMENT = 1
BN_ERR_TO_AFFINE = 2
BN_ERR_FE_ZERO = 3
BN_ERR_HIP = 4
BN_ERR_NO_DEVICE = 5
BN_ERR_INTERNAL = 6

FQ12_OPS = {"mul": 0, "sqr": 1, "inv": 2, "cyc_sqr": 3, "exp_by_neg_z": 4, "frob1": 5, "frob2": 6, "frob3": 7}

# every symbol include/bn254mi.h declares (checked by tests/test_capi_symbols.py)
EXPORTS = [
    "bn_ctx_create", "bn_ctx_destroy", "bn_last_error", "bn_ctx_stream",
    "bn_pairing_many", "bn_pairing_many_dev", "bn_pairing_batch", "bn_miller_loop_batch",
    "bn_final_exponentiation_many", "bn_miller_loop_many",
    "bn_g1_mul_many", "bn_g1_mul_many_dev", "bn_g2_mul_many", "bn_g2_mul_many_dev",
    "bn_fq12_op_many", "bn_workspace_bytes", "bn_reserve", "bn_set_phase_timing", "bn_get_phase_times",
    "bn_fq_from_slice_many", "bn_fq_to_big_endian_many", "bn_fq2_from_slice_many", "bn_fr_from_slice_many",
    "bn_fr_to_big_endian_many", "bn_fq_sqrt_many", "bn_fq2_sqrt_many", "bn_g1_affine_new_many",
    "bn_g2_affine_new_many", "bn_g2_affine_new_many_dev", "bn_g1_from_compressed_many", "bn_g2_from_compressed_many",
    "bn_g1_from_compressed_many_dev", "bn_g2_from_compressed_many_dev", "bn_gt_pow_many", "bn_gt_pow_many_dev",
    "bn_ctx_create_multi", "bn_ctx_num_devices", "bn_ctx_device", "bn_shard_range", "bn_pairing_many_allgather_dev",
    "bn_pairing_batch_dev", "bn_miller_loop_batch_dev", "bn_set_fe_wide_max", "bn_g2_precompute_many",
    "bn_set_latency_max", "bn_dev_status",
] + ["bn_%s_%s_many%s" % (g, op, dev) for g in ("g1", "g2") for op in ("add", "sub", "neg", "normalize", "eq")
     for dev in ("", "_dev")]
GROUP_OPS = ("add", "sub", "neg", "normalize", "eq")

# per-element status (bn_elem_status)
ST_OK, ST_FIELD_INVALID_SLICE_LENGTH, ST_FIELD_INVALID_U512, ST_FIELD_NOT_MEMBER = 0, 1, 2, 3
ST_CURVE_INVALID_ENCODING, ST_CURVE_NOT_MEMBER, ST_GROUP_NOT_ON_CURVE, ST_GROUP_NOT_IN_SUBGROUP = 4, 5, 6, 7


class BnError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("bn254mi error %d: %s" % (code, msg))
        self.code = code


_lib = None


def load():
    """Load the native library (raises if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError("libbn254mi.so not built: run `make -C paritytech-bn_amd` "
                          "(or __graft_entry__.build())")
    # One HIP runtime per process: torch ships its own libamdhip64.so.7 (and HSA
    # runtime).  Loaded first, it satisfies this library's libamdhip64.so.7 by
    # SONAME, so engine calls and torch tensors/streams/RCCL share one runtime;
    # loaded the other way round the process would hold two runtimes.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = ctypes.CDLL(LIB_PATH)
    vp, sz, i, u8p = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p
    sig = {
        "bn_ctx_create": ([i, ctypes.POINTER(vp)], i),
        "bn_ctx_destroy": ([vp], i),
        "bn_last_error": ([vp], ctypes.c_char_p),
        "bn_ctx_stream": ([vp], vp),
        "bn_pairing_many": ([vp, vp, vp, sz, vp], i),
        "bn_pairing_many_dev": ([vp, vp, vp, sz, vp, vp], i),
        "bn_pairing_batch": ([vp, vp, vp, sz, vp], i),
        "bn_miller_loop_batch": ([vp, vp, vp, sz, vp], i),
        "bn_final_exponentiation_many": ([vp, vp, sz, vp, u8p], i),
        "bn_miller_loop_many": ([vp, vp, vp, sz, vp], i),
        "bn_g1_mul_many": ([vp, vp, vp, sz, vp], i),
        "bn_g1_mul_many_dev": ([vp, vp, vp, sz, vp, vp], i),
        "bn_g2_mul_many": ([vp, vp, vp, sz, vp], i),
        "bn_g2_mul_many_dev": ([vp, vp, vp, sz, vp, vp], i),
        "bn_fq12_op_many": ([vp, i, vp, vp, sz, vp], i),
        "bn_workspace_bytes": ([sz], sz),
        "bn_reserve": ([vp, sz], i),
        "bn_set_phase_timing": ([vp, i], i),
        "bn_get_phase_times": ([vp, vp, vp], i),
        "bn_fq_from_slice_many": ([vp, vp, sz, vp, vp], i),
        "bn_fq_to_big_endian_many": ([vp, vp, sz, vp], i),
        "bn_fq2_from_slice_many": ([vp, vp, sz, vp, vp], i),
        "bn_fr_from_slice_many": ([vp, vp, sz, vp], i),
        "bn_fr_to_big_endian_many": ([vp, vp, sz, vp], i),
        "bn_fq_sqrt_many": ([vp, vp, sz, vp, vp], i),
        "bn_fq2_sqrt_many": ([vp, vp, sz, vp, vp], i),
        "bn_g1_affine_new_many": ([vp, vp, vp, sz, vp, vp], i),
        "bn_g2_affine_new_many": ([vp, vp, vp, sz, vp, vp], i),
        "bn_g2_affine_new_many_dev": ([vp, vp, vp, sz, vp, vp, vp], i),
        "bn_g1_from_compressed_many": ([vp, vp, sz, vp, vp], i),
        "bn_g2_from_compressed_many": ([vp, vp, sz, vp, vp], i),
        "bn_g1_from_compressed_many_dev": ([vp, vp, sz, vp, vp, vp], i),
        "bn_g2_from_compressed_many_dev": ([vp, vp, sz, vp, vp, vp], i),
        "bn_gt_pow_many": ([vp, vp, vp, sz, vp], i),
        "bn_gt_pow_many_dev": ([vp, vp, vp, sz, vp, vp], i),
        "bn_ctx_create_multi": ([vp, i, ctypes.POINTER(vp)], i),
        "bn_ctx_num_devices": ([vp], i),
        "bn_ctx_device": ([vp, i], vp),
        "bn_shard_range": ([sz, i, i, ctypes.POINTER(sz), ctypes.POINTER(sz)], None),
        "bn_pairing_many_allgather_dev": ([vp, vp, vp, sz, vp, vp], i),
        "bn_pairing_batch_dev": ([vp, vp, vp, sz, vp, vp, vp], i),
        "bn_miller_loop_batch_dev": ([vp, vp, vp, sz, vp, vp, vp], i),
        "bn_set_fe_wide_max": ([vp, sz], i),
        "bn_set_latency_max": ([vp, sz], i),
        "bn_g2_precompute_many": ([vp, vp, sz, vp], i),
        "bn_dev_status": ([vp, vp], i),
    }
    for g in ("g1", "g2"):
        for op in GROUP_OPS:
            unary = op in ("neg", "normalize")
            sig["bn_%s_%s_many" % (g, op)] = ([vp, vp, sz, vp] if unary else [vp, vp, vp, sz, vp], i)
            sig["bn_%s_%s_many_dev" % (g, op)] = ([vp, vp, sz, vp, vp] if unary else [vp, vp, vp, sz, vp, vp], i)
    ab_build = bool(os.environ.get("BN254MI_LIB"))  # an A/B build may predate newer entry points
    for name, (args, res) in sig.items():
        if ab_build and not hasattr(L, name):
            continue
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = res
    _lib = L
    return L


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _arr(a, width):
    a = np.ascontiguousarray(a, dtype=np.uint64)
    if a.size % width:
        raise ValueError("array of %d words is not a multiple of %d" % (a.size, width))
    return a.reshape(-1, width)


def _same_rows(*arrays):
    """Row count shared by paired inputs; a mismatch raises before any native call
    (the C ABI reads n rows from every buffer)."""
    n = arrays[0].shape[0]
    for a in arrays[1:]:
        if a.shape[0] != n:
            raise ValueError("paired inputs have %d and %d rows" % (n, a.shape[0]))
    return n


def shard_range(n, ndev, k):
    """[lo, hi) of shard k of n elements over ndev devices (the C ABI's split)."""
    lo, hi = ctypes.c_size_t(), ctypes.c_size_t()
    load().bn_shard_range(n, ndev, k, ctypes.byref(lo), ctypes.byref(hi))
    return lo.value, hi.value


class Context:
    """One device context (bn_ctx), or with `devices=[...]` one context over several
    devices of the node (bn_ctx_create_multi).  All arrays are reference memory images."""

    def __init__(self, device=0, devices=None):
        L = load()
        h = ctypes.c_void_p()
        if devices is None:
            rc = L.bn_ctx_create(device, ctypes.byref(h))
        else:
            arr = (ctypes.c_int * len(devices))(*devices)
            rc = L.bn_ctx_create_multi(arr, len(devices), ctypes.byref(h))
        if rc != BN_OK:
            raise BnError(rc, "bn_ctx_create(%s) failed" % (device if devices is None else devices))
        self._h = h
        self._L = L

    @property
    def num_devices(self):
        return self._L.bn_ctx_num_devices(self._h)

    def pairing_many_allgather_dev(self, d_p, d_q, n_per_dev, d_out, streams=None):
        """Config 4 in one process: per-device pointer lists (ints); every d_out[k]
        receives all num_devices * n_per_dev results in device order."""
        nd = len(d_p)
        vp = ctypes.c_void_p
        arr = lambda xs: (vp * nd)(*xs)  # noqa: E731
        self._check(self._L.bn_pairing_many_allgather_dev(self._h, arr(d_p), arr(d_q), n_per_dev, arr(d_out),
                                                          arr(streams) if streams else None))

    def device(self, k):
        """Device k's single-device context of a multi-device context (bn_ctx_device):
        owned by this context, valid while it lives."""
        h = self._L.bn_ctx_device(self._h, k)
        if not h:
            raise BnError(BN_ERR_INVALID_ARGUMENT, "no device %d in this context" % k)
        sub = Context.__new__(Context)
        sub._h = ctypes.c_void_p(h)
        sub._L = self._L
        sub._owner = self  # keeps the parent (which destroys it) alive
        return sub

    def dev_status(self, stream=None):
        """bn_dev_status: synchronize and raise on the sticky device outcome of the
        status-less _dev calls (BN_ERR_INTERNAL, BN_ERR_FE_ZERO); clears it."""
        self._check(self._L.bn_dev_status(self._h, stream))

    def close(self):
        if getattr(self, "_owner", None) is not None:  # a device of a multi-device context
            self._h = None
            return
        if getattr(self, "_h", None):
            self._L.bn_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc):
        if rc != BN_OK:
            raise BnError(rc, (self._L.bn_last_error(self._h) or b"").decode())

    @property
    def handle(self):
        return self._h

    @property
    def stream(self):
        return self._L.bn_ctx_stream(self._h)

    # ---- group law (lib.rs:388-423, 539-574)
    def group_op_many(self, group, op, a, b=None):
        """bn_{g1,g2}_{add,sub,neg,normalize,eq}_many: rows of a (and b); eq returns a
        uint8 array, the others point images."""
        w = {"g1": 12, "g2": 24}[group]
        a = _arr(a, w)
        args = [self._h, _ptr(a)]
        if op not in ("neg", "normalize"):
            b = _arr(b, w)
            _same_rows(a, b)
            args.append(_ptr(b))
        out = np.zeros(a.shape[0], np.uint8) if op == "eq" else np.zeros((a.shape[0], w), np.uint64)
        self._check(getattr(self._L, "bn_%s_%s_many" % (group, op))(*args, a.shape[0], _ptr(out)))
        return out

    def group_op_many_dev(self, group, op, d_a, d_b, n, d_out, stream=None):
        fn = getattr(self._L, "bn_%s_%s_many_dev" % (group, op))
        if op in ("neg", "normalize"):
            self._check(fn(self._h, d_a, n, d_out, stream))
        else:
            self._check(fn(self._h, d_a, d_b, n, d_out, stream))

    # ---- pairing path
    def pairing_many(self, p, q):
        p, q = _arr(p, 12), _arr(q, 24)
        _same_rows(p, q)
        out = np.zeros((p.shape[0], 48), np.uint64)
        self._check(self._L.bn_pairing_many(self._h, _ptr(p), _ptr(q), p.shape[0], _ptr(out)))
        return out

    def pairing_batch(self, p, q):
        p, q = _arr(p, 12), _arr(q, 24)
        _same_rows(p, q)
        out = np.zeros(48, np.uint64)
        self._check(self._L.bn_pairing_batch(self._h, _ptr(p), _ptr(q), p.shape[0], _ptr(out)))
        return out

    def miller_loop_batch(self, q, p):
        q, p = _arr(q, 24), _arr(p, 12)
        _same_rows(q, p)
        out = np.zeros(48, np.uint64)
        self._check(self._L.bn_miller_loop_batch(self._h, _ptr(q), _ptr(p), q.shape[0], _ptr(out)))
        return out

    def miller_loop_many(self, p, q):
        p, q = _arr(p, 12), _arr(q, 24)
        _same_rows(p, q)
        out = np.zeros((p.shape[0], 48), np.uint64)
        self._check(self._L.bn_miller_loop_many(self._h, _ptr(p), _ptr(q), p.shape[0], _ptr(out)))
        return out

    def g2_precompute_many(self, q):
        """AffineG2::precompute of each (Jacobian) q: (n, 87, 24) uint64 -- per coefficient
        ell_0, ell_vw, ell_vv (mod.rs:566-577, 701-727)."""
        q = _arr(q, 24)
        out = np.zeros((q.shape[0], 87, 24), np.uint64)
        self._check(self._L.bn_g2_precompute_many(self._h, _ptr(q), q.shape[0], _ptr(out)))
        return out

    def final_exponentiation_many(self, f):
        f = _arr(f, 48)
        out = np.zeros_like(f)
        ok = np.zeros(f.shape[0], np.uint8)
        self._check(self._L.bn_final_exponentiation_many(self._h, _ptr(f), f.shape[0], _ptr(out), _ptr(ok)))
        return out, ok

    # ---- group path
    def g1_mul_many(self, p, k):
        p, k = _arr(p, 12), _arr(k, 4)
        _same_rows(p, k)
        out = np.zeros_like(p)
        self._check(self._L.bn_g1_mul_many(self._h, _ptr(p), _ptr(k), p.shape[0], _ptr(out)))
        return out

    def g2_mul_many(self, p, k):
        p, k = _arr(p, 24), _arr(k, 4)
        _same_rows(p, k)
        out = np.zeros_like(p)
        self._check(self._L.bn_g2_mul_many(self._h, _ptr(p), _ptr(k), p.shape[0], _ptr(out)))
        return out

    def fq12_op_many(self, op, a, b=None):
        a = _arr(a, 48)
        bb = _arr(b, 48) if b is not None else None
        if op == "mul":
            if bb is None:
                raise ValueError("fq12 mul needs two operands")
            _same_rows(a, bb)
        out = np.zeros_like(a)
        self._check(self._L.bn_fq12_op_many(self._h, FQ12_OPS[op], _ptr(a), _ptr(bb) if bb is not None else None,
                                            a.shape[0], _ptr(out)))
        return out

    # ---- device-pointer variants (ints: device addresses, e.g. torch tensor.data_ptr())
    def pairing_many_dev(self, d_p, d_q, n, d_out, stream=None):
        self._check(self._L.bn_pairing_many_dev(self._h, d_p, d_q, n, d_out, stream))

    def g1_mul_many_dev(self, d_p, d_k, n, d_out, stream=None):
        self._check(self._L.bn_g1_mul_many_dev(self._h, d_p, d_k, n, d_out, stream))

    def g2_mul_many_dev(self, d_p, d_k, n, d_out, stream=None):
        self._check(self._L.bn_g2_mul_many_dev(self._h, d_p, d_k, n, d_out, stream))

    def pairing_batch_dev(self, d_p, d_q, n, d_out, d_status=None, stream=None):
        self._check(self._L.bn_pairing_batch_dev(self._h, d_p, d_q, n, d_out, d_status, stream))

    def miller_loop_batch_dev(self, d_q, d_p, n, d_out, d_status=None, stream=None):
        self._check(self._L.bn_miller_loop_batch_dev(self._h, d_q, d_p, n, d_out, d_status, stream))

    def set_fe_wide_max(self, n):
        """Batches of at most n elements use the 16-lane final exponentiation (latency path)."""
        self._check(self._L.bn_set_fe_wide_max(self._h, n))

    def set_latency_max(self, n):
        """Latency-path batches of at most n pairs run the one-launch k_pairing_latency."""
        self._check(self._L.bn_set_latency_max(self._h, n))

    def set_phase_timing(self, enable=True):
        self._check(self._L.bn_set_phase_timing(self._h, 1 if enable else 0))

    def phase_times(self):
        """(ms per phase [prepare, miller, final_exp, fe_out], launch sets) since the last read."""
        ms = np.zeros(4, np.float32)
        cnt = np.zeros(1, np.int32)
        self._check(self._L.bn_get_phase_times(self._h, _ptr(ms), _ptr(cnt)))
        return ms.astype(float), int(cnt[0])

    # ---- encodings / validation / square roots / decompression / Gt::pow
    def _bytes_in(self, b, width):
        b = np.ascontiguousarray(b, dtype=np.uint8)
        if b.size % width:
            raise ValueError("byte buffer of %d is not a multiple of %d" % (b.size, width))
        return b.reshape(-1, width)

    def fq_from_slice_many(self, be32):
        b = self._bytes_in(be32, 32)
        out = np.zeros((b.shape[0], 4), np.uint64)
        st = np.zeros(b.shape[0], np.uint8)
        self._check(self._L.bn_fq_from_slice_many(self._h, _ptr(b), b.shape[0], _ptr(out), _ptr(st)))
        return out, st

    def fq_to_big_endian_many(self, a):
        a = _arr(a, 4)
        out = np.zeros((a.shape[0], 32), np.uint8)
        self._check(self._L.bn_fq_to_big_endian_many(self._h, _ptr(a), a.shape[0], _ptr(out)))
        return out

    def fq2_from_slice_many(self, be64):
        b = self._bytes_in(be64, 64)
        out = np.zeros((b.shape[0], 8), np.uint64)
        st = np.zeros(b.shape[0], np.uint8)
        self._check(self._L.bn_fq2_from_slice_many(self._h, _ptr(b), b.shape[0], _ptr(out), _ptr(st)))
        return out, st

    def fr_from_slice_many(self, be32):
        b = self._bytes_in(be32, 32)
        out = np.zeros((b.shape[0], 4), np.uint64)
        self._check(self._L.bn_fr_from_slice_many(self._h, _ptr(b), b.shape[0], _ptr(out)))
        return out

    def fr_to_big_endian_many(self, a):
        a = _arr(a, 4)
        out = np.zeros((a.shape[0], 32), np.uint8)
        self._check(self._L.bn_fr_to_big_endian_many(self._h, _ptr(a), a.shape[0], _ptr(out)))
        return out

    def fq_sqrt_many(self, a):
        a = _arr(a, 4)
        out = np.zeros_like(a)
        ok = np.zeros(a.shape[0], np.uint8)
        self._check(self._L.bn_fq_sqrt_many(self._h, _ptr(a), a.shape[0], _ptr(out), _ptr(ok)))
        return out, ok

    def fq2_sqrt_many(self, a):
        a = _arr(a, 8)
        out = np.zeros_like(a)
        ok = np.zeros(a.shape[0], np.uint8)
        self._check(self._L.bn_fq2_sqrt_many(self._h, _ptr(a), a.shape[0], _ptr(out), _ptr(ok)))
        return out, ok

    def g1_affine_new_many(self, x, y):
        x, y = _arr(x, 4), _arr(y, 4)
        _same_rows(x, y)
        out = np.zeros((x.shape[0], 12), np.uint64)
        st = np.zeros(x.shape[0], np.uint8)
        self._check(self._L.bn_g1_affine_new_many(self._h, _ptr(x), _ptr(y), x.shape[0], _ptr(out), _ptr(st)))
        return out, st

    def g2_affine_new_many(self, x, y):
        x, y = _arr(x, 8), _arr(y, 8)
        _same_rows(x, y)
        out = np.zeros((x.shape[0], 24), np.uint64)
        st = np.zeros(x.shape[0], np.uint8)
        self._check(self._L.bn_g2_affine_new_many(self._h, _ptr(x), _ptr(y), x.shape[0], _ptr(out), _ptr(st)))
        return out, st

    def g1_from_compressed_many(self, b33):
        b = self._bytes_in(b33, 33)
        out = np.zeros((b.shape[0], 12), np.uint64)
        st = np.zeros(b.shape[0], np.uint8)
        self._check(self._L.bn_g1_from_compressed_many(self._h, _ptr(b), b.shape[0], _ptr(out), _ptr(st)))
        return out, st

    def g2_from_compressed_many(self, b65):
        b = self._bytes_in(b65, 65)
        out = np.zeros((b.shape[0], 24), np.uint64)
        st = np.zeros(b.shape[0], np.uint8)
        self._check(self._L.bn_g2_from_compressed_many(self._h, _ptr(b), b.shape[0], _ptr(out), _ptr(st)))
        return out, st

    def gt_pow_many(self, a, k):
        a, k = _arr(a, 48), _arr(k, 4)
        _same_rows(a, k)
        out = np.zeros_like(a)
        self._check(self._L.bn_gt_pow_many(self._h, _ptr(a), _ptr(k), a.shape[0], _ptr(out)))
        return out

    def g2_affine_new_many_dev(self, d_x, d_y, n, d_out, d_st, stream=None):
        self._check(self._L.bn_g2_affine_new_many_dev(self._h, d_x, d_y, n, d_out, d_st, stream))

    def g1_from_compressed_many_dev(self, d_b, n, d_out, d_st, stream=None):
        self._check(self._L.bn_g1_from_compressed_many_dev(self._h, d_b, n, d_out, d_st, stream))

    def g2_from_compressed_many_dev(self, d_b, n, d_out, d_st, stream=None):
        self._check(self._L.bn_g2_from_compressed_many_dev(self._h, d_b, n, d_out, d_st, stream))

    def gt_pow_many_dev(self, d_a, d_k, n, d_out, stream=None):
        self._check(self._L.bn_gt_pow_many_dev(self._h, d_a, d_k, n, d_out, stream))

    def reserve(self, n):
        self._check(self._L.bn_reserve(self._h, n))


def workspace_bytes(n):
    return load().bn_workspace_bytes(n)
