"""CPU-side checks of the product library: it loads without a GPU, exports every
symbol include/bn254mi.h declares, and refuses to run without a device."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "paritytech-bn_amd", "libbn254mi.so")
HDR = os.path.join(ROOT, "include", "bn254mi.h")


def declared():
    txt = open(HDR).read()
    return sorted(set(re.findall(r"\b(bn_[a-z0-9_]+)\s*\(", txt)))


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIB):
        pytest.skip("libbn254mi.so not built (run __graft_entry__.build())")
    return ctypes.CDLL(LIB)


def test_header_declares_the_path():
    names = declared()
    for must in ("bn_pairing_many", "bn_pairing_batch", "bn_miller_loop_batch", "bn_final_exponentiation_many",
                 "bn_g1_mul_many", "bn_pairing_many_dev"):
        assert must in names


def test_library_exports_every_declared_symbol(lib):
    missing = [n for n in declared() if not hasattr(lib, n)]
    assert not missing, missing


def test_python_binding_lists_every_export():
    from substrate_bn import _native
    assert sorted(_native.EXPORTS) == declared()


def test_no_device_is_an_error_not_a_fallback(lib):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    h = ctypes.c_void_p()
    lib.bn_ctx_create.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]
    rc = lib.bn_ctx_create(0, ctypes.byref(h))
    assert rc != 0 and not h.value


def test_workspace_size_is_sane(lib):
    lib.bn_workspace_bytes.restype = ctypes.c_size_t
    lib.bn_workspace_bytes.argtypes = [ctypes.c_size_t]
    per = lib.bn_workspace_bytes(1 << 16) / (1 << 16)
    assert 15_000 < per < 40_000   # ~19 KB of line coefficients + Fq12 slots per pairing


def test_shard_range_is_contiguous_and_covers(lib):
    """bn_shard_range (the multi-device split) -- host arithmetic, no GPU."""
    from substrate_bn import _native, parallel
    for n in (0, 1, 7, 65536, (1 << 20) + 3):
        for nd in (1, 2, 3, 8):
            lo_prev = 0
            for k in range(nd):
                lo, hi = _native.shard_range(n, nd, k)
                assert lo == lo_prev and hi >= lo
                assert (lo, hi) == tuple(parallel.shard_bounds(n, k, nd))
                lo_prev = hi
            assert lo_prev == n
    assert _native.shard_range(10, 2, 2) == (0, 0)  # k out of range
