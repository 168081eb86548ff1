"""ctypes wrapper of tests/native/libhostemul.so: the engine's device
arithmetic compiled for the host (TEST INFRASTRUCTURE ONLY)."""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "libhostemul.so")
_lib = None


def build():
    src = os.path.join(HERE, "host_emul.cpp")
    subprocess.check_call(["g++", "-O0", "-std=c++17", "-DBN_HOST_CHECKS", "-fPIC", "-shared", "-o", SO, src])


def lib():
    global _lib
    if _lib is None:
        hdr_dir = os.path.join(HERE, "..", "..", "paritytech-bn_amd", "csrc")
        newest = max(os.path.getmtime(os.path.join(hdr_dir, f)) for f in os.listdir(hdr_dir))
        newest = max(newest, os.path.getmtime(os.path.join(HERE, "host_emul.cpp")))
        if not os.path.exists(SO) or os.path.getmtime(SO) < newest:
            build()
        _lib = ctypes.CDLL(SO)
    return _lib


def call(name, *arrays, out_words, ints=(), ret=False):
    """arrays: uint64 memory images; returns the uint64 output of out_words u32
    words (and the function's int result with ret=True)."""
    fn = getattr(lib(), name)
    args = []
    keep = []
    for a in arrays:
        a = np.ascontiguousarray(a, dtype=np.uint64)
        keep.append(a)
        args.append(a.ctypes.data_as(ctypes.c_void_p))
    out = np.zeros(out_words // 2, dtype=np.uint64)
    args = args[:1] + [ctypes.c_int(i) for i in ints] + args[1:] if ints else args
    args.append(out.ctypes.data_as(ctypes.c_void_p))
    rc = fn(*args)
    return (out, rc) if ret else out
