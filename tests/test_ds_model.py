"""The digit-sliced Fq12 algorithm (paritytech-bn_amd/csrc/fq12_ds.h) in its lane-level
Python model (tools/ds_model.py): the Granger-Scott squaring and the Fq12 product,
lane by lane with every 64-bit column, 32-bit operand and signed range asserted,
against big-integer arithmetic (the formulas of fq12.rs:198-247 and 319-327), on
random folded inputs and on maximal-digit ones.  CPU only; the device code is
checked against the 16-lane functions by tests/test_gpu_ds.py."""
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import ds_model as M  # noqa: E402


def test_random_elements():
    random.seed(7)
    for _ in range(2):
        z = [M.rand_e() for _ in range(12)]
        w = [M.rand_e() for _ in range(12)]
        assert M.ref_vals(M.cyc(z)) == M.cyc_ref(M.ref_vals(z))
        assert M.ref_vals(M.mul(z, w)) == M.mul_ref(M.ref_vals(z), M.ref_vals(w))


def _maximal(fill):
    v = [0] * M.W
    for k in range(M.ND - 1):
        v[M.B + k] = fill()
    low = sum(v[M.B + k] << (M.DIG * k) for k in range(M.ND - 1))
    v[M.TOP] = (5 * M.P - 1 - low) >> (M.DIG * (M.ND - 1))  # the largest top digit of a folded value
    return v


def test_maximal_digits():
    random.seed(9)
    for fill in (lambda: (1 << M.DIG) + 2, lambda: 0):
        z = [_maximal(fill) for _ in range(12)]
        assert M.ref_vals(M.cyc(z)) == M.cyc_ref(M.ref_vals(z))
        assert M.ref_vals(M.mul(z, z)) == M.mul_ref(M.ref_vals(z), M.ref_vals(z))


def test_constants_match_the_header():
    """the digit tables of fq12_ds.h are the model's (p, p' = -p^-1 mod 2^260)"""
    src = open(os.path.join(ROOT, "paritytech-bn_amd", "csrc", "fq12_ds.h")).read()

    def table(name):
        i = src.index(name + "[10] = {")
        body = src[i:src.index("}", i)].split("{")[1]
        return [int(x.strip().rstrip("u"), 16) for x in body.split(",")]
    assert table("kDsP") == M.PD
    assert table("kDsPinv") == M.PID
    assert table("kDsS3") == M.spread(3)[M.B:M.TOP + 1]
    assert table("kDsS8") == M.spread(8)[M.B:M.TOP + 1]
