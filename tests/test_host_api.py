"""Host-side API checks that need no GPU: the Python mirror's argument
validation runs before any native call."""
import numpy as np
import pytest

import substrate_bn as bn
from substrate_bn import _native


def test_fr_from_str_matches_reference_rules():
    # fp.rs:23-43: to_digit(10) accepts ASCII 0-9 only; "" folds to zero
    assert bn.Fr.from_str("") == bn.Fr.zero()
    assert bn.Fr.from_str("7") == bn.Fr.from_int(7)
    assert bn.Fr.from_str(str(bn.R_ORDER + 5)) == bn.Fr.from_int(5)
    for bad in ("²", "12a", "-1", " 1", "٣"):
        assert bn.Fr.from_str(bad) is None


class _NoLib:
    """Stand-in for the ctypes library: any native call is a test failure."""
    def __getattr__(self, name):
        raise AssertionError("native call %s reached with mismatched inputs" % name)


def _ctx():
    c = _native.Context.__new__(_native.Context)
    c._h, c._L = None, _NoLib()
    return c


@pytest.mark.parametrize("call", [
    lambda c: c.pairing_many(np.zeros((3, 12)), np.zeros((2, 24))),
    lambda c: c.pairing_batch(np.zeros((3, 12)), np.zeros((2, 24))),
    lambda c: c.miller_loop_batch(np.zeros((3, 24)), np.zeros((2, 12))),
    lambda c: c.miller_loop_many(np.zeros((3, 12)), np.zeros((4, 24))),
    lambda c: c.g1_mul_many(np.zeros((3, 12)), np.zeros((2, 4))),
    lambda c: c.g2_mul_many(np.zeros((3, 24)), np.zeros((2, 4))),
    lambda c: c.fq12_op_many("mul", np.zeros((3, 48)), np.zeros((2, 48))),
    lambda c: c.g1_affine_new_many(np.zeros((3, 4)), np.zeros((2, 4))),
    lambda c: c.g2_affine_new_many(np.zeros((3, 8)), np.zeros((2, 8))),
    lambda c: c.gt_pow_many(np.zeros((3, 48)), np.zeros((2, 4))),
])
def test_mismatched_rows_raise_before_native_call(call):
    with pytest.raises(ValueError):
        call(_ctx())
