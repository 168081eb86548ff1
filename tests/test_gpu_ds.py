"""The digit-sliced Fq12 operations on the GPU (tools/ds_check.hip, built by
__graft_entry__.build()): every operation -- cyclotomic squaring, product, product
by a conjugate, Frobenius 1/2/3, conjugation, exp_by_neg_z and the whole last chunk
of the final exponentiation -- against the 16-lane functions of fq12_wide.h on 64
random and maximal-digit elements, canonical images compared word for word (the
reference formulas: fq12.rs:75-128, 198-247, 319-327)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tools", "ds_check")


@pytest.mark.gpu
def test_ds_operations_match_the_wide_layout():
    assert os.path.exists(BIN), "tools/ds_check not built: python -c 'import __graft_entry__ as g; g.build()'"
    r = subprocess.run([BIN, "64"], capture_output=True, text=True, timeout=180)
    assert r.returncode == 0 and "DS CHECK OK" in r.stdout, r.stdout[-3000:] + r.stderr[-2000:]
