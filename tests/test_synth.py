"""bench.py's synthetic-input helpers (substrate_bn/synth.py, no oracle) produce
exactly the data the oracle-side helpers describe: same scalar stream, same
generator images, same affine conversion and compressed records."""
import numpy as np

from oracle import oracle as O
from substrate_bn import synth
from tests.codec_util import compress_g2


def test_scalars_and_generators():
    for seed, lo in ((1, 1), (72, 0)):
        _, ref = O.random_scalars(50, seed, lo=lo)
        assert np.array_equal(synth.fr_images(50, seed, lo), ref)
    assert np.array_equal(synth.g1_one_image(), O.g1_one())
    assert np.array_equal(synth.g2_one_image(), O.g2_one())


def test_g2_affine_and_compression():
    _, t = O.random_scalars(12, 61)
    jac = O.g2_mul(O.g2_one(), t, 4)
    ref_aff, _ = O.g2_to_affine(jac)
    aff = synth.g2_jacobian_to_affine(jac)
    assert np.array_equal(aff, ref_aff)
    assert np.array_equal(synth.compress_g2(aff), compress_g2(ref_aff))
