"""Inputs whose z is one (points that came in affine: AffineG1::new / AffineG2::new
and `into()`, or Group::normalize): to_affine takes the reference's z == one branch
(mod.rs:199-216), and a wave whose every pair has z == one skips the binary-GCD
inversion (lines_wide.h pair_to_affine).  Checked on every path that converts
points: the one-launch latency kernel, the segmented path, the throughput kernel,
the segmented pairing_batch and miller_loop_batch (pre-FE Miller values, where the
affine points themselves are observable) -- against the oracle, and against the
same points in their Jacobian form (the same pairing, bit for bit).  Waves that
mix z == one with other z take the inversion for all lanes: also checked."""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu
NT = 16


@pytest.fixture(scope="module")
def pts():
    p, q, _, _ = O.random_pairs(96, seed=777, nthreads=NT)
    return p, q, O.g1_normalize(p), O.g2_normalize(q)


def test_normalized_images_have_z_one(pts):
    _, _, pa, qa = pts
    one = O.canon_to_mont_array([1]).reshape(4)
    assert all(np.array_equal(r[8:12], one) for r in pa)
    assert all(np.array_equal(r[16:20], one) and not r[20:24].any() for r in qa)


@pytest.mark.parametrize("path", ["latency", "segmented", "throughput"])
def test_pairing_many_affine_inputs(pts, path):
    from substrate_bn import Context
    p, q, pa, qa = pts
    c = Context(0)
    if path == "segmented":
        c.set_latency_max(0)
    if path == "throughput":
        c.set_latency_max(0)
        c.set_fe_wide_max(0)
    want = O.pairing_many(pa[:32], qa[:32], NT)
    assert np.array_equal(c.pairing_many(pa[:32], qa[:32]), want)
    # the same points in Jacobian form: the same reduced pairing
    assert np.array_equal(c.pairing_many(p[:32], q[:32]), want)
    # mixed waves: every other pair affine
    pm, qm = pa[:32].copy(), qa[:32].copy()
    pm[1::2], qm[1::2] = p[1:32:2], q[1:32:2]
    assert np.array_equal(c.pairing_many(pm, qm), want)
    # only one of the two points affine in every pair
    assert np.array_equal(c.pairing_many(pa[:32], q[:32]), want)


def test_throughput_kernel_full_waves_affine(pts):
    """k_pairing_full at a size past the latency paths: whole waves of z == one."""
    from substrate_bn import Context
    p, q, pa, qa = pts
    reps = 12000 // 96 + 1
    P, Q = np.tile(pa, (reps, 1)), np.tile(qa, (reps, 1))
    c = Context(0)
    out = c.pairing_many(P, Q)
    want = O.pairing_many(pa, qa, NT)
    assert np.array_equal(out, np.tile(want, (reps, 1)))


def test_pairing_batch_and_miller_values_affine(pts):
    from substrate_bn import Context
    p, q, pa, qa = pts
    c = Context(0)
    reps = 4224 // 96
    P, Q = np.tile(pa, (reps, 1)), np.tile(qa, (reps, 1))  # the segmented product (k_prepare_wide)
    got = c.pairing_batch(P, Q)
    assert np.array_equal(got, O.pairing_batch(P, Q, nthreads=NT))
    assert np.array_equal(got, c.pairing_batch(np.tile(p, (reps, 1)), np.tile(q, (reps, 1))))
    # miller_loop_batch (G2, G1): the Miller value depends on the affine points themselves
    _, want = O.miller_loop_batch(qa[:40], pa[:40])
    assert np.array_equal(c.miller_loop_batch(qa[:40], pa[:40]), want.reshape(48))
    _, want = O.miller_loop_batch(Q, P)
    assert np.array_equal(c.miller_loop_batch(Q, P), want.reshape(48))
