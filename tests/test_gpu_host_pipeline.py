"""bn_pairing_many on host buffers through the pinned double-buffered pipeline
(capi.hip pairing_many_host: pieces of 2^16 pairs, two bounce buffers, copy
streams): several pieces with a ragged last one, against the HBM-resident
bn_pairing_many_dev on the same inputs and against the oracle on sampled rows;
a zero point in a later piece; the pipeline forced on for one-piece calls
($BN254MI_HOST_PIPELINE=2; by default a single piece takes the pageable form);
and the pageable A/B form ($BN254MI_HOST_PIPELINE=0).  lib.rs:611-613.
Runs on the GPU box: python -m pytest tests -m gpu."""
import os

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu
PIECE = 1 << 16


@pytest.fixture(scope="module")
def setup():
    import torch

    from substrate_bn import Context, synth
    n = 3 * PIECE + 5  # four pieces: three full, one of 5 pairs (both buffers reused)
    dev = torch.device("cuda", 0)
    ctx = Context(0)
    s, t = synth.dataset_scalars(7, n)
    g1 = torch.from_numpy(np.tile(synth.g1_one_image().view(np.int64), (n, 1))).to(dev)
    g2 = torch.from_numpy(np.tile(synth.g2_one_image().view(np.int64), (n, 1))).to(dev)
    P = torch.empty((n, 12), dtype=torch.int64, device=dev)
    Q = torch.empty((n, 24), dtype=torch.int64, device=dev)
    stream = torch.cuda.Stream(dev)
    sh = stream.cuda_stream
    ctx.g1_mul_many_dev(g1.data_ptr(), torch.from_numpy(s.view(np.int64)).to(dev).data_ptr(), n, P.data_ptr(), sh)
    ctx.g2_mul_many_dev(g2.data_ptr(), torch.from_numpy(t.view(np.int64)).to(dev).data_ptr(), n, Q.data_ptr(), sh)
    torch.cuda.synchronize(dev)
    p = P.cpu().numpy().view(np.uint64).copy()
    q = Q.cpu().numpy().view(np.uint64).copy()
    p[PIECE + 3] = 0  # G1::zero() in the second piece: pairing is Gt::one()
    P.copy_(torch.from_numpy(p.view(np.int64)))
    out = torch.empty((n, 48), dtype=torch.int64, device=dev)
    ctx.pairing_many_dev(P.data_ptr(), Q.data_ptr(), n, out.data_ptr(), sh)
    torch.cuda.synchronize(dev)
    return ctx, p, q, out.cpu().numpy().view(np.uint64)


def test_pipeline_matches_device_path_and_oracle(setup):
    ctx, p, q, want = setup
    got = ctx.pairing_many(p, q)
    assert np.array_equal(got, want)
    rows = np.r_[0:8, PIECE - 2:PIECE + 6, 2 * PIECE - 1, 3 * PIECE - 1:3 * PIECE + 5]
    assert np.array_equal(got[rows], O.pairing_many(p[rows], q[rows], 16))
    assert np.array_equal(got[PIECE + 3], O.canon_to_mont_array([1] + [0] * 11))


def _ctx_with(mode, var="BN254MI_HOST_PIPELINE"):
    """a context created under $var=mode (read at creation)"""
    from substrate_bn import Context
    old = os.environ.get(var)
    os.environ[var] = mode
    try:
        return Context(0)
    finally:
        if old is None:
            del os.environ[var]
        else:
            os.environ[var] = old


@pytest.fixture(scope="module")
def ctx_always():
    return _ctx_with("2")


@pytest.mark.parametrize("n", [1, 5, PIECE, PIECE + 1, 2 * PIECE])
def test_pipeline_sizes(setup, ctx_always, n):
    """the pipeline forced on for every size (mode 2): one piece, exactly one
    full piece, a full piece plus one pair, two full pieces; a smaller call
    after a larger one reuses the grown buffers"""
    _, p, q, want = setup
    assert np.array_equal(ctx_always.pairing_many(p[:n], q[:n]), want[:n])


@pytest.mark.parametrize("n", [3, PIECE + 7])
def test_pageable_form_agrees(setup, n):
    _, p, q, want = setup
    ctx0 = _ctx_with("0")
    assert np.array_equal(ctx0.pairing_many(p[:n], q[:n]), want[:n])


def test_large_piece_path(setup):
    """the large-piece branch (pieces of host_piece once a call holds two of
    them; 2^17 by default, 2^15 here so the fixture exercises it): seven pieces,
    the last of 5 pairs"""
    _, p, q, want = setup
    ctx = _ctx_with(str(PIECE // 2), "BN254MI_HOST_PIECE")
    assert np.array_equal(ctx.pairing_many(p, q), want)
