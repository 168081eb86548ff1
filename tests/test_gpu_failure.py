"""The failure path of the capped LDS hand-offs.

The latency kernels hand lines and final-exponentiation items between waves
through LDS counters whose spin waits are capped (latency_kernel.h,
fq12_wide.h duo_wait), and the product's digit-sliced tail hands powers between its
squarer and multiplier blocks through global words whose polls are capped the same
way (fq12_ds.h ds_chan_ld).  A wait that runs out sets BN_ERR_INTERNAL and the call
must fail instead of returning a Gt computed from an unpublished slot -- the
reference panics rather than return a wrong value (src/groups/mod.rs:900).

libbn254mi_cap0.so (`make -C paritytech-bn_amd cap0`, built by
__graft_entry__.build()) is the product library with those units (and the tail) built at
spin cap 0, so the first wait of each kernel runs out deterministically (the
consumer's first line needs the producer's to_affine, tens of microseconds).
The library replaces the product one, so the calls run in a child process
(tests/failure_probe.py) with BN254MI_LIB pointing at it.
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CAP0 = os.path.join(ROOT, "paritytech-bn_amd", "libbn254mi_cap0.so")
BN_OK, BN_ERR_INTERNAL = 0, 6


@pytest.mark.gpu
def test_capped_handoff_fails_the_call():
    assert os.path.exists(CAP0), "libbn254mi_cap0.so not built: make -C paritytech-bn_amd cap0"
    env = dict(os.environ, BN254MI_LIB=CAP0)
    r = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "tests", "failure_probe.py")], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    # host-buffer calls through the one-launch latency kernel and the two-group FE fail, with no value
    assert res["pairing_many"] == BN_ERR_INTERNAL and not res["pairing_many_value_returned"], res
    assert res["pairing_batch"] == BN_ERR_INTERNAL and not res["pairing_batch_value_returned"], res
    assert res["miller_loop_batch"] == BN_ERR_INTERNAL, res
    assert res["final_exponentiation_many"] == BN_ERR_INTERNAL, res
    # the segmented product (4,224 terms): the digit-sliced tail's two-block channel,
    # failing promptly (within 1 s)
    assert res["pairing_batch_segmented"] == BN_ERR_INTERNAL, res
    assert not res["pairing_batch_segmented_value_returned"], res
    assert res["pairing_batch_segmented_s"] < 1.0, res
    # the status-less device call is accepted, and bn_dev_status reports the failure once
    assert res["pairing_many_dev_call"] == BN_OK, res
    assert res["dev_status_after"] == BN_ERR_INTERNAL, res
    assert res["dev_status_cleared"] == BN_OK, res
    # the device batch form writes BN_ERR_INTERNAL into its status word
    assert res["pairing_batch_dev_call"] == BN_OK, res
    assert res["pairing_batch_dev_status"] == BN_ERR_INTERNAL, res
    # the throughput kernel has no capped waits: the same library is still bit-exact there
    assert res["throughput_path"] == BN_OK and res["throughput_path_bit_exact"], res


def _tail_probe(lib, fused=1):
    path = os.path.join(ROOT, "paritytech-bn_amd", lib)
    assert os.path.exists(path), "%s not built: make -C paritytech-bn_amd chanfail latem" % lib
    env = dict(os.environ, BN254MI_LIB=path, BN254MI_TAIL_FUSED=str(fused), FAILURE_PROBE_TAIL="1")
    r = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "tests", "failure_probe.py")], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


@pytest.mark.gpu
@pytest.mark.parametrize("fused", [1, 0])
def test_tail_channel_fails_fast_after_one_expired_wait(fused):
    """Every store of the tail's global-memory channel dropped, at a spin cap of 2^20
    polls (~60 ms per expired wait): without the channel's sticky `dead` flag
    (fq12_ds.h ds_chan_ld) the multiplier's 80 takes and the squarer's 5 result
    reads would each spin out, ~5 s; with it each wave spins out once.  fused = 1:
    k_seg_tail (the segment chain's reads share the flag), 0: k_seg_fe1 + k_horner_tree2."""
    res = _tail_probe("libbn254mi_chanfail.so", fused)
    assert res["code"] == BN_ERR_INTERNAL and not res["value_returned"], res
    assert res["seconds_1"] < 1.5, res


@pytest.mark.gpu
@pytest.mark.parametrize("fused", [1, 0])
def test_tail_squarer_goes_on_alone_when_the_multiplier_is_late(fused):
    """The multiplier blocks starting ~2 ms late (as when other work holds the CUs):
    the squarer decides for the last chunk alone (kernels_tail.hip role word), the
    late blocks return, and the product is bit-exact (fused = 1: k_seg_tail's
    multiplier candidates; 0: k_horner_tree2's block 1)."""
    res = _tail_probe("libbn254mi_latem.so", fused)
    assert res["code"] == BN_OK and res["value_returned"] and res["bit_exact"], res


@pytest.mark.gpu
@pytest.mark.parametrize("fused", [1, 0])
def test_tail_forms_bit_exact(fused):
    """The product library's two tails on the 4,224-term segmented pairing_batch:
    k_seg_tail (default) and k_seg_fe1 + k_horner_tree2 (BN254MI_TAIL_FUSED=0)."""
    res = _tail_probe("libbn254mi.so", fused)
    assert res["code"] == BN_OK and res["value_returned"] and res["bit_exact"], res
