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
    # the segmented product (4,224 terms): the digit-sliced tail's two-block channel
    assert res["pairing_batch_segmented"] == BN_ERR_INTERNAL, res
    assert not res["pairing_batch_segmented_value_returned"], res
    # the status-less device call is accepted, and bn_dev_status reports the failure once
    assert res["pairing_many_dev_call"] == BN_OK, res
    assert res["dev_status_after"] == BN_ERR_INTERNAL, res
    assert res["dev_status_cleared"] == BN_OK, res
    # the device batch form writes BN_ERR_INTERNAL into its status word
    assert res["pairing_batch_dev_call"] == BN_OK, res
    assert res["pairing_batch_dev_status"] == BN_ERR_INTERNAL, res
    # the throughput kernel has no capped waits: the same library is still bit-exact there
    assert res["throughput_path"] == BN_OK and res["throughput_path_bit_exact"], res
