#!/usr/bin/env python3
"""Phase timing of config 5's tail (diagnostic build: tools/build_variant.sh tailstamps
-DBN_TAIL_STAMPS=1; run with BN254MI_LIB=ab/lib_tailstamps.so): five 2^14-term
bn_pairing_batch_dev products, then the s_memrealtime (100 MHz) stamps thread 0 of a
block wrote (fq12_ds.h TAIL_STAMP), in us from k_seg_fe1's start:
  k_seg_fe1, segment 0's block: start, first chunk done (the Fq12 inversion), squarings done;
  k_horner_tree2's squarer block S: start, tree done (k_seg_tail, BN254MI_TAIL_FUSED=1: no
  start stamp; "tree done" is the carrier of the segments' product starting the last chunk), then per exp_by_neg_z the end of its
  squarings and the arrival of M's product, and the last chunk done;
  its multiplier block M: start, role claimed, done.
Prints the median of the five per stamp as one JSON line."""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "paritytech-bn_amd"))
sys.path.insert(0, ROOT)
NAMES = {16: "fe1_start", 17: "fe1_first_chunk_done", 18: "fe1_squarings_done",
         0: "S_start", 1: "S_tree_done (k_seg_tail: the chain's product in)", 2: "S_exp1_squarings_done", 3: "S_exp1_result_in",
         4: "S_exp2_squarings_done", 5: "S_exp2_result_in", 6: "S_exp3_squarings_done", 7: "S_exp3_result_in",
         8: "S_last_chunk_done", 24: "M_start", 25: "M_claimed", 26: "M_done",
         27: "M1_claimed (k_seg_tail)", 28: "M1_done (k_seg_tail)"}


def main():
    import torch

    from substrate_bn import Context, synth
    from substrate_bn import _native
    dev = torch.device("cuda", 0)
    ctx = Context(0)
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 14
    s, t = synth.dataset_scalars(0, n)
    g1 = torch.from_numpy(np.tile(synth.g1_one_image().view(np.int64), (n, 1))).to(dev)
    g2 = torch.from_numpy(np.tile(synth.g2_one_image().view(np.int64), (n, 1))).to(dev)
    P = torch.empty((n, 12), dtype=torch.int64, device=dev)
    Q = torch.empty((n, 24), dtype=torch.int64, device=dev)
    st = torch.cuda.Stream(dev)
    ctx.g1_mul_many_dev(g1.data_ptr(), torch.from_numpy(s.view(np.int64)).to(dev).data_ptr(), n, P.data_ptr(),
                        st.cuda_stream)
    ctx.g2_mul_many_dev(g2.data_ptr(), torch.from_numpy(t.view(np.int64)).to(dev).data_ptr(), n, Q.data_ptr(),
                        st.cuda_stream)
    out = torch.empty(48, dtype=torch.int64, device=dev)
    lib = _native.load()
    fn = lib.bn_dbg_tail_stamps
    fn.argtypes = [ctypes.c_void_p]
    rows = []
    for rep in range(5):
        ctx.pairing_batch_dev(P.data_ptr(), Q.data_ptr(), n, out.data_ptr(), None, st.cuda_stream)
        torch.cuda.synchronize(dev)
        buf = np.zeros(32, np.uint64)
        assert fn(buf.ctypes.data_as(ctypes.c_void_p)) == 0
        t0 = int(buf[16])
        rows.append({NAMES[k]: (int(buf[k]) - t0) / 100.0 for k in NAMES})
    med = {k: sorted(r[k] for r in rows)[2] for k in rows[0]}
    print(json.dumps({"n": n, "us_from_fe1_start_median_of_5": med, "runs": rows}))


if __name__ == "__main__":
    main()
