#!/usr/bin/env python3
"""Where k_miller_seg's wave lifetime goes (diagnostic build: tools/build_variant.sh
segstamps -DBN_SEG_STAMPS=1; run with BN254MI_LIB=ab/lib_segstamps.so): one
2^14-term bn_pairing_batch_dev (BASELINE config 5), then every wave's s_memrealtime
(100 MHz) start and end and its segment.  Prints per segment the waves, K, and the
wave durations (min / mean / max, us) and end times from the kernel's first start,
and the kernel's wave-life fraction (mean duration / (last end - first start))."""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "paritytech-bn_amd"))
sys.path.insert(0, ROOT)


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
    fn = lib.bn_dbg_seg_stamps
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
    runs = []
    for rep in range(3):
        ctx.pairing_batch_dev(P.data_ptr(), Q.data_ptr(), n, out.data_ptr(), None, st.cuda_stream)
        torch.cuda.synchronize(dev)
        buf = np.zeros((4096, 4), np.uint64)
        nw = fn(buf.ctypes.data_as(ctypes.c_void_p), 4096)
        assert nw > 0
        w = buf[(buf[:, 0] > 0) & (buf[:, 1] > 0)]  # waves that ran a segment (not padding)
        t0 = int(w[:, 0].min())
        end = int(w[:, 1].max())
        dur = (w[:, 1].astype(np.int64) - w[:, 0].astype(np.int64)) / 100.0
        segs = {}
        for k in sorted(set(int(x) for x in w[:, 2])):
            m = w[:, 2] == k
            d = dur[m]
            e = (w[m, 1].astype(np.int64) - t0) / 100.0
            segs[k] = {"waves": int(m.sum()), "K": int(w[m, 3][0]), "dur_us": [round(float(d.min()), 1),
                       round(float(d.mean()), 1), round(float(d.max()), 1)],
                       "end_us": [round(float(e.min()), 1), round(float(e.max()), 1)]}
        runs.append({"kernel_us": (end - t0) / 100.0, "wave_life": float(dur.mean() / ((end - t0) / 100.0)),
                     "segments": segs})
    print(json.dumps({"n": n, "weights": os.environ.get("BN254MI_SEG_WEIGHTS", "36,39"), "runs": runs}))


if __name__ == "__main__":
    main()
