#!/usr/bin/env python3
"""Phase timing inside k_pairing_latency (diagnostic build: tools/build_variant.sh
stamps -DBN_LAT_STAMPS=1; run with BN254MI_LIB=exp/lib_stamps.so): one pairing
through bn_pairing_many_dev, then the s_memrealtime (100 MHz) stamps of block 0:
start, producer to_affine done, producer last line, consumer first line in,
consumer Miller loop done, consumer FE done.  Prints one JSON line (µs from start).
With --horner N: a bn_pairing_batch_dev of N terms (default 2^14, BASELINE config 5),
then k_horner_wide's stamps: start, g_0 in, first run of squarings, its load +
product, recombination done, final exponentiation done."""
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
    horner = "--horner" in sys.argv
    args = [a for a in sys.argv[1:] if a != "--horner"]
    n = int(args[0]) if args else (1 << 14 if horner else 1)
    s, t = synth.dataset_scalars(0, n)
    g1 = torch.from_numpy(np.tile(synth.g1_one_image().view(np.int64), (n, 1))).to(dev)
    g2 = torch.from_numpy(np.tile(synth.g2_one_image().view(np.int64), (n, 1))).to(dev)
    P = torch.empty((n, 12), dtype=torch.int64, device=dev)
    Q = torch.empty((n, 24), dtype=torch.int64, device=dev)
    sd = torch.from_numpy(s.view(np.int64)).to(dev)
    td = torch.from_numpy(t.view(np.int64)).to(dev)
    st = torch.cuda.Stream(dev)
    ctx.g1_mul_many_dev(g1.data_ptr(), sd.data_ptr(), n, P.data_ptr(), st.cuda_stream)
    ctx.g2_mul_many_dev(g2.data_ptr(), td.data_ptr(), n, Q.data_ptr(), st.cuda_stream)
    out = torch.empty((n, 48), dtype=torch.int64, device=dev)
    lib = _native.load()
    fn = lib.bn_dbg_hor_stamps if horner else lib.bn_dbg_lat_stamps
    fn.argtypes = [ctypes.c_void_p]
    rows = []
    for rep in range(5):
        if horner:
            ctx.pairing_batch_dev(P.data_ptr(), Q.data_ptr(), n, out.data_ptr(), None, st.cuda_stream)
        else:
            ctx.pairing_many_dev(P.data_ptr(), Q.data_ptr(), n, out.data_ptr(), st.cuda_stream)
        torch.cuda.synchronize(dev)
        buf = np.zeros(8, np.uint64)
        assert fn(buf.ctypes.data_as(ctypes.c_void_p)) == 0
        t0 = int(buf[0])
        rows.append([(int(x) - t0) / 100.0 for x in buf[:6]])  # 100 MHz -> µs
    names = (["start", "g0_in", "first_squarings", "first_load_mul", "horner_done", "fe_done"] if horner else
             ["start", "affine_done", "producer_done", "first_line_in", "miller_done", "fe_done"])
    med = [sorted(r[i] for r in rows)[2] for i in range(6)]
    print(json.dumps({"kernel": "k_horner_wide" if horner else "k_pairing_latency", "n": n, "us_from_start_median_of_5": dict(zip(names, med)), "runs": rows}))


if __name__ == "__main__":
    main()
