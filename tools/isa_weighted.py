#!/usr/bin/env python3
"""Trip-count-weighted VALU histogram of one kernel from its hipcc -S listing.

Every basic block is classified by the instruction classes of tools/isa_hist.py;
its execution count per lane comes from a signature table (the block's exact
v_mad_u64_u32 count, which identifies the Fq12 operation it implements) and the
operation counts of the algorithm (Miller loop digits, NAF
additions, the final-exponentiation step program).  Blocks without an entry
count once (setup, to_affine, the step-machine dispatch).  Output: per category
the weighted instruction count per lane and its share of all VALU.

    python tools/isa_weighted.py file.s KERNEL_SYMBOL SIG=WEIGHT[:NAME] ...
"""
import collections
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from isa_hist import blocks, cls  # noqa: E402

GROUPS = {
    "mad64 (v_mad_u64_u32)": ["mad64"],
    "carry/normalize (and, shifts, add3, lshl_add, alignbit)": ["valu_and", "valu_lshrrev", "valu_lshlrev", "shift64",
                                                                "vop3_3in", "valu_alignbit", "valu_bfe", "valu_ashrrev",
                                                                "valu_lshl", "valu_or", "valu_or3", "valu_bitop3"],
    "add/sub (digit-wise field add, sub, negation)": ["valu_add", "valu_sub", "valu_subrev", "carry"],
    "DPP / register moves": ["vmov", "agpr_mov"],
    "select (v_cndmask)": ["valu_cndmask"],
    "Montgomery digit (v_mul_lo_u32) + fold estimate (cvt, mul_f32)": ["mul32", "valu_cvt", "valu_mul", "valu_mad"],
}


def main():
    path, sym = sys.argv[1], sys.argv[2]
    table = {}
    for a in sys.argv[3:]:
        sig, rest = a.split("=")
        w, _, name = rest.partition(":")
        table[int(sig)] = (float(w), name or sig)
    bl = blocks(path, sym)
    tot = collections.Counter()
    seen = collections.Counter()
    per_op = {}
    for name, b in bl:
        c = collections.Counter(cls(x) for x in b)
        w, tag = table.get(c["mad64"], (1.0, None)) if c["mad64"] else (1.0, None)
        if tag:
            seen[tag] += 1
            per_op.setdefault(tag, (name, c))
        for k, v in c.items():
            tot[k] += v * w
    valu = {k: v for k, v in tot.items() if k in sum(GROUPS.values(), []) or k.startswith("valu_")}
    allv = sum(valu.values())
    print("kernel %s: %.0f weighted VALU per lane; blocks matched: %s" % (sym, allv, dict(seen)))
    rest = dict(valu)
    for g, ks in GROUPS.items():
        n = sum(rest.pop(k, 0) for k in ks)
        print("  %-62s %9.0f  %5.1f %%" % (g, n, 100 * n / allv))
    n = sum(rest.values())
    print("  %-62s %9.0f  %5.1f %%  %s" % ("other VALU", n, 100 * n / allv,
                                          ", ".join("%s=%.0f" % kv for kv in sorted(rest.items(), key=lambda x: -x[1])[:6])))
    # per matched operation: its block's VALU, VALU per MAD and category split (one execution)
    short = ["mad64", "carry/norm", "add/sub", "dpp/mov", "select", "mul_lo/fold"]
    print("\n  per operation (one execution of its block):")
    print("  %-14s %-10s %8s %8s %6s  %s" % ("op", "block", "VALU", "MAD", "V/MAD", "  ".join("%10s" % s for s in short)))
    for tag, (name, c) in per_op.items():
        v = {k: x for k, x in c.items() if k in sum(GROUPS.values(), []) or k.startswith("valu_")}
        nv = sum(v.values())
        cats = [sum(v.get(k, 0) for k in ks) for ks in GROUPS.values()]
        print("  %-14s %-10s %8d %8d %6.2f  %s" % (tag, name, nv, c["mad64"], nv / max(1, c["mad64"]),
                                                  "  ".join("%9.1f%%" % (100.0 * x / nv) for x in cats)))


if __name__ == "__main__":
    main()
