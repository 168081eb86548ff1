#!/usr/bin/env python3
"""Instruction census of one kernel in a hipcc -S listing: per basic block and
for every loop (a backward branch), count VALU / MAD / AGPR-move / memory / SALU
instructions.  Used to see where a kernel's VALU issue goes.

    python tools/isa_hist.py file.s KERNEL_SYMBOL [--top N]
"""
import collections
import re
import sys


def blocks(path, sym):
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith(sym + ":"))
    end = next(i for i in range(start, len(lines)) if lines[i].strip().startswith(".Lfunc_end"))
    out, cur, name = [], [], sym
    for l in lines[start + 1:end]:
        s = l.split(";")[0].strip()
        if not s:
            continue
        if s.endswith(":"):
            out.append((name, cur))
            name, cur = s[:-1], []
            continue
        if s.startswith("."):
            continue
        cur.append(s)
    out.append((name, cur))
    return out


def cls(ins):
    op = ins.split()[0]
    if op.startswith("v_mad_u64_u32"):
        return "mad64"
    if op.startswith("v_accvgpr"):
        return "agpr_mov"
    if op.startswith("v_mul_lo") or op.startswith("v_mul_hi"):
        return "mul32"
    if op.startswith("v_lshrrev_b64") or op.startswith("v_lshlrev_b64"):
        return "shift64"
    if op.startswith("v_add_co") or op.startswith("v_addc_co") or op.startswith("v_sub_co") or op.startswith("v_subb"):
        return "carry"
    if op.startswith("v_add3") or op.startswith("v_lshl_add") or op.startswith("v_and_or") or op.startswith("v_bfi") or op.startswith("v_bfe"):
        return "vop3_3in"
    if op.startswith("v_mov"):
        return "vmov"
    if op.startswith("v_"):
        return "valu_" + op.split("_e")[0][2:].split("_")[0]
    if op.startswith("buffer_") or op.startswith("global_") or op.startswith("scratch_") or op.startswith("flat_"):
        return "vmem_" + op.split("_")[0] + ("_st" if "store" in op else "_ld")
    if op.startswith("ds_"):
        return "lds"
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main():
    path, sym = sys.argv[1], sys.argv[2]
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 15
    bl = blocks(path, sym)
    idx = {n: i for i, (n, _) in enumerate(bl)}
    tot = collections.Counter()
    for _, b in bl:
        for ins in b:
            tot[cls(ins)] += 1
    print("kernel %s: %d instructions in %d blocks" % (sym, sum(tot.values()), len(bl)))
    print("  " + ", ".join("%s=%d" % kv for kv in tot.most_common()))
    # loops: a branch from block j back to block i <= j
    for j, (n, b) in enumerate(bl):
        for ins in b:
            m = re.match(r"s_(cbranch_\w+|branch)\s+(\S+)", ins)
            if m and m.group(2) in idx and idx[m.group(2)] <= j:
                i = idx[m.group(2)]
                c = collections.Counter()
                for _, bb in bl[i:j + 1]:
                    for x in bb:
                        c[cls(x)] += 1
                valu = sum(v for k, v in c.items() if k.startswith("v") and not k.startswith("vmem") or k in ("mad64", "agpr_mov", "mul32", "shift64", "carry", "vop3_3in"))
                print("loop %s..%s (%d blocks): %d instrs, VALU %d, mad64 %d | %s" % (
                    bl[i][0], n, j - i + 1, sum(c.values()), valu, c["mad64"],
                    ", ".join("%s=%d" % kv for kv in c.most_common(top))))


if __name__ == "__main__":
    main()
