#!/usr/bin/env python3
"""Extract the known-answer vectors of the reference's own tests as DATA.

Runs only in the build container (reads /root/reference as text; imports or
executes nothing from it).  Writes tests/golden/reference_kats.json, which is
committed and is what the tests read (the GPU box has no /root/reference).

Every number is stored as a canonical decimal integer (not Montgomery form):
  - `Fq::new(U256([lo, hi]))`  -> lo + hi * 2**128   (src/arith.rs:9-20)
  - `Fq::from_str("...")`      -> the decimal string (src/fields/fp.rs:23-43)
Sources (file:line in /root/reference):
  test_prepared_g2      src/groups/mod.rs:780-892
  test_miller_loop      src/groups/mod.rs:643-691
  test_reduced_pairing  src/groups/mod.rs:929-999
  fq12_test_vector      src/fields/mod.rs:94-227
  test_cyclotomic_exp   src/fields/mod.rs:230-344
  test_str              src/fields/mod.rs:68-81
"""
import json
import os
import re
import sys

REF = "/root/reference/src"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "reference_kats.json")

U256_RE = re.compile(r"U256\(\[\s*(\d+)\s*,\s*(\d+)\s*\]\)")
STR_RE = re.compile(r'from_str\(\s*"(\d+)"')


def fn_body(text, name):
    """Text of `fn name` up to the next top-level item."""
    start = text.index("fn " + name)
    nxt = re.compile(r"\n(#\[test\]|pub fn |fn |impl |#\[derive)")
    m = nxt.search(text, start + 3)
    return text[start: m.start() if m else len(text)], text[:start].count("\n") + 1


def u256s(body):
    return [str(int(lo) + (int(hi) << 128)) for lo, hi in U256_RE.findall(body)]


def strs(body):
    return STR_RE.findall(body)


def main():
    groups = open(os.path.join(REF, "groups/mod.rs")).read()
    fields = open(os.path.join(REF, "fields/mod.rs")).read()
    kats = {"_source": "risc0/paritytech-bn (substrate-bn 0.6.0) unit tests; canonical decimal integers"}

    body, line = fn_body(groups, "test_prepared_g2")
    scal = strs(body)
    vals = u256s(body)
    assert len(scal) == 1 and len(vals) == 4 + 87 * 6, (len(scal), len(vals))
    coeffs = [vals[4 + 6 * k: 4 + 6 * (k + 1)] for k in range(87)]
    kats["test_prepared_g2"] = {
        "where": "src/groups/mod.rs:%d" % line,
        "g2_scalar": scal[0],
        "q_affine": {"x": vals[0:2], "y": vals[2:4]},
        # order per EllCoeffs literal: ell_0 (c0,c1), ell_vw (c0,c1), ell_vv (c0,c1)
        "coeffs": coeffs,
    }

    body, line = fn_body(groups, "test_miller_loop")
    scal = strs(body)
    vals = u256s(body)
    assert len(scal) == 2 and len(vals) == 12
    kats["test_miller_loop"] = {"where": "src/groups/mod.rs:%d" % line, "g1_scalar": scal[0],
                                "g2_scalar": scal[1], "f": vals}

    body, line = fn_body(groups, "test_reduced_pairing")
    s = strs(body)
    assert len(s) == 14
    kats["test_reduced_pairing"] = {"where": "src/groups/mod.rs:%d" % line, "g1_scalar": s[0],
                                    "g2_scalar": s[1], "gt": s[2:]}

    body, line = fn_body(fields, "fq12_test_vector")
    s = strs(body)
    assert len(s) == 24
    kats["fq12_test_vector"] = {"where": "src/fields/mod.rs:%d" % line, "start": s[:12], "finally": s[12:],
                                "recipe": "next=start; 100x next*=start; cpy=next; 10x next=next^2; "
                                          "10x {next+=start; next-=cpy; next=-next}; next=next^2"}

    body, line = fn_body(fields, "test_cyclotomic_exp")
    s = strs(body)
    assert len(s) == 24
    kats["test_cyclotomic_exp"] = {"where": "src/fields/mod.rs:%d" % line, "orig": s[:12], "expected": s[12:]}

    body, line = fn_body(fields, "test_str")
    s = strs(body)
    assert len(s) == 2
    kats["test_str"] = {"where": "src/fields/mod.rs:%d" % line, "fr_minus_one": s[0], "fq_minus_one": s[1]}

    with open(OUT, "w") as fh:
        json.dump(kats, fh, indent=1)
    print("wrote", OUT)


if __name__ == "__main__":
    sys.exit(main())
