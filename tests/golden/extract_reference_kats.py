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
  sqrt_fq               src/fields/fp.rs:289-296
  sqrt_fq2              src/fields/fq2.rs:235-258
  g1_from_compressed    src/lib.rs:681-689
  g2_from_compressed    src/lib.rs:691-743
  testing_divrem        src/arith.rs:588-666 (the two fixed U512 cases)
  from_slice / to_big_endian  src/arith.rs:561-586
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

    fp = open(os.path.join(REF, "fields/fp.rs")).read()
    body, line = fn_body(fp, "sqrt_fq")
    s = strs(body)
    assert len(s) == 2
    kats["sqrt_fq"] = {"where": "src/fields/fp.rs:%d" % line, "root": s[0], "square": s[1]}

    fq2 = open(os.path.join(REF, "fields/fq2.rs")).read()
    body, line = fn_body(fq2, "sqrt_fq2")
    s = strs(body)
    assert len(s) == 6, s
    kats["sqrt_fq2"] = {"where": "src/fields/fq2.rs:%d" % line, "root": s[0:2], "square": s[2:4],
                        "minus_one_root": "i = (0, 1)", "no_root": s[4:6]}

    lib = open(os.path.join(REF, "lib.rs")).read()
    hex_re = re.compile(r'hex\("([0-9a-f]+)"\)')
    i1, i2 = lib.index("fn g1_from_compressed"), lib.index("fn g2_from_compressed")
    body, line = lib[i1:i2], lib[:i1].count("\n") + 1
    h, s = hex_re.findall(body), strs(body)
    assert len(h) == 1 and len(s) == 2
    kats["g1_from_compressed"] = {"where": "src/lib.rs:%d" % line, "bytes": h[0], "x": s[0], "y": s[1]}
    body, line = lib[i2:], lib[:i2].count("\n") + 1
    h, s = hex_re.findall(body), strs(body)
    assert len(h) == 3 and len(s) == 8 and s[4:8] == s[0:4], (len(h), len(s))
    kats["g2_from_compressed"] = {"where": "src/lib.rs:%d" % line, "bytes_0a": h[0], "bytes_0b_negated": h[1],
                                  "bytes_0c_invalid": h[2], "x": s[0:2], "y": s[2:4]}

    arith = open(os.path.join(REF, "arith.rs")).read()
    body, line = fn_body(arith, "testing_divrem")
    arr = re.findall(r"from\(\[([^\]]*)\]\)", body)
    words = [[int(w.strip(), 16) for w in a.split(",") if w.strip()] for a in arr]
    big = lambda ws: str(sum(w << (64 * i) for i, w in enumerate(ws)))
    # blocks in order: Fq modulus; p -> (1, 0); p^2-1 -> (q, r); p^2-2 -> (q, r);
    # "ridiculously large" -> (None, r); p^2 -> (None, 0); p^2+1 -> (None, 1);
    # Fr modulus, then "Fr modulus masked off" -> (Some(q < r), r' < r)
    assert [len(w) for w in words] == [4, 8, 8, 4, 4, 8, 4, 4, 8, 4, 8, 8, 4, 8], [len(w) for w in words]
    cases = [{"a": big(words[1]), "q": "1", "r": "0"},
             {"a": big(words[2]), "q": big(words[3]), "r": big(words[4])},
             {"a": big(words[5]), "q": big(words[6]), "r": big(words[7])},
             {"a": big(words[8]), "q": None, "r": big(words[9])},
             {"a": big(words[10]), "q": None, "r": "0"},
             {"a": big(words[11]), "q": None, "r": "1"}]
    kats["testing_divrem"] = {"where": "src/arith.rs:%d" % line, "modulo": big(words[0]), "cases": cases,
                              "fr_modulo": big(words[12]), "fr_masked_a": big(words[13])}
    kats["u256_one_big_endian"] = {"where": "src/arith.rs:561-586", "bytes": "00" * 31 + "01", "value": "1"}

    with open(OUT, "w") as fh:
        json.dump(kats, fh, indent=1)
    print("wrote", OUT)


if __name__ == "__main__":
    sys.exit(main())
