#!/usr/bin/env python3
"""Is there a cheaper chain for exp_by_neg_z (x^u, u = 4965661367192848881) in the
cyclotomic subgroup, where x^-d = conj(x^d) is free?  Prices a left-to-right chain
over a signed digit set D: the table (x^2 once, then one Fq12 product per further
odd entry) plus, for the digits, one product per nonzero digit after the top one and
one cyclotomic squaring per halving, at k_pairing_full's per-operation VALU
(profiles/r6_isa_histogram_k_pairing_full.txt: 3,053 per cyclotomic square, 7,528
per Fq12 product).  Contiguous odd windows up to 21 first, then random sets of up
to seven odd digits < 64.  Result: nothing beats the width-4
window's 16 products + 63 squarings by more than ~1 %.
"""
import functools, itertools
u = 4965661367192848881
S, M = 3053, 7528   # VALU per cyclotomic square / Fq12 product (k_pairing_full ISA)

def best(D):
    Ds = sorted(set(D) | {-d for d in D})
    @functools.lru_cache(None)
    def f(v):
        # returns (mults, sqrs) to compute x^v from table entries, top digit loaded free
        if v == 0: return None
        if v in D: return (0, 0)
        if v % 2 == 0:
            r = f(v // 2)
            return None if r is None else (r[0], r[1] + 1)
        res = None
        for d in Ds:
            w = v - d
            if w <= 0 or w % 2: continue
            r = f(w // 2)
            if r is None: continue
            c = (r[0] + 1, r[1] + 1)
            if res is None or c[0] * M + c[1] * S < res[0] * M + res[1] * S: res = c
        return res
    return f(u)

for k in range(1, 12):
    D = tuple(range(1, 2 * k, 2))
    r = best(D)
    table_m = k - 1
    table_s = 1 if k > 1 else 0
    m = r[0] + table_m; s = r[1] + table_s
    print("odd digits up to %2d: chain mults %2d sqrs %2d, table %d mults %d sqr -> %2d mults %2d sqrs cost %.0fk" % (2*k-1, r[0], r[1], table_m, table_s, m, s, (m*M + s*S)/1e3))

import random
def table_cost(D):
    # entries built in increasing order; each new odd entry e costs 1 mult if e = a + b (a, b in built, incl. 2 = x^2)
    built = {1, 2}
    m = 0
    for e in sorted(D):
        if e in built: continue
        if any((e - a) in built for a in built): m += 1; built.add(e); continue
        return None
    return m
bestc = None
random.seed(1)
cands = list(range(3, 64, 2))
for it in range(4000):
    k = random.randint(1, 6)
    D = tuple(sorted({1} | set(random.sample(cands, k))))
    tc = table_cost(D)
    if tc is None: continue
    r = best(D)
    if r is None: continue
    m = r[0] + tc; s = r[1] + 1
    c = m * M + s * S
    if bestc is None or c < bestc[0]:
        bestc = (c, D, m, s)
        print("%.0fk D=%s mults %d sqrs %d" % (c / 1e3, D, m, s))
