"""Generate inputs for / verify the ubench2 29-bit Montgomery prototype dump."""
import random, struct, sys
P = 0x30644E72E131A029B85045B68181585D97816A916871CA8D3C208C16D87CFD47
M = (1 << 29) - 1
def limbs(x): return [(x >> (29 * i)) & M for i in range(9)]
def val(l): return sum(v << (29 * i) for i, v in enumerate(l))
n = 4096
rnd = random.Random(5)
A = [rnd.randrange(2 * P) for _ in range(n)]
B = [rnd.randrange(2 * P) for _ in range(n)]
if sys.argv[1] == "gen":
    with open(sys.argv[2], "wb") as f:
        f.write(struct.pack("<i", n))
        for x in A + B:
            f.write(struct.pack("<9I", *limbs(x)))
else:
    data = open(sys.argv[2], "rb").read()
    bad = 0
    rinv = pow(1 << 261, -1, P)
    worst = 0
    for i in range(n):
        l = struct.unpack_from("<9I", data, 36 * i)
        v = val(l)
        worst = max(worst, v / P)
        if v % P != A[i] * B[i] * rinv % P or any(x > M for x in l[:8]):
            bad += 1
    print('{"bench": "mul29_check", "n": %d, "bad": %d, "max_out_over_p": %.4f}' % (n, bad, worst))
