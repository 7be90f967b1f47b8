"""Search the M-image chunk swizzle (csrc/kernels/ntn.hip mask_m) with the LDS bank model of bank_sim.py:
transposed full-K reads (rows 8q + 0..3 / + 4..7), transposed 16-deep tail reads (rows 32 + 4q + 0..3) and
the dC row reads (ds_read_b128, rows 16 ma + n, chunk pair 8 kb + 2q) must all be conflict-free."""
import itertools
import os
import random
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from bank_sim import G32, GB128, cyc_read  # noqa: E402


def score(X, MTH=3):
    def addr(row, chunk):
        return row * 128 + ((chunk ^ X[row & 15]) << 3)
    tot = 0
    for mb in range(MTH):
        for h in range(2):   # full K-step, lo / hi halves
            A = [addr(8 * (l >> 4) + 4 * h + ((l & 15) >> 2), 4 * mb + (l & 3)) for l in range(64)]
            tot += cyc_read(A, G32, 8)
        A = [addr(32 + 4 * (l >> 4) + ((l & 15) >> 2), 4 * mb + (l & 3)) for l in range(64)]   # tail
        tot += cyc_read(A, G32, 8)
    for ma in range(MTH):
        for kb in range(2):
            A = [addr(16 * ma + (l & 15), 8 * kb + 2 * (l >> 4)) for l in range(64)]
            tot += cyc_read(A, GB128, 16)
    return tot


if __name__ == "__main__":
    cur = [((a & 2) << 1) | (a & 8) for a in range(16)]
    print("current mask_m", score(cur))
    random.seed(0)
    best = None
    for _ in range(200000):
        X = [2 * random.randrange(8) for _ in range(16)]   # even: keeps 16-B pairs intact
        s = score(X)
        if best is None or s < best[0]:
            best = (s, X)
            print(best, flush=True)
            if s == 0:
                break


def structured():
    """X(a) = 4 * f(a bits) ^ 2 * g(...) candidates: all maps from the 4 row bits to the 3 chunk-pair bits
    that are linear over GF(2) (XOR of row-bit columns) -- 8^4 = 4096 candidates, exhaustive."""
    best = None
    for cols in itertools.product(range(8), repeat=4):
        X = []
        for a in range(16):
            y = 0
            for bit in range(4):
                if (a >> bit) & 1:
                    y ^= cols[bit]
            X.append(2 * y)
        s = score(X)
        if best is None or s < best[0]:
            best = (s, X, cols)
    return best
