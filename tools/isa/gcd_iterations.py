"""Outer iterations the key-cache inversion's binary GCD (fe_inv_vt.hpp, Pornin's
Algorithm 2 with k = 31: 62-bit approximations, 30 exact-parity steps per
iteration) needs before a = 0: per lane and as the maximum over a wave of 64
lanes, for uniformly random nonzero z < p.  The kernel leaves the loop when a = 0
in every lane of the wave.
Usage: python tools/isa/gcd_iterations.py [samples]"""
import random
import sys
from collections import Counter

P = 2 ** 255 - 19
M30 = (1 << 30) - 1


def iterations(z):
    a, b = z, P
    for it in range(17):
        if a == 0:
            return it
        nb = max(a.bit_length(), b.bit_length(), 62)
        A = (a & M30) | (((a >> (nb - 32)) & 0xffffffff) << 30)
        B = (b & M30) | (((b >> (nb - 32)) & 0xffffffff) << 30)
        f0, g0, f1, g1 = 1, 0, 0, 1
        for _ in range(30):
            if A & 1:
                if A < B:
                    A, B, f0, g0, f1, g1 = B, A, f1, g1, f0, g0
                A, f0, g0 = A - B, f0 - f1, g0 - g1
            A, f1, g1 = A >> 1, 2 * f1, 2 * g1
        a, b = abs((a * f0 + b * g0) >> 30), abs((a * f1 + b * g1) >> 30)
    return 17


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 6400
    rng = random.Random(1)
    v = [iterations(rng.randrange(1, P)) for _ in range(n)]
    print("per lane:", sorted(Counter(v).items()))
    print("wave of 64:", sorted(Counter(max(v[i:i + 64]) for i in range(0, n - 63, 64)).items()))


if __name__ == "__main__":
    main()
