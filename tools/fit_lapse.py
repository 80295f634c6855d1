#!/usr/bin/env python3
"""Coefficients of the lapse-rate power polynomial used by ngrtd_math.hpp lapse_rate_fast:

    (1 - .0065 E / 288.15) ** 5.2561   for E in [-500, 4500] m,  x = (E - 2000) / 2500

Chebyshev interpolant at 10 nodes in 50-digit arithmetic (mpmath), converted to monomial
coefficients in x, printed as C++ double literals with the maximum relative error of the
double-precision Horner evaluation over 4001 points.  (noble_gas_utils.py:103-113.)"""
import mpmath as mp

mp.mp.dps = 50
N = 10


def f(E):
    return mp.power(1 - mp.mpf("0.0065") * E / mp.mpf("288.15"), mp.mpf("5.2561"))


def main():
    nodes = [mp.cos(mp.pi * (k + mp.mpf(1) / 2) / N) for k in range(N)]
    fv = [f(2000 + 2500 * x) for x in nodes]
    ch = [(2 if j else 1) * sum(fv[k] * mp.cos(mp.pi * j * (k + mp.mpf(1) / 2) / N) for k in range(N)) / N
          for j in range(N)]
    T = [[mp.mpf(0)] * N for _ in range(N)]
    T[0][0] = 1
    T[1][1] = 1
    for j in range(2, N):
        for k in range(N):
            T[j][k] = (2 * T[j - 1][k - 1] if k else 0) - T[j - 2][k]
    mono = [float(sum(ch[j] * T[j][k] for j in range(k, N))) for k in range(N)]
    worst = 0.0
    for i in range(4001):
        E = -500.0 + 5000.0 * i / 4000
        x = (E - 2000.0) * (1.0 / 2500.0)
        b = mono[-1]
        for k in range(N - 2, -1, -1):
            b = b * x + mono[k]
        worst = max(worst, float(abs((mp.mpf(b) - f(mp.mpf(E))) / f(mp.mpf(E)))))
    print("max relative error %.3g" % worst)
    for k, m in enumerate(mono):
        print("    %s,   // x^%d" % (m.hex(), k))


if __name__ == "__main__":
    main()
