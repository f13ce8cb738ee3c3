#!/usr/bin/env python3
"""Coefficients of expm1_mid_f64's polynomial (gr-ldpc_ece535a_amd/csrc/ldpc_math.hpp).

expm1(r) = r + r^2 p(r) on |r| <= ln2/2.  p(r) = sum_k r^k / (k+2)! is
expanded to degree 22 in exact rational arithmetic, rewritten in Chebyshev
polynomials on [-h, h] (h = 0.3466 > ln2/2), truncated to degree D
(Chebyshev economisation: near-minimax, the error bounded by the dropped
coefficients' total, printed) and converted back to monomial coefficients,
rounded to double.

    python3 tools/gen_expm1_poly.py [D=9]
"""
import math
import sys
from fractions import Fraction as F

H = F(3466, 10000)
NT = 22


def cheb_of_monomials(a):
    """x^k = 2^(1-k) sum_j C(k, j) T_(k-2j), halved for the T_0 term."""
    c = [F(0)] * len(a)
    for k, ak in enumerate(a):
        for j in range(k // 2 + 1):
            n = k - 2 * j
            coef = F(math.comb(k, j), 2 ** k) * (2 if n > 0 else 1)
            c[n] += ak * coef
    return c


def mono_of_cheb(c, D):
    T = [[F(1)], [F(0), F(1)]]
    for n in range(2, D + 1):
        t = [F(0)] * (n + 1)
        for i, v in enumerate(T[n - 1]):
            t[i + 1] += 2 * v
        for i, v in enumerate(T[n - 2]):
            t[i] -= v
        T.append(t)
    m = [F(0)] * (D + 1)
    for n in range(D + 1):
        for i, v in enumerate(T[n]):
            m[i] += c[n] * v
    return m


def coefficients(D):
    taylor = [F(1, math.factorial(k + 2)) for k in range(NT + 1)]
    c = cheb_of_monomials([taylor[k] * H ** k for k in range(NT + 1)])  # r = H x
    m = mono_of_cheb(c, D)
    dropped = float(sum(abs(x) for x in c[D + 1:]))
    return [float(m[k] / H ** k) for k in range(D + 1)], dropped


def main():
    D = int(sys.argv[1]) if len(sys.argv) > 1 else 9
    coef, dropped = coefficients(D)
    print("// degree %d, dropped Chebyshev mass %.3g" % (D, dropped))
    print("  double p = %s;" % coef[-1].hex())
    for x in reversed(coef[:-1]):
        print("  p = fma_(p, r, %s);" % x.hex())


if __name__ == "__main__":
    main()
