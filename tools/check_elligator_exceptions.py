#!/usr/bin/env python3
"""The case analysis behind elligator2_h (csrc/verify.h): none of the
denominators it divides by can be zero, and its one-exponentiation
square-root bookkeeping is sound.  Each claim is a Legendre-symbol fact of
p = 2^255 - 19 and A = 486662:

  * D = 1 + 2 r^2 != 0            <=>  -1/2 (i.e. -2) is a non-square
  * W = D^2 (u^2 + A u + 1) != 0  <=>  A^2 - 4 is a non-square
  * m = Xn + D != 0               <=>  neither (A-1)/2 nor 1/(2(A-1)) is a square
  * chi(rho1) = chi(g(x1))        <=>  -(A + 2) is a square
  * 2/i = (1 - i)^2, 2/(-i) = (1 + i)^2 with i = sqrt(-1)

  python tools/check_elligator_exceptions.py   (exit status 0 = all hold)
"""
import sys

P = 2**255 - 19
A = 486662
I = pow(2, (P - 1) // 4, P)


def chi(x):
    return pow(x % P, (P - 1) // 2, P)


def inv(x):
    return pow(x % P, P - 2, P)


CLAIMS = [
    ("-2 non-square", chi(-2) == P - 1),
    ("A^2 - 4 non-square", chi(A * A - 4) == P - 1),
    ("(A-1)/2 non-square", chi((A - 1) * inv(2)) == P - 1),
    ("1/(2(A-1)) non-square", chi(inv(2 * (A - 1))) == P - 1),
    ("-(A+2) square", chi(-(A + 2)) == 1),
    ("i^2 = -1", I * I % P == P - 1),
    ("2/i = (1-i)^2", 2 * inv(I) % P == (1 - I) ** 2 % P),
    ("2/(-i) = (1+i)^2", 2 * inv(-I) % P == (1 + I) ** 2 % P),
]


def main():
    bad = 0
    for name, ok in CLAIMS:
        print(f"{'ok ' if ok else 'BAD'} {name}")
        bad += not ok
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
