#!/usr/bin/env python3
"""Check the GF(2^255-19) constants of ouroboros-network_amd/csrc/fe25519.h:
every fe_make(...) constant is parsed from the header, its canonical radix-2^25.5
limbs are checked, and its value is compared with the number it claims to be.

  python tools/check_fe_constants.py        (exit status 0 = all good)
"""
import os
import re
import sys

P = 2**255 - 19
A = 486662
SQRTM1 = pow(2, (P - 1) // 4, P)
D = (-121665 * pow(121666, P - 2, P)) % P
EXPECT = {
    "fe_d": D,
    "fe_d2": 2 * D % P,
    "fe_sqrtm1": SQRTM1,
    "fe_mont_a": A,
    "fe_mont_a2": A * A % P,
    "fe_mont_a2a": (A + 2) * A % P,
    "fe_one_plus_i": (1 + SQRTM1) % P,
    "fe_one_minus_i": (1 - SQRTM1) % P,
    "fe_zero": 0,
    "fe_one": 1,
    "fe_two": 2,
}
HDR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                   "ouroboros-network_amd", "csrc", "fe25519.h")


def value(limbs):
    v, sh = 0, 0
    for i, l in enumerate(limbs):
        bits = 26 if i % 2 == 0 else 25
        assert 0 <= l < (1 << bits), f"limb {i} = {l} not canonical"
        v += l << sh
        sh += bits
    return v


def main():
    src = open(HDR).read()
    found = {}
    for m in re.finditer(r"OURO_FI fe (fe_\w+)\(\) \{\s*return fe_make\(([^)]*)\);", src):
        found[m.group(1)] = [int(x) for x in m.group(2).replace("\n", " ").split(",")]
    bad = 0
    for name, want in EXPECT.items():
        if name not in found:
            print(f"missing {name}")
            bad += 1
            continue
        got = value(found[name])
        ok = got == want
        bad += not ok
        print(f"{'ok ' if ok else 'BAD'} {name}")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
