"""TEST INFRASTRUCTURE ONLY -- CPU oracle for the TPraos leader-threshold check.

Pure-Python exact-integer restatement of ledger-specs `checkLeaderValue`
(shelley-spec-ledger BlockChain.hs) with shelley-spec-non-integral's
`taylorExpCmp` over `FixedPoint = Data.Fixed E34`, as called from
ouroboros-consensus-shelley/src/Ouroboros/Consensus/Shelley/Protocol.hs:473-491
(`meetsLeaderThreshold`: `SL.checkLeaderValue (VRF.certifiedOutput certNat) r
(tpraosLeaderF tpraosParams)`).  Both packages are un-vendored git dependencies
absent from this container: PARITY UNPINNED -- no reference
output or fixture covers this function; the restatement follows the published
Haskell source as recalled and is checked here only against the independent
device restatement (csrc/leader.h).

Data.Fixed semantics (res = 10^34): a * b = floor(a b / res),
a / b = floor(a res / b), fromRational r = floor(r res), fromInteger i = i res.
"""
from __future__ import annotations

from fractions import Fraction

RES = 10**34


def _fix_mul(a: int, b: int) -> int:
    return (a * b) // RES


def _fix_div(a: int, b: int) -> int:
    return (a * RES) // b


def _from_rational(r: Fraction) -> int:
    return (r.numerator * RES) // r.denominator


def taylor_exp_cmp(bound_x: int, cmp: int, x: int, max_n: int = 1000):
    """taylorExpCmp boundX cmp x = go 1000 0 x 1 1 (mantissas in, verdict out):
    'ABOVE', 'BELOW' or 'MAX'."""
    err, acc, divisor = x, 1 * RES, 1 * RES
    for _ in range(max_n):
        divisor1 = divisor + 1 * RES
        err1 = _fix_div(_fix_mul(err, x), divisor1)
        acc1 = acc + err
        error_term = abs(_fix_mul(err1, bound_x))
        if cmp >= acc1 + error_term:
            return "ABOVE"
        if cmp < acc1 - error_term:
            return "BELOW"
        err, acc, divisor = err1, acc1, divisor1
    return "MAX"


def check_leader_value(beta: bytes, sigma: Fraction, active_slot_log: int,
                       f_is_one: bool = False) -> bool:
    """checkLeaderValue certVRF sigma f, with f given as its
    ActiveSlotCoeff fields: unActiveSlotLog (active_slot_log) and whether its
    unActiveSlotVal is exactly 1."""
    if f_is_one:
        return True
    cert_nat_max = 1 << (8 * len(beta))
    cert_nat = int.from_bytes(beta, "big")
    recip_q = _from_rational(Fraction(cert_nat_max, cert_nat_max - cert_nat))
    c = _fix_div(active_slot_log * RES, (10**34) * RES)  # activeSlotLog f
    x = -_fix_mul(_from_rational(Fraction(sigma)), c)
    r = taylor_exp_cmp(3 * RES, recip_q, x)
    return r == "BELOW"


def active_slot_log(f: Fraction, digits: int = 60) -> int:
    """floor(10^34 ln(1 - f)) from a high-precision decimal logarithm -- a test
    input generator, not the reference's `ln'` (which the device API takes
    precomputed, as the reference's ActiveSlotCoeff stores it)."""
    import decimal

    ctx = decimal.Context(prec=digits)
    v = ctx.ln(ctx.subtract(decimal.Decimal(1), ctx.divide(decimal.Decimal(f.numerator),
                                                           decimal.Decimal(f.denominator))))
    return int((v * decimal.Decimal(RES)).to_integral_value(rounding=decimal.ROUND_FLOOR))
