"""Leader threshold on the leader VRF output -- ledger-specs ``checkLeaderValue``.

Reference: ``meetsLeaderThreshold``
(ouroboros-consensus-shelley/src/Ouroboros/Consensus/Shelley/Protocol.hs:473-491)
calls ``SL.checkLeaderValue (VRF.certifiedOutput certNat) r (tpraosLeaderF
tpraosParams)`` with ``r`` the issuing pool's relative stake.  The reference
precomputes ``ActiveSlotCoeff``'s ``unActiveSlotLog = floor (10^34 ln (1 - f))``
once per network; this mirror takes that integer (``ActiveSlotCoeff`` below) so
the device never needs the reference's ``ln'``.

SURVEY.md §8(f) rank 3.  The batch runs on the GPU (``csrc/leader.h``); there is
no CPU fallback.  Parity is unpinned (the reference's packages are not in this
image): ``oracle/leader.py`` restates the same published algorithm
independently and the tests compare the two.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from fractions import Fraction
from typing import Sequence

import numpy as np

from . import _native
from ._pack import ptr

LEADER_NO = _native.LEADER_NO
LEADER_YES = _native.LEADER_YES
LEADER_BADARG = _native.LEADER_BADARG


@dataclass(frozen=True)
class ActiveSlotCoeff:
    """The reference's ``ActiveSlotCoeff``: ``unActiveSlotLog`` (a negative
    integer, floor(10^34 ln(1 - f))) and whether f is exactly 1."""

    un_active_slot_log: int
    is_one: bool = False

    def words(self):
        v = self.un_active_slot_log & ((1 << 128) - 1)
        lo = v & ((1 << 64) - 1)
        hi = v >> 64
        if hi >= 1 << 63:
            hi -= 1 << 64
        return hi, lo


def check_leader_values(beta_leader: np.ndarray, sigma: Sequence[Fraction],
                        f: ActiveSlotCoeff, host: bool = False) -> np.ndarray:
    """checkLeaderValue for every row of ``beta_leader`` (n x 64 u8) with the
    issuer's relative stake ``sigma[i]``; returns u8 LEADER_YES / LEADER_NO /
    LEADER_BADARG (sigma or f outside the supported domain).  host=True: the
    library's host path (ouro_leader_check_batch_host) instead of the GPU."""
    beta = np.ascontiguousarray(beta_leader, dtype=np.uint8).reshape(-1, 64)
    n = beta.shape[0]
    if len(sigma) != n:
        raise ValueError("one sigma per output")
    num = np.zeros(n, dtype=np.uint64)
    den = np.zeros(n, dtype=np.uint64)
    for i, s in enumerate(sigma):
        s = Fraction(s)
        if s.numerator < 0 or s.denominator >= 1 << 64 or s.numerator >= 1 << 64:
            raise ValueError("sigma must be a non-negative fraction of 64-bit integers")
        num[i], den[i] = s.numerator, s.denominator
    verdict = np.zeros(n, dtype=np.uint8)
    if n:
        hi, lo = f.words()
        name = "ouro_leader_check_batch" + ("_host" if host else "")
        rc = getattr(_native.load(), name)(n, ptr(beta), ptr(num), ptr(den), ctypes.c_int64(hi),
                                           ctypes.c_uint64(lo), 1 if f.is_one else 0,
                                           ptr(verdict))
        _native.check(rc, name)
    return verdict


def check_leader_value(beta: bytes, sigma: Fraction, f: ActiveSlotCoeff) -> bool:
    """The reference's single-item signature: Bool, True = eligible leader."""
    v = check_leader_values(np.frombuffer(bytes(beta), dtype=np.uint8).reshape(1, 64), [sigma], f)
    if v[0] == LEADER_BADARG:
        raise ValueError("sigma or active slot coefficient outside the supported domain")
    return bool(v[0] == LEADER_YES)
