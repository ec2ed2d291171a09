"""Sum6KES (SumKES^6 over SingleKES Ed25519DSIGN, Blake2b_256) on gfx950 --
mirror of cardano-crypto-class ``Cardano.Crypto.KES.Sum`` (verify side).

Reference surface: ``verifyKES :: ContextKES v -> VerKeyKES v -> Period -> a ->
SigKES v -> Either String ()`` / ``verifySignedKES``, called at
ouroboros-consensus-shelley/src/Ouroboros/Consensus/Shelley/Ledger/Integrity.hs:27
with t computed at Integrity.hs:38-44 (``kes_period`` below).
"""
from __future__ import annotations

import numpy as np

from . import _native
from ._pack import as_rows, msgs_arg, ptr

SIZE_VERKEY = 32
SIZE_SIG = 448
TOTAL_PERIODS = 64
PERIOD_MAX_U32 = 0xFFFFFFFF


def periods_u32(periods) -> np.ndarray:
    """The reference's ``Period`` is a 64-bit ``Word``; the C ABI takes 32 bits.
    SumKES.verifyKES goes right at a level when t >= half and subtracts half,
    so every t >= 63 (= 32 + 16 + ... + 1) takes the right branch at all six
    levels and ends on leaf 63 (SingleKES's ``assert (t == 0)`` is compiled
    out).  Saturating at 2^32 - 1 therefore keeps the reference's result for
    every Word; negative values are not periods and raise."""
    t = np.asarray(list(periods) if not isinstance(periods, np.ndarray) else periods)
    if t.size == 0:
        return np.zeros(0, np.uint32)
    if t.dtype == object or t.dtype.kind not in "iu":
        t = np.array([int(x) for x in t.ravel()], dtype=object)
        if any(x < 0 for x in t):
            raise ValueError("negative KES period")
        return np.array([min(int(x), PERIOD_MAX_U32) for x in t], np.uint32)
    if t.dtype.kind == "i" and (t < 0).any():
        raise ValueError("negative KES period")
    return np.ascontiguousarray(np.minimum(t.astype(np.uint64), PERIOD_MAX_U32).astype(np.uint32))


def kes_period(slot: int, slots_per_kes_period: int, start_of_kes_period: int) -> int:
    """t of verifyHeaderIntegrity (Integrity.hs:38-44): clamped at 0."""
    current = slot // slots_per_kes_period
    return current - start_of_kes_period if current >= start_of_kes_period else 0


class Sum6KES:
    @staticmethod
    def verify_kes(ctx, vk: bytes, period: int, msg: bytes, sig: bytes):
        """``verifyKES () vk t msg sig``: None (Right ()) or an error string."""
        if len(vk) != SIZE_VERKEY or len(sig) != SIZE_SIG:
            return "Reject"
        if int(period) < 0:
            raise ValueError("negative KES period")
        rc = _native.load().ouro_sum6kes_verify(vk, min(int(period), PERIOD_MAX_U32), msg,
                                                len(msg), sig)
        if rc == _native.OURO_OK:
            return None
        if rc == _native.OURO_INVALID:
            return "Reject"
        _native.check(rc, "ouro_sum6kes_verify")
        return "Reject"

    verify_signed_kes = verify_kes

    @staticmethod
    def verify_batch(vks, periods, msgs, sigs, host: bool = False) -> np.ndarray:
        """Batch verify; True = valid.  host=True: the library's host path
        (ouro_sum6kes_verify_batch_host) instead of the GPU."""
        vk = as_rows(vks, SIZE_VERKEY, "vk")
        sg = as_rows(sigs, SIZE_SIG, "sig")
        t = periods_u32(periods)
        buf, off, ln = msgs_arg(msgs)
        n = vk.shape[0]
        if sg.shape[0] != n or t.shape[0] != n or off.shape[0] != n:
            raise ValueError("vk, t, msg and sig batches differ in length")
        out = np.zeros(n, dtype=np.uint8)
        if n:
            name = "ouro_sum6kes_verify_batch" + ("_host" if host else "")
            rc = getattr(_native.load(), name)(
                n, ptr(vk), ptr(t), ptr(buf), ptr(off), ptr(ln), ptr(sg), ptr(out))
            _native.check(rc, name)
        return out.astype(bool)


verify_kes = Sum6KES.verify_kes
verify_signed_kes = Sum6KES.verify_signed_kes
verify_batch = Sum6KES.verify_batch
