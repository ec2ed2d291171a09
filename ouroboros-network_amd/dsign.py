"""Ed25519DSIGN on gfx950 -- mirror of cardano-crypto-class
``Cardano.Crypto.DSIGN.Ed25519`` (verify side).

Reference surface: ``verifyDSIGN :: ContextDSIGN v ->
VerKeyDSIGN v -> a -> SigDSIGN v -> Either String ()`` and
``verifySignedDSIGN``; the in-repo shape is visible in
ouroboros-consensus-byron/src/Ouroboros/Consensus/Byron/Crypto/DSIGN.hs:66-127.
Callers: the OCERT rule via
ouroboros-consensus-shelley/src/Ouroboros/Consensus/Shelley/Protocol.hs:435 and
the SingleKES leaf.  ``Right ()`` is returned as ``None``, ``Left e`` as the
string ``e``.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _native
from ._pack import as_rows, msgs_arg, ptr

SIZE_VERKEY = 32
SIZE_SIG = 64


class Ed25519DSIGN:
    """Verification half of Ed25519DSIGN (libsodium 1.0.18 acceptance rules)."""

    @staticmethod
    def verify_dsign(ctx, vk: bytes, msg: bytes, sig: bytes):
        """``verifyDSIGN () vk msg sig``: None (Right ()) or an error string."""
        if len(vk) != SIZE_VERKEY or len(sig) != SIZE_SIG:
            return "Verification failed"
        lib = _native.load()
        rc = lib.ouro_ed25519_verify(sig, msg, len(msg), vk)
        if rc == _native.OURO_OK:
            return None
        if rc == _native.OURO_INVALID:
            return "Verification failed"
        _native.check(rc, "ouro_ed25519_verify")
        return "Verification failed"  # unreachable: check() raised

    verify_signed_dsign = verify_dsign

    @staticmethod
    def verify_batch(vks, msgs, sigs, host: bool = False) -> np.ndarray:
        """Batch verify; returns a bool array (True = valid).  host=True runs
        the library's host path (ouro_ed25519_verify_batch_host: the kernels'
        lane routines on the CPU) instead of the GPU."""
        vk = as_rows(vks, SIZE_VERKEY, "vk")
        sg = as_rows(sigs, SIZE_SIG, "sig")
        buf, off, ln = msgs_arg(msgs)
        n = vk.shape[0]
        if sg.shape[0] != n or off.shape[0] != n:
            raise ValueError("vk, msg and sig batches differ in length")
        out = np.zeros(n, dtype=np.uint8)
        if n:
            name = "ouro_ed25519_verify_batch" + ("_host" if host else "")
            rc = getattr(_native.load(), name)(n, ptr(vk), ptr(sg), ptr(buf), ptr(off), ptr(ln),
                                               ptr(out))
            _native.check(rc, name)
        return out.astype(bool)


verify_dsign = Ed25519DSIGN.verify_dsign
verify_signed_dsign = Ed25519DSIGN.verify_signed_dsign
verify_batch = Ed25519DSIGN.verify_batch
