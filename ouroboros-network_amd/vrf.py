"""PraosVRF (ECVRF-ED25519-SHA512-Elligator2, IETF draft-03) on gfx950 --
mirror of cardano-crypto-praos ``Cardano.Crypto.VRF.Praos`` (verify side).

Reference surface: ``verifyVRF :: ContextVRF v -> VerKeyVRF v -> a ->
(OutputVRF v, CertVRF v) -> Bool`` and ``verifyCertified``; the mock-protocol
usage is ouroboros-consensus-mock/src/Ouroboros/Consensus/Mock/Protocol/Praos.hs:341-354,
the real call is the OVERLAY rule via
ouroboros-consensus-shelley/src/Ouroboros/Consensus/Shelley/Protocol.hs:435.

Claimed-output semantics: ``verify_vrf`` in mode
``"ref2020"`` (default, as recalled for cardano-base@4251c0bb) checks the proof
only; ``"strict"`` additionally requires the claimed output to equal the
proof's output.  ``output_from_proof`` is ``crypto_vrf_ietfdraft03_proof_to_hash``.

The range of the proof's s: ``s_mode="reduce"`` (default,
the fork as recalled: s reduced mod L) or ``"strict"`` (s >= L rejected,
OURO_VRF_STRICT_S).  Which one cardano-crypto-praos uses is unpinned -- no
reference fixture has s >= L -- so both are offered.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _native
from ._pack import as_rows, msgs_arg, ptr

SIZE_VERKEY = 32
SIZE_PROOF = 80
SIZE_OUTPUT = 64


S_MODES = {"reduce": 0, "strict": _native.VRF_STRICT_S}


def _s_flags(s_mode: str) -> int:
    if s_mode not in S_MODES:
        raise ValueError(f"s_mode: one of {sorted(S_MODES)}")
    return S_MODES[s_mode]


class PraosVRF:
    @staticmethod
    def verify(vk: bytes, msg: bytes, proof: bytes, s_mode: str = "reduce"):
        """crypto_vrf_ietfdraft03_verify: the 64-byte output, or None."""
        if len(vk) != SIZE_VERKEY or len(proof) != SIZE_PROOF:
            return None
        if _s_flags(s_mode):
            ok, beta = PraosVRF.verify_batch([vk], [msg], [proof], s_mode=s_mode)
            return bytes(beta[0]) if ok[0] else None
        out = ctypes.create_string_buffer(SIZE_OUTPUT)
        rc = _native.load().ouro_vrf03_verify(out, vk, proof, msg, len(msg))
        if rc == _native.OURO_OK:
            return out.raw
        if rc == _native.OURO_INVALID:
            return None
        _native.check(rc, "ouro_vrf03_verify")
        return None

    @staticmethod
    def verify_vrf(ctx, vk: bytes, msg: bytes, certified, mode: str = "ref2020",
                   s_mode: str = "reduce") -> bool:
        """``verifyVRF () vk msg (output, proof)``."""
        output, proof = certified
        beta = PraosVRF.verify(vk, msg, proof, s_mode=s_mode)
        if beta is None:
            return False
        return True if mode == "ref2020" else bytes(output) == beta

    verify_certified = verify_vrf

    @staticmethod
    def output_from_proof(proof: bytes):
        """crypto_vrf_ietfdraft03_proof_to_hash: 64 bytes, or None if Gamma
        does not decode."""
        out = ctypes.create_string_buffer(SIZE_OUTPUT)
        rc = _native.load().ouro_vrf03_proof_to_hash(out, proof)
        if rc == _native.OURO_OK:
            return out.raw
        if rc == _native.OURO_INVALID:
            return None
        _native.check(rc, "ouro_vrf03_proof_to_hash")
        return None

    @staticmethod
    def verify_batch(vks, alphas, proofs, s_mode: str = "reduce", host: bool = False):
        """Returns (valid bool array, outputs (n, 64) uint8; zero rows where
        invalid).  host=True: the library's host path
        (ouro_vrf03_verify_batch_host) instead of the GPU."""
        flags = _s_flags(s_mode)
        vk = as_rows(vks, SIZE_VERKEY, "vk")
        pf = as_rows(proofs, SIZE_PROOF, "proof")
        buf, off, ln = msgs_arg(alphas)
        n = vk.shape[0]
        if pf.shape[0] != n or off.shape[0] != n:
            raise ValueError("vk, alpha and proof batches differ in length")
        ver = np.zeros(n, dtype=np.uint8)
        beta = np.zeros((n, SIZE_OUTPUT), dtype=np.uint8)
        if n:
            name = "ouro_vrf03_verify_batch_host" if host else "ouro_vrf03_verify_batch_flags"
            rc = getattr(_native.load(), name)(
                n, ptr(vk), ptr(pf), ptr(buf), ptr(off), ptr(ln), ptr(beta), ptr(ver), flags)
            _native.check(rc, name)
        return ver.astype(bool), beta


verify_vrf = PraosVRF.verify_vrf
verify_certified = PraosVRF.verify_certified
output_from_proof = PraosVRF.output_from_proof
verify_batch = PraosVRF.verify_batch
