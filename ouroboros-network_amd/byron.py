"""ByronDSIGN on gfx950 -- mirror of the reference's in-repo instance
``ouroboros-consensus-byron/src/Ouroboros/Consensus/Byron/Crypto/DSIGN.hs:63-120``
(verify side), plus the Byron header slicer that feeds it (SURVEY.md §8(a)
row a11, §8(f) rank 4).

``verifyDSIGN (magic, genKey) (VerKeyByronDSIGN vk) a sig`` (DSIGN.hs:110-113)
verifies ``signTag magic (signTagFor genKey a) <> recoverBytes a`` under the
first 32 bytes of the 64-byte XPub ``vk`` with cardano-crypto's donna-derived
Ed25519, whose acceptance differs from libsodium's: only
``sig[63] & 0xE0`` and an undecodable key are rejected.  For a block,
``signTagFor genKey _ = SignBlock genKey`` (DSIGN.hs:60-61) and the tag bytes are
``"01" <> unXPub genKey <> "\\x09" <> serialize' magic`` (cardano-ledger-byron
``Cardano.Crypto.Signing.Tag.signTag`` [ext, recalled]; pinned by the golden
Byron header, whose block signature verifies under exactly this message).

Callers: PBFT header validation,
``ouroboros-consensus/src/Ouroboros/Consensus/Protocol/PBFT.hs:332-337``, and
the Byron storage integrity check,
``ouroboros-consensus-byron/src/Ouroboros/Consensus/Byron/Ledger/Integrity.hs:32-35``.
``Right ()`` is returned as ``None``, ``Left e`` as the string ``e``.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Sequence, Tuple

import numpy as np

from . import _native
from ._pack import as_rows, msgs_arg, ptr
from .header import CBORError, _head, array_items, bytes_at

SIZE_VERKEY = 64   # XPub = public key (32) || chain code (32)
SIZE_SIG = 64

ERR = "Verification failed"  # DSIGN.hs:113


def cbor_uint(v: int) -> bytes:
    """Canonical CBOR unsigned integer (``serialize'`` of a Word32/Word64)."""
    if v < 0:
        raise ValueError("negative")
    if v < 24:
        return bytes([v])
    for ai, width in ((24, 1), (25, 2), (26, 4), (27, 8)):
        if v < (1 << (8 * width)):
            return bytes([ai]) + v.to_bytes(width, "big")
    raise ValueError("too large")


def sign_tag_block(magic: int, gen_xpub: bytes) -> bytes:
    """``signTag magic (SignBlock genKey)``: "01" || XPub || 0x09 || CBOR(magic)."""
    if len(gen_xpub) != SIZE_VERKEY:
        raise ValueError("genesis key must be a 64-byte XPub")
    return b"01" + bytes(gen_xpub) + b"\x09" + cbor_uint(magic)


class ByronDSIGN:
    """Verification half of ByronDSIGN (DSIGN.hs:63-120)."""

    @staticmethod
    def verify_dsign(ctx: Tuple[int, bytes], vk: bytes, signable: bytes, sig: bytes):
        """``verifyDSIGN (magic, genKey) vk a sig`` with ``signable`` =
        ``recoverBytes a`` (the annotated ToSign bytes): None or an error string."""
        magic, gen_key = ctx
        if len(vk) != SIZE_VERKEY or len(sig) != SIZE_SIG:
            return ERR
        msg = sign_tag_block(magic, gen_key) + bytes(signable)
        rc = _native.load().ouro_byron_ed25519_verify(msg, len(msg), bytes(vk[:32]), bytes(sig))
        if rc == _native.OURO_OK:
            return None
        if rc == _native.OURO_INVALID:
            return ERR
        _native.check(rc, "ouro_byron_ed25519_verify")
        return ERR  # unreachable: check() raised

    verify_signed_dsign = verify_dsign

    @staticmethod
    def verify_batch(pks, msgs, sigs) -> np.ndarray:
        """Batch verify of complete messages (tag included) under 32-byte keys
        (XPub[0:32]) or 64-byte XPubs; returns a bool array."""
        if isinstance(pks, np.ndarray) and pks.ndim == 2 and pks.shape[1] == SIZE_VERKEY:
            pks = pks[:, :32]
        elif not isinstance(pks, np.ndarray):
            pks = [bytes(p)[:32] if len(p) == SIZE_VERKEY else bytes(p) for p in pks]
        pk = as_rows(pks, 32, "pk")
        sg = as_rows(sigs, SIZE_SIG, "sig")
        buf, off, ln = msgs_arg(msgs)
        n = pk.shape[0]
        if sg.shape[0] != n or off.shape[0] != n:
            raise ValueError("pk, msg and sig batches differ in length")
        out = np.zeros(n, dtype=np.uint8)
        if n:
            rc = _native.load().ouro_byron_ed25519_verify_batch(
                n, ptr(pk), ptr(sg), ptr(buf), ptr(off), ptr(ln), ptr(out))
            _native.check(rc, "ouro_byron_ed25519_verify_batch")
        return out.astype(bool)


# ---- Byron header slicer -----------------------------------------------------

@dataclass
class ByronHeader:
    """The fields of a Byron regular (non-EBB) header the block signature needs."""
    magic: int
    to_sign: bytes        # recoverBytes of ToSign: 0x85 || prevHash || bodyProof || slot || diff || extra
    issuer_xpub: bytes    # delegation certificate issuer = the genesis key of SignBlock
    delegate_xpub: bytes  # signing (delegate) key
    sig: bytes            # 64-byte block signature
    slot_raw: bytes

    def message(self) -> bytes:
        return sign_tag_block(self.magic, self.issuer_xpub) + self.to_sign


def parse_byron_header(raw: bytes) -> ByronHeader:
    """Slice a Byron N2N header, ``#6.24(bytes .cbor [1, header])`` with
    header = [magic, prevHash, bodyProof, consensusData, extraData] and
    consensusData = [slotId, leaderKey, difficulty, blockSig]; blockSig =
    [2, [dlgCert, sig]] (the delegated signature used on mainnet; golden fixture
    ouroboros-consensus-byron-test/test/golden/ByronNodeToNodeVersion1/Header_regular).
    The signed bytes are the raw encodings of the ToSign fields, never re-encoded."""
    mt, arg, j = _head(raw, 0)
    if mt != 6 or arg != 24:
        raise CBORError("Byron header: expected tag 24")
    mt, arg, k = _head(raw, j)
    if mt != 2:
        raise CBORError("Byron header: expected bytes")
    buf = raw[k:k + arg]
    outer = array_items(buf, 0)
    if len(outer) != 2:
        raise CBORError("Byron header: expected [kind, header]")
    kind = buf[outer[0][0]]
    if kind != 0x01:
        raise CBORError("Byron header: epoch-boundary headers carry no signature")
    hdr = array_items(buf, outer[1][0])
    if len(hdr) != 5:
        raise CBORError("Byron header: expected 5 fields")
    mt, magic, _ = _head(buf, hdr[0][0])
    if mt != 0:
        raise CBORError("Byron header: magic")
    cons = array_items(buf, hdr[3][0])
    if len(cons) != 4:
        raise CBORError("Byron header: consensus data")
    raw_of = lambda it: buf[it[0]:it[1]]  # noqa: E731
    to_sign = (b"\x85" + raw_of(hdr[1]) + raw_of(hdr[2]) + raw_of(cons[0]) + raw_of(cons[2])
               + raw_of(hdr[4]))
    bsig = array_items(buf, cons[3][0])
    mt, sigkind, _ = _head(buf, bsig[0][0])
    if sigkind != 2:
        raise CBORError(f"Byron header: block signature kind {sigkind} (only delegated, 2)")
    inner = array_items(buf, bsig[1][0])
    cert = array_items(buf, inner[0][0])
    issuer = bytes_at(buf, cert[1][0])
    delegate = bytes_at(buf, cert[2][0])
    sig = bytes_at(buf, inner[1][0])
    if len(issuer) != SIZE_VERKEY or len(delegate) != SIZE_VERKEY or len(sig) != SIZE_SIG:
        raise CBORError("Byron header: key/signature sizes")
    return ByronHeader(magic=magic, to_sign=to_sign, issuer_xpub=issuer, delegate_xpub=delegate,
                       sig=sig, slot_raw=raw_of(cons[0]))


def verify_byron_headers(headers: Sequence[ByronHeader]) -> np.ndarray:
    """PBFT block-signature check of a batch of Byron headers (PBFT.hs:332-337):
    one gfx950 launch, bool per header."""
    msgs: List[bytes] = [h.message() for h in headers]
    pks = [h.delegate_xpub[:32] for h in headers]
    sigs = [h.sig for h in headers]
    return ByronDSIGN.verify_batch(pks, msgs, sigs)


verify_dsign = ByronDSIGN.verify_dsign
verify_batch = ByronDSIGN.verify_batch
