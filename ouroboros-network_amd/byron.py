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
from typing import List, Optional, Sequence, Tuple, Union

import numpy as np

from . import _native
from ._pack import as_rows, msgs_arg, ptr
from .header import CBORError, _head, array_items, skip

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


# ---- delegation certificates ---------------------------------------------------
# A heavyweight delegation certificate (epoch, issuer XPub, delegate XPub,
# signature): cardano-ledger-byron's Delegation.Certificate [ext], the
# reference's PBftDelegationCert
# (ouroboros-consensus-byron/src/Ouroboros/Consensus/Byron/Protocol.hs:30) and
# the mempool's ByronDlg payload (.../Byron/Ledger/Mempool.hs:90).  The ledger
# verifies its signature under the issuer's key with the SignCertificate tag;
# the signed bytes below are pinned on the certificate the reference's golden
# Byron header carries (tests/test_byron_cert.py).  C ABI:
# ouro_byron_dlg_cert_{message,verify,verify_batch} (csrc/byron_dlg.cpp).
DLG_MSG_MAX = 96


def dlg_cert_message(magic: int, delegate_xpub: bytes, epoch: int) -> bytes:
    """0x0a || CBOR(magic) || CBOR bytes("00" || delegate XPub || CBOR(epoch))."""
    if len(delegate_xpub) != SIZE_VERKEY:
        raise ValueError("delegate key must be a 64-byte XPub")
    inner = b"00" + bytes(delegate_xpub) + cbor_uint(epoch)
    return b"\x0a" + cbor_uint(magic) + bytes([0x58, len(inner)]) + inner


def verify_delegation_certs(issuer_xpubs, delegate_xpubs, epochs, sigs,
                            protocol_magic: int) -> np.ndarray:
    """The certificates' signatures (ByronDSIGN acceptance) under the node's
    ProtocolMagicId, on the device (ouro_byron_dlg_cert_verify_batch); a
    bool array."""
    iss = as_rows(issuer_xpubs, SIZE_VERKEY, "issuer XPub")
    dlg = as_rows(delegate_xpubs, SIZE_VERKEY, "delegate XPub")
    sg = as_rows(sigs, SIZE_SIG, "sig")
    ep = np.ascontiguousarray(np.asarray(epochs, dtype=np.uint64).reshape(-1))
    n = iss.shape[0]
    if dlg.shape[0] != n or sg.shape[0] != n or ep.shape[0] != n:
        raise ValueError("certificate arrays differ in length")
    if not 0 <= int(protocol_magic) <= WORD32_MAX:
        raise ValueError("protocol magic outside Word32")
    out = np.zeros(n, dtype=np.uint8)
    if n:
        rc = _native.load().ouro_byron_dlg_cert_verify_batch(n, int(protocol_magic), ptr(iss),
                                                             ptr(dlg), ptr(ep), ptr(sg), ptr(out))
        _native.check(rc, "ouro_byron_dlg_cert_verify_batch")
    return out.astype(bool)


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
    def verify_batch(pks, msgs, sigs, host: bool = False) -> np.ndarray:
        """Batch verify of complete messages (tag included) under 32-byte keys
        (XPub[0:32]) or 64-byte XPubs; returns a bool array.  host=True: the
        library's host path (ouro_byron_ed25519_verify_batch_host)."""
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
            name = "ouro_byron_ed25519_verify_batch" + ("_host" if host else "")
            rc = getattr(_native.load(), name)(n, ptr(pk), ptr(sg), ptr(buf), ptr(off), ptr(ln),
                                               ptr(out))
            _native.check(rc, name)
        return out.astype(bool)


# ---- Byron header slicer -----------------------------------------------------
# Wire forms (ouroboros-consensus-byron/src/Ouroboros/Consensus/Byron/Node/Serialisation.hs):
#   F1  #6.24(bytes .cbor [kind, header])           Byron N2N v1 (:87-92), Cardano N2N v1
#   F2  [[kind, size], #6.24(bytes .cbor header)]   Byron N2N v2 (encodeDisk, :197-210)
#   F3  [0, F2]                                     Cardano N2N v2+ (HFC era 0)
# kind 1 = regular, 0 = epoch boundary (EBB).  The C slicer (csrc/cbor_byron.h,
# ouro_byron_pack_cbor) makes the same checks in the same order and reports
# the same status (tests/test_pack_byron.py).

PACK_OK, PACK_ECBOR, PACK_ESHAPE, PACK_ESIZE = 0, 1, 2, 3
PACK_EBB, PACK_ESHELLEY = 6, 7
WORD32_MAX = 0xFFFFFFFF
MSG_EXTRA = 80  # message slot per header: len + MSG_EXTRA bytes (cbor_byron.h)


class ByronPackError(CBORError):
    """A header the slicer rejects; .status is the OURO_PACK_* code."""

    def __init__(self, status: int, what: str):
        super().__init__(what)
        self.status = status


@dataclass
class ByronHeader:
    """The fields of a Byron regular (non-EBB) header the block signature needs."""
    magic: int            # the header's protocolMagic field
    to_sign: bytes        # recoverBytes of ToSign: 0x85 || prevHash || bodyProof || slot || diff || extra
    issuer_xpub: bytes    # delegation certificate issuer = the genesis key of SignBlock
    delegate_xpub: bytes  # signing (delegate) key
    sig: bytes            # 64-byte block signature
    slot_raw: bytes
    cert_epoch: int = 0   # the delegation certificate's epoch
    cert_sig: bytes = b""  # its signature (issuer key over dlg_cert_message)

    def message(self, protocol_magic: Union[int, str]) -> bytes:
        """signTag magic (SignBlock genKey) || signed bytes; magic = the node's
        configured ProtocolMagicId (mkByronContextDSIGN,
        ouroboros-consensus-byron/src/Ouroboros/Consensus/Byron/Ledger/PBFT.hs:43-44),
        or, only when asked for by name (protocol_magic=HEADER_MAGIC), the
        header's own field -- which the peer chose."""
        m = self.magic if _magic_arg(protocol_magic) < 0 else protocol_magic
        return sign_tag_block(m, self.issuer_xpub) + self.to_sign


def _fail(status: int, what: str):
    raise ByronPackError(status, what)


def _items(buf: bytes, i: int, want: int) -> List[Tuple[int, int]]:
    """A definite array of exactly `want` items (cbor_byron.h fixed_array)."""
    try:
        it = array_items(buf, i)
    except (CBORError, IndexError):
        _fail(PACK_ECBOR, f"malformed array at {i}")
    if len(it) != want:
        _fail(PACK_ESHAPE, f"expected {want} items at {i}")
    return it


def _uint(buf: bytes, i: int, mx: int, what: str) -> int:
    mt, arg, _ = _head(buf, i)
    if mt != 0 or arg < 0 or arg > mx:
        _fail(PACK_ESHAPE, what)
    return arg


def _bytes64(buf: bytes, i: int, what: str) -> bytes:
    mt, arg, j = _head(buf, i)
    if mt != 2 or arg < 0 or j + arg > len(buf):
        _fail(PACK_ESHAPE, what)
    if arg != SIZE_SIG:
        _fail(PACK_ESIZE, f"{what}: expected 64 bytes")
    return bytes(buf[j:j + arg])


def _parse(raw: bytes) -> Optional[ByronHeader]:
    buf = bytes(raw)
    mt, arg, j = _head(buf, 0)
    pos, kind = 0, 0
    nested = mt == 4 and arg == 2
    if nested:
        mt1, a1, j1 = _head(buf, j)
        if mt1 == 0:  # F3: the HFC era, then F2
            if a1 < 0:
                _fail(PACK_ESHAPE, "era")
            if a1 != 0:
                _fail(PACK_ESHELLEY, f"HFC era {a1}: not a Byron header")
            pos = j1
            mt, arg, j = _head(buf, pos)
            if mt != 4 or arg != 2:
                _fail(PACK_ESHAPE, "expected [[kind, size], header]")
        ks = _items(buf, j, 2)
        kind = _uint(buf, ks[0][0], 255, "kind: Word8")
        _uint(buf, ks[1][0], WORD32_MAX, "size: Word32")
        if kind > 1:
            _fail(PACK_ESHAPE, f"unknown header kind {kind}")
        pos = ks[1][1]
    mt, arg, j = _head(buf, pos)
    if mt != 6 or arg != 24:
        _fail(PACK_ESHAPE, "expected tag 24")
    mt, arg, k = _head(buf, j)
    if mt != 2 or arg < 0:
        _fail(PACK_ESHAPE, "expected definite CBOR-in-bytes")
    if k + arg != len(buf):
        _fail(PACK_ECBOR, "payload past the span or bytes after the header")
    h = k
    if not nested:  # F1: [kind, header]
        top = _items(buf, k, 2)
        kind = _uint(buf, top[0][0], 2**64 - 1, "kind")
        if kind > 1:
            _fail(PACK_ESHAPE, f"unknown header kind {kind}")
        h = top[1][0]
    if kind == 0:  # epoch boundary: no signature; its fields are not checked
        if skip(buf, h) != len(buf):
            _fail(PACK_ECBOR, "trailing bytes in CBOR-in-CBOR")
        return None
    f = _items(buf, h, 5)
    if f[4][1] != len(buf):
        _fail(PACK_ECBOR, "trailing bytes in CBOR-in-CBOR")
    magic = _uint(buf, f[0][0], WORD32_MAX, "protocol magic: Word32")
    cons = _items(buf, f[3][0], 4)
    bsig = _items(buf, cons[3][0], 2)
    mt, sigkind, _ = _head(buf, bsig[0][0])
    if mt != 0 or sigkind != 2:
        _fail(PACK_ESHAPE, "block signature kind (only delegated, 2)")
    inner = _items(buf, bsig[1][0], 2)
    cert = _items(buf, inner[0][0], 4)
    shape = []
    vals = []
    for at, what in ((cert[1][0], "issuer"), (cert[2][0], "delegate"), (inner[1][0], "sig")):
        try:
            vals.append(_bytes64(buf, at, what))
            shape.append(PACK_OK)
        except ByronPackError as e:
            vals.append(None)
            shape.append(e.status)
    if PACK_ESHAPE in shape:
        _fail(PACK_ESHAPE, "key/signature types")
    if PACK_ESIZE in shape:
        _fail(PACK_ESIZE, "key/signature sizes")
    raw_of = lambda it: buf[it[0]:it[1]]  # noqa: E731
    to_sign = (b"\x85" + raw_of(f[1]) + raw_of(f[2]) + raw_of(cons[0]) + raw_of(cons[2])
               + raw_of(f[4]))
    # the certificate's epoch and signature (not checked by PBFT's header
    # validation; dlg_cert_message / verify_delegation_certs): kept when well
    # formed, else left empty -- they never change the header's status
    cert_epoch, cert_sig = 0, b""
    try:
        mt, ep, _ = _head(buf, cert[0][0])
        mt2, ln, j2 = _head(buf, cert[3][0])
        if mt == 0 and ep >= 0 and mt2 == 2 and ln == SIZE_SIG and j2 + ln <= len(buf):
            cert_epoch, cert_sig = ep, bytes(buf[j2:j2 + ln])
    except (CBORError, IndexError):
        pass
    return ByronHeader(magic=magic, to_sign=to_sign, issuer_xpub=vals[0], delegate_xpub=vals[1],
                       sig=vals[2], slot_raw=raw_of(cons[0]), cert_epoch=cert_epoch,
                       cert_sig=cert_sig)


def byron_status(raw: bytes) -> Tuple[int, Optional[ByronHeader]]:
    """(OURO_PACK_* status, the header or None) -- what ouro_byron_pack_cbor
    reports for this header."""
    try:
        h = _parse(raw)
    except ByronPackError as e:
        return e.status, None
    except (CBORError, IndexError):
        return PACK_ECBOR, None
    return (PACK_EBB, None) if h is None else (PACK_OK, h)


def parse_byron_header(raw: bytes) -> ByronHeader:
    """Slice a regular Byron header in any of the wire forms F1-F3 above
    (golden fixtures: ouroboros-consensus-byron-test/test/golden/ByronNodeToNodeVersion1/Header_regular,
    ouroboros-consensus-cardano-test/test/golden/CardanoNodeToNodeVersion{1,2,3,4}/Header_Byron_regular).
    The signed bytes are the raw encodings of the ToSign fields, never
    re-encoded; the block signature is the delegated one, [2, [dlgCert, sig]].
    Raises CBORError (ByronPackError with the slicer's status) otherwise, an
    epoch-boundary header included."""
    st, h = byron_status(raw)
    if st != PACK_OK:
        raise ByronPackError(st, "epoch-boundary headers carry no signature" if st == PACK_EBB
                             else f"not a regular Byron header (status {st})")
    return h


@dataclass
class PackedByron:
    """ouro_byron_pack_cbor's output as arrays (views into its arena)."""
    pk: np.ndarray           # (n, 32)
    sig: np.ndarray          # (n, 64)
    genesis_vk: np.ndarray   # (n, 64)
    delegate_vk: np.ndarray  # (n, 64)
    magic: np.ndarray        # (n,) uint64
    msg: np.ndarray          # message bytes
    msg_off: np.ndarray      # (n,) uint64
    msg_len: np.ndarray      # (n,) uint32
    status: np.ndarray       # (n,) uint8 PACK_*
    _keep: tuple = ()

    def message(self, i: int) -> bytes:
        o = int(self.msg_off[i])
        return bytes(self.msg[o:o + int(self.msg_len[i])])


def _raw_arg(raw_headers):
    if isinstance(raw_headers, tuple) and len(raw_headers) == 3:
        buf, off, ln = raw_headers
        buf = np.frombuffer(buf, np.uint8) if isinstance(buf, (bytes, bytearray)) else \
            np.ascontiguousarray(buf, np.uint8).reshape(-1)
        return buf, np.ascontiguousarray(off, np.uint64), np.ascontiguousarray(ln, np.uint32)
    items = [bytes(r) for r in raw_headers]
    ln = np.array([len(r) for r in items], np.uint32)
    off = np.zeros(len(items), np.uint64)
    if len(items) > 1:
        off[1:] = np.cumsum(ln[:-1], dtype=np.uint64)
    return np.frombuffer(b"".join(items) or b"\0", np.uint8), off, ln


# protocol_magic = HEADER_MAGIC: sign with each header's own protocolMagic
# field instead of the node's configured ProtocolMagicId.  The reference
# always uses the configured one (Byron/Ledger/PBFT.hs:43-45 mkByronContextDSIGN,
# DSIGN.hs:111), so a header signed for another network fails there; the
# header's field is the peer's choice, hence an explicit opt-in, never a
# default.
HEADER_MAGIC = "header"


def _magic_arg(protocol_magic: Union[int, str]) -> int:
    if protocol_magic is None:
        raise ValueError("protocol_magic is required: the node's ProtocolMagicId "
                         "(or HEADER_MAGIC to use each header's own field)")
    if isinstance(protocol_magic, str):
        if protocol_magic != HEADER_MAGIC:
            raise ValueError(f"protocol_magic: a Word32 or {HEADER_MAGIC!r}")
        return -1
    if not 0 <= protocol_magic <= WORD32_MAX:
        raise ValueError("protocol_magic: a Word32")
    return int(protocol_magic)


def pack_byron_cbor(raw_headers, protocol_magic: Union[int, str],
                    nthreads: int = 0) -> PackedByron:
    """Raw Byron headers -> keys, signatures and signed messages through the C
    slicer (include/ouro_verify.h ouro_byron_pack_cbor, csrc/pack.cpp).
    raw_headers: a sequence of bytes, or (buf, off, len).  protocol_magic:
    the node's ProtocolMagicId for the sign tag (required; HEADER_MAGIC:
    each header's own field)."""
    import ctypes

    from .header import _pack_lib
    lib = _pack_lib() or _native.load()
    buf, off, ln = _raw_arg(raw_headers)
    n = int(off.size)
    if ln.size != n:
        raise ValueError("off / len: one entry per header")
    nbytes = int(lib.ouro_byron_pack_bytes(n, ptr(ln)))
    arena = np.empty(nbytes, np.uint8)
    status = np.zeros(max(n, 1), np.uint8)
    out = _native.ByronBatch()
    rc = lib.ouro_byron_pack_cbor(ptr(buf), buf.size, ptr(off), ptr(ln), n,
                                  _magic_arg(protocol_magic), ptr(arena), nbytes,
                                  ctypes.byref(out), ptr(status), nthreads)
    if rc != _native.OURO_OK:
        raise ValueError(f"ouro_byron_pack_cbor: {rc} (spans outside the buffer?)")
    base = arena.ctypes.data

    def view(addr, dt, w, cnt=None):
        if n == 0:
            return np.zeros((0, w) if w else 0, dt)
        cnt = cnt if cnt is not None else n * (w or 1)
        a = arena[addr - base: addr - base + cnt * np.dtype(dt).itemsize].view(dt)
        return a.reshape(n, w) if w else a

    return PackedByron(
        pk=view(out.pk, np.uint8, 32), sig=view(out.sig, np.uint8, 64),
        genesis_vk=view(out.genesis_vk, np.uint8, 64),
        delegate_vk=view(out.delegate_vk, np.uint8, 64), magic=view(out.magic, np.uint64, None),
        msg=arena[out.msg - base:] if n else np.zeros(0, np.uint8),
        msg_off=view(out.msg_off, np.uint64, None), msg_len=view(out.msg_len, np.uint32, None),
        status=status[:n], _keep=(arena, buf))


def verify_byron_cbor(raw_headers, protocol_magic: Union[int, str], devices=None):
    """Raw Byron headers -> (verdict bool array, status array) in one call
    (ouro_byron_verify_cbor: the raw-CBOR pipeline -- pinned staging, the
    device Byron slicer, the ByronDSIGN kernel): a regular header is valid
    when its block signature verifies, an epoch-boundary header always
    (PBFT.hs:327-328).  devices (a list of device indices, or "all"):
    ouro_byron_verify_cbor_multi, contiguous shards over those GPUs."""
    lib = _native.load()
    buf, off, ln = _raw_arg(raw_headers)
    n = int(off.size)
    status = np.zeros(max(n, 1), np.uint8)
    verdict = np.zeros(max(n, 1), np.uint8)
    if n and devices is not None:
        d = None if devices == "all" else np.ascontiguousarray(list(devices), np.int32)
        if d is not None and d.size == 0:
            raise ValueError("devices: at least one")
        rc = lib.ouro_byron_verify_cbor_multi(None if d is None else ptr(d),
                                              0 if d is None else int(d.size), ptr(buf),
                                              buf.size, ptr(off), ptr(ln), n,
                                              _magic_arg(protocol_magic), ptr(status),
                                              ptr(verdict))
        _native.check(rc, "ouro_byron_verify_cbor_multi")
    elif n:
        rc = lib.ouro_byron_verify_cbor(ptr(buf), buf.size, ptr(off), ptr(ln), n,
                                        _magic_arg(protocol_magic), ptr(status), ptr(verdict))
        _native.check(rc, "ouro_byron_verify_cbor")
    return verdict[:n].astype(bool), status[:n]


def verify_byron_headers(headers: Sequence[ByronHeader],
                         protocol_magic: Union[int, str]) -> np.ndarray:
    """PBFT block-signature check of a batch of parsed Byron headers
    (PBFT.hs:332-337): one gfx950 launch, bool per header.  Raw headers go
    through verify_byron_cbor instead (the C slicer, no per-header Python)."""
    msgs: List[bytes] = [h.message(protocol_magic) for h in headers]
    pks = [h.delegate_xpub[:32] for h in headers]
    sigs = [h.sig for h in headers]
    return ByronDSIGN.verify_batch(pks, msgs, sigs)


verify_dsign = ByronDSIGN.verify_dsign
verify_batch = ByronDSIGN.verify_batch
