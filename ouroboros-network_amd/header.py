"""Shelley-family header wire format -> SoA batch.

Wire shape (ouroboros-network/test/messages.cddl:27-34; decoder with the raw
bytes kept via Annotator at
ouroboros-consensus-shelley/src/Ouroboros/Consensus/Shelley/Ledger/Block.hs:216-217;
N2N wrapping at .../Shelley/Node/Serialisation.hs:88-90):

    header      = #6.24(bytes .cbor [header_body, kes_sig])          (N2N v1)
    hfc_header  = [era, #6.24(bytes .cbor [header_body, kes_sig])]   (Cardano N2N v2+)
    header_body = [blockNo, slot, prevHash, issuerVk, vrfVk, etaCert,
                   leaderCert, bodySize, bodyHash, hotVk, counter,
                   kesPeriod, sigma, protMajor, protMinor]
    cert        = [output(64 B), proof(80 B)]

The KES message is the *raw* header_body bytes, so the slicer records byte
spans instead of re-encoding anything.
"""
from __future__ import annotations

import hashlib
import os
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import numpy as np

from .kes import periods_u32
from .tpraos import HeaderBatch


class CBORError(ValueError):
    pass


def _head(buf: bytes, i: int) -> Tuple[int, int, int]:
    """(major type, argument, index after the head) of the item at i."""
    if i >= len(buf):
        raise CBORError("truncated")
    ib = buf[i]
    mt, ai = ib >> 5, ib & 31
    i += 1
    if ai < 24:
        return mt, ai, i
    if ai in (24, 25, 26, 27):
        n = 1 << (ai - 24)
        if i + n > len(buf):
            raise CBORError("truncated")
        return mt, int.from_bytes(buf[i:i + n], "big"), i + n
    if ai == 31:
        return mt, -1, i  # indefinite length
    raise CBORError(f"reserved additional info {ai}")


def skip(buf: bytes, i: int) -> int:
    """Index just past the CBOR data item starting at i."""
    mt, arg, j = _head(buf, i)
    if mt in (0, 1, 7):
        return j
    if mt in (2, 3):
        if arg < 0:
            while buf[j] != 0xFF:
                j = skip(buf, j)
            return j + 1
        if j + arg > len(buf):
            raise CBORError("truncated")  # (a short final string is not a shorter one)
        return j + arg
    if mt in (4, 5):
        count = arg * (2 if mt == 5 else 1)
        if arg < 0:
            while buf[j] != 0xFF:
                j = skip(buf, j)
            return j + 1
        for _ in range(count):
            j = skip(buf, j)
        return j
    if mt == 6:
        return skip(buf, j)
    raise CBORError("bad major type")


def array_items(buf: bytes, i: int) -> List[Tuple[int, int]]:
    """Spans [(start, end)] of the elements of the definite array at i."""
    mt, arg, j = _head(buf, i)
    if mt != 4 or arg < 0:
        raise CBORError(f"expected definite array at {i}")
    out = []
    for _ in range(arg):
        k = skip(buf, j)
        out.append((j, k))
        j = k
    return out


def uint_at(buf: bytes, i: int) -> int:
    mt, arg, _ = _head(buf, i)
    if mt != 0:
        raise CBORError(f"expected uint at {i}")
    return arg


def bytes_at(buf: bytes, i: int) -> bytes:
    mt, arg, j = _head(buf, i)
    if mt != 2 or arg < 0:
        raise CBORError(f"expected definite bytes at {i}")
    if j + arg > len(buf):
        raise CBORError("truncated")
    return bytes(buf[j:j + arg])


@dataclass
class ShelleyHeader:
    era: int                 # HFC era tag (1 Shelley, 2 Allegra, 3 Mary), 1 if unwrapped
    block_no: int
    slot: int
    issuer_vk: bytes
    vrf_vk: bytes
    eta_output: bytes
    eta_proof: bytes
    leader_output: bytes
    leader_proof: bytes
    hot_vk: bytes
    ocert_counter: int
    ocert_kes_period: int
    ocert_sigma: bytes
    body: bytes              # raw header_body CBOR = the KES message
    kes_sig: bytes
    body_span: Tuple[int, int]  # offsets of `body` inside the input bytes


def parse_header(raw: bytes) -> ShelleyHeader:
    """Parse an N2N (v1: tag-24 wrapped) or Cardano HFC-wrapped Shelley-era header.

    CBOR-in-CBOR as the reference decodes it (ouroboros-network/src/Ouroboros/
    Network/Block.hs:509-514): the tag-24 byte string is definite and inside
    `raw`; [header_body, kes_sig] is parsed from its payload alone and must end
    where the payload ends; nothing may follow the header."""
    buf = bytes(raw)
    era, i = 1, 0
    mt, arg, j = _head(buf, 0)
    if mt == 4 and arg == 2:  # [era, wrapped]
        era = uint_at(buf, j)
        if era == 0:
            raise CBORError("Byron header: not a TPraos header")
        i = skip(buf, j)
    mt, arg, j = _head(buf, i)
    if mt != 6 or arg != 24:
        raise CBORError("expected #6.24 wrapped header")
    mt, arg, k = _head(buf, j)
    if mt != 2 or arg < 0:
        raise CBORError("expected definite CBOR-in-bytes")
    if k + arg > len(buf):
        raise CBORError("truncated")
    if k + arg != len(buf):
        raise CBORError("trailing bytes after the header")
    buf = buf[:k + arg]  # (the same length: the payload bounds every parse below)
    inner_start = k
    top = array_items(buf, inner_start)
    if len(top) != 2:
        raise CBORError("header must be [body, sig]")
    (b0, b1), (s0, s1) = top
    if s1 != k + arg:
        raise CBORError("trailing bytes in CBOR-in-CBOR")
    f = array_items(buf, b0)
    if len(f) != 15:
        raise CBORError(f"header body must have 15 fields, got {len(f)}")
    eta = array_items(buf, f[5][0])
    lead = array_items(buf, f[6][0])
    if len(eta) != 2 or len(lead) != 2:
        raise CBORError("VRF certificates must be [output, proof]")
    hdr = ShelleyHeader(
        era=era,
        block_no=uint_at(buf, f[0][0]),
        slot=uint_at(buf, f[1][0]),
        issuer_vk=bytes_at(buf, f[3][0]),
        vrf_vk=bytes_at(buf, f[4][0]),
        eta_output=bytes_at(buf, eta[0][0]),
        eta_proof=bytes_at(buf, eta[1][0]),
        leader_output=bytes_at(buf, lead[0][0]),
        leader_proof=bytes_at(buf, lead[1][0]),
        hot_vk=bytes_at(buf, f[9][0]),
        ocert_counter=uint_at(buf, f[10][0]),
        ocert_kes_period=uint_at(buf, f[11][0]),
        ocert_sigma=bytes_at(buf, f[12][0]),
        body=buf[b0:b1],
        kes_sig=bytes_at(buf, s0),
        body_span=(b0, b1),
    )
    # rawDeserialise* of the fixed-size crypto types rejects any other length
    for name, want in (("issuer_vk", 32), ("vrf_vk", 32), ("eta_output", 64),
                       ("eta_proof", 80), ("leader_output", 64), ("leader_proof", 80),
                       ("hot_vk", 32), ("ocert_sigma", 64), ("kes_sig", 448)):
        if len(getattr(hdr, name)) != want:
            raise CBORError(f"{name}: expected {want} bytes")
    return hdr


def kes_t(slot: int, slots_per_kes_period: int, c0: int) -> int:
    """Integrity.hs:38-44: kesPeriod(slot) - c0, clamped at 0."""
    cur = slot // slots_per_kes_period
    return cur - c0 if cur >= c0 else 0


def pack(headers: Sequence[ShelleyHeader], eta_alpha: Optional[Sequence[bytes]] = None,
         leader_alpha: Optional[Sequence[bytes]] = None, slots_per_kes_period: int = 129600,
         *, claimed: bool = True, seeds: bool = False,
         epoch_nonce: Optional[bytes] = None) -> HeaderBatch:
    """SoA batch from parsed headers.

    VRF inputs: the caller's alphas (mkSeed values), or with seeds=True the
    header slots and `epoch_nonce` (eta0; None = NeutralNonce), from which the
    device derives them exactly as OVERLAY does.  claimed=True carries the
    headers' certifiedOutputs, so the verdict has the *_CLAIM_OK bits and the
    nonce output hashes the claimed eta output (the reference's semantics)."""
    n = len(headers)
    if not seeds and (eta_alpha is None or leader_alpha is None
                      or len(eta_alpha) != n or len(leader_alpha) != n):
        raise ValueError("one eta/leader alpha per header (or seeds=True)")
    if epoch_nonce is not None and len(epoch_nonce) != 32:
        raise ValueError("epoch_nonce: 32 bytes")

    def rows(get, w):
        return np.frombuffer(b"".join(get(h) for h in headers), np.uint8).reshape(n, w) if n \
            else np.zeros((0, w), np.uint8)

    lens = np.array([len(h.body) for h in headers], np.uint32)
    offs = np.zeros(n, np.uint64)
    if n > 1:
        offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    alphas = (None, None) if seeds else (
        np.frombuffer(b"".join(eta_alpha), np.uint8).reshape(n, 32),
        np.frombuffer(b"".join(leader_alpha), np.uint8).reshape(n, 32))
    return HeaderBatch(
        issuer_vk=rows(lambda h: h.issuer_vk, 32),
        vrf_vk=rows(lambda h: h.vrf_vk, 32),
        eta_proof=rows(lambda h: h.eta_proof, 80),
        leader_proof=rows(lambda h: h.leader_proof, 80),
        eta_alpha=alphas[0],
        leader_alpha=alphas[1],
        hot_vk=rows(lambda h: h.hot_vk, 32),
        ocert_counter=np.array([h.ocert_counter for h in headers], np.uint64),
        ocert_kes_period=np.array([h.ocert_kes_period for h in headers], np.uint64),
        ocert_sigma=rows(lambda h: h.ocert_sigma, 64),
        kes_t=periods_u32([kes_t(h.slot, slots_per_kes_period, h.ocert_kes_period)
                           for h in headers]),
        kes_sig=rows(lambda h: h.kes_sig, 448),
        body=np.frombuffer(b"".join(h.body for h in headers) or b"\0", np.uint8),
        body_off=offs,
        body_len=lens,
        eta_output=rows(lambda h: h.eta_output, 64) if claimed else None,
        leader_output=rows(lambda h: h.leader_output, 64) if claimed else None,
        slot=np.array([h.slot for h in headers], np.uint64) if seeds else None,
        epoch_nonce=np.frombuffer(epoch_nonce, np.uint8) if (seeds and epoch_nonce) else None,
    )


PACK_OK, PACK_ECBOR, PACK_ESHAPE, PACK_ESIZE, PACK_EBYRON, PACK_ESPAN = 0, 1, 2, 3, 4, 5


@dataclass
class PackedHeaders:
    """Result of :func:`pack_cbor`: the batch (arrays view the C arena and the
    raw buffer, which this object keeps alive), per-header status
    (PACK_*), slots and HFC eras."""
    batch: HeaderBatch
    status: np.ndarray
    slot: np.ndarray
    era: np.ndarray
    _keep: tuple = ()


_PACK_LIB = None


def _pack_lib():
    """TEST-ONLY: OURO_PACK_LIB names a library exporting just the slicer (the
    ASan/UBSan build of csrc/pack.cpp, tests/test_sanitizers.py)."""
    global _PACK_LIB
    path = os.environ.get("OURO_PACK_LIB")
    if not path:
        return None
    if _PACK_LIB is None:
        import ctypes

        from . import _native
        lib = ctypes.CDLL(path)
        for name in ("ouro_tpraos_pack_bytes", "ouro_tpraos_pack_cbor", "ouro_byron_pack_bytes",
                     "ouro_byron_pack_cbor"):
            res, args = _native.SIGNATURES[name]
            getattr(lib, name).restype = res
            getattr(lib, name).argtypes = args
        _PACK_LIB = lib
    return _PACK_LIB


def raw_triplet(raw_headers):
    """(buf, off, len) as contiguous uint8 / uint64 / uint32 arrays from either
    a sequence of bytes (one header each, concatenated) or a (buf, off, len)
    triple with the headers at buf[off[i]:off[i]+len[i]]."""
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


def pack_cbor(raw_headers, *, slots_per_kes_period: int = 129600,
              eta_alpha: Optional[np.ndarray] = None, leader_alpha: Optional[np.ndarray] = None,
              seeds: bool = False, epoch_nonce: Optional[bytes] = None, claimed: bool = True,
              nthreads: int = 0) -> PackedHeaders:
    """Raw header CBOR -> SoA batch through the C slicer of the product library
    (include/ouro_verify.h ouro_tpraos_pack_cbor; csrc/pack.cpp).  Same
    acceptance and arrays as parse_header + pack, without per-header Python.

    raw_headers: a sequence of bytes (one header each), or (buf, off, len)
    with the headers at buf[off[i]:off[i]+len[i]].  VRF inputs as for pack:
    the caller's alphas, or seeds=True (+ epoch_nonce) for mkSeed on device.
    Rejected headers (status != PACK_OK) get zero rows: they fail every check."""
    import ctypes

    from . import _native
    lib = _pack_lib() or _native.load()
    buf, off, ln = raw_triplet(raw_headers)
    n = int(off.size)
    if ln.size != n:
        raise ValueError("off / len: one entry per header")
    if epoch_nonce is not None and len(epoch_nonce) != 32:
        raise ValueError("epoch_nonce: 32 bytes")
    if not seeds and (eta_alpha is None or leader_alpha is None):
        raise ValueError("one eta/leader alpha per header (or seeds=True)")
    nbytes = int(lib.ouro_tpraos_pack_bytes(n))
    arena = np.empty(nbytes, np.uint8)
    status = np.zeros(max(n, 1), np.uint8)
    slot = np.zeros(max(n, 1), np.uint64)
    era = np.zeros(max(n, 1), np.uint8)
    out = _native.TPraosBatch()
    ptr = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    rc = lib.ouro_tpraos_pack_cbor(ptr(buf), buf.size, ptr(off), ptr(ln), n,
                                   slots_per_kes_period, ptr(arena), nbytes, ctypes.byref(out),
                                   ptr(slot), ptr(era), ptr(status), nthreads)
    if rc != _native.OURO_OK:
        raise ValueError(f"ouro_tpraos_pack_cbor: {rc} (spans outside the buffer?)")
    base = arena.ctypes.data

    def view(addr, dt, w):
        if n == 0:
            return np.zeros((0, w) if w else 0, dt)
        cnt = n * (w or 1)
        a = arena[addr - base: addr - base + cnt * np.dtype(dt).itemsize].view(dt)
        return a.reshape(n, w) if w else a

    batch = HeaderBatch(
        issuer_vk=view(out.issuer_vk, np.uint8, 32), vrf_vk=view(out.vrf_vk, np.uint8, 32),
        eta_proof=view(out.eta_proof, np.uint8, 80),
        leader_proof=view(out.leader_proof, np.uint8, 80),
        eta_alpha=None if seeds else eta_alpha, leader_alpha=None if seeds else leader_alpha,
        hot_vk=view(out.hot_vk, np.uint8, 32),
        ocert_counter=view(out.ocert_counter, np.uint64, None),
        ocert_kes_period=view(out.ocert_kes_period, np.uint64, None),
        ocert_sigma=view(out.ocert_sigma, np.uint8, 64), kes_t=view(out.kes_t, np.uint32, None),
        kes_sig=view(out.kes_sig, np.uint8, 448), body=buf,
        body_off=view(out.body_off, np.uint64, None), body_len=view(out.body_len, np.uint32, None),
        eta_output=view(out.eta_output, np.uint8, 64) if claimed else None,
        leader_output=view(out.leader_output, np.uint8, 64) if claimed else None,
        slot=slot[:n] if seeds else None,
        epoch_nonce=np.frombuffer(epoch_nonce, np.uint8) if (seeds and epoch_nonce) else None,
    )
    return PackedHeaders(batch, status[:n], slot[:n], era[:n], (arena, buf))


def _blake2b_256(m: bytes) -> bytes:
    return hashlib.blake2b(m, digest_size=32).digest()


SEED_ETA = _blake2b_256((0).to_bytes(8, "big"))  # mkNonceFromNumber 0
SEED_L = _blake2b_256((1).to_bytes(8, "big"))    # mkNonceFromNumber 1


def mk_seed(universal_nonce: Optional[bytes], slot: int, epoch_nonce: Optional[bytes]) -> bytes:
    """ledger-specs mkSeed on the host (the device computes the same when a
    batch carries slots): Blake2b_256(BE64(slot) || eta0) XOR ucNonce, eta0 =
    None for NeutralNonce; ucNonce = SEED_ETA / SEED_L (mkNonceFromNumber 0/1,
    pinned by the reference's golden ChainDepState, tests/test_nonce.py)."""
    h = _blake2b_256(slot.to_bytes(8, "big") + (epoch_nonce or b""))
    if universal_nonce is None:
        return h
    return bytes(a ^ b for a, b in zip(h, universal_nonce))


def _devices_arg(devices):
    """(int array or None, count) for the *_multi entries: None = every
    visible device"""
    if devices is None:
        return None, 0
    d = np.ascontiguousarray(list(devices), np.int32)
    if d.size == 0:
        raise ValueError("devices: at least one")
    return d, int(d.size)


def verify_integrity_cbor(raw_headers, slots_per_kes_period: int, host: bool = False,
                          devices=None):
    """verifyHeaderIntegrity over raw headers (KES only; the storage layer's
    check, ouroboros-consensus-shelley/src/Ouroboros/Consensus/Shelley/Ledger/
    Integrity.hs:20-44): returns (valid bool array, slicer status array).
    Default: ouro_integrity_verify_cbor (the raw-CBOR pipeline: header bytes
    gathered into pinned staging, the device slicer, the Sum6KES kernel).
    host=True: the same slicer, then the library's host path
    (ouro_sum6kes_verify_batch_host) -- no device touched.  devices (a list
    of device indices, or "all"): ouro_integrity_verify_cbor_multi, contiguous
    shards over those GPUs of this process."""
    import ctypes

    from . import _native
    buf, off, ln = raw_triplet(raw_headers)
    n = int(off.size)
    status = np.zeros(max(n, 1), np.uint8)
    verdict = np.zeros(max(n, 1), np.uint8)
    if n == 0:
        return verdict[:0].astype(bool), status[:0]
    ptr = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    lib = _native.load()
    if not host and devices is not None:
        d, nd = _devices_arg(None if devices == "all" else devices)
        rc = lib.ouro_integrity_verify_cbor_multi(ptr(d) if d is not None else None, nd,
                                                  ptr(buf), buf.size, ptr(off), ptr(ln), n,
                                                  slots_per_kes_period, ptr(status),
                                                  ptr(verdict))
        _native.check(rc, "ouro_integrity_verify_cbor_multi")
        return verdict[:n].astype(bool), status[:n]
    if not host:
        rc = lib.ouro_integrity_verify_cbor(ptr(buf), buf.size, ptr(off), ptr(ln), n,
                                            slots_per_kes_period, ptr(status), ptr(verdict))
        _native.check(rc, "ouro_integrity_verify_cbor")
        return verdict[:n].astype(bool), status[:n]
    p = pack_cbor((buf, off, ln), slots_per_kes_period=slots_per_kes_period, seeds=True,
                  claimed=False)
    b = p.batch
    rc = lib.ouro_sum6kes_verify_batch_host(n, ptr(b.hot_vk), ptr(b.kes_t), ptr(b.body),
                                            ptr(b.body_off), ptr(b.body_len), ptr(b.kes_sig),
                                            ptr(verdict))
    _native.check(rc, "ouro_sum6kes_verify_batch_host")
    ok = (verdict[:n] != 0) & (p.status == PACK_OK)
    return ok, p.status.copy()


def verify_headers_cbor(raw_headers, slots_per_kes_period: int, *,
                        epoch_nonce: Optional[bytes] = None,
                        eta_alpha: Optional[np.ndarray] = None,
                        leader_alpha: Optional[np.ndarray] = None, nonce: bool = False,
                        devices=None):
    """The full TPraos header check straight from raw header CBOR in host
    memory, one call (include/ouro_verify.h ouro_tpraos_verify_cbor): the
    crypto of TPraos.updateChainDepState (ouroboros-consensus-shelley/src/
    Ouroboros/Consensus/Shelley/Protocol.hs:433-442) over every header.
    VRF inputs: eta_alpha / leader_alpha (n x 32 each) when given, else mkSeed
    from each header's slot and epoch_nonce (None = NeutralNonce) on the
    device.  Returns (verdict, beta_eta, beta_leader, status[, eta_nonce]):
    verdict = OURO_HDR_* bits (0 where the header does not slice).
    devices (a list of device indices, or "all"): ouro_tpraos_verify_cbor_multi,
    contiguous shards over those GPUs of this process."""
    import ctypes

    from . import _native
    buf, off, ln = raw_triplet(raw_headers)
    n = int(off.size)
    if ln.size != n:
        raise ValueError("off / len: one entry per header")
    if epoch_nonce is not None and len(epoch_nonce) != 32:
        raise ValueError("epoch_nonce: 32 bytes")
    if (eta_alpha is None) != (leader_alpha is None):
        raise ValueError("give both alpha arrays or neither")
    m = max(n, 1)
    status = np.zeros(m, np.uint8)
    verdict = np.zeros(m, np.uint8)
    be = np.zeros((m, 64), np.uint8)
    bl = np.zeros((m, 64), np.uint8)
    en = np.zeros((m, 32), np.uint8) if nonce else None
    ptr = lambda a: None if a is None else a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    ea = la = None
    if eta_alpha is not None:
        ea = np.ascontiguousarray(eta_alpha, np.uint8).reshape(n, 32)
        la = np.ascontiguousarray(leader_alpha, np.uint8).reshape(n, 32)
    eta0 = None if epoch_nonce is None else np.frombuffer(bytes(epoch_nonce), np.uint8)
    if n:
        lib = _native.load()
        if devices is not None:
            d, nd = _devices_arg(None if devices == "all" else devices)
            rc = lib.ouro_tpraos_verify_cbor_multi(ptr(d), nd, ptr(buf), buf.size, ptr(off),
                                                   ptr(ln), n, slots_per_kes_period, ptr(eta0),
                                                   ptr(ea), ptr(la), ptr(status), ptr(verdict),
                                                   ptr(be), ptr(bl), ptr(en))
            _native.check(rc, "ouro_tpraos_verify_cbor_multi")
        else:
            rc = lib.ouro_tpraos_verify_cbor(ptr(buf), buf.size, ptr(off), ptr(ln), n,
                                             slots_per_kes_period, ptr(eta0), ptr(ea), ptr(la),
                                             ptr(status), ptr(verdict), ptr(be), ptr(bl), ptr(en))
            _native.check(rc, "ouro_tpraos_verify_cbor")
    out = (verdict[:n], be[:n], bl[:n], status[:n])
    return out + (en[:n],) if nonce else out
