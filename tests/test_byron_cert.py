"""Byron heavyweight delegation certificates (VERDICT r05 missing item 5:
the certificate signature's layout, SURVEY.md Appendix C, was unpinned).

A certificate (epoch, issuer XPub, delegate XPub, signature) is
cardano-ledger-byron's Delegation.Certificate [ext] -- the reference's
PBftDelegationCert (ouroboros-consensus-byron/src/Ouroboros/Consensus/Byron/
Protocol.hs:30) and the mempool's ByronDlg payload (.../Byron/Ledger/
Mempool.hs:90).  The reference's golden Byron header carries one inside its
block signature; its signature verifies under exactly

    0x0a || CBOR(protocol magic) || CBOR bytes("00" || delegate XPub || CBOR(epoch))

(the SignCertificate tag bytes, then the CBOR serialisation of the signed
ByteString) and under none of the unwrapped orders tried before -- which is
what pins the layout.  CPU tests: the pin (libsodium directly and the
oracle's donna-style verify), the C message builder against the Python one,
the single-certificate entry on the host path, argument checks; and on the
GPU (marked gpu) the device batch against the oracle.
"""
import ctypes
import json
import os

import numpy as np
import pytest

import oracle_ffi as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def golden():
    from ouroboros_network_amd import byron as B

    with open(os.path.join(ROOT, "tests", "golden", "reference_kats.json")) as f:
        k = json.load(f)
    raws = [bytes.fromhex(k["byron"]["raw"])] + [bytes.fromhex(w["raw"]) for w in k["byron_wire"]]
    hs = []
    for r in raws:
        st, h = B.byron_status(r)
        if st == B.PACK_OK:
            hs.append(h)
    assert hs
    return hs


def _sodium_verify(s, sig, m, pk):
    return s.crypto_sign_ed25519_verify_detached(sig, m, ctypes.c_ulonglong(len(m)), pk) == 0


def test_layout_pinned_by_the_golden_certificate(golden):
    from ouroboros_network_amd import byron as B

    s = O.sodium()
    for h in golden:
        assert len(h.cert_sig) == 64
        m = B.dlg_cert_message(h.magic, h.delegate_xpub, h.cert_epoch)
        assert O.ed25519_verify_byron(h.cert_sig, m, h.issuer_xpub[:32])
        if s is not None:
            assert _sodium_verify(s, h.cert_sig, m, h.issuer_xpub[:32])
        # the unwrapped orders (SURVEY.md App. C's search) do not verify
        ep = B.cbor_uint(h.cert_epoch)
        mg = B.cbor_uint(h.magic)
        for wrong in (b"00" + h.delegate_xpub + b"\x0a" + mg + ep,
                      b"\x0a" + mg + b"00" + h.delegate_xpub + ep,
                      b"00" + h.delegate_xpub + ep,
                      b"\x0a" + m[1 + len(mg) + 2:]):  # no magic
            assert not O.ed25519_verify_byron(h.cert_sig, wrong, h.issuer_xpub[:32])


def test_c_message_builder_matches_python():
    from ouroboros_network_amd import _native
    from ouroboros_network_amd import byron as B

    lib = _native.load()
    rng = np.random.default_rng(5)
    buf = ctypes.create_string_buffer(B.DLG_MSG_MAX)
    for magic in (0, 1, 23, 24, 255, 256, 65535, 65536, 764824073, 2**32 - 1):
        for epoch in (0, 1, 23, 24, 255, 256, 2**16, 2**32 - 1, 2**32, 2**64 - 1):
            d = rng.bytes(64)
            want = B.dlg_cert_message(magic, d, epoch)
            n = lib.ouro_byron_dlg_cert_message(buf, magic, d, epoch)
            assert n == len(want) <= B.DLG_MSG_MAX
            assert buf.raw[:n] == want
    assert lib.ouro_byron_dlg_cert_message(None, 1, bytes(64), 0) == 0


def test_single_certificate_on_the_host_path(golden):
    """ouro_byron_dlg_cert_verify (host path, no GPU): the golden certificate
    under its magic; the wrong magic or epoch, and a flipped bit in the
    signature or either key, against the oracle's verdict."""
    from ouroboros_network_amd import _native
    from ouroboros_network_amd import byron as B

    lib = _native.load()
    h = golden[0]
    assert lib.ouro_byron_dlg_cert_verify(h.magic, h.issuer_xpub, h.delegate_xpub, h.cert_epoch,
                                          h.cert_sig) == 0
    assert lib.ouro_byron_dlg_cert_verify(764824073, h.issuer_xpub, h.delegate_xpub,
                                          h.cert_epoch, h.cert_sig) == -1
    assert lib.ouro_byron_dlg_cert_verify(h.magic, h.issuer_xpub, h.delegate_xpub,
                                          h.cert_epoch + 1, h.cert_sig) == -1
    rng = np.random.default_rng(11)
    for _ in range(60):
        which = int(rng.integers(0, 3))
        iss, dlg, sig = bytearray(h.issuer_xpub), bytearray(h.delegate_xpub), bytearray(h.cert_sig)
        tgt = (iss, dlg, sig)[which]
        lim = 32 if which == 0 else 64  # only XPub[0:32] is the issuer's key
        tgt[int(rng.integers(0, lim))] ^= 1 << int(rng.integers(0, 8))
        want = O.ed25519_verify_byron(bytes(sig), B.dlg_cert_message(h.magic, bytes(dlg),
                                                                     h.cert_epoch), bytes(iss[:32]))
        rc = lib.ouro_byron_dlg_cert_verify(h.magic, bytes(iss), bytes(dlg), h.cert_epoch,
                                            bytes(sig))
        assert rc == (0 if want else -1)
    assert lib.ouro_byron_dlg_cert_verify(h.magic, None, h.delegate_xpub, 0, h.cert_sig) \
        == _native.OURO_EINVAL


def test_batch_argument_checks():
    from ouroboros_network_amd import _native
    from ouroboros_network_amd import byron as B

    lib = _native.load()
    assert lib.ouro_byron_dlg_cert_verify_batch(0, 1, None, None, None, None, None) == 0
    assert lib.ouro_byron_dlg_cert_verify_batch(3, 1, None, None, None, None, None) \
        == _native.OURO_EINVAL
    with pytest.raises(ValueError):
        B.verify_delegation_certs(np.zeros((2, 64), np.uint8), np.zeros((3, 64), np.uint8),
                                  [0, 0], np.zeros((2, 64), np.uint8), 1)
    with pytest.raises(ValueError):
        B.verify_delegation_certs(np.zeros((1, 64), np.uint8), np.zeros((1, 64), np.uint8),
                                  [0], np.zeros((1, 64), np.uint8), 2**32)


def synth_certs(n: int, magic: int, seed: int = 3):
    """n certificates signed by the oracle's Ed25519 (test infrastructure),
    one in eight corrupted; the expected verdicts from the oracle's
    donna-style verify."""
    from ouroboros_network_amd import byron as B

    rng = np.random.default_rng(seed)
    iss, dlg, eps, sigs, want = [], [], [], [], []
    keys = [O.ed25519_keypair(rng.bytes(32)) for _ in range(8)]
    for i in range(n):
        pk, sk = keys[i % 8]
        ix = pk + rng.bytes(32)  # XPub = key || chain code
        dx = rng.bytes(64)
        ep = int(rng.integers(0, 2**40)) if i % 3 else int(rng.integers(0, 400))
        sig = O.ed25519_sign(sk, B.dlg_cert_message(magic, dx, ep))
        if rng.integers(0, 8) == 0:
            what = int(rng.integers(0, 4))
            if what == 0:
                b = bytearray(sig)
                b[int(rng.integers(0, 64))] ^= 1 << int(rng.integers(0, 8))
                sig = bytes(b)
            elif what == 1:
                b = bytearray(ix)
                b[int(rng.integers(0, 32))] ^= 1 << int(rng.integers(0, 8))
                ix = bytes(b)
            elif what == 2:
                b = bytearray(dx)
                b[int(rng.integers(0, 64))] ^= 1 << int(rng.integers(0, 8))
                dx = bytes(b)
            else:
                ep ^= 1
        iss.append(ix)
        dlg.append(dx)
        eps.append(ep)
        sigs.append(sig)
        want.append(O.ed25519_verify_byron(sig, B.dlg_cert_message(magic, dx, ep), ix[:32]))
    arr = lambda xs: np.frombuffer(b"".join(xs), np.uint8).reshape(len(xs), -1)  # noqa: E731
    return arr(iss), arr(dlg), np.array(eps, np.uint64), arr(sigs), np.array(want)


def test_synthetic_certificates_single_items_host():
    """A few hundred oracle-signed certificates through the single-item
    (host-path) entry against the oracle's verdicts."""
    from ouroboros_network_amd import _native

    lib = _native.load()
    iss, dlg, eps, sigs, want = synth_certs(240, 764824073)
    assert 0 < want.sum() < len(want)
    for i in range(len(want)):
        rc = lib.ouro_byron_dlg_cert_verify(764824073, bytes(iss[i]), bytes(dlg[i]), int(eps[i]),
                                            bytes(sigs[i]))
        assert rc == (0 if want[i] else -1), i


@pytest.mark.gpu
def test_gpu_delegation_certificate_batch(gpu_lib, golden):
    """ouro_byron_dlg_cert_verify_batch on the device: 4,096 oracle-signed
    certificates (1/8 corrupted in the signature, either key or the epoch)
    plus the golden certificate and its single-byte corruptions, against the
    oracle; then the same certificates under another magic all fail."""
    from ouroboros_network_amd import byron as B

    magic = 764824073
    iss, dlg, eps, sigs, want = synth_certs(4096, magic)
    got = B.verify_delegation_certs(iss, dlg, eps, sigs, magic)
    np.testing.assert_array_equal(got, want)
    assert not B.verify_delegation_certs(iss, dlg, eps, sigs, magic + 1).any()
    h = golden[0]
    rows_i, rows_d, rows_s, rows_w = [], [], [], []
    for pos in range(64 + 32 + 64):
        ix, dx, sg = bytearray(h.issuer_xpub), bytearray(h.delegate_xpub), bytearray(h.cert_sig)
        if pos < 64:
            sg[pos] ^= 0x10
        elif pos < 96:
            ix[pos - 64] ^= 0x10
        else:
            dx[pos - 96] ^= 0x10
        rows_i.append(bytes(ix))
        rows_d.append(bytes(dx))
        rows_s.append(bytes(sg))
        rows_w.append(O.ed25519_verify_byron(bytes(sg), B.dlg_cert_message(h.magic, bytes(dx),
                                                                           h.cert_epoch),
                                             bytes(ix[:32])))
    rows_i.append(h.issuer_xpub)
    rows_d.append(h.delegate_xpub)
    rows_s.append(h.cert_sig)
    rows_w.append(True)
    arr = lambda xs: np.frombuffer(b"".join(xs), np.uint8).reshape(len(xs), -1)  # noqa: E731
    got = B.verify_delegation_certs(arr(rows_i), arr(rows_d), [h.cert_epoch] * len(rows_i),
                                    arr(rows_s), h.magic)
    np.testing.assert_array_equal(got, np.array(rows_w))
    assert got[-1] and not got[:-1].all()
