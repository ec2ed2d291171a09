"""The one-call raw-CBOR entries at the C ABI without a device (CPU suite):
ouro_tpraos_verify_cbor and ouro_integrity_verify_cbor reject bad arguments
with OURO_EINVAL before touching a device -- a span outside raw_bytes (as
ouro_tpraos_pack_cbor does), only one of the two alpha arrays, a zero KES
period, NULL outputs -- accept n = 0, and on a host with no GPU return
OURO_ENODEV leaving the verdicts untouched (never recomputed behind the
caller's back, never "valid").  The GPU parity tests are tests/test_gpu_cbor.py.
"""
import ctypes

import numpy as np
import pytest

EINVAL, ENODEV = -3, -4


@pytest.fixture(scope="module")
def lib():
    from ouroboros_network_amd import _native

    return _native.load()


def _args(kats):
    raws = [bytes.fromhex(h["raw"]) for h in kats["headers"]]
    buf = np.frombuffer(b"".join(raws), np.uint8)
    ln = np.array([len(r) for r in raws], np.uint32)
    off = np.concatenate([[0], np.cumsum(ln)[:-1]]).astype(np.uint64)
    return buf, off, ln


def P(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def _verify(lib, buf, off, ln, n, spkp=100, eta0=None, ea=None, la=None, status=True,
            verdict=None):
    st = np.zeros(max(n, 1), np.uint8) if status else None
    v = verdict if verdict is not None else np.full(max(n, 1), 0xEE, np.uint8)
    return lib.ouro_tpraos_verify_cbor(P(buf), buf.size, P(off), P(ln), n, spkp, P(eta0), P(ea),
                                       P(la), P(st), P(v), None, None, None), v


def test_bad_arguments_are_einval(lib, kats):
    buf, off, ln = _args(kats)
    n = off.size
    a = np.zeros((n, 32), np.uint8)
    off_bad = off.copy()
    off_bad[-1] = buf.size - 3  # span past the end of raw
    assert _verify(lib, buf, off_bad, ln, n)[0] == EINVAL
    assert b"span outside raw_bytes" in lib.ouro_last_error()
    big = off.copy()
    big[2] = 2**64 - 8  # an offset that would wrap
    assert _verify(lib, buf, big, ln, n)[0] == EINVAL
    assert _verify(lib, buf, off, ln, n, ea=a)[0] == EINVAL
    assert _verify(lib, buf, off, ln, n, la=a)[0] == EINVAL
    assert _verify(lib, buf, off, ln, n, spkp=0)[0] == EINVAL
    assert _verify(lib, buf, off, ln, n, status=False)[0] == EINVAL
    st = np.zeros(n, np.uint8)
    v = np.zeros(n, np.uint8)
    assert lib.ouro_integrity_verify_cbor(P(buf), buf.size, P(off_bad), P(ln), n, 100, P(st),
                                          P(v)) == EINVAL
    assert lib.ouro_integrity_verify_cbor(P(buf), buf.size, P(off), P(ln), n, 0, P(st),
                                          P(v)) == EINVAL
    assert lib.ouro_integrity_verify_cbor(P(buf), buf.size, P(off), P(ln), n, 100, None,
                                          P(v)) == EINVAL


def test_empty_batch_is_ok(lib, kats):
    buf, off, ln = _args(kats)
    assert _verify(lib, buf, off, ln, 0)[0] == 0
    assert lib.ouro_integrity_verify_cbor(None, 0, None, None, 0, 100, None, None) == 0


def test_no_device_is_an_error_not_an_accept(lib, kats):
    import torch

    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    buf, off, ln = _args(kats)
    rc, v = _verify(lib, buf, off, ln, off.size, eta0=np.zeros(32, np.uint8))
    assert rc == ENODEV and (v == 0xEE).all()
    st = np.zeros(off.size, np.uint8)
    v = np.full(off.size, 0xEE, np.uint8)
    assert lib.ouro_integrity_verify_cbor(P(buf), buf.size, P(off), P(ln), off.size, 100, P(st),
                                          P(v)) == ENODEV
    assert (v == 0xEE).all()


def test_python_mirror_checks_its_arguments(kats):
    from ouroboros_network_amd import header as H

    raws = [bytes.fromhex(h["raw"]) for h in kats["headers"]]
    with pytest.raises(ValueError):
        H.verify_headers_cbor(raws, 100, epoch_nonce=b"\0" * 31)
    with pytest.raises(ValueError):
        H.verify_headers_cbor(raws, 100, eta_alpha=np.zeros((len(raws), 32), np.uint8))
    v, be, bl, st = H.verify_headers_cbor([], 100)
    assert v.size == 0 and st.size == 0


def test_multi_entries_without_a_device(lib, kats):
    """The multi-device raw entries check every span, the
    period, the alpha pair, the protocol magic and the device list before any
    shard starts (OURO_EINVAL), accept n = 0, and with no GPU return
    OURO_ENODEV with the verdicts untouched."""
    import torch

    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    buf, off, ln = _args(kats)
    n = off.size
    st = np.zeros(n, np.uint8)
    v = np.full(n, 0xEE, np.uint8)
    a = np.zeros((n, 32), np.uint8)
    devs = np.array([0, 0], np.int32)
    I = ctypes.c_int

    def hdr(d, nd, o=off, spkp=100, ea=None, la=None, count=n):
        return lib.ouro_tpraos_verify_cbor_multi(P(d), I(nd), P(buf), buf.size, P(o), P(ln), count,
                                                 spkp, None, P(ea), P(la), P(st), P(v), None,
                                                 None, None)

    def kes(d, nd, o=off, spkp=100):
        return lib.ouro_integrity_verify_cbor_multi(P(d), I(nd), P(buf), buf.size, P(o), P(ln),
                                                    n, spkp, P(st), P(v))

    def byron(d, nd, magic=-1, o=off):
        return lib.ouro_byron_verify_cbor_multi(P(d), I(nd), P(buf), buf.size, P(o), P(ln), n,
                                                magic, P(st), P(v))

    bad = off.copy()
    bad[-1] = buf.size - 3
    for call in (lambda: hdr(devs, 2, o=bad), lambda: kes(devs, 2, o=bad),
                 lambda: byron(devs, 2, o=bad), lambda: hdr(devs, 2, spkp=0),
                 lambda: kes(devs, 2, spkp=0), lambda: hdr(devs, 2, ea=a),
                 lambda: byron(devs, 2, magic=2**32), lambda: byron(devs, 2, magic=-2),
                 lambda: hdr(devs, 0), lambda: kes(devs, -1), lambda: byron(devs, 65)):
        assert call() == EINVAL, lib.ouro_last_error()
    assert hdr(devs, 2, count=0) == 0
    for call in (lambda: hdr(devs, 2), lambda: kes(None, 0), lambda: byron(devs, 1)):
        assert call() == ENODEV
    assert (v == 0xEE).all()
