"""The raw-CBOR entries over several GPUs of one process:
ouro_tpraos_verify_cbor_multi, ouro_integrity_verify_cbor_multi and
ouro_byron_verify_cbor_multi -- what an 8-GPU node's bulk callers hold
(ChainDB's suffix re-validation, ouroboros-consensus/src/Ouroboros/Consensus/
Storage/ChainDB/Impl/LgrDB.hs:350-368; storage integrity,
.../Storage/ImmutableDB/Impl/Validation.hs:358-365,
.../Storage/VolatileDB/Impl/Parser.hs:66-85; Byron PBFT,
ouroboros-consensus/src/Ouroboros/Consensus/Protocol/PBFT.hs:332-338).

On the one-GPU box the device lists are [0], [0, 0] (two shards on two
pooled workers of the one GPU), [0, 0, 0] and "all"; the expected values are
the pinned host slicers + the oracle (tests/test_gpu_cbor.py's _expect), the
golden headers with every single-byte corruption and truncations.  Two
threads calling at once show the calls are no longer serialised.
"""
import threading

import numpy as np
import pytest

import oracle_ffi as O
from test_gpu_cbor import SPKP, _expect, _golden_cases

pytestmark = pytest.mark.gpu

DEVICE_LISTS = [[0], [0, 0], [0, 0, 0], "all"]


@pytest.mark.parametrize("devices", DEVICE_LISTS, ids=["d0", "d00", "d000", "all"])
def test_tpraos_cbor_multi_golden(gpu_lib, kats, small_chunks, devices):
    from ouroboros_network_amd import header as H

    small_chunks(CHUNK=256)  # several chunks per shard
    raws, ea, la = _golden_cases(kats, stride=2)
    want = _expect(raws, SPKP, ea, la)
    v, be, bl, st, en = H.verify_headers_cbor(raws, SPKP, eta_alpha=ea, leader_alpha=la,
                                              nonce=True, devices=devices)
    np.testing.assert_array_equal(st, want[4])
    np.testing.assert_array_equal(v, want[0])
    ok = st == H.PACK_OK
    np.testing.assert_array_equal(be[ok], want[1][ok])
    np.testing.assert_array_equal(bl[ok], want[2][ok])
    np.testing.assert_array_equal(en[ok], want[3][ok])
    assert (v & 0x3F == 0x3F).sum() >= len(kats["headers"])
    # the single-device call agrees row for row
    one = H.verify_headers_cbor(raws, SPKP, eta_alpha=ea, leader_alpha=la, nonce=True)
    for a, b in zip(one, (v, be, bl, st, en)):
        np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("devices", DEVICE_LISTS, ids=["d0", "d00", "d000", "all"])
def test_tpraos_cbor_multi_seeded(gpu_lib, kats, devices):
    """mkSeed inputs on the device under an epoch nonce, across shards."""
    import hdr_cases as C
    from ouroboros_network_amd import header as H

    eta0 = b"\x33" * 32
    raws, _ = C.seeded_raw(kats, eta0, 24, spkp=SPKP)
    want = _expect(raws, SPKP, epoch_nonce=eta0)
    v, be, bl, st, en = H.verify_headers_cbor(raws, SPKP, epoch_nonce=eta0, nonce=True,
                                              devices=devices)
    np.testing.assert_array_equal(st, want[4])
    np.testing.assert_array_equal(v, want[0])
    np.testing.assert_array_equal(en, want[3])


@pytest.mark.parametrize("devices", DEVICE_LISTS, ids=["d0", "d00", "d000", "all"])
def test_integrity_cbor_multi_golden(gpu_lib, kats, small_chunks, devices):
    from ouroboros_network_amd import header as H

    small_chunks(CHUNK=256)
    raws, _, _ = _golden_cases(kats, stride=2)
    want_ok, want_st = H.verify_integrity_cbor(raws, SPKP, host=True)
    ok, st = H.verify_integrity_cbor(raws, SPKP, devices=devices)
    np.testing.assert_array_equal(st, want_st)
    np.testing.assert_array_equal(ok, want_ok)
    assert 0 < ok.sum() < len(raws)


def _byron_cases(kats):
    from ouroboros_network_amd import byron as B

    wires = [bytes.fromhex(w["raw"]) for w in kats["byron_wire"]]
    regular = [w for w, d in zip(wires, kats["byron_wire"]) if d["kind"] == "regular"]
    raws = list(wires)
    for g in (regular[0], regular[2]):  # n2n v1, hfc
        for pos in range(len(g)):
            m = bytearray(g)
            m[pos] ^= 0x04
            raws.append(bytes(m))
        raws += [g[:k] for k in (0, 1, 50, len(g) - 1)]
    want, want_st = [], []
    for r in raws:
        st, h = B.byron_status(r)
        want_st.append(st)
        if st == B.PACK_EBB:
            want.append(True)
        elif st != B.PACK_OK:
            want.append(False)
        else:
            want.append(O.ed25519_verify_byron(h.sig, h.message(B.HEADER_MAGIC),
                                               h.delegate_xpub[:32]))
    return raws, np.array(want), np.array(want_st, np.uint8)


@pytest.mark.parametrize("devices", [None] + DEVICE_LISTS, ids=["one", "d0", "d00", "d000", "all"])
def test_byron_cbor_pipeline_and_multi(gpu_lib, kats, small_chunks, devices):
    """ouro_byron_verify_cbor on the chunked engine (device Byron slicer +
    ByronDSIGN kernel) and its multi-device form: every golden wire form,
    every single-byte corruption and truncations of the v1 and HFC regular
    headers, against the Python slicer + the oracle's donna-style verify."""
    from ouroboros_network_amd import byron as B

    small_chunks(CHUNK=256, SLOTS=3)
    raws, want, want_st = _byron_cases(kats)
    got, st = B.verify_byron_cbor(raws, B.HEADER_MAGIC, devices=devices)
    np.testing.assert_array_equal(st, want_st)
    np.testing.assert_array_equal(got, want)
    assert 0 < got.sum() < len(raws)
    # the configured magic: the golden one verifies, another does not
    regular = [r for r, s in zip(raws, want_st) if s == B.PACK_OK][:3]
    ok, _ = B.verify_byron_cbor(regular, kats["byron"]["magic"], devices=devices)
    bad, _ = B.verify_byron_cbor(regular, 764824073, devices=devices)
    assert not bad.any()
    want_cfg = [O.ed25519_verify_byron(h.sig, h.message(kats["byron"]["magic"]),
                                       h.delegate_xpub[:32])
                for h in (B.byron_status(r)[1] for r in regular)]
    np.testing.assert_array_equal(ok, np.array(want_cfg))


def test_byron_cbor_many_chunks_large(gpu_lib, kats, small_chunks):
    """200,000 Byron headers (the golden wire forms repeated, one in 50
    corrupted) through the pipeline in 64 K chunks: the pattern's verdicts
    repeat exactly."""
    from ouroboros_network_amd import byron as B

    raws, want, want_st = _byron_cases(kats)
    pat = [raws[i] for i in range(len(raws))]
    n = 200_000
    idx = np.arange(n) % len(pat)
    ln = np.array([len(pat[i]) for i in idx], np.uint32)
    off = np.zeros(n, np.uint64)
    off[1:] = np.cumsum(ln[:-1], dtype=np.uint64)
    buf = np.frombuffer(b"".join(pat[i] for i in idx), np.uint8)
    got, st = B.verify_byron_cbor((buf, off, ln), B.HEADER_MAGIC)
    np.testing.assert_array_equal(st, want_st[idx])
    np.testing.assert_array_equal(got, want[idx])
    got2, st2 = B.verify_byron_cbor((buf, off, ln), B.HEADER_MAGIC, devices=[0, 0])
    np.testing.assert_array_equal(got2, got)
    np.testing.assert_array_equal(st2, st)


def test_multi_calls_run_concurrently(gpu_lib, kats):
    """Two threads (a ChainSync-like caller and a ChainDB-like one) each make
    multi-device calls at the same time, each borrowing pooled workers of
    its own (no process-wide lock since round 6): both get the oracle's
    verdicts on every call."""
    import ctypes

    from ouroboros_network_amd import header as H

    raws, ea, la = _golden_cases(kats, stride=5)
    want = _expect(raws, SPKP, ea, la)
    want_ok, _ = H.verify_integrity_cbor(raws, SPKP, host=True)
    errors = []

    def hdr_caller():
        try:
            for _ in range(6):
                v = H.verify_headers_cbor(raws, SPKP, eta_alpha=ea, leader_alpha=la,
                                          devices=[0, 0])[0]
                assert (v == want[0]).all()
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    def kes_caller():
        try:
            for _ in range(6):
                ok, _ = H.verify_integrity_cbor(raws, SPKP, devices=[0, 0])
                assert (ok == want_ok).all()
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    ts = [threading.Thread(target=hdr_caller), threading.Thread(target=kes_caller)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=300)
    assert not errors, errors
    devs = np.zeros(64, np.int32)
    k = gpu_lib.ouro_debug_multi_workers(devs.ctypes.data_as(ctypes.c_void_p), None, None, 64)
    assert k >= 2 and (devs[:min(k, 64)] == 0).all()  # pooled workers, all on device 0


def test_multi_rejects_bad_arguments(gpu_lib, kats):
    from ouroboros_network_amd import _native
    from ouroboros_network_amd import header as H

    raws = [bytes.fromhex(kats["headers"][0]["raw"])] * 3
    buf, off, ln = H.raw_triplet(raws)
    off = off.copy()
    off[2] = buf.size  # a span past the buffer: rejected before any shard starts
    with pytest.raises(ValueError):
        H.verify_integrity_cbor((buf, off, ln), SPKP, devices=[0, 0])
    with pytest.raises(_native.NativeUnavailable):
        H.verify_integrity_cbor(raws, SPKP, devices=[0, 99])


@pytest.mark.device_error
def test_multi_cbor_device_error_recomputes_on_the_host_path(gpu_lib, kats, small_chunks):
    """OURO_TEST_DEVICE_ERROR (test build): every launch of every shard fails;
    each shard is recomputed on the host path and the three multi entries
    still return the oracle's verdicts (never an accept the device did not
    make)."""
    from ouroboros_network_amd import _native
    from ouroboros_network_amd import byron as B
    from ouroboros_network_amd import header as H

    raws, ea, la = _golden_cases(kats, stride=13)
    want = _expect(raws, SPKP, ea, la)
    want_ok, want_st = H.verify_integrity_cbor(raws, SPKP, host=True)
    braws, bwant, bwant_st = _byron_cases(kats)
    with _native.knob_env(OURO_TEST_DEVICE_ERROR="1", OURO_CBOR_CHUNK="256"):
        v, be, bl, st = H.verify_headers_cbor(raws, SPKP, eta_alpha=ea, leader_alpha=la,
                                              devices=[0, 0])
        np.testing.assert_array_equal(st, want[4])
        np.testing.assert_array_equal(v, want[0])
        ok, ist = H.verify_integrity_cbor(raws, SPKP, devices=[0, 0])
        np.testing.assert_array_equal(ok, want_ok)
        np.testing.assert_array_equal(ist, want_st)
        got, bst = B.verify_byron_cbor(braws, B.HEADER_MAGIC, devices=[0, 0])
        np.testing.assert_array_equal(got, bwant)
        np.testing.assert_array_equal(bst, bwant_st)
        got1, _ = B.verify_byron_cbor(braws, B.HEADER_MAGIC)
        np.testing.assert_array_equal(got1, bwant)
        msg = gpu_lib.ouro_last_error().decode()
        assert "recomputed on the host path" in msg, msg
