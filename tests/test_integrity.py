"""Storage integrity over raw headers -- verifyHeaderIntegrity
(ouroboros-consensus-shelley/src/Ouroboros/Consensus/Shelley/Ledger/Integrity.hs:20-44),
the KES-only check the VolatileDB parser (Storage/VolatileDB/Impl/Parser.hs:66-85)
and ImmutableDB chunk validation (Storage/ImmutableDB/Impl/Validation.hs:358-365)
run on every stored block -- as one call from raw CBOR:
ouro_integrity_verify_cbor / _device and header.verify_integrity_cbor.

Expected verdicts come from the pinned Python slicer (header.parse_header,
tests/test_pack.py) and the oracle's Sum6KES (oracle/kes.c) with the period
computed as Integrity.hs:38-44 does (header.kes_t): the golden headers of the
reference, every single-byte corruption of them, truncations, and slots on
both sides of the opcert's KES period.  The CPU test runs the library's host
path; the GPU tests the one-call device path and the HBM-resident one.
"""
import numpy as np
import pytest

import oracle_ffi as O

SPKP = 129600  # tpraosSlotsPerKESPeriod of the golden examples' mainnet-like config


def _cases(kats, stride=1):
    raws = []
    golden = [bytes.fromhex(h["raw"]) for h in kats["headers"]]
    for g in golden:
        raws.append(g)
        for pos in range(0, len(g), stride):
            m = bytearray(g)
            m[pos] ^= 0x08
            raws.append(bytes(m))
        raws += [g[:k] for k in (0, 1, 100, len(g) - 1)]
    return raws


def _expect(raws, spkp):
    from ouroboros_network_amd import header as H

    want = []
    for r in raws:
        try:
            h = H.parse_header(r)
        except Exception:  # noqa: BLE001 -- any rejection by the pinned slicer
            want.append(False)
            continue
        t = H.kes_t(h.slot, spkp, h.ocert_kes_period)
        want.append(O.kes_verify(h.hot_vk, t, h.body, h.kes_sig))
    return np.array(want)


def test_integrity_host_path_matches_oracle(kats):
    from ouroboros_network_amd import header as H

    raws = _cases(kats, stride=3)
    for spkp in (SPKP, 1, 10**9):
        ok, status = H.verify_integrity_cbor(raws, spkp, host=True)
        np.testing.assert_array_equal(ok, _expect(raws, spkp))
        assert (ok <= (status == H.PACK_OK)).all()
    golden = [bytes.fromhex(h["raw"]) for h in kats["headers"]]
    ok, _ = H.verify_integrity_cbor(golden, SPKP, host=True)
    assert ok.all()
    # slots_per_kes_period = 1: the golden headers' t = slot - c0 is no longer 0
    ok1, _ = H.verify_integrity_cbor(golden, 1, host=True)
    assert not ok1.any()


@pytest.mark.gpu
def test_integrity_one_call_matches_oracle(gpu_lib, kats):
    from ouroboros_network_amd import header as H

    raws = _cases(kats, stride=1)
    for spkp in (SPKP, 1):
        ok, status = H.verify_integrity_cbor(raws, spkp)
        np.testing.assert_array_equal(ok, _expect(raws, spkp))
        hok, hst = H.verify_integrity_cbor(raws, spkp, host=True)
        np.testing.assert_array_equal(ok, hok)
        np.testing.assert_array_equal(status, hst)


@pytest.mark.gpu
def test_integrity_device_resident(gpu_lib, kats):
    """ouro_integrity_verify_cbor_device on HBM-resident raw headers (spans
    padded apart, one outside raw_bytes): verdicts and statuses equal the
    one-call host-buffer form."""
    import ctypes

    import torch

    from ouroboros_network_amd import _native
    from ouroboros_network_amd import header as H

    raws = _cases(kats, stride=5)
    parts, off, ln, at = [], [], [], 0
    for k, r in enumerate(raws):
        pad = bytes(k % 7)
        parts += [pad, r]
        off.append(at + len(pad))
        ln.append(len(r))
        at += len(pad) + len(r)
    buf = b"".join(parts)
    off.append(len(buf) - 3)  # a span past the end: OURO_PACK_ESPAN on the device
    ln.append(10)
    n = len(off)
    dev = torch.device("cuda", 0)
    d_raw = torch.tensor(np.frombuffer(buf, np.uint8).copy(), device=dev)
    d_off = torch.tensor(np.array(off, np.int64), device=dev)
    d_len = torch.tensor(np.array(ln, np.int32), device=dev)
    nb = int(gpu_lib.ouro_tpraos_pack_bytes(n))
    arena = torch.zeros(nb, dtype=torch.uint8, device=dev)
    status = torch.zeros(n, dtype=torch.uint8, device=dev)
    verdict = torch.full((n,), 7, dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream()
    rc = gpu_lib.ouro_integrity_verify_cbor_device(
        ctypes.c_void_p(st.cuda_stream), d_raw.data_ptr(), len(buf), d_off.data_ptr(),
        d_len.data_ptr(), n, SPKP, arena.data_ptr(), nb, status.data_ptr(), verdict.data_ptr())
    _native.check(rc, "ouro_integrity_verify_cbor_device")
    torch.cuda.synchronize()
    ok, hst = H.verify_integrity_cbor(raws, SPKP)
    np.testing.assert_array_equal(verdict.cpu().numpy()[:-1].astype(bool), ok)
    np.testing.assert_array_equal(status.cpu().numpy()[:-1], hst)
    assert status[-1].item() == H.PACK_ESPAN and verdict[-1].item() == 0
