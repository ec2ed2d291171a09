"""Raw header CBOR in host memory -> verdicts in ONE call:
ouro_tpraos_verify_cbor (header.verify_headers_cbor) and the pipelined
ouro_integrity_verify_cbor, the entries the reference's bulk callers would
bind -- ChainDB's suffix re-validation
(ouroboros-consensus/src/Ouroboros/Consensus/Storage/ChainDB/Impl/LgrDB.hs:350-368),
ChainSync windows (.../MiniProtocol/ChainSync/Client.hs:792) and storage
integrity (.../Storage/VolatileDB/Impl/Parser.hs:66-85,
ouroboros-consensus-shelley/src/Ouroboros/Consensus/Shelley/Ledger/Integrity.hs:20-44).

Expected values: the pinned host slicer (header.pack_cbor = header.parse_header
item for item, tests/test_pack.py) feeding the oracle's header combiner
(oracle/tpraos.c), verdicts masked to 0 where the header does not slice.
Cases: the reference's golden headers, every single-byte corruption of each,
truncations; headers re-proved for mkSeed inputs under an epoch nonce and
under NeutralNonce (forged claims, a wrong slot); buffers with gaps,
shuffled and shared spans; the pipeline cut into many small chunks over
every slot count; a device error recomputed on the host path.
"""
import os

import numpy as np
import pytest

import hdr_cases as C
import oracle_ffi as O

SPKP = 100  # the golden examples' slots per KES period (Examples.hs)


def _golden_cases(kats, stride=1):
    golden = [bytes.fromhex(h["raw"]) for h in kats["headers"]]
    ea = [bytes.fromhex(h["eta_alpha"]) for h in kats["headers"]]
    la = [bytes.fromhex(h["leader_alpha"]) for h in kats["headers"]]
    raws, ra, rl = [], [], []
    for g, a, b in zip(golden, ea, la):
        variants = [g] + [g[:k] for k in (0, 1, 100, len(g) - 1)]
        for pos in range(0, len(g), stride):
            m = bytearray(g)
            m[pos] ^= 0x08
            variants.append(bytes(m))
        raws += variants
        ra += [a] * len(variants)
        rl += [b] * len(variants)
    return raws, np.frombuffer(b"".join(ra), np.uint8).reshape(-1, 32), \
        np.frombuffer(b"".join(rl), np.uint8).reshape(-1, 32)


def _expect(raws, spkp, ea=None, la=None, epoch_nonce=None):
    """host slicer + oracle, masked by the slicer's status"""
    from ouroboros_network_amd import header as H

    seeds = ea is None
    p = H.pack_cbor(raws, slots_per_kes_period=spkp, eta_alpha=ea, leader_alpha=la, seeds=seeds,
                    epoch_nonce=epoch_nonce)
    v, be, bl, en = O.tpraos_verify_batch_nonce(p.batch)
    ok = p.status == H.PACK_OK
    v = np.where(ok, v, 0).astype(np.uint8)
    return v, be, bl, en, p.status.copy()


def _check(raws, spkp, ea=None, la=None, epoch_nonce=None, triple=None):
    from ouroboros_network_amd import header as H

    want = _expect(raws, spkp, ea, la, epoch_nonce)
    got = H.verify_headers_cbor(triple or raws, spkp, epoch_nonce=epoch_nonce, eta_alpha=ea,
                                leader_alpha=la, nonce=True)
    v, be, bl, st, en = got
    np.testing.assert_array_equal(st, want[4])
    np.testing.assert_array_equal(v, want[0])
    ok = st == H.PACK_OK
    # outputs of the rows that slice (a rejected header's outputs are unspecified zeros)
    np.testing.assert_array_equal(be[ok], want[1][ok])
    np.testing.assert_array_equal(bl[ok], want[2][ok])
    np.testing.assert_array_equal(en[ok], want[3][ok])
    return v, st


@pytest.mark.gpu
def test_golden_corruptions_truncations(gpu_lib, kats):
    from ouroboros_network_amd import header as H

    raws, ea, la = _golden_cases(kats)
    v, st = _check(raws, SPKP, ea, la)
    golden_rows = [i for i, r in enumerate(raws) if r in
                   {bytes.fromhex(h["raw"]) for h in kats["headers"]}]
    assert ((v[golden_rows] & 0x3F) == 0x3F).all()  # every check and both claims
    assert (st != H.PACK_OK).any() and (v[st != H.PACK_OK] == 0).all()


def _ramp_chunks(n, per, ramp=True):
    """chunk count of kernels.hip raw_chunks / raw_chunk_target (the golden
    headers are far below the 96 MiB byte cap)"""
    count, j, i = 0, 0, 0
    while i < n:
        t = per
        if ramp:
            t = per // 4 if j == 0 else (per // 2 if j == 1 else per)
            left = n - i
            if left <= per + per // 2:
                t = min(t, max(per // 4, left // 2))
            t = max(t, 256)
        i += t
        j += 1
        count += 1
    return count


@pytest.mark.gpu
@pytest.mark.parametrize("chunk,slots,ramp", [(256, 1, 1), (256, 3, 0), (512, 8, 1),
                                              (1024, 2, 1), (1024, 2, 0)])
def test_golden_in_small_chunks(gpu_lib, kats, small_chunks, chunk, slots, ramp):
    raws, ea, la = _golden_cases(kats, stride=2)
    small_chunks(CHUNK=chunk, SLOTS=slots, RAMP=ramp)
    _check(raws, SPKP, ea, la)
    stats = np.zeros(6)
    gpu_lib.ouro_debug_cbor_stats(stats.ctypes.data)
    assert stats[3] == _ramp_chunks(len(raws), chunk, bool(ramp)) and stats[4] == slots


@pytest.mark.gpu
@pytest.mark.parametrize("nonce", [b"\x5a" * 32, None])
def test_seeded_headers(gpu_lib, kats, nonce):
    """mkSeed from each header's slot and eta0 on the device; claims forged on
    some rows, a header whose slot no longer matches its proofs."""
    from ouroboros_network_amd import header as H

    raws, slots = C.seeded_raw(kats, nonce, 40, spkp=SPKP)
    v, _ = _check(raws, SPKP, epoch_nonce=nonce)
    assert ((v & 0x3F) == 0x3F).all()
    # the wrong eta0 fails both VRFs everywhere
    other = b"\x01" * 32 if nonce is None else None
    got = H.verify_headers_cbor(raws, SPKP, epoch_nonce=other)[0]
    assert ((got & 0x0C) == 0).all() and ((got & 0x03) == 0x03).all()
    # a forged claimed output (a byte of the certs' output changed inside the
    # body: the KES signature then fails too, exactly as the oracle says)
    bad = []
    for r in raws[:6]:
        h = H.parse_header(r)
        off = r.index(h.leader_output)
        m = bytearray(r)
        m[off + 3] ^= 1
        bad.append(bytes(m))
    _check(bad, SPKP, epoch_nonce=nonce)


@pytest.mark.gpu
def test_buffer_layouts(gpu_lib, kats, small_chunks):
    """Headers anywhere in the caller's buffer: gaps, reversed order, one span
    listed twice, the last header ending at the buffer's end; results equal
    the packed-in-order call row for row."""
    from ouroboros_network_amd import header as H

    raws, ea, la = _golden_cases(kats, stride=7)
    rng = np.random.default_rng(5)
    order = rng.permutation(len(raws))
    parts, off, at = [], np.zeros(len(raws), np.uint64), 0
    for k in order:
        pad = bytes(int(rng.integers(0, 40)))
        parts.append(pad)
        at += len(pad)
        off[k] = at
        parts.append(raws[k])
        at += len(raws[k])
    buf = np.frombuffer(b"".join(parts), np.uint8)
    ln = np.array([len(r) for r in raws], np.uint32)
    small_chunks(CHUNK=256)
    v, st = _check(raws, SPKP, ea, la, triple=(buf, off, ln))
    # one span twice (rows 0 and 1 the same header)
    off2, ln2 = off.copy(), ln.copy()
    off2[1], ln2[1] = off2[0], ln2[0]
    ea2, la2 = ea.copy(), la.copy()
    ea2[1], la2[1] = ea2[0], la2[0]
    got = H.verify_headers_cbor((buf, off2, ln2), SPKP, eta_alpha=ea2, leader_alpha=la2)
    assert got[0][1] == got[0][0] == v[0] and got[3][1] == st[0]


@pytest.mark.gpu
def test_integrity_in_small_chunks(gpu_lib, kats, small_chunks):
    """ouro_integrity_verify_cbor on the same pipeline, many chunks."""
    from ouroboros_network_amd import header as H

    raws, _, _ = _golden_cases(kats, stride=3)
    want_ok, want_st = H.verify_integrity_cbor(raws, SPKP, host=True)
    for chunk, slots in ((256, 2), (4096, 6)):
        small_chunks(CHUNK=chunk, SLOTS=slots)
        ok, st = H.verify_integrity_cbor(raws, SPKP)
        np.testing.assert_array_equal(ok, want_ok)
        np.testing.assert_array_equal(st, want_st)


@pytest.mark.gpu
def test_synthetic_headers_match_the_soa_path(gpu_lib):
    """Device-synthesised raw headers (bench.synth_raw_headers) through the one
    call from pageable memory, in several chunks: every header valid, results
    equal the HBM-resident SoA path's."""
    import torch

    import bench
    from ouroboros_network_amd import header as H
    from ouroboros_network_amd import verify_headers

    n = 20000
    t, raw, rl = bench.synth_raw_headers(n, 64, torch.device("cuda", 0))
    buf = raw.cpu().numpy()
    ea = t["eta_alpha"].cpu().numpy().reshape(n, 32)
    la = t["leader_alpha"].cpu().numpy().reshape(n, 32)
    off = np.arange(n, dtype=np.uint64) * rl
    ln = np.full(n, rl, np.uint32)
    v, be, bl, st = H.verify_headers_cbor((buf, off, ln), 129600, eta_alpha=ea, leader_alpha=la)
    assert (st == 0).all() and ((v & 0x3F) == 0x3F).all()
    p = H.pack_cbor((buf, off, ln), slots_per_kes_period=129600, eta_alpha=ea, leader_alpha=la)
    rv, rbe, rbl = verify_headers(p.batch)
    np.testing.assert_array_equal(v, rv)
    np.testing.assert_array_equal(be, rbe)
    np.testing.assert_array_equal(bl, rbl)


@pytest.mark.gpu
@pytest.mark.device_error
def test_device_error_recomputes_on_the_host_path(gpu_lib, kats, small_chunks):
    """OURO_TEST_DEVICE_ERROR (test build hook): every launch reports an error;
    both raw entries return the oracle's verdicts from the host path."""
    from ouroboros_network_amd import _native
    from ouroboros_network_amd import header as H

    if not _native.test_hooks():
        pytest.skip("the library was built without test hooks")
    raws, ea, la = _golden_cases(kats, stride=11)
    with _native.knob_env(OURO_TEST_DEVICE_ERROR="1", OURO_CBOR_CHUNK="256"):
        _check(raws, SPKP, ea, la)
        nraws, _ = C.seeded_raw(kats, b"\x07" * 32, 8, spkp=SPKP)
        _check(nraws, SPKP, epoch_nonce=b"\x07" * 32)
        ok, st = H.verify_integrity_cbor(raws, SPKP)
        hok, hst = H.verify_integrity_cbor(raws, SPKP, host=True)
        np.testing.assert_array_equal(ok, hok)
        msg = gpu_lib.ouro_last_error().decode()
        assert "recomputed on the host path" in msg, msg


@pytest.mark.gpu
def test_c_callers(gpu_lib, kats, tmp_path):
    """tests/c/cbor_callers.c: 8 pthreads call ouro_tpraos_verify_cbor and
    ouro_integrity_verify_cbor -- four of them the multi-device forms with
    devices {0} and {0, 0} -- through the C ABI on the golden cases (every
    single-byte corruption and truncations), each result checked against the
    pinned host slicer + oracle."""
    import subprocess

    from ouroboros_network_amd import header as H

    exe = os.path.join(os.path.dirname(os.path.abspath(__file__)), "c", "build", "cbor_callers")
    assert os.path.exists(exe), "build tests/c (make -C tests/c)"
    raws, ea, la = _golden_cases(kats, stride=3)
    v, be, bl, _en, st = _expect(raws, SPKP, ea, la)
    ok, _ = H.verify_integrity_cbor(raws, SPKP, host=True)
    buf, off, ln = H.raw_triplet(raws)
    n = len(raws)
    path = tmp_path / "cbor_input.bin"
    with open(path, "wb") as f:
        f.write(np.array([n, buf.size, SPKP], np.uint64).tobytes())
        for a in (buf, off, ln, ea, la, st, v, be, bl, ok.astype(np.uint8)):
            f.write(np.ascontiguousarray(a).tobytes())
    r = subprocess.run([exe, str(path), "8", "3"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and r.stdout.startswith("ok"), (r.stdout, r.stderr[-2000:])
