"""GPU parity: the gfx950 kernels (through the C ABI) against the CPU oracle and
the reference's golden vectors.  Bit-exact: verdicts and 64-byte VRF outputs.

Inputs: seeded synthetic batches (oracle signer, SURVEY.md §8(d) seeds), with
1/8 of items corrupted applyCorruption-style (one byte incremented at a seeded
offset; ouroboros-consensus-test/src/Test/Util/Corruption.hs), plus the fixed
edge-case sets in edge_cases.py.
"""
import os

import numpy as np
import pytest

import hdr_cases as HC
import oracle_ffi as O
from edge_cases import L as edge_L
from edge_cases import ed25519_edge_cases, vrf_edge_cases

pytestmark = pytest.mark.gpu


def corrupt_rows(rng, arrays, frac=8):
    """Increment one byte of 1/frac of the rows of one of `arrays` (in place)."""
    n = arrays[0].shape[0]
    idx = np.nonzero(rng.integers(0, frac, n) == 0)[0]
    for i in idx:
        a = arrays[rng.integers(0, len(arrays))]
        j = rng.integers(0, a.shape[1])
        a[i, j] = (int(a[i, j]) + 1) & 0xFF
    return idx


@pytest.fixture(params=["wave_per_item", "lane_per_item"])
def small_path(request, monkeypatch):
    """Batches up to OURO_WIDE_SMALL_MAX items run one item per wave
    (wide_cores.h, the single-item latency path); 0 forces the one-lane
    throughput kernels.  Both must agree with the oracle."""
    if request.param == "lane_per_item":
        monkeypatch.setenv("OURO_WIDE_SMALL_MAX", "0")
    return request.param


def test_ed25519_batch_matches_oracle(small_path, gpu_lib):
    from ouroboros_network_amd import Ed25519DSIGN

    rng = np.random.default_rng(7)
    pk, sig, msg = O.synth_ed25519(2048, first=1000)
    bad = corrupt_rows(rng, [pk, sig, msg])
    got = Ed25519DSIGN.verify_batch(pk, msg, sig)
    buf, off, ln = msg.reshape(-1), np.arange(2048, dtype=np.uint64) * 32, np.full(2048, 32, np.uint32)
    want = O.ed25519_verify_batch(pk, sig, buf, off, ln)
    assert want.sum() > 2048 - 2 * len(bad)
    np.testing.assert_array_equal(got, want)


def test_ed25519_edge_cases(small_path, gpu_lib):
    from ouroboros_network_amd import Ed25519DSIGN

    cases = ed25519_edge_cases()
    got = Ed25519DSIGN.verify_batch([c[0] for c in cases], [c[2] for c in cases],
                                    [c[1] for c in cases])
    want = np.array([O.ed25519_verify(c[1], c[2], c[0]) for c in cases])
    np.testing.assert_array_equal(got, want)


def test_sodium_shim_matches_libsodium_rules(gpu_lib):
    """lib/libouro_sodium_shim.so's crypto_sign_ed25519_verify_detached (the
    opt-in link alias of ouro_ed25519_verify) on the edge-case set: the
    oracle's (= libsodium 1.0.18's) verdict for every case."""
    import ctypes
    import os

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    shim = ctypes.CDLL(os.path.join(root, "ouroboros-network_amd", "lib",
                                    "libouro_sodium_shim.so"))
    fn = shim.crypto_sign_ed25519_verify_detached
    fn.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_ulonglong, ctypes.c_char_p]
    cases = ed25519_edge_cases()
    for pk, sig, msg in cases[:24]:
        want = 0 if O.ed25519_verify(sig, msg, pk) else -1
        assert fn(sig, msg, len(msg), pk) == want


def test_ed25519_variable_messages(small_path, gpu_lib):
    from ouroboros_network_amd import Ed25519DSIGN

    rng = np.random.default_rng(3)
    msgs, pks, sigs = [], [], []
    for i in range(300):
        seed = rng.bytes(32)
        pk, sk = O.ed25519_keypair(seed)
        m = rng.bytes(int(rng.integers(0, 700)))
        s = O.ed25519_sign(sk, m)
        if i % 5 == 0:
            m = m + b"x"
        msgs.append(m)
        pks.append(pk)
        sigs.append(s)
    got = Ed25519DSIGN.verify_batch(pks, msgs, sigs)
    want = np.array([O.ed25519_verify(s, m, k) for k, m, s in zip(pks, msgs, sigs)])
    np.testing.assert_array_equal(got, want)


def test_vrf_batch_matches_oracle(small_path, gpu_lib):
    from ouroboros_network_amd import PraosVRF

    rng = np.random.default_rng(11)
    pk, proof, alpha = O.synth_vrf(512, first=77)
    corrupt_rows(rng, [pk, proof, alpha])
    ok, beta = PraosVRF.verify_batch(pk, alpha, proof)
    wok, wbeta = O.vrf_verify_batch(pk, proof, alpha)
    np.testing.assert_array_equal(ok, wok)
    np.testing.assert_array_equal(beta, wbeta)


def test_vrf_draft03_vectors(small_path, gpu_lib, kats):
    from ouroboros_network_amd import PraosVRF

    vs = kats["vrf_draft03"]
    ok, beta = PraosVRF.verify_batch([bytes.fromhex(v["pk"]) for v in vs],
                                     [bytes.fromhex(v["alpha"]) for v in vs],
                                     [bytes.fromhex(v["pi"]) for v in vs])
    assert ok.all()
    for b, v in zip(beta, vs):
        assert bytes(b).hex() == v["beta"]
    for v in vs:
        assert PraosVRF.output_from_proof(bytes.fromhex(v["pi"])).hex() == v["beta"]


@pytest.mark.parametrize("s_mode", ["reduce", "strict"])
def test_vrf_edge_cases(small_path, gpu_lib, s_mode):
    """Both readings of the proof's s: reduced mod L (the
    default) and strict (s >= L rejected, OURO_VRF_STRICT_S); the s + L cases
    split them."""
    from ouroboros_network_amd import PraosVRF

    cases = vrf_edge_cases()
    ok, beta = PraosVRF.verify_batch([c[0] for c in cases], [c[2] for c in cases],
                                     [c[1] for c in cases], s_mode=s_mode)
    split = 0
    for (pk, pi, a), o, b in zip(cases, ok, beta):
        w = O.vrf_verify_mode(pk, pi, a, strict_s=s_mode == "strict")
        assert o == (w is not None)
        assert bytes(b) == (w if w is not None else bytes(64))
        split += (O.vrf_verify_mode(pk, pi, a, False) is not None) != \
            (O.vrf_verify_mode(pk, pi, a, True) is not None)
    assert split >= 4  # the s + L rows of the four valid proofs
    # the single-item form agrees
    pk, pi, a = next(c for c in cases if int.from_bytes(c[1][48:], "little") >= HC.L)
    got = PraosVRF.verify(pk, a, pi, s_mode=s_mode)
    assert got == O.vrf_verify_mode(pk, pi, a, strict_s=s_mode == "strict")


def test_kes_batch_matches_oracle(gpu_lib):
    from ouroboros_network_amd import Sum6KES

    rng = np.random.default_rng(5)
    n = 256
    seeds = [rng.bytes(32) for _ in range(4)]
    vks = [O.kes_keygen(s) for s in seeds]
    rows_vk, ts, msgs, sigs = [], [], [], []
    for i in range(n):
        k = i % 4
        t = int(rng.integers(0, 64))
        m = rng.bytes(int(rng.integers(100, 700)))
        sig = O.kes_sign(seeds[k], t, m)
        if i % 7 == 3:
            t = (t + 1) % 64  # wrong period
        rows_vk.append(vks[k])
        ts.append(t)
        msgs.append(m)
        sigs.append(sig)
    sig_a = np.frombuffer(b"".join(sigs), np.uint8).reshape(n, 448).copy()
    corrupt_rows(rng, [sig_a], frac=9)
    got = Sum6KES.verify_batch(rows_vk, ts, msgs, sig_a)
    want = np.array([O.kes_verify(v, t, m, bytes(s)) for v, t, m, s in zip(rows_vk, ts, msgs, sig_a)])
    assert want.sum() > n // 2
    np.testing.assert_array_equal(got, want)


def test_golden_headers(gpu_lib, kats):
    from ouroboros_network_amd import header as H
    from ouroboros_network_amd import verify_headers

    hs = kats["headers"]
    parsed = [H.parse_header(bytes.fromhex(h["raw"])) for h in hs]
    batch = H.pack(parsed, [bytes.fromhex(h["eta_alpha"]) for h in hs],
                   [bytes.fromhex(h["leader_alpha"]) for h in hs], slots_per_kes_period=100)
    verdict, be, bl = verify_headers(batch)
    for h, v, e, l in zip(hs, verdict, be, bl):
        assert int(v) & 0x0F == h["expect_verdict"], h["name"]
        assert int(v) & 0x30 == 0x30, h["name"]  # claimed outputs = computed
        assert bytes(e).hex() == h["expect_beta_eta"]
        assert bytes(l).hex() == h["expect_beta_leader"]


def test_golden_headers_single_byte_corruption(gpu_lib, kats):
    """prop_detectCorruption_Header-style: every byte of one golden header's
    crypto-relevant payload incremented, verdict bits equal to the oracle's."""
    from ouroboros_network_amd import header as H
    from ouroboros_network_amd import verify_headers

    h0 = kats["headers"][0]
    raw = bytes.fromhex(h0["raw"])
    base = H.parse_header(raw)
    variants = []
    for off in range(base.body_span[0], len(raw)):
        r = bytearray(raw)
        r[off] = (r[off] + 1) & 0xFF
        try:
            variants.append(H.parse_header(bytes(r)))
        except Exception:
            continue  # no longer decodes: the reference rejects before crypto
    ea = [bytes.fromhex(h0["eta_alpha"])] * len(variants)
    la = [bytes.fromhex(h0["leader_alpha"])] * len(variants)
    batch = H.pack(variants, ea, la, slots_per_kes_period=100)
    verdict, be, bl = verify_headers(batch)
    wv, wbe, wbl = O.tpraos_verify_batch(batch)
    np.testing.assert_array_equal(verdict, wv)
    np.testing.assert_array_equal(be, wbe)
    np.testing.assert_array_equal(bl, wbl)
    assert (verdict & 0x0F != 15).sum() > len(variants) // 2


def test_golden_tx_witnesses(gpu_lib, kats):
    from ouroboros_network_amd import Ed25519DSIGN

    ws = kats["tx_witnesses"]
    got = Ed25519DSIGN.verify_batch([bytes.fromhex(w["pk"]) for w in ws],
                                    [bytes.fromhex(w["msg"]) for w in ws],
                                    [bytes.fromhex(w["sig"]) for w in ws])
    assert got.all()


@pytest.fixture(params=["gpu", "host"])
def single_route(request):
    """Single items on both routes (VERDICT r04 hygiene): the host path (the
    default since round 4) and the GPU (OURO_SINGLE_ITEM=gpu), so the -m gpu
    set exercises the device's single-item route too."""
    from ouroboros_network_amd import _native

    with _native.knob_env(OURO_SINGLE_ITEM=request.param):
        yield request.param


def test_single_item_abi(gpu_lib, kats, single_route):
    from ouroboros_network_amd import Ed25519DSIGN, PraosVRF, Sum6KES
    from ouroboros_network_amd import header as H

    h0 = kats["headers"][0]
    hd = H.parse_header(bytes.fromhex(h0["raw"]))
    msg = hd.hot_vk + hd.ocert_counter.to_bytes(8, "big") + hd.ocert_kes_period.to_bytes(8, "big")
    assert Ed25519DSIGN.verify_dsign((), hd.issuer_vk, msg, hd.ocert_sigma) is None
    assert Ed25519DSIGN.verify_dsign((), hd.issuer_vk, msg + b"!", hd.ocert_sigma) is not None
    assert Sum6KES.verify_kes((), hd.hot_vk, 0, hd.body, hd.kes_sig) is None
    assert Sum6KES.verify_kes((), hd.hot_vk, 1, hd.body, hd.kes_sig) is not None
    cert = (hd.eta_output, hd.eta_proof)
    assert PraosVRF.verify_vrf((), hd.vrf_vk, bytes.fromhex(h0["eta_alpha"]), cert)
    assert PraosVRF.verify_vrf((), hd.vrf_vk, bytes.fromhex(h0["eta_alpha"]), cert, mode="strict")
    assert not PraosVRF.verify_vrf((), hd.vrf_vk, bytes.fromhex(h0["leader_alpha"]), cert)


def test_empty_batches(gpu_lib):
    from ouroboros_network_amd import Ed25519DSIGN, PraosVRF

    assert Ed25519DSIGN.verify_batch(np.zeros((0, 32), np.uint8), [], np.zeros((0, 64), np.uint8)).size == 0
    ok, beta = PraosVRF.verify_batch(np.zeros((0, 32), np.uint8), [], np.zeros((0, 80), np.uint8))
    assert ok.size == 0 and beta.shape == (0, 64)


def _golden_variants(kats):
    """Golden headers + every decodable single-byte corruption of the first."""
    return HC.golden_variants(kats, stride=1)


LAT_FORMS = {
    "wide_fused": {},  # default: every core on one wave, the last core finishes
    "wide_finish_launch": {"OURO_LAT_FUSE": "0"},
    "lane_quads": {"OURO_LAT_WIDE": "0", "OURO_LAT_QUAD": "1"},
    "one_lane": {"OURO_LAT_WIDE": "0", "OURO_LAT_QUAD": "0"},
}


@pytest.mark.parametrize("form", list(LAT_FORMS))
def test_lowlat_equals_throughput_and_oracle(gpu_lib, kats, monkeypatch, form):
    """Latency mode (eight cores per header: each on one wave with wave-wide
    field arithmetic, its last core finishing the header -- or with a finish
    launch -- or each on a DPP lane quad that splits every group operation's
    products, or on one lane) gives the same verdict bits and outputs as the
    throughput kernel and the oracle."""
    from ouroboros_network_amd.tpraos import verify_headers, verify_headers_lowlat

    for k, v in LAT_FORMS[form].items():
        monkeypatch.setenv(k, v)

    batch = _golden_variants(kats)
    wv, wbe, wbl = O.tpraos_verify_batch(batch)
    for fn in (verify_headers, verify_headers_lowlat):
        v, be, bl = fn(batch)
        np.testing.assert_array_equal(v, wv)
        np.testing.assert_array_equal(be, wbe)
        np.testing.assert_array_equal(bl, wbl)
    for lo, hi in [(0, 1), (3, 67), (10, 10)]:
        v, be, bl = verify_headers_lowlat(batch.slice(lo, hi))
        np.testing.assert_array_equal(v, wv[lo:hi])
        np.testing.assert_array_equal(bl, wbl[lo:hi])


@pytest.mark.parametrize("form", ["wide_fused", "wide_finish_launch"])
def test_lowlat_kes_body_lengths(gpu_lib, kats, monkeypatch, form):
    """KES leaf messages around every SHA-512 block boundary, up to past the
    latency mode's wave-hash capacity (8 blocks; longer bodies hash on the
    lane): latency and throughput verdicts equal the oracle's, and every
    re-signed row verifies while its one-byte-changed twin fails KES only."""
    from ouroboros_network_amd.tpraos import verify_headers, verify_headers_lowlat

    for k, v in LAT_FORMS[form].items():
        monkeypatch.setenv(k, v)
    batch = HC.kes_body_lengths(kats)
    wv, wbe, wbl = O.tpraos_verify_batch(batch)
    assert (wv[0::2] == 0x3F).all() and (wv[1::2] == 0x3D).all()
    for fn in (verify_headers, verify_headers_lowlat):
        v, be, bl = fn(batch)
        np.testing.assert_array_equal(v, wv)
        np.testing.assert_array_equal(be, wbe)
        np.testing.assert_array_equal(bl, wbl)


def test_pipelined_host_batches(gpu_lib, kats, monkeypatch):
    """Host-buffer header batches larger than one chunk go through the
    two-stream pipeline (kernels.hip hdr_batch_pipelined): same verdicts and
    outputs as one-piece staging and the oracle, for ragged chunk sizes, rows
    in shuffled order (bodies not monotonic in the buffer, with gaps) and an
    empty body in the middle of a chunk."""
    from ouroboros_network_amd.tpraos import HeaderBatch, verify_headers

    base = _golden_variants(kats)
    n = len(base)
    rng = np.random.default_rng(11)
    order = rng.permutation(n)
    # re-lay the bodies: reversed row order, 3-byte gaps between them
    blens = base.body_len.astype(np.int64)
    new_off = np.zeros(n, dtype=np.uint64)
    chunks, pos = [], 0
    for i in reversed(range(n)):
        o = int(base.body_off[i])
        chunks.append(bytes(3) + base.body[o:o + int(blens[i])].tobytes())
        new_off[i] = pos + 3
        pos += 3 + int(blens[i])
    body = np.frombuffer(b"".join(chunks), dtype=np.uint8)
    kw = {k: getattr(base, k) for k in HeaderBatch.__dataclass_fields__ if k != "body"}
    kw["body_off"] = new_off
    batch = HeaderBatch(body=body, **kw).rows(order)
    batch.body_len[5] = 0  # an empty body: its KES leaf check fails, nothing else
    wv, wbe, wbl = O.tpraos_verify_batch(batch)
    assert wv[5] & 0x02 == 0
    for chunk in ("0", "1", "7", "64", str(n - 1)):
        monkeypatch.setenv("OURO_HOST_CHUNK", chunk)
        v, be, bl = verify_headers(batch)
        np.testing.assert_array_equal(v, wv)
        np.testing.assert_array_equal(be, wbe)
        np.testing.assert_array_equal(bl, wbl)


def test_multi_device_shards(gpu_lib, kats, monkeypatch):
    """ouro_tpraos_verify_batch_multi: contiguous shards on persistent worker
    threads (here several pipelines sharing the one GPU of the box, and every
    visible device) give the single-call results and the oracle's, for
    shard counts that do not divide the batch and with small pipeline chunks."""
    from ouroboros_network_amd import _native
    from ouroboros_network_amd.tpraos import verify_headers, verify_headers_multi

    batch = _golden_variants(kats)
    wv, wbe, wbl = O.tpraos_verify_batch(batch)
    assert _native.load().ouro_device_count() >= 1
    monkeypatch.setenv("OURO_HOST_CHUNK", "50")
    for devices in ([0], [0, 0], [0, 0, 0], None, [0] * 7):
        for _ in range(2):  # the workers persist between calls
            v, be, bl = verify_headers_multi(batch, devices)
            np.testing.assert_array_equal(v, wv)
            np.testing.assert_array_equal(be, wbe)
            np.testing.assert_array_equal(bl, wbl)
    v, _, _ = verify_headers_multi(batch.slice(0, 2), [0, 0, 0])  # fewer headers than shards
    np.testing.assert_array_equal(v, wv[:2])
    with pytest.raises(ValueError):
        verify_headers_multi(batch, [])
    with pytest.raises(Exception):
        verify_headers_multi(batch, [0, 99])  # no such device: an error, never a verdict
    np.testing.assert_array_equal(verify_headers(batch)[0], wv)


def test_header_plan_replays(gpu_lib, kats):
    """The captured-graph plan over 64-header windows (BASELINE configs[4]):
    every window and a ragged tail match the oracle; replays are independent
    (a window after a different one gives the same answer); oversize batches
    are rejected, never silently truncated."""
    from ouroboros_network_amd.tpraos import HeaderPlan

    batch = _golden_variants(kats)
    n = len(batch)
    assert n > 128
    wv, wbe, wbl = O.tpraos_verify_batch(batch)
    plan = HeaderPlan(max_headers=64, max_body_bytes=int(batch.body.size))
    try:
        for lo in list(range(0, n, 64)) + [0]:
            hi = min(n, lo + 64)
            v, be, bl = plan.run(batch.slice(lo, hi))
            np.testing.assert_array_equal(v, wv[lo:hi])
            np.testing.assert_array_equal(be, wbe[lo:hi])
            np.testing.assert_array_equal(bl, wbl[lo:hi])
        v, _, _ = plan.run(batch.slice(5, 6))
        assert int(v[0]) == int(wv[5])
        assert plan.run(batch.slice(0, 0))[0].size == 0
        with pytest.raises(ValueError):
            plan.run(batch.slice(0, 65))
    finally:
        plan.close()


def test_plan_submit_wait_windows_in_flight(gpu_lib, kats):
    """Asynchronous plans (ouro_tpraos_plan_submit / _wait): four 64-header
    windows in flight on four plans at once, inputs overwritten right after
    submit, results collected in reverse order -- each equals the oracle.
    Misuse (second submit before wait, wait with nothing in flight) is an
    error, never a stale or silent result."""
    from ouroboros_network_amd.tpraos import HeaderPlan

    batch = _golden_variants(kats)
    n = len(batch)
    wv, wbe, wbl = O.tpraos_verify_batch(batch)
    plans = [HeaderPlan(max_headers=64, max_body_bytes=int(batch.body.size)) for _ in range(4)]
    try:
        for rnd in range(2):
            lows = [(rnd * 256 + 64 * k) % (n - 64) for k in range(4)]
            for plan, lo in zip(plans, lows):
                w = batch.slice(lo, lo + 64)
                w = type(w)(**{k: None if getattr(w, k) is None else getattr(w, k).copy()
                               for k in w.__dataclass_fields__})
                plan.submit(w)
                w.ocert_sigma[:] = 0  # the plan staged its own copy
                w.body[:] = 0
            for plan, lo in reversed(list(zip(plans, lows))):
                v, be, bl = plan.wait()
                np.testing.assert_array_equal(v, wv[lo:lo + 64])
                np.testing.assert_array_equal(be, wbe[lo:lo + 64])
                np.testing.assert_array_equal(bl, wbl[lo:lo + 64])
        plans[0].submit(batch.slice(0, 3))
        with pytest.raises(ValueError):
            plans[0].submit(batch.slice(3, 6))
        v, _, _ = plans[0].wait()
        np.testing.assert_array_equal(v, wv[0:3])
        with pytest.raises(ValueError):
            plans[0].wait()
    finally:
        for plan in plans:
            plan.close()


# ---- ByronDSIGN ------------------------------

def test_byron_golden_header(small_path, gpu_lib, kats):
    from ouroboros_network_amd import ByronDSIGN, parse_byron_header, verify_byron_headers

    b = kats["byron"]
    h = parse_byron_header(bytes.fromhex(b["raw"]))
    ctx = (h.magic, h.issuer_xpub)
    assert ByronDSIGN.verify_dsign(ctx, h.delegate_xpub, h.to_sign, h.sig) is None
    assert ByronDSIGN.verify_dsign(ctx, h.delegate_xpub, h.to_sign[:-1] + b"\x00", h.sig) \
        == "Verification failed"
    assert ByronDSIGN.verify_dsign((h.magic + 1, h.issuer_xpub), h.delegate_xpub, h.to_sign,
                                   h.sig) == "Verification failed"
    assert verify_byron_headers([h, h], protocol_magic=b["magic"]).tolist() == [True, True]
    # a header signed for another network's magic fails under the configured one
    assert verify_byron_headers([h], protocol_magic=764824073).tolist() == [False]


def test_byron_batch_matches_oracle(small_path, gpu_lib):
    """Synthetic signatures with 1/8 corrupted, the Ed25519 edge-case set and
    the Byron-specific corners (S + L < 2^253 accepted, top bits of S set):
    verdicts bit-exact with the oracle's donna-style rule."""
    from ouroboros_network_amd import ByronDSIGN

    rng = np.random.default_rng(11)
    pk, sig, msg = O.synth_ed25519(1024, first=5000)
    corrupt_rows(rng, [pk, sig, msg])
    # S -> S + L on every 5th row (valid under Byron rules, invalid under libsodium's)
    for i in range(0, 1024, 5):
        s = int.from_bytes(sig[i, 32:].tobytes(), "little") + edge_L
        if s < 2**253:
            sig[i, 32:] = np.frombuffer(s.to_bytes(32, "little"), np.uint8)
    sig[3::97, 63] |= 0x20  # a top bit of S set
    cases = [(bytes(pk[i]), bytes(sig[i]), bytes(msg[i])) for i in range(1024)]
    cases += ed25519_edge_cases()
    got = ByronDSIGN.verify_batch([c[0] for c in cases], [c[2] for c in cases],
                                  [c[1] for c in cases])
    want = np.array([O.ed25519_verify_byron(c[1], c[2], c[0]) for c in cases])
    np.testing.assert_array_equal(got, want)
    assert want.sum() > 700


def test_byron_raw_headers_to_verdicts(small_path, gpu_lib, kats):
    """ouro_byron_verify_cbor: the golden Byron headers in every wire form
    (regular + epoch boundary) and every single-byte corruption of the v1 and
    HFC regular ones, raw CBOR -> verdicts in one call; the expected verdict
    is the Python slicer's status + the oracle's donna-style verify of the
    message it assembles (EBB: valid, PBFT.hs:327-328).  Then the configured
    protocol magic: the golden magic verifies, another one does not."""
    from ouroboros_network_amd import byron as B

    wires = [bytes.fromhex(w["raw"]) for w in kats["byron_wire"]]
    regular = [w for w, d in zip(wires, kats["byron_wire"]) if d["kind"] == "regular"]
    raws = list(wires)
    for g in (regular[0], regular[2]):  # n2n v1, hfc
        for pos in range(len(g)):
            m = bytearray(g)
            m[pos] ^= 0x04
            raws.append(bytes(m))
    got, status = B.verify_byron_cbor(raws, B.HEADER_MAGIC)
    want = []
    for r in raws:
        st, h = B.byron_status(r)
        if st == B.PACK_EBB:
            want.append(True)
        elif st != B.PACK_OK:
            want.append(False)
        else:
            want.append(O.ed25519_verify_byron(h.sig, h.message(B.HEADER_MAGIC), h.delegate_xpub[:32]))
        assert status[len(want) - 1] == st
    np.testing.assert_array_equal(got, np.array(want))
    assert got[:len(wires)].all()
    assert 0 < got[len(wires):].sum() < len(raws) - len(wires)
    ok, _ = B.verify_byron_cbor(regular, protocol_magic=kats["byron"]["magic"])
    assert ok.all()
    bad, st = B.verify_byron_cbor(regular, protocol_magic=764824073)
    assert not bad.any() and (st == B.PACK_OK).all()


def test_kes_periods_beyond_the_tree(gpu_lib, single_route):
    """Periods >= 64 (the reference's Period is a 64-bit Word): every t >= 63
    walks right at all six levels to leaf 63 (SumKES.verifyKES; SingleKES's
    assert is compiled out), so a leaf-63 signature verifies and others do
    not.  The host layer saturates Word periods at 2^32 - 1 for the ABI."""
    from ouroboros_network_amd import Sum6KES

    rng = np.random.default_rng(11)
    seed = rng.bytes(32)
    vk = O.kes_keygen(seed)
    m = rng.bytes(544)
    sig63, sig62 = O.kes_sign(seed, 63, m), O.kes_sign(seed, 62, m)
    periods = [62, 63, 64, 65, 100, 127, 128, 1 << 20, (1 << 32) - 1, 1 << 32, (1 << 64) - 1]
    rows = [(t, s) for t in periods for s in (sig63, sig62)]
    got = Sum6KES.verify_batch([vk] * len(rows), [t for t, _ in rows], [m] * len(rows),
                               np.frombuffer(b"".join(s for _, s in rows), np.uint8).reshape(-1, 448))
    want = [O.kes_verify(vk, min(t, (1 << 32) - 1), m, s) for t, s in rows]
    np.testing.assert_array_equal(got, want)
    # leaf 63 for every t >= 63, leaf 62 only at t = 62
    assert list(got) == [t == 62 if s is sig62 else t >= 63 for t, s in rows]
    for t, s in rows:
        assert (Sum6KES.verify_kes((), vk, t, m, s) is None) == (t == 62 if s is sig62 else t >= 63)
