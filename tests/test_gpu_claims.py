"""GPU parity of the header boundary's optional members (include/ouro_verify.h):

* claimed VRF outputs -> OURO_HDR_ETA_CLAIM_OK / _LEADER_CLAIM_OK.  The
  reference accepts on the proof (verifyCertified) and then uses the CLAIMED
  output (Shelley/Protocol.hs:484-486, Shelley/Ledger/TPraos.hs:40); a forged
  claimed output on a valid proof must give PROOF ok and CLAIM clear;
* VRF inputs derived on the device from (slot, eta0) by mkSeed;
* the eta_nonce output (mkNonceFromOutputVRF of the claimed eta output),
  folded by ouro_nonce_fold exactly as oracle/nonce.py's UPDN.

Every path -- throughput kernel (one piece and pipelined chunks), latency
kernels (lane quads and one lane), captured plans (run, submit/wait) and the
multi-device workers -- against the oracle (oracle/tpraos.c), bit for bit.
"""
import contextlib
import os

import numpy as np
import pytest

import hdr_cases as HC
import oracle_ffi as O

pytestmark = pytest.mark.gpu


def _oracle(batch):
    import ctypes

    n = len(batch)
    en = np.zeros((n, 32), np.uint8)
    s = batch.c_struct(en)
    v = np.zeros(n, np.uint8)
    be = np.zeros((n, 64), np.uint8)
    bl = np.zeros((n, 64), np.uint8)
    O.lib().orc_tpraos_verify_batch(ctypes.addressof(s), O.p(v), O.p(be), O.p(bl), 8)
    return v, be, bl, en


def _cases(kats):
    rng = np.random.default_rng(31)
    forged, _ = HC.forge_claims(HC.golden_variants(kats, stride=3), rng)
    return {
        "forged_claims": forged,
        "no_claims": HC.golden_variants(kats, stride=5, claimed=False),
        "seeded_eta0": HC.seeded(kats, bytes(range(100, 132)), copies=6),
        "seeded_neutral": HC.seeded(kats, None, copies=3),
    }


def _check(got, want):
    for g, w in zip(got, want):
        np.testing.assert_array_equal(g, w)


@pytest.mark.parametrize("chunk", ["0", "5"], ids=["one_piece", "pipelined"])
def test_throughput_paths(gpu_lib, kats, monkeypatch, chunk):
    from ouroboros_network_amd.tpraos import verify_headers

    monkeypatch.setenv("OURO_HOST_CHUNK", chunk)
    for name, batch in _cases(kats).items():
        want = _oracle(batch)
        _check(verify_headers(batch, nonce=True), want)
        v = verify_headers(batch)[0]
        np.testing.assert_array_equal(v, want[0])
    seeded = _cases(kats)["seeded_eta0"]
    v = verify_headers(seeded)[0]
    assert list(v[:6]) == [0x3F, 0x3F, 0x03, 0x2B, 0x1F, 0x2F]


LAT_FORMS = {
    "wide_fused": {},
    "wide_finish_launch": {"OURO_LAT_FUSE": "0"},
    "lane_quads": {"OURO_LAT_WIDE": "0", "OURO_LAT_QUAD": "1"},
    "one_lane": {"OURO_LAT_WIDE": "0", "OURO_LAT_QUAD": "0"},
}


@pytest.mark.parametrize("form", list(LAT_FORMS))
def test_latency_paths(gpu_lib, kats, monkeypatch, form):
    from ouroboros_network_amd.tpraos import HeaderPlan, verify_headers_lowlat

    for k, v in LAT_FORMS[form].items():
        monkeypatch.setenv(k, v)
    cases = _cases(kats)
    for name, batch in cases.items():
        want = _oracle(batch)
        _check(verify_headers_lowlat(batch, nonce=True), want)
    # one plan serves batches with and without each optional member in turn
    plan = HeaderPlan(max_headers=64, max_body_bytes=64 * 1400)
    try:
        for _ in range(2):
            for name, batch in cases.items():
                want = _oracle(batch)
                for lo in range(0, len(batch), 64):
                    hi = min(len(batch), lo + 64)
                    w = batch.slice(lo, hi)
                    got = plan.run(w, nonce=True)
                    _check(got, tuple(x[lo:hi] for x in want))
                    plan.submit(w, nonce=(lo // 64) % 2 == 0)
                    got = plan.wait()
                    _check(got, tuple(x[lo:hi] for x in want)[:len(got)])
    finally:
        plan.close()


def test_multi_device_paths(gpu_lib, kats):
    from ouroboros_network_amd.tpraos import verify_headers_multi

    for name, batch in _cases(kats).items():
        want = _oracle(batch)
        for devices in ([0], [0, 0, 0]):
            _check(verify_headers_multi(batch, devices, nonce=True), want)


def test_nonce_fold_from_device_outputs(gpu_lib, kats):
    """eta_nonce rows from the kernel, folded by ouro_nonce_fold, equal the
    oracle's UPDN fold over Blake2b-256 of the CLAIMED outputs; with claimed
    outputs forged, the fold follows the claimed (not the computed) output,
    as the reference's PRTCL rule does."""
    from ouroboros_network_amd.tpraos import nonce_fold, verify_headers

    ON = O.nonce_module()
    batch = HC.seeded(kats, bytes(32), copies=2)
    v, be, bl, en = verify_headers(batch, nonce=True)
    claimed = [bytes(r) for r in batch.eta_output]
    assert [bytes(r) for r in en] == [ON.mk_nonce_from_output_vrf(c) for c in claimed]
    assert bytes(en[5]) != ON.mk_nonce_from_output_vrf(bytes(be[5]))  # forged claim row
    slots = np.sort(batch.slot)
    for fsne in (int(slots[len(slots) // 2]) + 10, 2**63):
        got = nonce_fold(en, slots, fsne, 7, None, b"\x11" * 32)
        assert got == ON.fold(None, b"\x11" * 32, [bytes(r) for r in en], slots, fsne, 7)


@contextlib.contextmanager
def _poisoned_submit():
    """The plan test hook (kernels.hip plan_poison; the test build only),
    reached through the environment: every submit while it is set first
    poisons the counters."""
    from ouroboros_network_amd import _native

    with _native.knob_env(OURO_TEST_PLAN_POISON="1"):
        yield


@pytest.mark.hooks
def test_plan_counters_from_cut_off_launch(gpu_lib, kats):
    """A plan whose arrival counters were left mid-count by an earlier launch
    that never completed (simulated: with OURO_TEST_PLAN_POISON set,
    ouro_tpraos_plan_submit first leaves every counter one arrival short of its
    finish, tagged with the last launch's generation) must still give the oracle's verdicts and outputs on the next
    window: each launch counts in its own generation (wide_cores.h
    arrive_last), so no header finishes early on the stale counts -- and no
    verdict carries an earlier window's result.  The second window holds other
    headers than the first, so a stale record would show."""
    from ouroboros_network_amd.tpraos import HeaderPlan

    rng = np.random.default_rng(41)
    forged, _ = HC.forge_claims(HC.golden_variants(kats, stride=3), rng)
    first, second = forged.slice(0, 64), forged.slice(64, 128)
    w1, w2 = _oracle(first), _oracle(second)
    plan = HeaderPlan(64, 64 * 1400)
    try:
        _check(plan.run(first, nonce=True), w1)
        for _ in range(3):
            with _poisoned_submit():
                _check(plan.run(second, nonce=True), w2)
            with _poisoned_submit():
                _check(plan.run(first, nonce=True), w1)
        # and a partial window after a poisoned full one
        with _poisoned_submit():
            _check(plan.run(second.slice(5, 17), nonce=True), tuple(a[5:17] for a in w2))
    finally:
        plan.close()


@pytest.mark.hooks
def test_plan_results_never_stale(gpu_lib, kats):
    """ADVICE r04 (the done word): with OURO_TEST_PLAN_SENTINEL (test build)
    every result byte of the plan's pinned output block is overwritten with a
    sentinel before each launch, so a wait that returned before all of the
    tail's stores were visible -- the verdict and both outputs, written by
    several lanes of the tail wave -- would return the sentinel.  Windows
    alternate between two different batches; every one must equal the oracle."""
    from ouroboros_network_amd import tpraos as T

    a = HC.golden_variants(kats, stride=13).slice(0, 64)
    b = HC.seeded(kats, bytes(range(32)), copies=4).slice(0, 40)
    wa, wb = O.tpraos_verify_batch_nonce(a), O.tpraos_verify_batch_nonce(b)
    plan = T.HeaderPlan(64, 64 * 1400)
    from ouroboros_network_amd import _native

    try:
        with _native.knob_env(OURO_TEST_PLAN_SENTINEL="1"):
            for k in range(200):
                batch, want = (a, wa) if k % 2 == 0 else (b, wb)
                got = plan.run(batch, nonce=True)
                for g, w in zip(got, want):
                    np.testing.assert_array_equal(g, w)
    finally:
        plan.close()
