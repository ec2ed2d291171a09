"""Device errors on a real GPU box: every host-buffer call recomputes on the
product's host path (csrc/host_path.hip) and returns the oracle's verdicts,
never an unverified accept (SURVEY.md §5 and §8(b) "Errors"; VERDICT r03 next
item 4).  The device error is forced through the library's test hook
(OURO_TEST_DEVICE_ERROR in the environment: every launch reports
OURO_EDEVICE); OURO_ON_DEVICE_ERROR=fail turns the recompute off, and the call
must then return the error and leave the verdicts untouched.

Also: the single-item calls on both routes (the host path, the default, and
OURO_SINGLE_ITEM=gpu) against the oracle on the edge-case sets.

Every other GPU test runs with the recompute counter watched (conftest.py):
none of them may pass on the host path unnoticed.
"""
import contextlib
import ctypes
import os
from fractions import Fraction

import numpy as np
import pytest

import hdr_cases as HC
import oracle_ffi as O
from edge_cases import ed25519_edge_cases, vrf_edge_cases

pytestmark = [pytest.mark.gpu, pytest.mark.device_error]


def env(**kv):
    """the switches set for a block, the library re-reading them (knobs.h)"""
    from ouroboros_network_amd import _native

    return _native.knob_env(**kv)


def recomputed(lib):
    a, b = ctypes.c_ulonglong(), ctypes.c_ulonglong()
    lib.ouro_debug_host_path(ctypes.byref(a), ctypes.byref(b))
    return b.value


@contextlib.contextmanager
def device_error(lib, calls, same_thread=True):
    """Every launch inside fails; `calls` host-buffer calls must recompute
    (and, on the calling thread, say so in ouro_last_error)."""
    r0 = recomputed(lib)
    with env(OURO_TEST_DEVICE_ERROR=1):
        yield
    assert recomputed(lib) - r0 == calls
    if same_thread:
        assert b"recomputed on the host path" in lib.ouro_last_error()


def test_ed25519_and_byron_batches_recompute(gpu_lib):
    from ouroboros_network_amd import Ed25519DSIGN
    from ouroboros_network_amd.byron import ByronDSIGN  # noqa: F401

    cases = ed25519_edge_cases()
    pks, sigs, msgs = [c[0] for c in cases], [c[1] for c in cases], [c[2] for c in cases]
    want = np.array([O.ed25519_verify(s, m, k) for k, s, m in cases])
    with device_error(gpu_lib, 1):
        got = Ed25519DSIGN.verify_batch(pks, msgs, sigs)
    np.testing.assert_array_equal(got, want)
    # larger than the wave-per-item limit: the lane kernel's launch fails
    pk, sig, msg = O.synth_ed25519(3000, first=5)
    sig = sig.copy()
    sig[::7, 3] ^= 1
    want = O.ed25519_verify_batch(pk, sig, msg.reshape(-1), np.arange(3000, dtype=np.uint64) * 32,
                                  np.full(3000, 32, np.uint32))
    with device_error(gpu_lib, 1):
        got = Ed25519DSIGN.verify_batch(pk, msg, sig)
    np.testing.assert_array_equal(got, want)
    # ByronDSIGN acceptance through the same recompute
    n = len(cases)
    pka = np.frombuffer(b"".join(pks), np.uint8).reshape(n, 32)
    sga = np.frombuffer(b"".join(sigs), np.uint8).reshape(n, 64)
    buf = np.frombuffer(b"".join(msgs) or b"\0", np.uint8)
    ln = np.array([len(m) for m in msgs], np.uint32)
    off = np.concatenate([[0], np.cumsum(ln)[:-1]]).astype(np.uint64)
    v = np.zeros(n, np.uint8)
    with device_error(gpu_lib, 1):
        assert gpu_lib.ouro_byron_ed25519_verify_batch(n, O.p(pka), O.p(sga), O.p(buf), O.p(off),
                                                       O.p(ln), O.p(v)) == 0
    np.testing.assert_array_equal(v.astype(bool),
                                  np.array([O.ed25519_verify_byron(s, m, k) for k, s, m in cases]))


@pytest.mark.parametrize("s_mode", ["reduce", "strict"])
def test_vrf_batch_recompute(gpu_lib, s_mode):
    from ouroboros_network_amd import PraosVRF

    pk, proof, alpha = O.synth_vrf(200, first=31)
    proof = proof.copy()
    proof[::9, 50] ^= 2
    for i in range(3, 200, 17):
        proof[i] = np.frombuffer(HC.with_s_plus_l(bytes(proof[i])), np.uint8)
    with device_error(gpu_lib, 1):
        ok, beta = PraosVRF.verify_batch(pk, alpha, proof, s_mode=s_mode)
    for i in range(200):
        want = O.vrf_verify_mode(bytes(pk[i]), bytes(proof[i]), bytes(alpha[i]), s_mode == "strict")
        assert ok[i] == (want is not None)
        assert bytes(beta[i]) == (want or bytes(64))


def test_kes_batch_recompute(gpu_lib, kats):
    from ouroboros_network_amd import Sum6KES
    from ouroboros_network_amd import header as H

    hds = [H.parse_header(bytes.fromhex(h["raw"])) for h in kats["headers"]]
    vks = [h.hot_vk for h in hds] * 2
    ts = [0] * len(hds) + [1] * len(hds)
    bodies = [h.body for h in hds] * 2
    sigs = [h.kes_sig for h in hds] * 2
    with device_error(gpu_lib, 1):
        got = Sum6KES.verify_batch(vks, ts, bodies, sigs)
    assert list(got) == [True] * len(hds) + [False] * len(hds)


def _check(got, want):
    for g, w in zip(got, want):
        if w is not None:
            np.testing.assert_array_equal(g, w)


def test_header_paths_recompute(gpu_lib, kats):
    """Throughput (one piece and pipelined chunks), latency, multi-device,
    plans (run and submit/wait): all recompute and equal the oracle, the
    optional members (claimed outputs, seeds, eta nonce) included."""
    from ouroboros_network_amd import tpraos as T

    rng = np.random.default_rng(3)
    forged, _ = HC.forge_claims(HC.golden_variants(kats, stride=9), rng)
    seeded = HC.seeded(kats, bytes(range(32)), copies=2)
    for batch in (forged, seeded):
        want = O.tpraos_verify_batch_nonce(batch)
        with device_error(gpu_lib, 1):
            _check(T.verify_headers(batch, nonce=True), want)
        with env(OURO_HOST_CHUNK=16), device_error(gpu_lib, 1):
            _check(T.verify_headers(batch, nonce=True), want)
        with device_error(gpu_lib, 1):
            _check(T.verify_headers_lowlat(batch, nonce=True), want)
        with device_error(gpu_lib, 2, same_thread=False):  # two shards, one per worker
            _check(T.verify_headers_multi(batch, devices=[0, 0], nonce=True), want)
    w = O.tpraos_verify_batch_nonce(forged.slice(0, 40))
    plan = T.HeaderPlan(64, 64 * 1400)
    try:
        with device_error(gpu_lib, 1):
            _check(plan.run(forged.slice(0, 40), nonce=True), w)
        r0 = recomputed(gpu_lib)
        with env(OURO_TEST_DEVICE_ERROR=1):  # the launch fails at submit ...
            plan.submit(forged.slice(0, 40), nonce=True)
        _check(plan.wait(), w)  # ... and wait recomputes from the staged inputs
        assert recomputed(gpu_lib) == r0 + 1
        # and the plan is healthy again afterwards
        r0 = recomputed(gpu_lib)
        _check(plan.run(forged.slice(0, 40), nonce=True), w)
        assert recomputed(gpu_lib) == r0
    finally:
        plan.close()


def test_leader_and_byron_cbor_recompute(gpu_lib, kats):
    import test_leader as TL
    from ouroboros_network_amd import leader as LD
    from ouroboros_network_amd.byron import verify_byron_cbor

    items = [(b, s) for b, s, L in TL.cases(seed=5, n_random=100) if L == TL.cases()[0][2]]
    L = TL.cases()[0][2]
    beta = np.frombuffer(b"".join(b for b, _ in items), np.uint8).reshape(-1, 64)
    with device_error(gpu_lib, 1):
        got = LD.check_leader_values(beta, [s for _, s in items], LD.ActiveSlotCoeff(L))
    want = [LD.LEADER_YES if TL.OL.check_leader_value(b, s, L) else LD.LEADER_NO for b, s in items]
    assert list(got) == want
    raw = bytes.fromhex(kats["byron"]["raw"])
    with device_error(gpu_lib, 1):
        verdict, status = verify_byron_cbor([raw, raw, raw],
                                            protocol_magic=kats["byron"]["magic"])
    assert list(status) == [0, 0, 0] and verdict.all()
    with device_error(gpu_lib, 1):
        verdict, status = verify_byron_cbor([raw], protocol_magic=764824073)
    assert list(status) == [0] and not verdict.any()


def test_recompute_off_returns_the_error(gpu_lib, kats):
    """OURO_ON_DEVICE_ERROR=fail: the error comes back and the verdicts stay
    as they were -- never reported valid."""
    from ouroboros_network_amd import _native
    from ouroboros_network_amd import tpraos as T

    batch = HC.golden_variants(kats, stride=40)
    n = len(batch)
    s = batch.c_struct()
    v = np.full(n, 0xEE, np.uint8)
    be = np.zeros((n, 64), np.uint8)
    bl = np.zeros((n, 64), np.uint8)
    from ouroboros_network_amd import Ed25519DSIGN

    plan = T.HeaderPlan(64, 64 * 1400)  # (its capture launches too: made before the hook)
    r0 = recomputed(gpu_lib)
    try:
        with env(OURO_TEST_DEVICE_ERROR=1, OURO_ON_DEVICE_ERROR="fail"):
            rc = gpu_lib.ouro_tpraos_verify_batch(ctypes.byref(s), O.p(v), O.p(be), O.p(bl))
            assert rc == _native.OURO_EDEVICE
            assert (v == 0xEE).all()
            pk, sig, msg = O.synth_ed25519(8, first=1)
            with pytest.raises(_native.DeviceError):
                Ed25519DSIGN.verify_batch(pk, msg, sig)
            assert gpu_lib.ouro_tpraos_plan_submit(plan._p, ctypes.byref(s)) == _native.OURO_EDEVICE
    finally:
        plan.close()
    assert recomputed(gpu_lib) == r0


@pytest.mark.parametrize("route", ["host", "gpu"])
def test_single_items_both_routes(gpu_lib, kats, route):
    """ouro_ed25519_verify / ouro_vrf03_verify / ouro_vrf03_proof_to_hash /
    ouro_sum6kes_verify / ouro_byron_ed25519_verify on the host path (the
    default) and on the GPU (OURO_SINGLE_ITEM=gpu), edge cases vs the oracle."""
    from ouroboros_network_amd import header as H

    kw = {"OURO_SINGLE_ITEM": "gpu"} if route == "gpu" else {"OURO_SINGLE_ITEM": "host"}
    with env(**kw):
        for pk, sig, m in ed25519_edge_cases()[:40]:
            assert (gpu_lib.ouro_ed25519_verify(sig, m, len(m), pk) == 0) == \
                O.ed25519_verify(sig, m, pk)
            assert (gpu_lib.ouro_byron_ed25519_verify(m, len(m), pk, sig) == 0) == \
                O.ed25519_verify_byron(sig, m, pk)
        out = ctypes.create_string_buffer(64)
        for pk, pi, a in vrf_edge_cases()[:30]:
            want = O.vrf_verify(pk, pi, a)
            rc = gpu_lib.ouro_vrf03_verify(out, pk, pi, a, len(a))
            assert (rc == 0) == (want is not None)
            if want is not None:
                assert out.raw == want
            want_h = O.vrf_proof_to_hash(pi)
            rc = gpu_lib.ouro_vrf03_proof_to_hash(out, pi)
            assert (rc == 0) == (want_h is not None)
            if want_h is not None:
                assert out.raw == want_h
        hd = H.parse_header(bytes.fromhex(kats["headers"][0]["raw"]))
        assert gpu_lib.ouro_sum6kes_verify(hd.hot_vk, 0, hd.body, len(hd.body), hd.kes_sig) == 0
        assert gpu_lib.ouro_sum6kes_verify(hd.hot_vk, 2, hd.body, len(hd.body), hd.kes_sig) == -1
