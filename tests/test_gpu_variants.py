"""The non-default launch forms kept as A/B switches, against the oracle on
the GPU (their measurements: DESIGN.md §4 "Measured design alternatives"):

* OURO_SPLIT=1 -- the split kernels (pre / dsm at 4 waves per SIMD / post)
  for headers, Ed25519 and Sum6KES (rejected on time, kept bit-exact); the
  product fixes the choice at compile time, so these run on the test-hook
  build (tests/test_gpu_hooks.py);
* OURO_PLAN_STAGE=0 / 1 / 2 / 3 -- a latency plan's window copies (2, the
  default: copy kernel in, results written by the latency kernel straight
  into the pinned block), with and without the eta nonce output;
* OURO_PLAN_GRAPH=1 -- the plan's launches captured into one hipGraph
  instead of issued per submit (the default since r04m);
* OURO_PLAN_FLAG=0 -- the plan's wait on the stream's completion instead of
  the kernel's done word in the pinned output block.

Every form must give the oracle's verdicts and outputs; a switch that drifts
from it fails here even while it is off by default.
"""
import numpy as np
import pytest

import hdr_cases as HC
import oracle_ffi as O

pytestmark = pytest.mark.gpu


def _corrupt(rng, a, frac=8):
    idx = np.nonzero(rng.integers(0, frac, a.shape[0]) == 0)[0]
    for i in idx:
        a[i, int(rng.integers(0, a.shape[1]))] ^= 0x10
    return idx


@pytest.mark.hooks  # the product fixes OURO_SPLIT at compile time
def test_split_headers_match_oracle(gpu_lib, kats, monkeypatch):
    from ouroboros_network_amd import tpraos as T

    monkeypatch.setenv("OURO_SPLIT", "1")
    batch = HC.golden_variants(kats, stride=5)
    wv, wbe, wbl = O.tpraos_verify_batch(batch)
    v, be, bl = T.verify_headers(batch)
    np.testing.assert_array_equal(v, wv)
    np.testing.assert_array_equal(be, wbe)
    np.testing.assert_array_equal(bl, wbl)
    # claims, (slot, eta0) seeds and the eta nonce through the split path
    seeded = HC.seeded(kats, bytes(range(32)), copies=3)
    got = T.verify_headers(seeded, nonce=True)
    want = O.tpraos_verify_batch_nonce(seeded)
    for g, w in zip(got, want):
        np.testing.assert_array_equal(g, w)


@pytest.mark.hooks  # the product fixes OURO_SPLIT at compile time
def test_split_ed25519_and_kes_match_oracle(gpu_lib, monkeypatch):
    from ouroboros_network_amd import Ed25519DSIGN, Sum6KES

    monkeypatch.setenv("OURO_SPLIT", "1")
    monkeypatch.setenv("OURO_WIDE_SMALL_MAX", "0")  # the lane kernels, not wave-per-item
    rng = np.random.default_rng(17)
    n = 4096
    pk, sig, msg = O.synth_ed25519(n, first=300)
    _corrupt(rng, sig)
    got = Ed25519DSIGN.verify_batch(pk, msg, sig)
    buf, off, ln = msg.reshape(-1), np.arange(n, dtype=np.uint64) * 32, np.full(n, 32, np.uint32)
    want = O.ed25519_verify_batch(pk, sig, buf, off, ln)
    assert 0 < want.sum() < n
    np.testing.assert_array_equal(got, want)

    seeds = [rng.bytes(32) for _ in range(3)]
    vks = [O.kes_keygen(s) for s in seeds]
    rows_vk, ts, msgs, sigs = [], [], [], []
    for i in range(96):
        k, t = i % 3, int(rng.integers(0, 64))
        m = rng.bytes(int(rng.integers(1, 600)))
        s = O.kes_sign(seeds[k], t, m)
        if i % 5 == 2:
            t = (t + 3) % 64
        rows_vk.append(vks[k])
        ts.append(t)
        msgs.append(m)
        sigs.append(s)
    sig_a = np.frombuffer(b"".join(sigs), np.uint8).reshape(len(sigs), 448).copy()
    _corrupt(rng, sig_a, frac=9)
    got = Sum6KES.verify_batch(rows_vk, ts, msgs, sig_a)
    want = np.array([O.kes_verify(v, t, m, bytes(s)) for v, t, m, s in zip(rows_vk, ts, msgs, sig_a)])
    assert 0 < want.sum() < len(sigs)
    np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("stage,graph,flag", [("0", "1", "1"), ("1", "1", "1"), ("2", "1", "1"),
                                              ("3", "1", "1"), ("0", "0", "1"), ("2", "0", "1"),
                                              ("2", "0", "0")])
def test_plan_stage_forms_match_oracle(gpu_lib, kats, monkeypatch, stage, graph, flag):
    from ouroboros_network_amd.tpraos import HeaderPlan

    monkeypatch.setenv("OURO_PLAN_STAGE", stage)  # read when the plan is created
    monkeypatch.setenv("OURO_PLAN_GRAPH", graph)  # 1: the launches captured into a hipGraph
    monkeypatch.setenv("OURO_PLAN_FLAG", flag)  # 0: wait on the stream, not the done word
    batch = HC.golden_variants(kats, stride=9)
    wv, wbe, wbl = O.tpraos_verify_batch(batch)
    plan = HeaderPlan(max_headers=64, max_body_bytes=int(batch.body.size))
    try:
        for lo in range(0, len(batch), 64):
            hi = min(len(batch), lo + 64)
            v, be, bl = plan.run(batch.slice(lo, hi))
            np.testing.assert_array_equal(v, wv[lo:hi])
            np.testing.assert_array_equal(be, wbe[lo:hi])
            np.testing.assert_array_equal(bl, wbl[lo:hi])
    finally:
        plan.close()
    seeded = HC.seeded(kats, bytes(range(32)), copies=2)
    want = O.tpraos_verify_batch_nonce(seeded)
    plan = HeaderPlan(max_headers=64, max_body_bytes=int(seeded.body.size))
    try:
        got = plan.run(seeded, nonce=True)
        for g, w in zip(got, want):
            np.testing.assert_array_equal(g, w)
    finally:
        plan.close()
