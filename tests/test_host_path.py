"""The product library's HOST path (csrc/host_path.hip; round 4) against the
oracle, on the CPU -- no GPU needed.

Since round 4 the single-item entry points (ouro_ed25519_verify,
ouro_byron_ed25519_verify, ouro_vrf03_verify, ouro_vrf03_proof_to_hash,
ouro_sum6kes_verify) run on the CPU, and every host-buffer batch whose device
run fails is recomputed on that path (include/ouro_verify.h).  Since round 5
the path's field and group arithmetic is its own 64-bit implementation
(csrc/host_fast.h: 5 x 51-bit limbs); OURO_HOST_IMPL=lanes selects the
kernels' lane routines compiled for the CPU instead, and every test here runs
both.  The explicit *_batch_host entry points expose it for
batches.  These tests load the product library itself (lib/libouro_verify.so)
and compare with the oracle (oracle/, test infrastructure only) on the same
edge-case sets the GPU parity tests use; nothing under oracle/ is linked into
the product (test_product_links_no_oracle).  tests/test_gpu_host_path.py
forces device errors on a GPU box and checks the recompute.
"""
import ctypes
import os
import subprocess
from fractions import Fraction

import numpy as np
import pytest

import hdr_cases as HC
import oracle_ffi as O
from edge_cases import ed25519_edge_cases, vrf_edge_cases

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "ouroboros-network_amd", "lib", "libouro_verify.so")


@pytest.fixture(scope="module", params=["fast", "lanes"])
def lib(request):
    from ouroboros_network_amd import _native

    lib = _native.load()
    with _native.knob_env(OURO_HOST_IMPL=request.param):
        yield lib


@pytest.fixture(params=["fast", "lanes"])
def impl(request):
    """the host path's implementation for tests that call through Python"""
    from ouroboros_network_amd import _native

    _native.load()
    with _native.knob_env(OURO_HOST_IMPL=request.param):
        yield request.param


def test_host_entries_check_their_spans(lib):
    """the *_batch_host entries run the device calls' span checks --
    a NULL message with a nonzero length and an offset that wraps are
    OURO_EINVAL, never a read of invalid memory."""
    P = ctypes.c_void_p
    n = 2
    pk = np.zeros((n, 32), np.uint8)
    sig = np.zeros((n, 64), np.uint8)
    v = np.zeros(n, np.uint8)
    ln = np.array([0, 5], np.uint32)
    off = np.array([0, 0], np.uint64)
    wrap = np.array([0, 2**64 - 2], np.uint64)
    msg = np.zeros(16, np.uint8)
    for fn in (lib.ouro_ed25519_verify_batch_host, lib.ouro_byron_ed25519_verify_batch_host):
        assert fn(n, O.p(pk), O.p(sig), None, O.p(off), O.p(ln), O.p(v)) == -3
        assert fn(n, O.p(pk), O.p(sig), O.p(msg), O.p(wrap), O.p(ln), O.p(v)) == -3
    pi = np.zeros((n, 80), np.uint8)
    assert lib.ouro_vrf03_verify_batch_host(n, O.p(pk), O.p(pi), None, O.p(off), O.p(ln), None,
                                            O.p(v), 0) == -3
    t = np.zeros(n, np.uint32)
    ks = np.zeros((n, 448), np.uint8)
    assert lib.ouro_sum6kes_verify_batch_host(n, O.p(pk), O.p(t), O.p(msg), O.p(wrap), O.p(ln),
                                              O.p(ks), O.p(v)) == -3
    # a header batch whose body span wraps
    batch = HC.golden_variants(__import__("json").load(open(os.path.join(
        ROOT, "tests", "golden", "reference_kats.json"))), stride=400, s_rows=False)
    bo = batch.body_off.copy()
    bo[-1] = 2**64 - 3
    s = batch.c_struct()
    s.body_off = bo.ctypes.data  # (HeaderBatch itself rejects such offsets)
    vv = np.zeros(len(batch), np.uint8)
    assert lib.ouro_tpraos_verify_batch_host(ctypes.byref(s), O.p(vv), None, None) == -3
    # zero-length spans need no buffer at all
    z = np.zeros(n, np.uint32)
    assert lib.ouro_ed25519_verify_batch_host(n, O.p(pk), O.p(sig), None, O.p(off), O.p(z),
                                              O.p(v)) == 0


def _counts(lib):
    a, b = ctypes.c_ulonglong(), ctypes.c_ulonglong()
    lib.ouro_debug_host_path(ctypes.byref(a), ctypes.byref(b))
    return a.value, b.value


def test_single_items_run_on_the_host_path(lib):
    """The single-item calls need no device: they verify here, in a container
    without a GPU, and count as host-path items."""
    s0, _ = _counts(lib)
    pk, sig, msg = O.synth_ed25519(4, first=3)
    for i in range(4):
        m = bytes(msg[i])
        assert lib.ouro_ed25519_verify(bytes(sig[i]), m, len(m), bytes(pk[i])) == 0
        bad = bytearray(sig[i])
        bad[40] ^= 1
        assert lib.ouro_ed25519_verify(bytes(bad), m, len(m), bytes(pk[i])) == -1
    assert _counts(lib)[0] == s0 + 8


def test_ed25519_single_edge_cases(lib):
    for pk, sig, m in ed25519_edge_cases():
        got = lib.ouro_ed25519_verify(sig, m, len(m), pk)
        assert got in (0, -1)
        assert (got == 0) == O.ed25519_verify(sig, m, pk)


def test_ed25519_batch_host_corrupted_and_ragged(impl):
    """Batches over host threads: synthetic signatures with 1/3 corrupted,
    messages of ragged lengths (0..300 B, unaligned offsets)."""
    from ouroboros_network_amd import dsign

    rng = np.random.default_rng(5)
    n = 96
    vks, sigs, msgs, want = [], [], [], []
    for i in range(n):
        seed = rng.bytes(32)
        pk, sk = O.ed25519_keypair(seed)
        m = rng.bytes(int(rng.integers(0, 300)))
        s = bytearray(O.ed25519_sign(sk, m))
        if i % 3 == 1:
            s[int(rng.integers(0, 64))] ^= 1 << int(rng.integers(0, 8))
        vks.append(pk)
        sigs.append(bytes(s))
        msgs.append(m)
        want.append(O.ed25519_verify(bytes(s), m, pk))
    got = dsign.verify_batch(vks, msgs, sigs, host=True)
    np.testing.assert_array_equal(got, np.array(want))
    assert 0 < got.sum() < n


_POOL_CHILD = r"""
import sys
sys.path[:0] = [%r, %r]
import numpy as np
import oracle_ffi as O
from ouroboros_network_amd import dsign
rng = np.random.default_rng(11)
vks, sigs, msgs, want = [], [], [], []
for i in range(150):
    pk, sk = O.ed25519_keypair(rng.bytes(32))
    m = rng.bytes(int(rng.integers(0, 200)))
    s = bytearray(O.ed25519_sign(sk, m))
    if i %% 4 == 2:
        s[int(rng.integers(0, 64))] ^= 1
    vks.append(pk); sigs.append(bytes(s)); msgs.append(m)
    want.append(O.ed25519_verify(bytes(s), m, pk))
got = dsign.verify_batch(vks, msgs, sigs, host=True)
assert (got == np.array(want)).all() and 0 < got.sum() < len(want)
print("ok", int(got.sum()))
"""


@pytest.mark.parametrize("threads", ["1", "3"])
def test_host_pool_serial_and_narrow(threads):
    """the host path's task pool (csrc/task_pool.cpp)
    with no worker threads at all (OURO_HOST_THREADS=1: the calling thread
    runs every task, as when no worker can be spawned) and with two workers
    gives the oracle's verdicts."""
    env = dict(os.environ, OURO_HOST_THREADS=threads)
    r = subprocess.run(["python3", "-c", _POOL_CHILD % (ROOT, os.path.join(ROOT, "tests"))],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.startswith("ok")


def test_byron_single_and_batch(lib, kats):
    from ouroboros_network_amd import dsign  # noqa: F401  (loads the library)

    b = kats["byron"]
    pk, sig, msg = (bytes.fromhex(b[k]) for k in ("pk", "sig", "msg"))
    assert lib.ouro_byron_ed25519_verify(msg, len(msg), pk, sig) == 0
    bad = bytearray(msg)
    bad[7] ^= 1
    assert lib.ouro_byron_ed25519_verify(bytes(bad), len(bad), pk, sig) == -1
    # the donna-style corners against the oracle's Byron rule
    cases = list(ed25519_edge_cases())
    n = len(cases)
    pks = np.frombuffer(b"".join(c[0] for c in cases), np.uint8).reshape(n, 32)
    sgs = np.frombuffer(b"".join(c[1] for c in cases), np.uint8).reshape(n, 64)
    buf = np.frombuffer(b"".join(c[2] for c in cases) or b"\0", np.uint8)
    ln = np.array([len(c[2]) for c in cases], np.uint32)
    off = np.concatenate([[0], np.cumsum(ln)[:-1]]).astype(np.uint64)
    v = np.zeros(n, np.uint8)
    assert lib.ouro_byron_ed25519_verify_batch_host(n, O.p(pks), O.p(sgs), O.p(buf), O.p(off),
                                                    O.p(ln), O.p(v)) == 0
    want = [O.ed25519_verify_byron(c[1], c[2], c[0]) for c in cases]
    np.testing.assert_array_equal(v.astype(bool), np.array(want))


def test_vrf_single_vectors_and_edges(lib, kats):
    out = ctypes.create_string_buffer(64)
    for v in kats["vrf_draft03"]:
        a = bytes.fromhex(v["alpha"])
        assert lib.ouro_vrf03_verify(out, bytes.fromhex(v["pk"]), bytes.fromhex(v["pi"]), a,
                                     len(a)) == 0
        assert out.raw.hex() == v["beta"]
        assert lib.ouro_vrf03_proof_to_hash(out, bytes.fromhex(v["pi"])) == 0
        assert out.raw.hex() == v["beta"]
    for pk, pi, a in vrf_edge_cases():
        out = ctypes.create_string_buffer(b"\xaa" * 64, 64)
        rc = lib.ouro_vrf03_verify(out, pk, pi, a, len(a))
        want = O.vrf_verify(pk, pi, a)
        assert (rc == 0) == (want is not None)
        if want is not None:
            assert out.raw == want
        else:
            assert out.raw == b"\xaa" * 64  # written only on success
        h = ctypes.create_string_buffer(64)
        rc = lib.ouro_vrf03_proof_to_hash(h, pi)
        want_h = O.vrf_proof_to_hash(pi)
        assert (rc == 0) == (want_h is not None)
        if want_h is not None:
            assert h.raw == want_h


def test_vrf_batch_host_both_s_modes(impl):
    from ouroboros_network_amd import vrf

    pk, proof, alpha = O.synth_vrf(40, first=11)
    proof = proof.copy()
    for i in range(0, 40, 5):
        proof[i] = np.frombuffer(HC.with_s_plus_l(bytes(proof[i])), np.uint8)
    for i in range(2, 40, 7):
        proof[i, 60] ^= 4
    for s_mode in ("reduce", "strict"):
        ok, beta = vrf.verify_batch(pk, alpha, proof, s_mode=s_mode, host=True)
        for i in range(40):
            want = O.vrf_verify_mode(bytes(pk[i]), bytes(proof[i]), bytes(alpha[i]),
                                     s_mode == "strict")
            assert ok[i] == (want is not None), (s_mode, i)
            assert bytes(beta[i]) == (want or bytes(64))


def test_kes_single_and_batch(lib, kats):
    from ouroboros_network_amd import header as H
    from ouroboros_network_amd import kes

    for h in kats["headers"]:
        hd = H.parse_header(bytes.fromhex(h["raw"]))
        assert lib.ouro_sum6kes_verify(hd.hot_vk, 0, hd.body, len(hd.body), hd.kes_sig) == 0
        assert lib.ouro_sum6kes_verify(hd.hot_vk, 1, hd.body, len(hd.body), hd.kes_sig) == -1
    # every period of one synthetic tree, some corrupted, over host threads
    seed = b"\x05" * 32
    vk = O.kes_keygen(seed)
    rng = np.random.default_rng(9)
    ts, msgs, sigs, want = [], [], [], []
    for t in range(0, 64, 3):
        m = rng.bytes(int(rng.integers(0, 700)))
        s = bytearray(O.kes_sign(seed, t, m))
        tt = t
        if t % 4 == 1:
            s[int(rng.integers(0, 448))] ^= 0x20
        if t % 9 == 2:
            tt = t + 1
        ts.append(tt)
        msgs.append(m)
        sigs.append(bytes(s))
        want.append(O.kes_verify(vk, tt, m, bytes(s)))
    got = kes.verify_batch([vk] * len(ts), ts, msgs, sigs, host=True)
    np.testing.assert_array_equal(got, np.array(want))
    assert 0 < got.sum() < len(ts)


def _oracle_hdr(batch, nonce=False):
    return O.tpraos_verify_batch_nonce(batch) if nonce else O.tpraos_verify_batch(batch)


def test_headers_host_golden_variants(kats, impl):
    """k_tpraos_verify's body on the host: golden headers and every kind of
    single-field corruption hdr_cases makes, equal to the oracle's verdict
    bits and outputs."""
    from ouroboros_network_amd.tpraos import verify_headers_host

    batch = HC.golden_variants(kats, stride=5)
    got = verify_headers_host(batch)
    want = _oracle_hdr(batch)
    for g, w in zip(got, want):
        np.testing.assert_array_equal(g, w)
    assert (got[0] & 0x0F != 15).sum() > 10


def test_headers_host_claims_seeds_nonces(kats, impl):
    from ouroboros_network_amd.tpraos import verify_headers_host

    rng = np.random.default_rng(21)
    forged, _ = HC.forge_claims(HC.golden_variants(kats, stride=23), rng)
    for batch in (forged, HC.golden_variants(kats, stride=23, claimed=False),
                  HC.seeded(kats, bytes(range(32)), copies=2), HC.seeded(kats, None, copies=1)):
        got = verify_headers_host(batch, nonce=True)
        want = _oracle_hdr(batch, nonce=True)
        for g, w in zip(got, want):
            np.testing.assert_array_equal(g, w)


def test_leader_host_matches_oracle():
    import test_leader as TL
    from ouroboros_network_amd import leader as LD

    by_L = {}
    for b, s, L in TL.cases(seed=13, n_random=300):
        by_L.setdefault(L, []).append((b, s))
    for L, items in by_L.items():
        beta = np.frombuffer(b"".join(b for b, _ in items), dtype=np.uint8).reshape(-1, 64)
        got = LD.check_leader_values(beta, [s for _, s in items], LD.ActiveSlotCoeff(L),
                                     host=True)
        want = np.array([LD.LEADER_YES if TL.OL.check_leader_value(b, s, L) else LD.LEADER_NO
                         for b, s in items], dtype=np.uint8)
        np.testing.assert_array_equal(got, want)
    beta = np.frombuffer(b"\xff" * 128, dtype=np.uint8).reshape(2, 64)
    got = LD.check_leader_values(beta, [Fraction(1), Fraction(1)], LD.ActiveSlotCoeff(1),
                                 host=True)
    assert list(got) == [LD.LEADER_BADARG, LD.LEADER_BADARG]


def test_host_path_unaligned_buffers(lib):
    """Host callers' buffers need not be 16-B aligned (common.h host accessors)."""
    pk, sig, msg = O.synth_ed25519(8, first=21)
    raw = bytearray(1 + 8 * 96)
    for i in range(8):
        raw[1 + 96 * i:1 + 96 * i + 32] = bytes(pk[i])
        raw[1 + 96 * i + 32:1 + 96 * (i + 1)] = bytes(sig[i])
    buf = (ctypes.c_uint8 * len(raw)).from_buffer(raw)
    base = ctypes.addressof(buf) + 1
    for i in range(8):
        m = bytes(msg[i])
        assert lib.ouro_ed25519_verify(ctypes.c_void_p(base + 96 * i + 32), m, len(m),
                                       ctypes.c_void_p(base + 96 * i)) == 0


def test_product_links_no_oracle():
    """The host path is the product's own code: nothing under oracle/ is linked
    into or named by lib/libouro_verify.so."""
    syms = subprocess.run(["nm", "-D", "--defined-only", LIB], check=True, capture_output=True,
                          text=True).stdout
    assert "orc_" not in syms
    needed = subprocess.run(["readelf", "-d", LIB], check=True, capture_output=True,
                            text=True).stdout
    assert "oracle" not in needed and "sodium" not in needed
    src = open(os.path.join(ROOT, "ouroboros-network_amd", "csrc", "host_path.hip")).read()
    includes = [ln for ln in src.splitlines() if ln.startswith("#include")]
    assert includes and not any("oracle" in ln for ln in includes)
