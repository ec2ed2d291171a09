"""The product's host path (csrc/host_path.hip, host_fast.h, task_pool.cpp)
against the oracle, run only inside tests/test_sanitizers.py's child process
on lib/libouro_hostpath_asan.so (AddressSanitizer + UBSan build with a
test-only shim, csrc/hostpath_asan_shim.cpp); skipped elsewhere."""
import ctypes
import json
import os

import numpy as np
import pytest

import hdr_cases as HC
import oracle_ffi as O

LIB = os.environ.get("OURO_HOSTPATH_ASAN_LIB")
pytestmark = pytest.mark.skipif(not LIB, reason="only under tests/test_sanitizers.py")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def hp():
    lib = ctypes.CDLL(LIB)
    P, N, U32 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32
    lib.hp_ed_batch.argtypes = [N, P, P, P, P, P, P, U32]
    lib.hp_vrf_batch.argtypes = [N, P, P, P, P, P, P, P, U32]
    lib.hp_kes_batch.argtypes = [N, P, P, P, P, P, P, P]
    lib.hp_hdr_batch.argtypes = [P, P, P, P]
    return lib


def _ragged(msgs):
    off = np.zeros(len(msgs), np.uint64)
    ln = np.array([len(m) for m in msgs], np.uint32)
    buf = bytearray(b"\x00")  # unaligned first offset
    for i, m in enumerate(msgs):
        off[i] = len(buf)
        buf += m
    return np.frombuffer(bytes(buf) + b"\x00", np.uint8).copy(), off, ln


def test_ed25519_host_batch(hp):
    rng = np.random.default_rng(21)
    pks, sigs, msgs, want = [], [], [], []
    for i in range(120):
        pk, sk = O.ed25519_keypair(rng.bytes(32))
        m = rng.bytes(int(rng.integers(0, 260)))
        s = bytearray(O.ed25519_sign(sk, m))
        if i % 3 == 1:
            s[int(rng.integers(0, 64))] ^= 1 << int(rng.integers(0, 8))
        pks.append(pk)
        sigs.append(bytes(s))
        msgs.append(m)
        want.append(O.ed25519_verify(bytes(s), m, pk))
    buf, off, ln = _ragged(msgs)
    pk = np.frombuffer(b"".join(pks), np.uint8).copy()
    sig = np.frombuffer(b"".join(sigs), np.uint8).copy()
    v = np.zeros(len(msgs), np.uint8)
    assert hp.hp_ed_batch(len(msgs), O.p(pk), O.p(sig), O.p(buf), O.p(off), O.p(ln), O.p(v), 0) == 0
    np.testing.assert_array_equal(v != 0, np.array(want))


def test_vrf_host_batch(hp):
    n = 48
    pk, proof, alpha = O.synth_vrf(n)
    proof[1::3, 50] ^= 4
    want, wbeta = O.vrf_verify_batch(pk, proof, alpha)
    off = (np.arange(n) * 32).astype(np.uint64)
    ln = np.full(n, 32, np.uint32)
    beta = np.zeros((n, 64), np.uint8)
    v = np.zeros(n, np.uint8)
    assert hp.hp_vrf_batch(n, O.p(pk), O.p(proof), O.p(alpha), O.p(off), O.p(ln), O.p(beta),
                           O.p(v), 0) == 0
    np.testing.assert_array_equal(v != 0, want)
    np.testing.assert_array_equal(beta[want], wbeta[want])


def test_kes_host_batch(hp):
    rng = np.random.default_rng(22)
    vks, ts, sigs, msgs, want = [], [], [], [], []
    for i in range(24):
        seed = rng.bytes(32)
        t = int(rng.integers(0, 64))
        m = rng.bytes(int(rng.integers(0, 700)))
        sig = bytearray(O.kes_sign(seed, t, m))
        if i % 4 == 3:
            sig[int(rng.integers(0, 448))] ^= 2
        vk = O.kes_keygen(seed)
        vks.append(vk)
        ts.append(t)
        sigs.append(bytes(sig))
        msgs.append(m)
        want.append(O.kes_verify(vk, t, m, bytes(sig)))
    buf, off, ln = _ragged(msgs)
    vk = np.frombuffer(b"".join(vks), np.uint8).copy()
    sg = np.frombuffer(b"".join(sigs), np.uint8).copy()
    t = np.array(ts, np.uint32)
    v = np.zeros(len(msgs), np.uint8)
    assert hp.hp_kes_batch(len(msgs), O.p(vk), O.p(t), O.p(buf), O.p(off), O.p(ln), O.p(sg),
                           O.p(v)) == 0
    np.testing.assert_array_equal(v != 0, np.array(want))


def test_header_host_batch(hp):
    kats = json.load(open(os.path.join(ROOT, "tests", "golden", "reference_kats.json")))
    batch = HC.golden_variants(kats, stride=16)
    want, wbe, wbl = O.tpraos_verify_batch(batch)
    n = len(batch)
    s = batch.c_struct()
    v = np.zeros(n, np.uint8)
    be = np.zeros((n, 64), np.uint8)
    bl = np.zeros((n, 64), np.uint8)
    assert hp.hp_hdr_batch(ctypes.addressof(s), O.p(v), O.p(be), O.p(bl)) == 0
    np.testing.assert_array_equal(v, want)
    np.testing.assert_array_equal(be, wbe)
    np.testing.assert_array_equal(bl, wbl)
