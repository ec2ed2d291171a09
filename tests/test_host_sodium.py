"""The product's host path against libsodium 1.0.18 DIRECTLY (VERDICT r05
weak item 1 / item 6): no oracle anywhere in these checks, so a defect the
host path's field layer (csrc/host_fast.h) shared with oracle/curve.c could
not pass both.

libsodium 1.0.18 is the version the reference's CI pins
(.github/workflows/build.yml:77,98) and the function the reference calls for
Ed25519 (crypto_sign_ed25519_verify_detached; caller
shape ouroboros-consensus-byron/src/Ouroboros/Consensus/Byron/Crypto/DSIGN.hs:110-113).
The VRF proofs are made here by a draft-03 prover written with libsodium's
own group and scalar primitives (crypto_core_ed25519_from_uniform -- the
Elligator2 map the VRF fork calls --, crypto_scalarmult_ed25519_*,
crypto_core_ed25519_scalar_*), pinned first on the three IETF draft-03
vectors; the product's verdicts and beta outputs are then compared with what
that prover says.  Every call here runs the product's host path (single
items by default, `*_batch_host` for batches); no GPU.
"""
import ctypes
import hashlib

import numpy as np
import pytest

import oracle_ffi as O
from edge_cases import ed25519_edge_cases

L = 2**252 + 27742317777372353535851937790883648493


@pytest.fixture(scope="module")
def na():
    s = O.sodium()
    if s is None:
        pytest.skip("libsodium 1.0.18 not present")
    from ouroboros_network_amd import _native

    return s, _native.load()


def _sodium_verify(s, sig, m, pk):
    return s.crypto_sign_ed25519_verify_detached(sig, m, ctypes.c_ulonglong(len(m)), pk) == 0


def _sodium_keypair(s, seed):
    pk, sk = ctypes.create_string_buffer(32), ctypes.create_string_buffer(64)
    assert s.crypto_sign_ed25519_seed_keypair(pk, sk, seed) == 0
    return pk.raw, sk.raw


def _sodium_sign(s, sk, m):
    sig = ctypes.create_string_buffer(64)
    assert s.crypto_sign_ed25519_detached(sig, None, m, ctypes.c_ulonglong(len(m)), sk) == 0
    return sig.raw


def test_ed25519_edge_cases_single_and_batch(na):
    """Every edge case (S >= L, small-order R / A, non-canonical and
    undecodable encodings, mixed-order keys with torsion-consistent R, ...):
    the product's single-item call and its host batch give libsodium's own
    verdict."""
    s, lib = na
    cases = ed25519_edge_cases()
    want = [_sodium_verify(s, sig, m, pk) for pk, sig, m in cases]
    assert 0 < sum(want) < len(cases)
    for (pk, sig, m), w in zip(cases, want):
        assert (lib.ouro_ed25519_verify(sig, m, len(m), pk) == 0) == w
    n = len(cases)
    pks = np.frombuffer(b"".join(c[0] for c in cases), np.uint8)
    sgs = np.frombuffer(b"".join(c[1] for c in cases), np.uint8)
    buf = np.frombuffer(b"".join(c[2] for c in cases) + b"\0", np.uint8)
    ln = np.array([len(c[2]) for c in cases], np.uint32)
    off = np.concatenate([[0], np.cumsum(ln[:-1])]).astype(np.uint64)
    v = np.zeros(n, np.uint8)
    assert lib.ouro_ed25519_verify_batch_host(n, O.p(pks), O.p(sgs), O.p(buf), O.p(off),
                                              O.p(ln), O.p(v)) == 0
    np.testing.assert_array_equal(v.astype(bool), np.array(want))


def test_ed25519_ten_thousand_seeded_one_eighth_corrupted(na):
    """10^4 keypairs and signatures made by libsodium over ragged messages
    (0..700 B at unaligned offsets), 1/8 corrupted by one flipped bit in the
    signature, key or message: the product's host batch against
    crypto_sign_ed25519_verify_detached item by item."""
    s, lib = na
    rng = np.random.default_rng(20251018)
    n = 10_000
    pks, sigs, msgs = [], [], []
    for i in range(n):
        pk, sk = _sodium_keypair(s, rng.bytes(32))
        m = rng.bytes(int(rng.integers(0, 700)))
        sig = _sodium_sign(s, sk, m)
        if rng.integers(0, 8) == 0:
            what = int(rng.integers(0, 3))
            if what == 0:
                b = bytearray(sig)
                b[int(rng.integers(0, 64))] ^= 1 << int(rng.integers(0, 8))
                sig = bytes(b)
            elif what == 1:
                b = bytearray(pk)
                b[int(rng.integers(0, 32))] ^= 1 << int(rng.integers(0, 8))
                pk = bytes(b)
            elif m:
                b = bytearray(m)
                b[int(rng.integers(0, len(m)))] ^= 1 << int(rng.integers(0, 8))
                m = bytes(b)
        pks.append(pk)
        sigs.append(sig)
        msgs.append(m)
    want = np.array([_sodium_verify(s, g, m, k) for k, g, m in zip(pks, sigs, msgs)])
    assert 0.8 * n < want.sum() < n
    # messages one byte apart from the previous one's end: unaligned offsets
    parts, off, at = [], np.zeros(n, np.uint64), 0
    for i, m in enumerate(msgs):
        parts.append(b"\x5a" * (i % 3))
        at += i % 3
        off[i] = at
        parts.append(m)
        at += len(m)
    buf = np.frombuffer(b"".join(parts) + b"\0", np.uint8)
    ln = np.array([len(m) for m in msgs], np.uint32)
    pk_a = np.frombuffer(b"".join(pks), np.uint8)
    sg_a = np.frombuffer(b"".join(sigs), np.uint8)
    v = np.zeros(n, np.uint8)
    assert lib.ouro_ed25519_verify_batch_host(n, O.p(pk_a), O.p(sg_a), O.p(buf), O.p(off),
                                              O.p(ln), O.p(v)) == 0
    np.testing.assert_array_equal(v.astype(bool), want)
    # and the single-item route on a sample
    for i in range(0, n, 97):
        assert (lib.ouro_ed25519_verify(sigs[i], msgs[i], len(msgs[i]), pks[i]) == 0) == want[i]


# ---- a draft-03 prover from libsodium's primitives --------------------------

def _sc(x: int) -> bytes:
    return (x % L).to_bytes(32, "little")


class SodiumVRF:
    """ECVRF-ED25519-SHA512-Elligator2 (draft-03) written with libsodium
    1.0.18's public primitives only: H from
    crypto_core_ed25519_from_uniform on SHA-512(0x04 || 0x01 || Y || alpha)'s
    first 32 bytes with bit 255 cleared, the nonce SHA-512(h[32:64] || H)
    mod L, c the first 16 bytes of SHA-512(0x04 || 0x02 || H || Gamma ||
    kB || kH), s = k + c x mod L, beta = SHA-512(0x04 || 0x03 || [8]Gamma)."""

    def __init__(self, s):
        self.s = s

    def _mul(self, k: bytes, p: bytes) -> bytes:
        out = ctypes.create_string_buffer(32)
        assert self.s.crypto_scalarmult_ed25519_noclamp(out, k, p) == 0
        return out.raw

    def _base(self, k: bytes) -> bytes:
        out = ctypes.create_string_buffer(32)
        assert self.s.crypto_scalarmult_ed25519_base_noclamp(out, k) == 0
        return out.raw

    def hash_to_curve(self, y: bytes, alpha: bytes) -> bytes:
        r = bytearray(hashlib.sha512(b"\x04\x01" + y + alpha).digest()[:32])
        r[31] &= 0x7F
        h = ctypes.create_string_buffer(32)
        assert self.s.crypto_core_ed25519_from_uniform(h, bytes(r)) == 0
        return h.raw

    def keypair(self, seed: bytes):
        hsk = hashlib.sha512(seed).digest()
        x = bytearray(hsk[:32])
        x[0] &= 248
        x[31] &= 127
        x[31] |= 64
        xi = int.from_bytes(bytes(x), "little")
        return self._base(_sc(xi)), (xi % L, hsk[32:])

    def prove(self, sk, y: bytes, alpha: bytes) -> bytes:
        x, trunc = sk
        H = self.hash_to_curve(y, alpha)
        gamma = self._mul(_sc(x), H)
        k = int.from_bytes(hashlib.sha512(trunc + H).digest(), "little") % L
        c = hashlib.sha512(b"\x04\x02" + H + gamma + self._base(_sc(k))
                           + self._mul(_sc(k), H)).digest()[:16]
        s = (k + int.from_bytes(c, "little") * x) % L
        return gamma + c + s.to_bytes(32, "little")

    def beta(self, proof: bytes) -> bytes:
        return hashlib.sha512(b"\x04\x03" + self._mul(_sc(8), proof[:32])).digest()


def test_sodium_prover_reproduces_the_draft03_vectors(na, kats):
    """The libsodium-built prover is right: it reproduces the IETF draft-03
    vectors' pk, proof and beta byte for byte."""
    s, _ = na
    vrf = SodiumVRF(s)
    for v in kats["vrf_draft03"]:
        pk, sk = vrf.keypair(bytes.fromhex(v["sk"])[:32])
        assert pk.hex() == v["pk"]
        pi = vrf.prove(sk, pk, bytes.fromhex(v["alpha"]))
        assert pi.hex() == v["pi"]
        assert vrf.beta(pi).hex() == v["beta"]


def test_vrf_random_inputs_against_sodium_prover(na):
    """Elligator2 on 3,000 random inputs: honest proofs over random alphas
    (each alpha a fresh uniform Elligator2 input) from the libsodium-built
    prover verify on the product's host path (single items and the host
    batch) with libsodium's beta; one flipped bit anywhere in 1/8 of the
    proofs is rejected."""
    s, lib = na
    vrf = SodiumVRF(s)
    rng = np.random.default_rng(7)
    keys = [vrf.keypair(rng.bytes(32)) for _ in range(16)]
    n = 3000
    pks, proofs, alphas, want_ok, want_beta = [], [], [], [], []
    for i in range(n):
        pk, sk = keys[i % 16]
        alpha = rng.bytes(32)
        pi = vrf.prove(sk, pk, alpha)
        ok = True
        if rng.integers(0, 8) == 0:
            b = bytearray(pi)
            b[int(rng.integers(0, 80))] ^= 1 << int(rng.integers(0, 8))
            pi = bytes(b)
            ok = False
        pks.append(pk)
        proofs.append(pi)
        alphas.append(alpha)
        want_ok.append(ok)
        want_beta.append(vrf.beta(pi) if ok else bytes(64))
    want_ok = np.array(want_ok)
    pk_a = np.frombuffer(b"".join(pks), np.uint8)
    pr_a = np.frombuffer(b"".join(proofs), np.uint8)
    al_a = np.frombuffer(b"".join(alphas), np.uint8)
    off = (np.arange(n) * 32).astype(np.uint64)
    ln = np.full(n, 32, np.uint32)
    beta = np.zeros((n, 64), np.uint8)
    v = np.zeros(n, np.uint8)
    assert lib.ouro_vrf03_verify_batch_host(n, O.p(pk_a), O.p(pr_a), O.p(al_a), O.p(off),
                                            O.p(ln), O.p(beta), O.p(v), 0) == 0
    np.testing.assert_array_equal(v.astype(bool), want_ok)
    for i in np.nonzero(want_ok)[0]:
        assert bytes(beta[i]) == want_beta[i], i
    out = ctypes.create_string_buffer(64)
    for i in range(0, n, 53):
        rc = lib.ouro_vrf03_verify(out, pks[i], proofs[i], alphas[i], 32)
        assert (rc == 0) == want_ok[i]
        if want_ok[i]:
            assert out.raw == want_beta[i]
            assert lib.ouro_vrf03_proof_to_hash(out, proofs[i]) == 0 and out.raw == want_beta[i]
