"""Pin the CPU oracle before trusting it (CPU-only).

* SHA-512 / Blake2b against hashlib and libsodium 1.0.18 (the reference CI's
  pin, conda copy) -- differential, random lengths incl. block boundaries.
* Ed25519 keygen/sign/verify and Elligator2 against libsodium 1.0.18,
  including the fixed edge-case set.
* VRF against the IETF draft-03 vectors (verify, output, and the prover).
* Everything against the reference's golden headers / witnesses / Byron sig.
"""
import ctypes
import hashlib

import numpy as np
import pytest

import oracle_ffi as O
from edge_cases import ed25519_edge_cases, small_order_encodings

sodium = O.sodium()
needs_sodium = pytest.mark.skipif(sodium is None, reason="libsodium 1.0.18 not in this image")


def test_hashes_match_hashlib():
    rng = np.random.default_rng(0)
    for n in [0, 1, 63, 64, 111, 112, 127, 128, 129, 239, 240, 255, 256, 1000]:
        m = rng.bytes(n)
        assert O.sha512(m) == hashlib.sha512(m).digest()
        assert O.blake2b_256(m) == hashlib.blake2b(m, digest_size=32).digest()


@needs_sodium
def test_ed25519_against_libsodium():
    rng = np.random.default_rng(1)
    for i in range(64):
        seed = rng.bytes(32)
        pk, sk = O.ed25519_keypair(seed)
        pk2, sk2 = ctypes.create_string_buffer(32), ctypes.create_string_buffer(64)
        sodium.crypto_sign_ed25519_seed_keypair(pk2, sk2, seed)
        assert pk == pk2.raw
        m = rng.bytes(int(rng.integers(0, 300)))
        sig = O.ed25519_sign(sk, m)
        s2 = ctypes.create_string_buffer(64)
        sodium.crypto_sign_ed25519_detached(s2, None, m, ctypes.c_ulonglong(len(m)), sk2)
        assert sig == s2.raw
        bad = bytearray(sig)
        bad[i % 64] = (bad[i % 64] + 1) & 0xFF
        for s in (sig, bytes(bad)):
            want = sodium.crypto_sign_ed25519_verify_detached(s, m, ctypes.c_ulonglong(len(m)), pk) == 0
            assert O.ed25519_verify(s, m, pk) == want


@needs_sodium
def test_ed25519_edge_cases_against_libsodium():
    for pk, sig, m in ed25519_edge_cases():
        want = sodium.crypto_sign_ed25519_verify_detached(sig, m, ctypes.c_ulonglong(len(m)), pk) == 0
        assert O.ed25519_verify(sig, m, pk) == want, (pk.hex(), sig.hex())


@needs_sodium
def test_small_order_blocklist_matches_libsodium():
    # crypto_core_ed25519_is_valid_point rejects small order (and non-canonical)
    for e in small_order_encodings():
        assert sodium.crypto_core_ed25519_is_valid_point(e) == 0


@needs_sodium
def test_elligator2_against_libsodium():
    rng = np.random.default_rng(2)
    for _ in range(64):
        r = bytearray(rng.bytes(32))
        r[31] &= 0x7F
        want = ctypes.create_string_buffer(32)
        sodium.crypto_core_ed25519_from_uniform(want, bytes(r))
        assert O.elligator2(bytes(r)) == want.raw


def test_vrf_draft03_vectors(kats):
    for v in kats["vrf_draft03"]:
        pk, sk = O.vrf_keypair(bytes.fromhex(v["sk"]))
        assert pk.hex() == v["pk"]
        alpha = bytes.fromhex(v["alpha"])
        assert O.vrf_prove(sk, alpha).hex() == v["pi"]
        assert O.vrf_verify(pk, bytes.fromhex(v["pi"]), alpha).hex() == v["beta"]
        assert O.vrf_proof_to_hash(bytes.fromhex(v["pi"])).hex() == v["beta"]
        assert O.vrf_verify(pk, bytes.fromhex(v["pi"]), alpha + b"\0") is None


def test_golden_headers(kats):
    from ouroboros_network_amd import header as H

    for h in kats["headers"]:
        hd = H.parse_header(bytes.fromhex(h["raw"]))
        msg = hd.hot_vk + hd.ocert_counter.to_bytes(8, "big") + hd.ocert_kes_period.to_bytes(8, "big")
        assert O.ed25519_verify(hd.ocert_sigma, msg, hd.issuer_vk)
        assert O.kes_verify(hd.hot_vk, h["kes_t"], hd.body, hd.kes_sig)
        assert not O.kes_verify(hd.hot_vk, h["kes_t"] + 1, hd.body, hd.kes_sig)
        be = O.vrf_verify(hd.vrf_vk, hd.eta_proof, bytes.fromhex(h["eta_alpha"]))
        bl = O.vrf_verify(hd.vrf_vk, hd.leader_proof, bytes.fromhex(h["leader_alpha"]))
        assert be.hex() == h["expect_beta_eta"]
        assert bl.hex() == h["expect_beta_leader"]


def test_golden_header_examples_keys(kats):
    """Examples.hs:167-194: DSIGN and VRF keys come from seed 32 x 0x01."""
    from ouroboros_network_amd import header as H

    hd = H.parse_header(bytes.fromhex(kats["headers"][0]["raw"]))
    pk, _ = O.ed25519_keypair(b"\x01" * 32)
    assert hd.issuer_vk == pk
    vpk, vsk = O.vrf_keypair(b"\x01" * 32)
    assert hd.vrf_vk == vpk
    # the prover reproduces the golden eta proof bit-exactly
    assert O.vrf_prove(vsk, bytes.fromhex(kats["headers"][0]["eta_alpha"])) == hd.eta_proof


def test_golden_tx_witnesses_and_byron(kats):
    for w in kats["tx_witnesses"]:
        assert O.ed25519_verify(bytes.fromhex(w["sig"]), bytes.fromhex(w["msg"]), bytes.fromhex(w["pk"]))
    b = kats["byron"]
    assert O.ed25519_verify_byron(bytes.fromhex(b["sig"]), bytes.fromhex(b["msg"]), bytes.fromhex(b["pk"]))


def test_kes_sign_verify_roundtrip():
    seed = bytes(range(32))
    vk = O.kes_keygen(seed)
    for t in (0, 1, 31, 32, 63):
        m = b"body-%d" % t
        sig = O.kes_sign(seed, t, m)
        assert O.kes_verify(vk, t, m, sig)
        assert not O.kes_verify(vk, (t + 1) % 64, m, sig)
        assert not O.kes_verify(vk, t, m + b"!", sig)


def test_threaded_batches_equal_serial():
    pk, sig, msg = O.synth_ed25519(256, first=5, threads=4)
    buf = msg.reshape(-1)
    off = np.arange(256, dtype=np.uint64) * 32
    ln = np.full(256, 32, np.uint32)
    sig[7, 3] ^= 1
    got = O.ed25519_verify_batch(pk, sig, buf, off, ln, threads=4)
    want = np.array([O.ed25519_verify(bytes(sig[i]), bytes(msg[i]), bytes(pk[i])) for i in range(256)])
    np.testing.assert_array_equal(got, want)
    assert got.sum() == 255
