"""mkSeed, mkNonceFromNumber and the nonce fold, CPU.

Pinning: the reference's golden ChainDepState
(ouroboros-consensus-shelley-test/test/golden/disk/ChainDepState, committed
as data in tests/golden/reference_kats.json by tools/make_golden.py) is built
at ouroboros-consensus-shelley-test/src/Test/Consensus/Shelley/Examples.hs:520-537
with every Nonce = SL.mkNonceFromNumber 1 -- that pins mkNonceFromNumber, the
function that makes seedEta (0) and seedL (1).  The composition around it
(mkSeed's BE64(slot) || eta0 hash XOR seed, UPDN, Nonce <>) follows the
un-vendored shelley-spec-ledger as restated in oracle/nonce.py and
oracle/tpraos.c: PARITY UNPINNED by any reference fixture, checked here
between three independent statements (oracle C, oracle Python, device code
compiled for the host) and, on the GPU, the kernels (test_gpu_claims.py).
"""
import ctypes
import hashlib
import os
import subprocess

import numpy as np
import pytest

import oracle_ffi as O
from ouroboros_network_amd import header as H

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DH = os.path.join(ROOT, "ouroboros-network_amd", "lib", "libouro_devhost_test.so")
ON = O.nonce_module()


def _cbor_nonces(buf: bytes):
    """Every Nonce value [1, bytes(32)] and NeutralNonce [0] in a CBOR item."""
    found, neutral = [], 0

    def walk(i):
        nonlocal neutral
        mt, arg, j = H._head(buf, i)
        if mt == 4 and arg >= 0:
            items = H.array_items(buf, i)
            if arg == 2:
                m0, a0, _ = H._head(buf, items[0][0])
                m1, a1, k1 = H._head(buf, items[1][0])
                if m0 == 0 and a0 == 1 and m1 == 2 and a1 == 32:
                    found.append(bytes(buf[k1:k1 + 32]))
                    return items[-1][1]
            if arg == 1:
                m0, a0, _ = H._head(buf, items[0][0])
                if m0 == 0 and a0 == 0:
                    neutral += 1
            for a, _ in items:
                walk(a)
            return items[-1][1] if items else j
        if mt == 5 and arg >= 0:
            k = j
            for _ in range(2 * arg):
                k = walk(k)
            return k
        if mt == 6:
            return walk(j)
        return H.skip(buf, i)

    walk(0)
    return found, neutral


def test_mk_nonce_from_number_pinned_by_golden_chain_dep_state(kats):
    cds = kats["chain_dep_state"]
    nonces, neutral = _cbor_nonces(bytes.fromhex(cds["raw"]))
    k = cds["nonce_number"]
    assert len(nonces) >= 4 and neutral >= 1  # csTickn has one NeutralNonce
    want = O.mk_nonce_from_number(k)
    assert all(x == want for x in nonces)
    assert want == hashlib.blake2b(k.to_bytes(8, "big"), digest_size=32).digest()
    assert ON.mk_nonce_from_number(k) == want
    # the seeds mkSeed uses (same function, 0 and 1)
    assert H.SEED_L == want == O.mk_nonce_from_number(1)
    assert H.SEED_ETA == O.mk_nonce_from_number(0) == ON.mk_nonce_from_number(0)


@pytest.fixture(scope="module")
def dh():
    if not os.path.exists(DH):
        subprocess.run(["make", "-C", os.path.join(ROOT, "ouroboros-network_amd"),
                        "lib/libouro_devhost_test.so"], check=True, stdout=subprocess.DEVNULL)
    lib = ctypes.CDLL(DH)
    lib.dh_mk_seed.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_uint64, ctypes.c_void_p]
    return lib


def test_mk_seed_device_code_equals_oracles(dh):
    """hdr_seed (the header kernels' path) = oracle C = oracle Python =
    header.mk_seed, for edge and random slots, with and without eta0."""
    rng = np.random.default_rng(5)
    slots = [0, 1, 9, 255, 256, 2**32 - 1, 2**32, 2**63, 2**64 - 1] + \
        [int(x) for x in rng.integers(0, 2**63, 40, dtype=np.int64)]
    out = ctypes.create_string_buffer(32)
    for s in slots:
        for eta0 in (None, rng.bytes(32), bytes(32)):
            for leader, uc in ((0, H.SEED_ETA), (1, H.SEED_L)):
                want = O.mk_seed(uc, s, eta0)
                assert want == ON.mk_seed(uc, s, eta0) == H.mk_seed(uc, s, eta0)
                dh.dh_mk_seed(out, leader, s, eta0)
                assert out.raw == want, (s, leader, eta0)
    # NeutralNonce ucNonce: no XOR
    assert O.mk_seed(None, 7, None) == hashlib.blake2b((7).to_bytes(8, "big"),
                                                       digest_size=32).digest()


def test_nonce_fold_matches_restatement():
    """ouro_nonce_fold (product, host-only) = oracle/nonce.py's UPDN fold:
    random eta nonces, slots on both sides of the stability-window cut,
    Neutral and non-Neutral starting states, n = 0."""
    from ouroboros_network_amd.tpraos import nonce_fold

    rng = np.random.default_rng(17)
    fsne, sp = 432000, 129600
    for trial in range(60):
        n = int(rng.integers(0, 40))
        etas = [rng.bytes(32) for _ in range(n)]
        base = int(rng.integers(fsne - sp - 30, fsne - sp + 10))
        slots = sorted(base + int(x) for x in rng.integers(0, 40, n))
        ev = None if trial % 3 == 0 else rng.bytes(32)
        ec = None if trial % 4 == 0 else rng.bytes(32)
        got = nonce_fold(np.frombuffer(b"".join(etas), np.uint8), np.array(slots, np.uint64),
                         fsne, sp, ev, ec)
        assert got == ON.fold(ev, ec, etas, slots, fsne, sp)
    # SlotNo arithmetic is Word64: s + sp wraps exactly as in the reference
    e = rng.bytes(32)
    assert nonce_fold(np.frombuffer(e, np.uint8), np.array([2**64 - 5], np.uint64), 10, 7,
                      None, None) == ON.fold(None, None, [e], [2**64 - 5], 10, 7) == (e, e)


def test_header_batch_optional_members():
    from ouroboros_network_amd.tpraos import HeaderBatch

    n = 4
    z = lambda w: np.zeros((n, w), np.uint8)  # noqa: E731
    base = dict(issuer_vk=z(32), vrf_vk=z(32), eta_proof=z(80), leader_proof=z(80),
                hot_vk=z(32), ocert_counter=np.zeros(n, np.uint64),
                ocert_kes_period=np.zeros(n, np.uint64), ocert_sigma=z(64),
                kes_t=np.zeros(n, np.uint32), kes_sig=z(448), body=np.zeros(8, np.uint8),
                body_off=np.zeros(n, np.uint64), body_len=np.zeros(n, np.uint32))
    with pytest.raises(ValueError):
        HeaderBatch(eta_alpha=None, leader_alpha=None, **base)  # no alphas, no slots
    hb = HeaderBatch(eta_alpha=None, leader_alpha=None, slot=np.arange(n, dtype=np.uint64),
                     epoch_nonce=np.arange(32, dtype=np.uint8), eta_output=z(64),
                     leader_output=z(64), **base)
    s = hb.c_struct()
    assert s.eta_alpha is None and s.slot and s.epoch_nonce and s.eta_output and not s.eta_nonce
    part = hb.rows([3, 1])
    assert list(part.slot) == [3, 1] and np.shares_memory(part.epoch_nonce, hb.epoch_nonce)
    assert part.eta_output.shape == (2, 64) and part.eta_alpha is None
    with pytest.raises(ValueError):
        HeaderBatch(eta_alpha=z(32), leader_alpha=z(32), epoch_nonce=np.zeros(31, np.uint8),
                    **base)
    with pytest.raises(ValueError):  # a uint64 offset + length that wraps is caught
        HeaderBatch(eta_alpha=z(32), leader_alpha=z(32),
                    **{**base, "body_off": np.full(n, 2**64 - 2, np.uint64),
                       "body_len": np.full(n, 4, np.uint32)})


def test_pack_seeded_and_claimed(kats):
    hs = kats["headers"]
    parsed = [H.parse_header(bytes.fromhex(h["raw"])) for h in hs]
    b = H.pack(parsed, seeds=True, epoch_nonce=bytes(range(32)), slots_per_kes_period=100)
    assert b.eta_alpha is None and list(b.slot) == [p.slot for p in parsed]
    assert bytes(b.eta_output[0]) == parsed[0].eta_output
    b2 = H.pack(parsed, [bytes(32)] * len(parsed), [bytes(32)] * len(parsed), 100, claimed=False)
    assert b2.eta_output is None and b2.slot is None
    with pytest.raises(ValueError):
        H.pack(parsed, None, None, 100)
