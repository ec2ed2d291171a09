"""The kernels' lane routines (verify.h), compiled for the host by hipcc, against
the oracle and exact integer arithmetic (CPU-only; no GPU needed).

This checks the arithmetic the gfx950 kernels execute -- same source, same
limb representation -- before any GPU time is spent.  It is not the product
path: the product library only runs these routines inside kernels.
"""
import ctypes
import os
import subprocess

import numpy as np
import pytest

import hdr_cases as HC
import oracle_ffi as O
from edge_cases import ed25519_edge_cases, vrf_edge_cases

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# OURO_DEVHOST_LIB: the ASan/UBSan build (tests/test_sanitizers.py)
SO = os.environ.get("OURO_DEVHOST_LIB") or os.path.join(
    ROOT, "ouroboros-network_amd", "lib", "libouro_devhost_test.so")
P = 2**255 - 19
L = 2**252 + 27742317777372353535851937790883648493


@pytest.fixture(scope="module")
def dh():
    if not os.path.exists(SO):
        subprocess.run(["make", "-C", os.path.join(ROOT, "ouroboros-network_amd"),
                        "lib/libouro_devhost_test.so"], check=True, stdout=subprocess.DEVNULL)
    return ctypes.CDLL(SO)


def enc(x):
    return (x % P).to_bytes(32, "little")


def dec(b):
    return int.from_bytes(b, "little")


def test_field_ops(dh):
    rng = np.random.default_rng(0)
    out = ctypes.create_string_buffer(32)
    specials = [0, 1, 2, P - 1, P - 2, 19, 2**255 - 20, 2**254, (P - 1) // 2]
    vals = specials + [int.from_bytes(rng.bytes(32), "little") % P for _ in range(300)]
    for i, x in enumerate(vals):
        y = vals[(7 * i + 3) % len(vals)]
        dh.dh_fe_mul(out, enc(x), enc(y))
        assert dec(out.raw) == x * y % P
        dh.dh_fe_sq(out, enc(x))
        assert dec(out.raw) == x * x % P
        dh.dh_fe_sub(out, enc(x), enc(y))
        assert dec(out.raw) == (x - y) % P
    for x in specials[1:6] + vals[20:40]:
        dh.dh_fe_invert(out, enc(x))
        assert dec(out.raw) == pow(x, P - 2, P)


def test_invert_vartime(dh):
    """modinv.h's divsteps inversion equals z^(p-2) (0 -> 0) on edge values,
    random canonical values, values >= p and unreduced limb vectors."""
    rng = np.random.default_rng(5)
    out = ctypes.create_string_buffer(32)
    specials = [0, 1, 2, 3, 19, P - 1, P - 2, (P - 1) // 2, (P + 1) // 2, 2**254, 2**255 - 20,
                2**128 - 1, 2**30, 2**30 - 1, 2**240 + 1, 5**100 % P]
    vals = specials + [int.from_bytes(rng.bytes(32), "little") % P for _ in range(3000)]
    vals += [int.from_bytes(rng.bytes(32), "little") >> int(rng.integers(0, 250))
             for _ in range(500)]
    for x in vals:
        dh.dh_fe_invert_vartime(out, enc(x % P))
        assert dec(out.raw) == pow(x, P - 2, P), x
        # the latency mode's divsteps, at most 10 bits per step (wide_inv.h)
        dh.dh_fe_invert_vartime_cap10(out, enc(x % P))
        assert dec(out.raw) == pow(x, P - 2, P), x
        dh.dh_fe_invert_vartime_sel(out, enc(x % P))
        assert dec(out.raw) == pow(x, P - 2, P), x
        dh.dh_fe_invert_vartime_spec(out, enc(x % P))
        assert dec(out.raw) == pow(x, P - 2, P), x
    E = [0, 26, 51, 77, 102, 128, 153, 179, 204, 230]
    for _ in range(500):
        top = int(rng.choice([1 << 26, 1 << 28, 1 << 31]))
        limbs = [int(rng.integers(0, top)) for _ in range(10)]
        arr = (ctypes.c_uint32 * 10)(*limbs)
        dh.dh_fe_invert_vartime_limbs(out, arr)
        x = sum(l << E[i] for i, l in enumerate(limbs)) % P
        assert dec(out.raw) == pow(x, P - 2, P)


def test_tobytes_canonicalises_unreduced_limbs(dh):
    """fe_to_words on unsigned limb vectors at and beyond the 'reduced' bounds
    (anything below 2^31 per limb)."""
    rng = np.random.default_rng(1)
    E = [0, 26, 51, 77, 102, 128, 153, 179, 204, 230]
    out = ctypes.create_string_buffer(32)
    for _ in range(500):
        top = int(rng.choice([1 << 26, 1 << 28, 1 << 31]))
        limbs = [int(rng.integers(0, top)) for _ in range(10)]
        arr = (ctypes.c_uint32 * 10)(*limbs)
        dh.dh_fe_limbs_tobytes(out, arr)
        want = sum(l << E[i] for i, l in enumerate(limbs)) % P
        assert dec(out.raw) == want


def test_table_entry_packing(dh):
    """verify.h fe_pack256 / fe_unpack256 (the per-lane table entries, one
    128-B line each): every limb vector the tables store (limbs < 2^28) packs
    to 256 bits congruent to it mod p, and unpacks to limbs within their
    widths (limb 9 within 26 bits) whose value is exactly the packed word."""
    rng = np.random.default_rng(11)
    E = [0, 26, 51, 77, 102, 128, 153, 179, 204, 230]
    words = (ctypes.c_uint32 * 8)()
    back = (ctypes.c_uint32 * 10)()
    cases = [[(1 << 28) - 1] * 10, [0] * 10, [(1 << 26) - 1, (1 << 25) - 1] * 5,
             [1 << 26, 1 << 25] * 5, [(1 << 26) - 19] + [(1 << 25) - 1, (1 << 26) - 1] * 4 + [(1 << 25) - 1]]
    for _ in range(2000):
        top = int(rng.choice([1 << 25, 1 << 26, 1 << 27, 1 << 28]))
        cases.append([int(rng.integers(0, top)) for _ in range(10)])
    for limbs in cases:
        dh.dh_fe_pack256(words, back, (ctypes.c_uint32 * 10)(*limbs))
        w = sum(int(x) << (32 * i) for i, x in enumerate(words))
        x = sum(l << E[i] for i, l in enumerate(limbs))
        assert w % P == x % P
        out = list(back)
        assert all(out[i] < (1 << (26 if i % 2 == 0 else 25)) for i in range(9))
        assert out[9] < (1 << 26)
        assert sum(l << E[i] for i, l in enumerate(out)) == w


def test_scalar_reduce(dh):
    rng = np.random.default_rng(2)
    out = ctypes.create_string_buffer(32)
    for v in [b"\xff" * 64, bytes(64), L.to_bytes(64, "little"), (L - 1).to_bytes(64, "little"),
              (2 * L).to_bytes(64, "little")] + [rng.bytes(64) for _ in range(200)]:
        dh.dh_sc_reduce64(out, v)
        assert dec(out.raw) == dec(v) % L


def _half(dh, h):
    c0 = ctypes.create_string_buffer(32)
    c1 = ctypes.create_string_buffer(32)
    neg = ctypes.c_int(0)
    bits = dh.dh_half_scalars(h.to_bytes(32, "little"), c0, c1, ctypes.byref(neg))
    a, b = dec(c0.raw), dec(c1.raw)
    return (-a if neg.value else a), b, bits


def test_half_scalars(dh):
    """lattice.h: c0 = c1 h (mod 8L), c1 odd, and both about half size -- the
    conditions under which the half-size Ed25519 equation is equivalent to
    libsodium's (the relation and parity are what correctness rests on; the
    size only decides speed)."""
    rng = np.random.default_rng(5)
    hs = [0, 1, 2, 3, 8, L - 1, L - 2, 2**252, 2**128, 2**128 + 1, 2**127, (L - 1) // 2,
          8 * 3**80 % L, 2**200 + 7]
    rand = [int.from_bytes(rng.bytes(64), "little") % L for _ in range(3000)]
    sizes = []
    for k, h in enumerate(hs + rand):
        c0, c1, bits = _half(dh, h)
        assert c1 % 2 == 1 and 0 < c1 < L
        assert (c0 - c1 * h) % (8 * L) == 0
        assert max(abs(c0).bit_length(), c1.bit_length()) == bits
        if k >= len(hs):
            sizes.append(bits)
    # structured h (L - 1, 2^252, ...) have no short odd vector and use (h, 1);
    # hash outputs do: about half size
    assert max(sizes) <= 142 and np.median(sizes) <= 128, (max(sizes), np.median(sizes))


def test_half_scalars_v2_equals_v1(dh):
    """lattice.h's round-6 Lehmer step (32-bit cofactor magnitudes, a
    Newton-refined reciprocal; the product path) makes the same quotients and
    breaks as the round-1 step, so the pairs are identical bit for bit: on
    structured values and 20,000 random h < 2^253 (uniform, and below L)."""
    rng = np.random.default_rng(21)
    hs = [0, 1, 2, 3, 8, L - 1, L - 2, 2**252, 2**253 - 1, 2**128, 2**128 + 1, 2**127,
          (L - 1) // 2, 8 * 3**80 % L, 2**200 + 7, 2**129 - 1, 3 * 2**160 + 5]
    hs += [int.from_bytes(rng.bytes(32), "little") >> 3 for _ in range(10000)]
    hs += [int.from_bytes(rng.bytes(64), "little") % L for _ in range(10000)]
    bufs = [ctypes.create_string_buffer(32) for _ in range(4)]
    n1, n2 = ctypes.c_int(0), ctypes.c_int(0)
    for h in hs:
        hb = h.to_bytes(32, "little")
        b2 = dh.dh_half_scalars(hb, bufs[0], bufs[1], ctypes.byref(n2))
        b1 = dh.dh_half_scalars_v1(hb, bufs[2], bufs[3], ctypes.byref(n1))
        assert (b2, bufs[0].raw, bufs[1].raw, n2.value) == (b1, bufs[2].raw, bufs[3].raw,
                                                            n1.value), hex(h)


def test_hashes(dh):
    import hashlib

    rng = np.random.default_rng(3)
    out = ctypes.create_string_buffer(64)
    for n in [0, 1, 47, 48, 49, 63, 64, 65, 175, 176, 177, 544, 1000]:
        pre, m = rng.bytes(64), rng.bytes(n)
        dh.dh_sha512_prefixed64(out, pre, m, n)
        assert out.raw == hashlib.sha512(pre + m).digest()
    x = rng.bytes(64)
    dh.dh_blake2b256_64(out, x)
    assert out.raw[:32] == hashlib.blake2b(x, digest_size=32).digest()


def test_elligator2(dh):
    rng = np.random.default_rng(4)
    out = ctypes.create_string_buffer(32)
    for _ in range(40):
        r = bytearray(rng.bytes(32))
        r[31] &= 0x7F
        dh.dh_elligator2(out, bytes(r))
        assert out.raw == O.elligator2(bytes(r))


def test_ed25519_lane(dh):
    pk, sig, msg = O.synth_ed25519(48, first=9)
    for i in range(48):
        s = bytearray(sig[i])
        if i % 3 == 1:
            s[i % 64] ^= 0x10
        m = bytes(msg[i])
        assert (dh.dh_ed25519_verify(bytes(s), m, len(m), bytes(pk[i])) == 0) == \
            O.ed25519_verify(bytes(s), m, bytes(pk[i]))


def test_ed25519_lane_edge_cases(dh):
    for pk, sig, m in ed25519_edge_cases():
        assert (dh.dh_ed25519_verify(sig, m, len(m), pk) == 0) == O.ed25519_verify(sig, m, pk)


def test_vrf_lane(dh, kats):
    out = ctypes.create_string_buffer(64)
    for v in kats["vrf_draft03"]:
        a = bytes.fromhex(v["alpha"])
        assert dh.dh_vrf03_verify(out, bytes.fromhex(v["pk"]), bytes.fromhex(v["pi"]), a, len(a)) == 0
        assert out.raw.hex() == v["beta"]
    for pk, pi, a in vrf_edge_cases():
        rc = dh.dh_vrf03_verify(out, pk, pi, a, len(a))
        want = O.vrf_verify(pk, pi, a)
        assert (rc == 0) == (want is not None)
        if want is not None:
            assert out.raw == want


def test_kes_lane_golden(dh, kats):
    from ouroboros_network_amd import header as H

    for h in kats["headers"]:
        hd = H.parse_header(bytes.fromhex(h["raw"]))
        assert dh.dh_sum6kes_verify(hd.hot_vk, 0, hd.body, len(hd.body), hd.kes_sig) == 0
        assert dh.dh_sum6kes_verify(hd.hot_vk, 1, hd.body, len(hd.body), hd.kes_sig) != 0


def _run_drivers(dh, batch, mode, nonce=False):
    n = len(batch)
    en = np.zeros((n, 32), np.uint8) if nonce else None
    s = batch.c_struct(en)
    verdict = np.zeros(n, np.uint8)
    be = np.zeros((n, 64), np.uint8)
    bl = np.zeros((n, 64), np.uint8)
    dh.dh_tpraos_verify.argtypes = [ctypes.c_void_p, ctypes.c_int] + [ctypes.c_void_p] * 3
    assert dh.dh_tpraos_verify(ctypes.addressof(s), mode, O.p(verdict), O.p(be), O.p(bl)) == 0
    return verdict, be, bl, en


def _oracle(batch, nonce=False):
    n = len(batch)
    en = np.zeros((n, 32), np.uint8) if nonce else None
    s = batch.c_struct(en)
    verdict = np.zeros(n, np.uint8)
    be = np.zeros((n, 64), np.uint8)
    bl = np.zeros((n, 64), np.uint8)
    O.lib().orc_tpraos_verify_batch(ctypes.addressof(s), O.p(verdict), O.p(be), O.p(bl), 8)
    return verdict, be, bl, en


MODES = pytest.mark.parametrize("mode", [0, 1, 2, 3],
                                ids=["throughput", "latency", "latency_quad", "split_phases"])


@MODES
def test_header_drivers(dh, kats, mode):
    """tpraos.h's cores + single-inversion finish, in the throughput schedule
    (one lane, VRF key table shared) and the latency schedule (a lane per
    core), equal the oracle's verdict bits and outputs."""
    batch = HC.golden_variants(kats, stride=7)
    got = _run_drivers(dh, batch, mode)
    want = _oracle(batch)
    for g, w in zip(got[:3], want[:3]):
        np.testing.assert_array_equal(g, w)
    for h, v in zip(kats["headers"], got[0]):
        assert int(v) & 0x0F == h["expect_verdict"]
        assert int(v) & 0x30 == 0x30  # claimed outputs = computed (golden)
    assert (got[0] & 0x0F != 15).sum() > 10


@MODES
def test_header_drivers_claims_seeds_nonces(dh, kats, mode):
    """The optional members: forged claimed outputs on valid proofs (PROOF bit
    set, CLAIM bit clear), no claimed outputs (no CLAIM bits), VRF inputs
    derived on the device from (slot, eta0) incl. NeutralNonce, and the
    eta_nonce output -- all equal to the oracle."""
    rng = np.random.default_rng(21)
    forged, idx = HC.forge_claims(HC.golden_variants(kats, stride=23), rng)
    cases = [forged, HC.golden_variants(kats, stride=23, claimed=False),
             HC.seeded(kats, bytes(range(32)), copies=2),
             HC.seeded(kats, None, copies=1)]
    for batch in cases:
        got = _run_drivers(dh, batch, mode, nonce=True)
        want = _oracle(batch, nonce=True)
        for g, w in zip(got, want):
            np.testing.assert_array_equal(g, w)
    v = _run_drivers(dh, forged, mode)[0]
    assert ((v[idx] & 0x0F) == 15).sum() > 0 and ((v[idx] & 0x30) != 0x30).all()
    sv = _run_drivers(dh, cases[2], mode)[0]
    assert list(sv[:6]) == [0x3F, 0x3F, 0x03, 0x2B, 0x1F, 0x2F]


def test_zero_bound_violations(dh):
    """Every multiplier input seen by the tests above stayed inside the limb
    bounds fe25519.h's overflow analysis assumes (run last in this module)."""
    dh.dh_bound_violations.restype = ctypes.c_ulonglong
    # exercise the VRF / Elligator paths once more on fresh random inputs
    rng = np.random.default_rng(99)
    out = ctypes.create_string_buffer(32)
    for _ in range(200):
        r = bytearray(rng.bytes(32))
        r[31] &= 0x7F
        dh.dh_elligator2(out, bytes(r))
    assert dh.dh_bound_violations() == 0
