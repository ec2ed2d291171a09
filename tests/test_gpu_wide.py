"""The wave-wide arithmetic of the latency mode (csrc/wide.h) against the
lane-local routines it replaces, on the device: conversions, products,
squaring chains, z^(2^252-3), doubling, addition/subtraction, [s]P against
double-and-add, the identity, and the latency mode's [s]H item (wide_vrf.h).  One wave per case (random + edge field
elements: p - 1, 0); csrc/wide_test.hip is a test-only library.  The
latency items' Elligator2 and encoding are also checked against the oracle
directly (test_wide_elligator2_matches_oracle), and their inversion against
exact Python integers (test_wide_invert_matches_python); the wave [s]P and
its encoding against exact affine arithmetic, torsion components included
(test_wide_scalarmult_matches_python); the wave SHA-512 against hashlib
(test_wide_sha512_matches_hashlib)."""
import ctypes
import os

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "ouroboros-network_amd", "lib", "libouro_wide_test.so")
NAMES = ["convert", "mul", "sq_chain", "pow22523", "dbl", "add_sub", "scalarmult", "identity",
         "vrf_sh_H", "vrf_sh_V"]


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [1, 0x5eed])
def test_wide_arithmetic_matches_lane_routines(gpu_lib, seed):
    lib = ctypes.CDLL(LIB)
    lib.ouro_wide_selftest.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]
    waves = 512
    out = np.zeros(waves * len(NAMES), dtype=np.int32)
    dbg = np.zeros(24, dtype=np.int32)
    assert lib.ouro_wide_selftest(waves, seed, out.ctypes.data, dbg.ctypes.data) == 0
    res = out.reshape(waves, len(NAMES))
    bad = {NAMES[t]: int((res[:, t] != 1).sum()) for t in range(len(NAMES))}
    assert all(v == 0 for v in bad.values()), (bad, dbg.tolist())


@pytest.mark.gpu
def test_wide_elligator2_matches_oracle(gpu_lib):
    """The latency items' hash-to-curve (wide_cores.h elligator2_wide, cofactor
    cleared) and one-point encoding (encode1_wide: the vector-pass conversion
    and the three zero tests) against the oracle's Elligator2
    (oracle/vrf03.c orc_elligator2_from_uniform, pinned to libsodium's
    crypto_core_ed25519_from_uniform in test_oracle.py), byte for byte.
    Inputs as the VRF hands them over (top bit clear): zero, small values,
    the non-canonical range p .. 2^255 - 1 and seeded random strings."""
    import oracle_ffi as O

    p = 2**255 - 19
    vals = [0, 1, 2, 3, 4, 5, p - 1, p, p + 1, p + 7, 2**255 - 1]
    rs = [v.to_bytes(32, "little") for v in vals]
    rng = np.random.default_rng(11)
    for _ in range(245):
        r = bytearray(rng.bytes(32))
        r[31] &= 0x7F
        rs.append(bytes(r))
    n = len(rs)
    lib = ctypes.CDLL(LIB)
    lib.ouro_wide_elligator2.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_void_p]
    out = ctypes.create_string_buffer(32 * n)
    assert lib.ouro_wide_elligator2(n, b"".join(rs), out) == 0
    bad = [i for i in range(n) if out.raw[32 * i:32 * i + 32] != O.elligator2(rs[i])]
    assert not bad, [rs[i].hex() for i in bad[:4]]


@pytest.mark.gpu
def test_wide_invert_matches_python(gpu_lib):
    """The latency encodings' inversion (wide_inv.h fe_invert_wave: divsteps
    with the operand updates on the lanes, early exit, 0 -> 0) against exact
    Python integers, pow(z, p - 2, p), on inputs read as fe_from_words does
    (bit 255 ignored): 0, 1, 2, p - 1, p (= 0), p + 1 .. 2^255 - 1
    (non-canonical), powers of two and seeded random words."""
    p = 2**255 - 19
    vals = [0, 1, 2, 19, p - 2, p - 1, p, p + 1, p + 18, 2**255 - 1, 2**254, 2**128, 2**64 - 1]
    rng = np.random.default_rng(12)
    for _ in range(243):
        vals.append(int.from_bytes(rng.bytes(32), "little"))
    n = len(vals)
    zb = b"".join(v.to_bytes(32, "little") for v in vals)
    lib = ctypes.CDLL(LIB)
    lib.ouro_wide_invert.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_void_p]
    out = ctypes.create_string_buffer(32 * n)
    assert lib.ouro_wide_invert(n, zb, out) == 0
    bad = []
    for i, v in enumerate(vals):
        z = (v & (2**255 - 1)) % p
        want = pow(z, p - 2, p)  # 0 for z = 0, as the kernel documents
        if int.from_bytes(out.raw[32 * i:32 * i + 32], "little") != want:
            bad.append(hex(v))
    assert not bad, bad[:4]


@pytest.mark.gpu
def test_wide_scalarmult_matches_python(gpu_lib):
    """The latency chains' [s]P on the wave (wide.h pw_scalarmult: table,
    signed width-4 windows, additions, doublings) and encode1_wide against
    exact affine arithmetic in Python (edge_cases.smul), s reduced mod L as
    the kernel reads it: prime-order points, the identity, an order-8 point and
    mixed-order points (a torsion component the chain must carry exactly),
    scalars 0, 1, L - 1, L, L + 1, 2^256 - 1 and seeded random ones."""
    import edge_cases as E

    rng = np.random.default_rng(13)
    rnd = lambda: int.from_bytes(rng.bytes(32), "little")  # noqa: E731
    pts = [E.BASE, (0, 1), E.T8, ((-E.BASE[0]) % E.P, E.BASE[1])]
    for _ in range(6):
        pts.append(E.smul(rnd() % E.L, E.BASE))
    pts.append(E.add(E.smul(rnd() % E.L, E.BASE), E.T8))
    pts.append(E.add(E.BASE, E.smul(3, E.T8)))
    scal = [0, 1, E.L - 1, E.L, E.L + 1, 2**256 - 1]
    cases = [(pt, s) for pt in pts[:4] for s in scal]
    for pt in pts:
        for _ in range(3):
            cases.append((pt, rnd()))
    n = len(cases)
    pe = b"".join(E.enc_pt(pt) for pt, _ in cases)
    sc = b"".join(s.to_bytes(32, "little") for _, s in cases)
    lib = ctypes.CDLL(LIB)
    lib.ouro_wide_scalarmult.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_char_p,
                                         ctypes.c_void_p, ctypes.c_void_p]
    out = ctypes.create_string_buffer(32 * n)
    ok = np.zeros(n, dtype=np.int32)
    assert lib.ouro_wide_scalarmult(n, pe, sc, out, ok.ctypes.data) == 0
    assert ok.all()
    bad = [i for i, (pt, s) in enumerate(cases)
           if out.raw[32 * i:32 * i + 32] != E.enc_pt(E.smul(s % E.L, pt))]
    assert not bad, [(E.enc_pt(cases[i][0]).hex(), hex(cases[i][1])) for i in bad[:3]]


@pytest.mark.gpu
def test_wide_sha512_matches_hashlib(gpu_lib):
    """The latency items' wave SHA-512 (sha512.h sha512_prefixed_wave: every
    block's schedule on its own lane, the rounds from LDS) against hashlib:
    a 64-byte prefix plus a global-memory tail of every length around the
    block and padding boundaries up to the wave form's 8 blocks, and the
    tail's two-messages-per-wave form over 130-byte challenge strings."""
    import hashlib

    rng = np.random.default_rng(14)
    lens = sorted({0, 1, 7, 8, 46, 47, 48, 49, 63, 64, 65, 110, 111, 112, 113, 127, 128,
                   175, 176, 177, 239, 240, 241, 367, 368, 544, 623, 624, 751, 752, 879, 880, 943})
    n = len(lens)
    pre = rng.bytes(64 * n)
    msg = bytearray(1024 * n)
    for i, ln in enumerate(lens):
        msg[1024 * i:1024 * i + ln] = rng.bytes(ln)
    lib = ctypes.CDLL(LIB)
    lib.ouro_wide_sha512_prefixed.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_char_p,
                                              ctypes.c_void_p, ctypes.c_void_p]
    ln_arr = np.array(lens, dtype=np.uint32)
    out = ctypes.create_string_buffer(64 * n)
    assert lib.ouro_wide_sha512_prefixed(n, pre, bytes(msg), ln_arr.ctypes.data, out) == 0
    bad = [ln for i, ln in enumerate(lens)
           if out.raw[64 * i:64 * i + 64]
           != hashlib.sha512(pre[64 * i:64 * i + 64] + bytes(msg[1024 * i:1024 * i + ln])).digest()]
    assert not bad, bad

    pairs = 16
    msgs = [rng.bytes(130) for _ in range(2 * pairs)]
    lib.ouro_wide_sha512_130_pairs.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_void_p]
    out2 = ctypes.create_string_buffer(64 * 2 * pairs)
    assert lib.ouro_wide_sha512_130_pairs(pairs, b"".join(m + b"\0\0" for m in msgs), out2) == 0
    bad2 = [i for i, m in enumerate(msgs) if out2.raw[64 * i:64 * i + 64] != hashlib.sha512(m).digest()]
    assert not bad2, bad2
