"""Fixed edge-case sets for Ed25519 and the draft-03 VRF (SURVEY.md §4, §7
step 1): the acceptance corners libsodium 1.0.18 pins (S >= L, the 7
small-order encodings with and without the sign bit, non-canonical y, the x = 0
sign-bit case, undecodable points, mixed-order keys, the identity-key and
identity-Gamma forgeries) plus honest items around them.  Points are built
with exact integer arithmetic here; the expected verdicts come from the oracle
at test time.
"""
from __future__ import annotations

import hashlib

import oracle_ffi as O

P = 2**255 - 19
L = 2**252 + 27742317777372353535851937790883648493
D = (-121665 * pow(121666, P - 2, P)) % P
SQRTM1 = pow(2, (P - 1) // 4, P)


def enc_int(y: int, sign: int = 0) -> bytes:
    b = bytearray(y.to_bytes(32, "little"))
    b[31] |= sign << 7
    return bytes(b)


def recover_x(y: int, sign: int):
    x2 = (y * y - 1) * pow(D * y * y + 1, P - 2, P) % P
    x = pow(x2, (P + 3) // 8, P)
    if (x * x - x2) % P:
        x = x * SQRTM1 % P
    if (x * x - x2) % P:
        return None
    if x & 1 != sign:
        x = (-x) % P
    return x


def add(p1, p2):
    (x1, y1), (x2, y2) = p1, p2
    t = D * x1 * x2 * y1 * y2 % P
    return ((x1 * y2 + y1 * x2) * pow(1 + t, P - 2, P) % P,
            (y1 * y2 + x1 * x2) * pow(1 - t, P - 2, P) % P)


def enc_pt(pt) -> bytes:
    x, y = pt
    return enc_int(y, x & 1)


def dec_pt(b: bytes):
    y = int.from_bytes(b, "little") & ((1 << 255) - 1)
    return (recover_x(y, b[31] >> 7), y)


Y8 = 0x05FC536D880238B13933C6D305ACDFD5F098EFF289F4C345B027B2C28F95E826
SMALL_Y = [0, 1, Y8, P - Y8, P - 1, P, P + 1]
T8 = (recover_x(Y8, 0), Y8)  # an order-8 point


def smul(k: int, pt):
    """[k]pt by double-and-add (exact, slow; test data only)."""
    acc = (0, 1)
    while k:
        if k & 1:
            acc = add(acc, pt)
        pt = add(pt, pt)
        k >>= 1
    return acc


BASE = (recover_x(4 * pow(5, P - 2, P) % P, 0), 4 * pow(5, P - 2, P) % P)


def torsion_consistent_cases(per_order: int = 2):
    """Signatures over a mixed-order key A = aB + T_A whose R carries exactly
    the torsion -[h]T_A, so that [S]B - [h]A == R holds exactly: cofactorless
    verification (libsodium 1.0.18) accepts them, and a verifier that reduced
    the coefficient of A modulo L instead of 8L would not.  Also the same
    signatures with R's torsion off by one step (rejected).  T_A of order 2, 4
    and 8.  [(pk, sig, msg)]"""
    out = []
    rng_seed = 0
    for k in (4, 2, 1):  # [k]T8 has order 8 / k
        TA = smul(k, T8)
        made = 0
        while made < per_order:
            rng_seed += 1
            a = int.from_bytes(hashlib.sha512(b"tors-a%d" % rng_seed).digest(), "little") % L
            r = int.from_bytes(hashlib.sha512(b"tors-r%d" % rng_seed).digest(), "little") % L
            A = add(smul(a, BASE), TA)
            pk = enc_pt(A)
            msg = b"torsion %d" % rng_seed
            rB = smul(r, BASE)
            for j in range(8):
                R = add(rB, smul(j, T8))
                Rb = enc_pt(R)
                h = int.from_bytes(hashlib.sha512(Rb + pk + msg).digest(), "little") % L
                # [j]T8 == -[h k]T8  <=>  j = -h k (mod 8)
                if (j + h * k) % 8 == 0:
                    S = (r + h * a) % L
                    out.append((pk, Rb + S.to_bytes(32, "little"), msg))
                    Rw = enc_pt(add(R, T8))
                    hw = int.from_bytes(hashlib.sha512(Rw + pk + msg).digest(), "little") % L
                    Sw = (r + hw * a) % L
                    out.append((pk, Rw + Sw.to_bytes(32, "little"), msg))
                    made += 1
                    break
    return out


def small_order_encodings():
    out = []
    for y in SMALL_Y:
        for s in (0, 1):
            out.append(enc_int(y, s))
    return out


def non_square_y() -> int:
    y = 2
    while recover_x(y, 0) is not None:
        y += 1
    return y


def ed25519_edge_cases():
    """[(pk, sig, msg)]"""
    cases = []
    seed = hashlib.sha512(b"edge").digest()[:32]
    pk, sk = O.ed25519_keypair(seed)
    msg = b"edge-case message"
    sig = O.ed25519_sign(sk, msg)
    R, S = sig[:32], int.from_bytes(sig[32:], "little")
    cases.append((pk, sig, msg))                                   # honest
    cases.append((pk, sig, b""))                                   # wrong msg
    cases.append((pk, R + (S + L).to_bytes(32, "little"), msg))    # S + L
    cases.append((pk, R + L.to_bytes(32, "little"), msg))          # S = L
    cases.append((pk, R + (L - 1).to_bytes(32, "little"), msg))
    cases.append((pk, R + b"\xff" * 32, msg))
    for e in small_order_encodings():
        cases.append((pk, e + sig[32:], msg))                      # small-order R
        cases.append((e, sig, msg))                                # small-order A
        cases.append((e, e + bytes(32), msg))                      # A = R small, S = 0
    # identity-key forgery (OpenSSL accepts, libsodium must reject)
    ident = enc_int(1)
    cases.append((ident, ident + bytes(32), msg))
    # non-canonical A: y + p for small y that decode
    for y in range(2, 19):
        if recover_x(y, 0) is not None:
            cases.append((enc_int(y + P), sig, msg))
    # undecodable A and R
    ns = non_square_y()
    cases.append((enc_int(ns), sig, msg))
    cases.append((pk, enc_int(ns) + sig[32:], msg))
    # non-canonical R (y >= p) of a real R
    ry = int.from_bytes(R, "little") & ((1 << 255) - 1)
    if ry + P < 2**255:
        cases.append((pk, enc_int(ry + P, R[31] >> 7) + sig[32:], msg))
    # mixed-order key A + T8 with the honest signature
    A = dec_pt(pk)
    cases.append((enc_pt(add(A, T8)), sig, msg))
    # honest signatures over a mixed-order key: sign with scalar, publish A+T
    # (cofactorless verification decides; the oracle gives the answer)
    # every byte of the honest signature flipped in turn
    for j in range(0, 64, 7):
        b = bytearray(sig)
        b[j] ^= 0x40
        cases.append((pk, bytes(b), msg))
    # sign bit of pk flipped
    b = bytearray(pk)
    b[31] ^= 0x80
    cases.append((bytes(b), sig, msg))
    # mixed-order keys with torsion-consistent R (accepted) and off-by-one R
    cases += torsion_consistent_cases()
    return cases


def vrf_edge_cases():
    """[(pk, proof, alpha)]"""
    seed = hashlib.sha512(b"vrf-edge").digest()[:32]
    pk, sk = O.vrf_keypair(seed)
    out = []
    for alpha in (b"", b"\x00", bytes(32), bytes(range(200))):
        pi = O.vrf_prove(sk, alpha)
        out.append((pk, pi, alpha))
        out.append((pk, pi, alpha + b"\x01"))
        G, c, s = pi[:32], pi[32:48], int.from_bytes(pi[48:], "little")
        if s + L < 2**256:
            out.append((pk, G + c + (s + L).to_bytes(32, "little"), alpha))  # s + L
        b = bytearray(pi)
        b[33] ^= 1
        out.append((pk, bytes(b), alpha))                                   # c changed
    alpha = b"edge"
    pi = O.vrf_prove(sk, alpha)
    for e in small_order_encodings():
        out.append((e, pi, alpha))                    # small-order pk
        out.append((pk, e + pi[32:], alpha))          # small-order Gamma (decodes; c fails)
    ns = non_square_y()
    out.append((enc_int(ns), pi, alpha))
    out.append((pk, enc_int(ns) + pi[32:], alpha))
    for y in range(2, 19):
        if recover_x(y, 0) is not None:
            out.append((enc_int(y + P), pi, alpha))   # non-canonical pk
            out.append((pk, enc_int(y + P) + pi[32:], alpha))  # non-canonical Gamma
            break
    # universal forgery attempt with the identity key (must be rejected by the
    # key check): Gamma = I, s = 0, c = H(4,2,H,I,I,I)[:16]
    ident = enc_int(1)
    out.append((ident, ident + bytes(16) + bytes(32), alpha))
    # Gamma with x = 0 and the sign bit set (y = 1 -> identity)
    out.append((pk, enc_int(1, 1) + pi[32:], alpha))
    return out
