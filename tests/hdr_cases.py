"""Header batches for the header-combiner tests (CPU and GPU), built from the
reference's golden headers (tests/golden/reference_kats.json).

* golden_variants: the 7 golden headers plus decodable single-byte
  corruptions of the first (every `stride`-th byte of its body and KES
  signature), VRF inputs as the golden examples use them
  (Examples.hs:457-458), claimed outputs carried (or not);
* seeded: the golden headers re-proved for mkSeed inputs -- the golden VRF
  key is the seed 32 x 0x01 key -- so the device derives
  alpha from (slot, eta0); plus rows with a wrong slot, a wrong proof and
  forged claimed outputs;
* forge_claims: valid proofs with the claimed output changed (the
  ref2020-vs-strict split of SURVEY.md App. B.3).
"""
import numpy as np

import oracle_ffi as O
from ouroboros_network_amd import header as H

GOLDEN_VRF_SEED = b"\x01" * 32
L = 2**252 + 27742317777372353535851937790883648493


def with_s_plus_l(proof: bytes) -> bytes:
    """The same proof with s replaced by s + L: draft-03 as the fork reads it
    (s reduced mod L) still verifies it; a strict-s reading rejects it
    (the OURO_HDR_*_S_UNREDUCED bits)."""
    s = int.from_bytes(proof[48:80], "little")
    return proof[:48] + (s + L).to_bytes(32, "little")


def golden_variants(kats, stride=1, claimed=True, s_rows=True):
    hs = kats["headers"]
    parsed = [H.parse_header(bytes.fromhex(h["raw"])) for h in hs]
    ea = [bytes.fromhex(h["eta_alpha"]) for h in hs]
    la = [bytes.fromhex(h["leader_alpha"]) for h in hs]
    raw = bytes.fromhex(hs[0]["raw"])
    for off in range(parsed[0].body_span[0], len(raw), stride):
        r = bytearray(raw)
        r[off] = (r[off] + 1) & 0xFF
        try:
            parsed.append(H.parse_header(bytes(r)))
        except Exception:
            continue  # no longer decodes: the reference rejects before crypto
        ea.append(ea[0])
        la.append(la[0])
    batch = H.pack(parsed, ea, la, slots_per_kes_period=100, claimed=claimed)
    if not s_rows:
        return batch
    # the first golden header three more times: the eta proof's s, the
    # leader proof's s, both, replaced by s + L
    rows = batch.rows([0, 0, 0])
    ep, lp = rows.eta_proof.copy(), rows.leader_proof.copy()
    for r, (e, l) in enumerate(((1, 0), (0, 1), (1, 1))):
        if e:
            ep[r] = np.frombuffer(with_s_plus_l(ep[r].tobytes()), np.uint8)
        if l:
            lp[r] = np.frombuffer(with_s_plus_l(lp[r].tobytes()), np.uint8)
    extra = rows.with_(eta_proof=ep, leader_proof=lp)
    return concat(batch, extra)


def concat(a, b):
    """Rows of a then rows of b (b's body offsets rebased past a's body)."""
    from dataclasses import fields

    kw = {}
    for f in fields(a):
        x, y = getattr(a, f.name), getattr(b, f.name)
        if f.name == "body":
            kw[f.name] = np.concatenate([x, y])
        elif f.name == "body_off":
            kw[f.name] = np.concatenate([x, y + np.uint64(a.body.size)])
        elif f.name == "epoch_nonce":
            kw[f.name] = x
        elif x is None:
            kw[f.name] = None
        else:
            kw[f.name] = np.concatenate([x, y])
    return type(a)(**kw)


def forge_claims(batch, rng, frac=4):
    """Copy of `batch` with one byte of the claimed eta or leader output
    changed on 1/frac of the rows; returns (batch, forged row indices)."""
    eo, lo = batch.eta_output.copy(), batch.leader_output.copy()
    idx = np.nonzero(rng.integers(0, frac, len(batch)) == 0)[0]
    idx = np.union1d(idx, [0])  # a golden row: valid proofs, forged output
    for i in idx:
        a = eo if rng.integers(0, 2) else lo
        a[i, rng.integers(0, 64)] ^= 1 << int(rng.integers(0, 8))
    return batch.with_(eta_output=eo, leader_output=lo), idx


def seeded(kats, epoch_nonce, copies=4, rng=None):
    """Golden headers with VRF proofs over mkSeed seedEta/seedL slot eta0, the
    slots varied per copy (epoch_nonce None = NeutralNonce)."""
    rng = rng or np.random.default_rng(3)
    _, sk = O.vrf_keypair(GOLDEN_VRF_SEED)
    hs = kats["headers"]
    parsed = [H.parse_header(bytes.fromhex(h["raw"])) for h in hs] * copies
    slots = [int(x) for x in rng.integers(0, 2**40, len(parsed))]
    slots[0], slots[1] = 0, 2**64 - 1
    batch = H.pack(parsed, seeds=True, epoch_nonce=epoch_nonce, slots_per_kes_period=100)
    ep, lp = batch.eta_proof.copy(), batch.leader_proof.copy()
    eo, lo = batch.eta_output.copy(), batch.leader_output.copy()
    for i, s in enumerate(slots):
        for uc, proofs, outs in ((H.SEED_ETA, ep, eo), (H.SEED_L, lp, lo)):
            pi = O.vrf_prove(sk, O.mk_seed(uc, s, epoch_nonce))
            proofs[i] = np.frombuffer(pi, np.uint8)
            outs[i] = np.frombuffer(O.vrf_proof_to_hash(pi), np.uint8)
    sl = np.array(slots, np.uint64)
    sl[2] += 1            # proofs for another slot: both VRFs fail
    ep[3, 70] ^= 4        # a corrupted eta proof
    lo[4, 5] ^= 1         # a forged claimed leader output on a valid proof
    eo[5, 63] ^= 0x80     # a forged claimed eta output on a valid proof
    return batch.with_(eta_proof=ep, leader_proof=lp, eta_output=eo, leader_output=lo, slot=sl)


# SHA-512 block boundaries of the KES leaf message R || A || body (64 + len
# bytes): lengths around every nb-block limit (64 + len + 17 = 128 nb), up to
# past the latency mode's wave-hash capacity (8 blocks: len <= 943), and 0.
KES_BODY_LENGTHS = [0, 1, 7, 8, 46, 47, 48, 49, 111, 112, 175, 176, 303, 431, 544, 559, 560,
                    687, 815, 942, 943, 944, 1000, 1200]


def kes_body_lengths(kats, lengths=KES_BODY_LENGTHS, seed=b"\x07" * 32):
    """The first golden header re-signed for bodies of the given lengths: a
    fresh Sum6KES key (hot vk), its OCERT signed by the golden cold key (the
    seed 32 x 0x01 key), the body random bytes, the KES
    signature over it at the header's period.  Each length twice: valid, and
    with one body byte (or, for the empty body, one leaf-signature byte)
    changed after signing, so that KES alone fails."""
    import dataclasses

    h0 = H.parse_header(bytes.fromhex(kats["headers"][0]["raw"]))
    cold_pk, cold_sk = O.ed25519_keypair(GOLDEN_VRF_SEED)
    assert cold_pk == h0.issuer_vk
    hot = O.kes_keygen(seed)
    t = H.kes_t(h0.slot, 100, h0.ocert_kes_period)
    ocert_msg = hot + h0.ocert_counter.to_bytes(8, "big") + h0.ocert_kes_period.to_bytes(8, "big")
    sigma = O.ed25519_sign(cold_sk, ocert_msg)
    rng = np.random.default_rng(2024)
    rows = []
    for n in lengths:
        body = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        sig = O.kes_sign(seed, t, body)
        rows.append(dataclasses.replace(h0, hot_vk=hot, ocert_sigma=sigma, body=body, kes_sig=sig))
        if n:
            bad = bytearray(body)
            bad[(n * 7) // 11] ^= 0x10
            rows.append(dataclasses.replace(rows[-1], body=bytes(bad)))
        else:  # nothing to change in an empty body: the leaf signature's R
            bad = bytearray(sig)
            bad[5] ^= 0x10
            rows.append(dataclasses.replace(rows[-1], kes_sig=bytes(bad)))
    ea = [bytes.fromhex(kats["headers"][0]["eta_alpha"])] * len(rows)
    la = [bytes.fromhex(kats["headers"][0]["leader_alpha"])] * len(rows)
    return H.pack(rows, ea, la, slots_per_kes_period=100)


# ---- raw wire headers (for the raw-CBOR entries) ------------------------------
def _cbor_head(mt: int, v: int) -> bytes:
    if v < 24:
        return bytes([mt << 5 | v])
    for ai, w in ((24, 1), (25, 2), (26, 4), (27, 8)):
        if v < 1 << (8 * w):
            return bytes([mt << 5 | ai]) + v.to_bytes(w, "big")
    raise ValueError(v)


def cbor_uint(v: int) -> bytes:
    return _cbor_head(0, v)


def cbor_bytes(b: bytes) -> bytes:
    return _cbor_head(2, len(b)) + b


def wire_header(fields, kes_sig: bytes, era=None) -> bytes:
    """[header_body, kes_sig] CBOR-in-CBOR wrapped as N2N v1 (#6.24 bytes), or
    as the Cardano HFC form [era, #6.24 bytes] when era is given
    (ouroboros-network/test/messages.cddl:27-34).  `fields` are the 15 encoded
    header_body items."""
    body = _cbor_head(4, 15) + b"".join(fields)
    inner = b"\x82" + body + cbor_bytes(kes_sig)
    wrapped = b"\xd8\x18" + cbor_bytes(inner)
    return wrapped if era is None else b"\x82" + cbor_uint(era) + wrapped


def seeded_raw(kats, epoch_nonce, n, spkp=100, rng=None, era_every=3):
    """n raw wire headers that verify completely under mkSeed inputs: the first
    golden header's fields re-encoded with a slot per header, both VRF certs
    proved by the golden VRF key (seed 32 x 0x01) over
    mkSeed seedEta / seedL slot eta0 (epoch_nonce None = NeutralNonce), a fresh
    Sum6KES key whose OCERT the golden cold key signs, and the KES signature at
    t = slot // spkp - kesPeriod over the re-encoded body.  Every era_every-th
    header is HFC-wrapped.  Returns (list of raw headers, slots)."""
    rng = rng or np.random.default_rng(11)
    h0 = H.parse_header(bytes.fromhex(kats["headers"][0]["raw"]))
    f0 = H.array_items(h0.body, 0)
    keep = lambda k: h0.body[f0[k][0]:f0[k][1]]  # noqa: E731
    cold_pk, cold_sk = O.ed25519_keypair(GOLDEN_VRF_SEED)
    _, vrf_sk = O.vrf_keypair(GOLDEN_VRF_SEED)
    kes_seed = b"\x05" * 32
    hot = O.kes_keygen(kes_seed)
    out, slots = [], []
    for i in range(n):
        slot = int(rng.integers(0, 2**40)) if i % 5 else int(rng.integers(0, 2**20))
        t = int(rng.integers(0, 64))
        c0 = max(0, slot // spkp - t)
        t = slot // spkp - c0
        counter = int(rng.integers(0, 2**16))
        sigma = O.ed25519_sign(cold_sk, hot + counter.to_bytes(8, "big") + c0.to_bytes(8, "big"))
        certs = []
        for uc in (H.SEED_ETA, H.SEED_L):
            pi = O.vrf_prove(vrf_sk, O.mk_seed(uc, slot, epoch_nonce))
            certs.append(b"\x82" + cbor_bytes(O.vrf_proof_to_hash(pi)) + cbor_bytes(pi))
        fields = [keep(0), cbor_uint(slot), keep(2), cbor_bytes(cold_pk), keep(4), certs[0],
                  certs[1], keep(7), keep(8), cbor_bytes(hot), cbor_uint(counter), cbor_uint(c0),
                  cbor_bytes(sigma), keep(13), keep(14)]
        body = _cbor_head(4, 15) + b"".join(fields)
        sig = O.kes_sign(kes_seed, min(t, 63) if t < 64 else 63, body)
        out.append(wire_header(fields, sig, era=(2 if i % era_every == 0 else None)))
        slots.append(slot)
    return out, np.array(slots, np.uint64)
