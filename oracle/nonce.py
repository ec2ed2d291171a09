"""Nonce evolution restated in plain Python -- TEST INFRASTRUCTURE ONLY.

The host-side fold that follows the header crypto in SL.updateChainDepState
(reached via ouroboros-consensus-shelley/src/Ouroboros/Consensus/Shelley/Protocol.hs:433-442),
from shelley-spec-ledger (un-vendored; cabal.project:168-187):
  * PRTCL: eta = mkNonceFromOutputVRF (certifiedOutput bheaderEta), i.e.
    Blake2b-256 of the header's CLAIMED 64-byte eta output;
  * UPDN (Updn.hs): with s the header slot, sp the stability window and
    firstSlotNextEpoch the first slot of the epoch after s's,
        if s +* Duration sp < firstSlotNextEpoch
            then (eta_v <> eta, eta_v <> eta)   -- candidate follows
            else (eta_v <> eta, eta_c)          -- candidate frozen
  * Nonce composition (BaseTypes.hs): Nonce a <> Nonce b = Nonce
    (Blake2b-256(a || b)); x <> NeutralNonce = x; NeutralNonce <> x = x.
None stands for NeutralNonce.  Only tests/ import this file.
"""
import hashlib

MASK64 = (1 << 64) - 1


def blake2b_256(m: bytes) -> bytes:
    return hashlib.blake2b(m, digest_size=32).digest()


def mk_nonce_from_number(k: int) -> bytes:
    return blake2b_256(k.to_bytes(8, "big"))


def mk_nonce_from_output_vrf(out64: bytes) -> bytes:
    return blake2b_256(out64)


def compose(a, b):
    if a is None:
        return b
    if b is None:
        return a
    return blake2b_256(a + b)


def mk_seed(uc, slot: int, eta0) -> bytes:
    h = blake2b_256(slot.to_bytes(8, "big") + (eta0 or b""))
    return h if uc is None else bytes(x ^ y for x, y in zip(h, uc))


def updn(eta_v, eta_c, eta: bytes, slot: int, first_slot_next_epoch: int, sp: int):
    new_v = compose(eta_v, eta)
    if ((slot + sp) & MASK64) < first_slot_next_epoch:  # SlotNo is a Word64
        return new_v, new_v
    return new_v, eta_c


def fold(eta_v, eta_c, etas, slots, first_slot_next_epoch: int, sp: int):
    for eta, s in zip(etas, slots):
        eta_v, eta_c = updn(eta_v, eta_c, eta, int(s), first_slot_next_epoch, sp)
    return eta_v, eta_c
