/*
 * ed25519.c -- Ed25519 sign/verify for the oracle.  TEST INFRASTRUCTURE ONLY.
 *
 * orc_ed25519_verify restates libsodium 1.0.18
 * _crypto_sign_ed25519_verify_detached (non-ED25519_COMPAT build), the C
 * function behind cardano-crypto-class Ed25519DSIGN.verifyDSIGN (SURVEY.md
 * §8(a) row a1, App. B.1).  Reference call sites: the OCERT rule via
 * ouroboros-consensus-shelley/src/Ouroboros/Consensus/Shelley/Protocol.hs:435,
 * the SingleKES leaf (Shelley/Ledger/Integrity.hs:27), and the Cardano
 * DSIGN ~ Ed25519DSIGN constraint at
 * ouroboros-consensus-cardano/src/Ouroboros/Consensus/Cardano/CanHardFork.hs:360.
 *
 * orc_ed25519_verify_byron restates the donna-derived cardano-crypto verify
 * behind ByronDSIGN (ouroboros-consensus-byron/src/Ouroboros/Consensus/Byron/
 * Crypto/DSIGN.hs:110-113): parity pinned by the one Byron
 * golden header only.
 */
#include "internal.h"
#include <string.h>

void orc_ed25519_seed_keypair(uint8_t pk[32], uint8_t sk[64], const uint8_t seed[32]) {
  uint8_t h[64];
  ge A;
  orc_sha512(h, seed, 32);
  h[0] &= 248;
  h[31] &= 127;
  h[31] |= 64;
  ge_scalarmult_base(&A, h);
  ge_tobytes(pk, &A);
  memcpy(sk, seed, 32);
  memcpy(sk + 32, pk, 32);
}

void orc_ed25519_sign(uint8_t sig[64], const uint8_t *m, size_t mlen, const uint8_t sk[64]) {
  uint8_t az[64], nonce[64], hram[64], r[32], k[32];
  orc_sha512_ctx c;
  ge R;
  orc_sha512(az, sk, 32);
  az[0] &= 248;
  az[31] &= 127;
  az[31] |= 64;
  orc_sha512_init(&c);
  orc_sha512_update(&c, az + 32, 32);
  orc_sha512_update(&c, m, mlen);
  orc_sha512_final(&c, nonce);
  sc_reduce(r, nonce, 64);
  ge_scalarmult_base(&R, r);
  ge_tobytes(sig, &R);
  orc_sha512_init(&c);
  orc_sha512_update(&c, sig, 32);
  orc_sha512_update(&c, sk + 32, 32);
  orc_sha512_update(&c, m, mlen);
  orc_sha512_final(&c, hram);
  sc_reduce(k, hram, 64);
  sc_muladd(sig + 32, k, az, r);
}

/* R' = [h](-A) + [S]B, compared byte-exactly with R */
static int verify_core(const uint8_t sig[64], const uint8_t *m, size_t mlen, const uint8_t pk[32],
                       const ge *negA) {
  uint8_t hram[64], h[32], rcheck[32];
  orc_sha512_ctx c;
  ge Rp;
  orc_sha512_init(&c);
  orc_sha512_update(&c, sig, 32);
  orc_sha512_update(&c, pk, 32);
  orc_sha512_update(&c, m, mlen);
  orc_sha512_final(&c, hram);
  sc_reduce(h, hram, 64);
  ge_double_scalarmult(&Rp, h, negA, sig + 32, &cc()->B);
  ge_tobytes(rcheck, &Rp);
  return memcmp(rcheck, sig, 32) == 0 ? 0 : -1;
}

int orc_ed25519_verify(const uint8_t sig[64], const uint8_t *m, size_t mlen,
                       const uint8_t pk[32]) {
  ge negA;
  if (!sc_is_canonical(sig + 32) || ge_has_small_order(sig)) return -1;
  if (!ge_is_canonical(pk) || ge_has_small_order(pk)) return -1;
  if (ge_frombytes_negate(&negA, pk) != 0) return -1;
  return verify_core(sig, m, mlen, pk, &negA);
}

int orc_ed25519_verify_byron(const uint8_t sig[64], const uint8_t *m, size_t mlen,
                             const uint8_t pk[32]) {
  ge negA;
  if (sig[63] & 0xE0) return -1;
  if (ge_frombytes_negate(&negA, pk) != 0) return -1;
  return verify_core(sig, m, mlen, pk, &negA);
}
