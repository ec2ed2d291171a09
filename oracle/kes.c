/*
 * kes.c -- Sum6KES (SumKES^6 over SingleKES Ed25519DSIGN, Blake2b_256) for the
 * oracle.  TEST INFRASTRUCTURE ONLY.
 *
 * Restates cardano-crypto-class SumKES.verifyKES / SingleKES.verifyKES
 * (SURVEY.md §8(a) row a3, App. B.2), reached from
 * ouroboros-consensus-shelley/src/Ouroboros/Consensus/Shelley/Ledger/Integrity.hs:27
 * (SL.verifySignedKES () ocertVkHot t hdrBody hdrSignature) and from the OCERT
 * rule via Shelley/Protocol.hs:435.  Pinned by the three golden Shelley /
 * Allegra / Mary headers (tests/golden/).
 *
 * Signature layout (rawSerialiseSigKES of SumKES, recursively sigma || vk0 || vk1):
 *   sig[0:64] = leaf Ed25519 signature, then for level k = 1..6 (bottom-up) the
 *   pair (vk0_k, vk1_k) at offset 64 + 64 (k - 1).
 */
#include "internal.h"
#include <string.h>

int orc_sum6kes_verify(const uint8_t vk[32], uint32_t t, const uint8_t *m, size_t mlen,
                       const uint8_t sig[ORC_KES_SIGBYTES]) {
  uint8_t cur[32], h[32];
  memcpy(cur, vk, 32);
  for (int k = ORC_KES_DEPTH; k >= 1; k--) {
    const uint8_t *pair = sig + 64 + 64 * (k - 1);
    orc_blake2b_256(h, pair, 64);
    if (memcmp(h, cur, 32) != 0) return -1;
    uint32_t half = 1u << (k - 1);
    if (t < half) {
      memcpy(cur, pair, 32);
    } else {
      memcpy(cur, pair + 32, 32);
      t -= half;
    }
  }
  /* SingleKES: assert (t == 0) is compiled out; the leaf is plain Ed25519 */
  return orc_ed25519_verify(sig, m, mlen, cur);
}

/* ---- synthetic tree (test data only) ----
 * leaf i seed = SHA-512(tree seed || LE32(i))[0:32]; the device synthesiser
 * (ouroboros-network_amd/csrc/synth.hip) derives the same keys. */
static void leaf_seed(uint8_t out[32], const uint8_t seed[32], uint32_t i) {
  uint8_t buf[36], h[64];
  memcpy(buf, seed, 32);
  buf[32] = (uint8_t)i;
  buf[33] = (uint8_t)(i >> 8);
  buf[34] = (uint8_t)(i >> 16);
  buf[35] = (uint8_t)(i >> 24);
  orc_sha512(h, buf, sizeof buf);
  memcpy(out, h, 32);
}

/* level[0] = 64 leaf vks, level[k] = 64 >> k node hashes */
static void build_tree(uint8_t nodes[7][64][32], const uint8_t seed[32]) {
  for (uint32_t i = 0; i < 64; i++) {
    uint8_t ls[32], sk[64];
    leaf_seed(ls, seed, i);
    orc_ed25519_seed_keypair(nodes[0][i], sk, ls);
  }
  for (int k = 1; k <= ORC_KES_DEPTH; k++) {
    for (int i = 0; i < (64 >> k); i++) {
      uint8_t pair[64];
      memcpy(pair, nodes[k - 1][2 * i], 32);
      memcpy(pair + 32, nodes[k - 1][2 * i + 1], 32);
      orc_blake2b_256(nodes[k][i], pair, 64);
    }
  }
}

void orc_sum6kes_keygen(uint8_t root_vk[32], const uint8_t seed[32]) {
  static __thread uint8_t nodes[7][64][32];
  build_tree(nodes, seed);
  memcpy(root_vk, nodes[ORC_KES_DEPTH][0], 32);
}

void orc_sum6kes_sign(uint8_t sig[ORC_KES_SIGBYTES], const uint8_t seed[32], uint32_t t,
                      const uint8_t *m, size_t mlen) {
  static __thread uint8_t nodes[7][64][32];
  uint8_t ls[32], pk[32], sk[64];
  t &= 63;
  build_tree(nodes, seed);
  leaf_seed(ls, seed, t);
  orc_ed25519_seed_keypair(pk, sk, ls);
  orc_ed25519_sign(sig, m, mlen, sk);
  for (int k = 1; k <= ORC_KES_DEPTH; k++) {
    uint32_t idx = t >> (k - 1); /* index of the path node at level k-1 */
    uint32_t base = idx & ~1u;
    memcpy(sig + 64 + 64 * (k - 1), nodes[k - 1][base], 32);
    memcpy(sig + 64 + 64 * (k - 1) + 32, nodes[k - 1][base + 1], 32);
  }
}
