/*
 * oracle.h -- CPU restatement of the Praos/TPraos header-crypto hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product library links, loads or
 * calls this code.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may use it, and only as the checker (or as the timed CPU
 * baseline), never as the thing measured or shipped.
 *
 * What it restates (the reference keeps this arithmetic in un-vendored C
 * dependencies):
 *   - libsodium 1.0.18 (pinned by the reference's CI,
 *     .github/workflows/build.yml:77,98): SHA-512, Blake2b (unkeyed),
 *     crypto_sign_ed25519_verify_detached acceptance rules,
 *     ge25519_from_uniform (Elligator2, App. B.3).
 *   - cardano-crypto-praos @ cardano-base 4251c0bb (cabal.project:156-166):
 *     crypto_vrf_ietfdraft03_{verify,proof_to_hash,prove} (App. B.3, B.3').
 *   - cardano-crypto-class SumKES/SingleKES verify (App. B.2), called from
 *     ouroboros-consensus-shelley/src/Ouroboros/Consensus/Shelley/Ledger/Integrity.hs:27
 *   - the crypto subset of SL.updateChainDepState reached via
 *     ouroboros-consensus-shelley/src/Ouroboros/Consensus/Shelley/Protocol.hs:433-442
 *
 * Parity pinning: libsodium 1.0.18 (conda copy, same version as the CI pin) for
 * SHA-512/Blake2b/Ed25519/Elligator2 via differential tests; IETF draft-03
 * ECVRF vectors and the reference's golden Shelley/Allegra/Mary headers for the
 * VRF, Sum6KES and opcert paths (tests/golden/).  VRF acceptance rules beyond
 * honest inputs (s >= L handling) are "parity unpinned" (SURVEY.md App. B.3).
 *
 * Representation is deliberately different from the device code: 5x51-bit
 * limbs with 128-bit products (device: 10 limbs radix 2^25.5).
 */
#ifndef OURO_ORACLE_H
#define OURO_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- hashes ---- */
void orc_sha512(uint8_t out[64], const uint8_t *in, size_t len);
void orc_blake2b(uint8_t *out, size_t outlen, const uint8_t *in, size_t len);
void orc_blake2b_256(uint8_t out[32], const uint8_t *in, size_t len);

/* ---- Ed25519 (libsodium 1.0.18 semantics) ---- */
void orc_ed25519_seed_keypair(uint8_t pk[32], uint8_t sk[64], const uint8_t seed[32]);
void orc_ed25519_sign(uint8_t sig[64], const uint8_t *m, size_t mlen, const uint8_t sk[64]);
/* 0 = valid, -1 = invalid (libsodium crypto_sign_ed25519_verify_detached) */
int orc_ed25519_verify(const uint8_t sig[64], const uint8_t *m, size_t mlen, const uint8_t pk[32]);
/* Byron / cardano-crypto (donna-derived) acceptance: only sig[63]&0xE0 and A decode */
int orc_ed25519_verify_byron(const uint8_t sig[64], const uint8_t *m, size_t mlen,
                             const uint8_t pk[32]);

/* ---- ECVRF-ED25519-SHA512-Elligator2, IETF draft-03 ---- */
void orc_elligator2_from_uniform(uint8_t out[32], const uint8_t r[32]);
/* strict_s = 1: also reject a proof whose s is not below L */
int orc_vrf03_verify_mode(uint8_t out[64], const uint8_t pk[32], const uint8_t pi[80],
                          const uint8_t *m, size_t mlen, int strict_s);
int orc_vrf03_verify(uint8_t out[64], const uint8_t pk[32], const uint8_t proof[80],
                     const uint8_t *m, size_t mlen);
int orc_vrf03_proof_to_hash(uint8_t out[64], const uint8_t proof[80]);
/* sk = seed(32) || pk(32), as crypto_vrf_ietfdraft03_keypair_from_seed */
void orc_vrf03_keypair(uint8_t pk[32], uint8_t sk[64], const uint8_t seed[32]);
int orc_vrf03_prove(uint8_t proof[80], const uint8_t sk[64], const uint8_t *m, size_t mlen);

/* ---- Sum6KES (SumKES^6 over SingleKES Ed25519DSIGN, Blake2b_256) ---- */
#define ORC_KES_DEPTH 6
#define ORC_KES_SIGBYTES 448
int orc_sum6kes_verify(const uint8_t vk[32], uint32_t t, const uint8_t *m, size_t mlen,
                       const uint8_t sig[ORC_KES_SIGBYTES]);
/* Synthetic tree (test data only): 64 leaf seeds = SHA-512(seed || LE32(i))[0:32].
 * Writes the root vk; sign produces the 448-B signature for period t. */
void orc_sum6kes_keygen(uint8_t root_vk[32], const uint8_t seed[32]);
void orc_sum6kes_sign(uint8_t sig[ORC_KES_SIGBYTES], const uint8_t seed[32], uint32_t t,
                      const uint8_t *m, size_t mlen);

/* ---- TPraos header crypto (SoA batch; layout mirrors include/ouro_verify.h) ---- */
typedef struct orc_tpraos_batch {
  size_t n;
  const uint8_t *issuer_vk;   /* n x 32  cold key (opcert signer)         */
  const uint8_t *vrf_vk;      /* n x 32                                     */
  const uint8_t *eta_proof;   /* n x 80                                     */
  const uint8_t *leader_proof;/* n x 80                                     */
  const uint8_t *eta_alpha;   /* n x 32  mkSeed seedEta slot eta0           */
  const uint8_t *leader_alpha;/* n x 32  mkSeed seedL   slot eta0           */
  const uint8_t *hot_vk;      /* n x 32  ocert.hotVk = Sum6 root            */
  const uint64_t *ocert_counter; /* n */
  const uint64_t *ocert_kes_period; /* n  (c0) */
  const uint8_t *ocert_sigma; /* n x 64                                     */
  const uint32_t *kes_t;      /* n  t = kesPeriod(slot) - c0 (Integrity.hs:38-44) */
  const uint8_t *kes_sig;     /* n x 448                                    */
  const uint8_t *body;        /* concatenated header-body CBOR              */
  const uint64_t *body_off;   /* n                                          */
  const uint32_t *body_len;   /* n                                          */
  /* optional (NULL = not used), as include/ouro_verify.h */
  const uint8_t *eta_output;  /* n x 64  claimed certifiedOutput (eta)      */
  const uint8_t *leader_output; /* n x 64 claimed certifiedOutput (leader)  */
  const uint64_t *slot;       /* n  -> alphas = mkSeed seedEta/seedL slot eta0 */
  const uint8_t *epoch_nonce; /* 32  eta0 (NULL: NeutralNonce)              */
  uint8_t *eta_nonce;         /* n x 32 OUT  mkNonceFromOutputVRF           */
} orc_tpraos_batch;

#define ORC_HDR_OCERT_OK 1u
#define ORC_HDR_KES_OK 2u
#define ORC_HDR_VRF_ETA_OK 4u
#define ORC_HDR_VRF_LEADER_OK 8u
#define ORC_HDR_ALL_OK 15u
#define ORC_HDR_ETA_CLAIM_OK 16u
#define ORC_HDR_LEADER_CLAIM_OK 32u
/* the proof's s is not reduced (s >= L): draft-03's decode_proof as
 * libsodium's fork reduces it (accepted); a strict-s caller rejects it
 * (parity of the default unpinned) */
#define ORC_HDR_ETA_S_UNREDUCED 64u
#define ORC_HDR_LEADER_S_UNREDUCED 128u

/* ledger-specs mkNonceFromNumber: Blake2b-256(BE64(k)) (a Nonce hash) */
void orc_mk_nonce_from_number(uint8_t out[32], uint64_t k);
/* ledger-specs mkSeed ucNonce slot eta0 (called at
 * ouroboros-consensus-shelley/src/Ouroboros/Consensus/Shelley/Protocol.hs:409-410):
 * Blake2b-256(BE64(slot) || eta0) XOR ucNonce; eta0 = NULL is NeutralNonce
 * (nothing appended); uc = NULL is a NeutralNonce ucNonce (no XOR). */
void orc_mk_seed(uint8_t out[32], const uint8_t *uc, uint64_t slot, const uint8_t *eta0);

void orc_tpraos_verify_one(const orc_tpraos_batch *b, size_t i, uint8_t *verdict,
                           uint8_t beta_eta[64], uint8_t beta_leader[64]);

/* ---- threaded batch drivers (cpu_baseline leg of bench.py) ---- */
void orc_ed25519_verify_batch(size_t n, const uint8_t *pk, const uint8_t *sig,
                              const uint8_t *msg, const uint64_t *msg_off,
                              const uint32_t *msg_len, uint8_t *verdict, int threads);
void orc_vrf03_verify_batch(size_t n, const uint8_t *pk, const uint8_t *proof,
                            const uint8_t *alpha, size_t alpha_len, uint8_t *beta,
                            uint8_t *verdict, int threads);
void orc_sum6kes_verify_batch(size_t n, const uint8_t *vk, const uint32_t *t,
                              const uint8_t *msg, const uint64_t *msg_off,
                              const uint32_t *msg_len, const uint8_t *sig, uint8_t *verdict,
                              int threads);
void orc_tpraos_verify_batch(const orc_tpraos_batch *b, uint8_t *verdict, uint8_t *beta_eta,
                             uint8_t *beta_leader, int threads);

/* libsodium's crypto_sign_ed25519_verify_detached over a batch (dlopen of
 * so_path), the reference's own Ed25519 for the CPU baseline; -1 if absent */
int orc_sodium_ed25519_verify_batch(const char *so_path, size_t n, const uint8_t *pk,
                                    const uint8_t *sig, const uint8_t *msg32, uint8_t *verdict,
                                    int threads);

/* synthesis helpers (threaded) used by tests to build inputs;
 * seed(tag, i) = SHA-512("ouro-mi355x/" || tag zero-padded to 12 B || LE64(i))[0:32] */
void orc_seed(uint8_t out[32], const char *tag, uint64_t i);
void orc_synth_ed25519(size_t n, uint64_t first, uint8_t *pk, uint8_t *sig, uint8_t *msg32,
                       int threads);
void orc_synth_vrf(size_t n, uint64_t first, uint8_t *pk, uint8_t *proof, uint8_t *alpha32,
                   int threads);

#ifdef __cplusplus
}
#endif
#endif
