/*
 * vrf03.c -- ECVRF-ED25519-SHA512-Elligator2, IETF draft-03, for the oracle.
 * TEST INFRASTRUCTURE ONLY.
 *
 * Restates cardano-crypto-praos (cardano-base@4251c0bb, cabal.project:156-166)
 * crypto_vrf_ietfdraft03_{verify,proof_to_hash,prove}, the C behind
 * PraosVRF.verifyVRF / verifyCertified / certifiedOutput (SURVEY.md §8(a) rows
 * a5-a7, App. B.3/B.3').  Reference call sites: the OVERLAY rule's vrfChecks
 * via ouroboros-consensus-shelley/src/Ouroboros/Consensus/Shelley/Protocol.hs:435
 * (2 VRFs per header), certifiedOutput at Shelley/Ledger/TPraos.hs:40 and
 * Shelley/Protocol.hs:484-486; mock-protocol shape at
 * ouroboros-consensus-mock/src/Ouroboros/Consensus/Mock/Protocol/Praos.hs:341-354.
 *
 * Pinned by the three IETF draft-03 vectors and the two golden-header proofs
 * (tests/golden/).  Elligator2 is libsodium 1.0.18 ge25519_from_uniform, pinned
 * differentially against crypto_core_ed25519_from_uniform.  Handling of s >= L
 * (reduce, as recalled for the fork) is parity unpinned.
 */
#include "internal.h"
#include <string.h>

#define SUITE 0x04

/* libsodium 1.0.18 ge25519_from_uniform (x_sign taken from r[31] bit 7) */
void orc_elligator2_from_uniform(uint8_t out[32], const uint8_t r[32]) {
  const curve_consts *k = cc();
  uint8_t s[32];
  fe rr2, x, x2, x3, e, negx, one, t;
  memcpy(s, r, 32);
  uint8_t x_sign = s[31] & 0x80;
  s[31] &= 0x7f;
  fe_frombytes(&rr2, s);
  fe_sq(&rr2, &rr2);
  fe_add(&rr2, &rr2, &rr2);  /* 2 r^2 */
  fe_1(&one);
  fe_add(&rr2, &rr2, &one);  /* 1 + 2 r^2 */
  fe_invert(&rr2, &rr2);
  fe_mul(&x, &k->mont_a, &rr2);
  fe_neg(&x, &x);            /* x = -A / (1 + 2 r^2) */
  fe_sq(&x2, &x);
  fe_mul(&x3, &x, &x2);
  fe_add(&e, &x3, &x);
  fe_mul(&x2, &x2, &k->mont_a);
  fe_add(&e, &x2, &e);       /* e = x^3 + A x^2 + x */
  /* chi(e) = e^((p-1)/2) = (e^(2^252-3))^2... computed as e^(2^254-10) */
  {
    fe z = e, r1;
    /* (p-1)/2 = 2^254 - 10 = 4*(2^252 - 3) + 2 */
    fe_pow22523(&r1, &z);
    fe_sq(&r1, &r1);
    fe_sq(&r1, &r1);
    fe_sq(&t, &z);
    fe_mul(&e, &r1, &t);
  }
  uint8_t eb[32];
  fe_tobytes(eb, &e);
  int e_is_minus_1 = eb[1] & 1;
  fe_neg(&negx, &x);
  if (e_is_minus_1) {
    x = negx;
    fe_sub(&x, &x, &k->mont_a); /* x = -x - A */
  }
  /* y_ed = (x - 1) / (x + 1) */
  fe xp1, xm1;
  fe_add(&xp1, &x, &one);
  fe_sub(&xm1, &x, &one);
  fe_invert(&xp1, &xp1);
  fe_mul(&t, &xm1, &xp1);
  fe_tobytes(s, &t);
  s[31] |= x_sign;
  ge P, P2;
  if (ge_frombytes(&P, s) != 0) {
    memset(out, 0, 32); /* unreachable for field inputs (libsodium aborts) */
    return;
  }
  ge_dbl(&P2, &P);
  ge_dbl(&P2, &P2);
  ge_dbl(&P2, &P2);
  ge_tobytes(out, &P2);
}

static int string_to_point(ge *P, const uint8_t s[32]) {
  if (!ge_is_canonical(s) || ge_frombytes(P, s) != 0) return -1;
  return 0;
}

static void hash_to_curve(uint8_t H[32], const uint8_t Y[32], const uint8_t *m, size_t mlen) {
  orc_sha512_ctx c;
  uint8_t r[64];
  const uint8_t pre[2] = {SUITE, 0x01};
  orc_sha512_init(&c);
  orc_sha512_update(&c, pre, 2);
  orc_sha512_update(&c, Y, 32);
  orc_sha512_update(&c, m, mlen);
  orc_sha512_final(&c, r);
  r[31] &= 0x7f;
  orc_elligator2_from_uniform(H, r);
}

static void hash_points(uint8_t c[16], const uint8_t H[32], const uint8_t G[32],
                        const uint8_t U[32], const uint8_t V[32]) {
  uint8_t str[2 + 128], out[64];
  str[0] = SUITE;
  str[1] = 0x02;
  memcpy(str + 2, H, 32);
  memcpy(str + 34, G, 32);
  memcpy(str + 66, U, 32);
  memcpy(str + 98, V, 32);
  orc_sha512(out, str, sizeof str);
  memcpy(c, out, 16);
}

int orc_vrf03_proof_to_hash(uint8_t beta[64], const uint8_t pi[80]) {
  ge G, G8;
  uint8_t in[34];
  if (string_to_point(&G, pi) != 0) return -1;
  ge_dbl(&G8, &G);
  ge_dbl(&G8, &G8);
  ge_dbl(&G8, &G8);
  in[0] = SUITE;
  in[1] = 0x03;
  ge_tobytes(in + 2, &G8);
  orc_sha512(beta, in, sizeof in);
  return 0;
}

/* draft-03 leaves the range of s to the implementation: the fork's
 * decode_proof reduces it mod L (recalled, unpinned);
 * strict_s selects the other reading, s >= L rejected. */
int orc_vrf03_verify_mode(uint8_t out[64], const uint8_t pk[32], const uint8_t pi[80],
                          const uint8_t *m, size_t mlen, int strict_s) {
  if (strict_s && !sc_is_canonical(pi + 48)) return -1;
  return orc_vrf03_verify(out, pk, pi, m, mlen);
}

int orc_vrf03_verify(uint8_t out[64], const uint8_t pk[32], const uint8_t pi[80],
                     const uint8_t *m, size_t mlen) {
  ge Y, G, H, negY, negG, U, V;
  uint8_t Ys[32], Hs[32], Gs[32], Us[32], Vs[32], c[32], s[32], cp[16];
  /* validate_key */
  if (ge_has_small_order(pk) || string_to_point(&Y, pk) != 0) return -1;
  /* decode_proof */
  if (string_to_point(&G, pi) != 0) return -1;
  memset(c, 0, 32);
  memcpy(c, pi + 32, 16);
  sc_reduce(s, pi + 48, 32);
  /* H = hash_to_curve(encode(Y), alpha) */
  ge_tobytes(Ys, &Y);
  hash_to_curve(Hs, Ys, m, mlen);
  ge_frombytes(&H, Hs);
  /* U = sB - cY, V = sH - cG */
  ge_neg(&negY, &Y);
  ge_neg(&negG, &G);
  ge_double_scalarmult(&U, s, &cc()->B, c, &negY);
  ge_double_scalarmult(&V, s, &H, c, &negG);
  ge_tobytes(Gs, &G);
  ge_tobytes(Us, &U);
  ge_tobytes(Vs, &V);
  hash_points(cp, Hs, Gs, Us, Vs);
  if (memcmp(cp, c, 16) != 0) return -1;
  return orc_vrf03_proof_to_hash(out, pi);
}

void orc_vrf03_keypair(uint8_t pk[32], uint8_t sk[64], const uint8_t seed[32]) {
  orc_ed25519_seed_keypair(pk, sk, seed);
}

int orc_vrf03_prove(uint8_t pi[80], const uint8_t sk[64], const uint8_t *m, size_t mlen) {
  uint8_t az[64], Hs[32], Gs[32], kb[32], kh[32], nonce[64], kk[32], c[32];
  orc_sha512_ctx ctx;
  ge H, G, KB, KH;
  orc_sha512(az, sk, 32);
  az[0] &= 248;
  az[31] &= 127;
  az[31] |= 64;
  hash_to_curve(Hs, sk + 32, m, mlen);
  if (ge_frombytes(&H, Hs) != 0) return -1;
  ge_scalarmult(&G, az, &H);
  ge_tobytes(Gs, &G);
  orc_sha512_init(&ctx);
  orc_sha512_update(&ctx, az + 32, 32);
  orc_sha512_update(&ctx, Hs, 32);
  orc_sha512_final(&ctx, nonce);
  sc_reduce(kk, nonce, 64);
  ge_scalarmult_base(&KB, kk);
  ge_scalarmult(&KH, kk, &H);
  ge_tobytes(kb, &KB);
  ge_tobytes(kh, &KH);
  memset(c, 0, 32);
  hash_points(c, Hs, Gs, kb, kh);
  memcpy(pi, Gs, 32);
  memcpy(pi + 32, c, 16);
  sc_muladd(pi + 48, c, az, kk);
  return 0;
}
