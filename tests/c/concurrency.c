/*
 * Concurrent callers of the C ABI (include/ouro_verify.h: "All calls are
 * thread-safe and reentrant").  The reference calls its crypto from one
 * ChainSync client thread per peer plus ChainDB's chain-selection thread
 * (ouroboros-consensus/src/Ouroboros/Consensus/Network/NodeToNode.hs:173-176),
 * so T threads here interleave single-item calls (the libsodium /
 * cardano-crypto-praos ABI, the crypto_vrf_* names through the opt-in shim
 * lib/libouro_vrf_shim.so) with batch calls on their own data, each result
 * checked against the CPU oracle computed up front.  Then CHURN short-lived
 * threads, one after another, each make one batch call (GHC's FFI worker
 * pool grows and shrinks like this): the per-thread context pool must hand
 * each the context the previous one returned at its exit, so the contexts
 * created grow by at most one.  Test infrastructure: links the product
 * library, the shim and the oracle.
 *
 * usage: concurrency THREADS ROUNDS [CHURN]
 *        -> prints "ok <calls> <contexts created by the churn>" or "FAIL ..."
 */
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"
#include "ouro_verify.h"
#include "ouro_verify_debug.h"

int crypto_vrf_ietfdraft03_verify(unsigned char *, const unsigned char *, const unsigned char *,
                                  const unsigned char *, unsigned long long);
int crypto_vrf_proof_to_hash(unsigned char *, const unsigned char *);

#define NED 512
#define NVRF 256
#define NKES 64
#define MLEN 96

static uint8_t ed_pk[NED][32], ed_sig[NED][64], ed_msg[NED][32], ed_ok[NED];
static uint8_t v_pk[NVRF][32], v_pi[NVRF][80], v_al[NVRF][32], v_ok[NVRF], v_beta[NVRF][64];
static uint8_t k_vk[NKES][32], k_sig[NKES][448], k_msg[NKES][MLEN], k_ok[NKES];
static uint32_t k_t[NKES];
static int g_rounds;
static int g_fail;
static long g_calls[64];

static uint64_t rnd(uint64_t *s) {
  *s ^= *s << 13;
  *s ^= *s >> 7;
  *s ^= *s << 17;
  return *s;
}

#define CHECK(cond, ...)                  \
  do {                                    \
    if (!(cond)) {                        \
      fprintf(stderr, __VA_ARGS__);       \
      __sync_fetch_and_add(&g_fail, 1);   \
      return NULL;                        \
    }                                     \
  } while (0)

/* one Ed25519 batch call, then the thread exits (returning its context) */
static void *short_lived(void *arg) {
  const int lo = (int)(long)arg % (NED - 64);
  uint64_t off[64];
  uint32_t len[64];
  uint8_t v[64];
  for (int k = 0; k < 64; k++) {
    off[k] = 32ull * (uint64_t)(lo + k);
    len[k] = 32;
  }
  CHECK(ouro_ed25519_verify_batch(64, ed_pk[lo], ed_sig[lo], &ed_msg[0][0], off, len, v) == 0,
        "short-lived batch rc\n");
  for (int k = 0; k < 64; k++) CHECK(v[k] == ed_ok[lo + k], "short-lived %d\n", lo + k);
  return NULL;
}

static void *worker(void *arg) {
  const int id = (int)(long)arg;
  uint64_t s = 0x9e3779b97f4a7c15ull * (id + 1);
  long calls = 0;
  if (id % 3 == 2) CHECK(ouro_set_device(0) == OURO_OK, "set_device\n");
  for (int r = 0; r < g_rounds; r++) {
    const int kind = (int)(rnd(&s) % 6);
    if (kind == 0) {  /* single Ed25519 */
      const int i = (int)(rnd(&s) % NED);
      const int rc = ouro_ed25519_verify(ed_sig[i], ed_msg[i], 32, ed_pk[i]);
      CHECK(rc == (ed_ok[i] ? 0 : -1), "t%d ed %d rc %d want %d\n", id, i, rc, ed_ok[i]);
    } else if (kind == 1) {  /* Ed25519 batch of a random window */
      const int lo = (int)(rnd(&s) % NED), m = 1 + (int)(rnd(&s) % (NED - lo));
      uint64_t off[NED];
      uint32_t len[NED];
      uint8_t v[NED];
      for (int k = 0; k < m; k++) {
        off[k] = 32ull * (uint64_t)(lo + k);
        len[k] = 32;
      }
      /* absolute offsets into the whole message array: only the window uploads */
      CHECK(ouro_ed25519_verify_batch((size_t)m, ed_pk[lo], ed_sig[lo], &ed_msg[0][0], off, len,
                                      v) == 0, "t%d ed batch rc\n", id);
      for (int k = 0; k < m; k++) CHECK(v[k] == ed_ok[lo + k], "t%d ed batch %d\n", id, lo + k);
    } else if (kind == 2) {  /* single VRF through the cardano-crypto-praos name */
      const int i = (int)(rnd(&s) % NVRF);
      uint8_t out[64];
      memset(out, 0xee, 64);
      const int rc = crypto_vrf_ietfdraft03_verify(out, v_pk[i], v_pi[i], v_al[i], 32);
      CHECK(rc == (v_ok[i] ? 0 : -1), "t%d vrf %d rc %d\n", id, i, rc);
      if (v_ok[i]) CHECK(memcmp(out, v_beta[i], 64) == 0, "t%d vrf beta %d\n", id, i);
      else CHECK(out[0] == 0xee && out[63] == 0xee, "t%d vrf wrote output on failure\n", id);
    } else if (kind == 3) {  /* VRF batch */
      const int lo = (int)(rnd(&s) % NVRF), m = 1 + (int)(rnd(&s) % (NVRF - lo));
      uint64_t off[NVRF];
      uint32_t len[NVRF];
      uint8_t v[NVRF], beta[NVRF][64];
      for (int k = 0; k < m; k++) {
        off[k] = 32ull * (uint64_t)k;
        len[k] = 32;
      }
      CHECK(ouro_vrf03_verify_batch((size_t)m, v_pk[lo], v_pi[lo], v_al[lo], off, len, &beta[0][0],
                                    v) == 0, "t%d vrf batch rc\n", id);
      for (int k = 0; k < m; k++) {
        CHECK(v[k] == v_ok[lo + k], "t%d vrf batch %d\n", id, lo + k);
        if (v[k]) CHECK(memcmp(beta[k], v_beta[lo + k], 64) == 0, "t%d vrf batch beta\n", id);
      }
    } else if (kind == 4) {  /* single Sum6KES + proof_to_hash */
      const int i = (int)(rnd(&s) % NKES);
      const int rc = ouro_sum6kes_verify(k_vk[i], k_t[i], k_msg[i], MLEN, k_sig[i]);
      CHECK(rc == (k_ok[i] ? 0 : -1), "t%d kes %d rc %d\n", id, i, rc);
      const int j = (int)(rnd(&s) % NVRF);
      uint8_t out[64], want[64];
      const int wr = orc_vrf03_proof_to_hash(want, v_pi[j]);
      const int gr = crypto_vrf_proof_to_hash(out, v_pi[j]);
      CHECK(gr == wr, "t%d p2h rc\n", id);
      if (!wr) CHECK(memcmp(out, want, 64) == 0, "t%d p2h\n", id);
    } else {  /* Sum6KES batch */
      const int lo = (int)(rnd(&s) % NKES), m = 1 + (int)(rnd(&s) % (NKES - lo));
      uint64_t off[NKES];
      uint32_t len[NKES];
      uint8_t v[NKES];
      for (int k = 0; k < m; k++) {
        off[k] = (uint64_t)MLEN * (uint64_t)k;
        len[k] = MLEN;
      }
      CHECK(ouro_sum6kes_verify_batch((size_t)m, k_vk[lo], &k_t[lo], k_msg[lo], off, len,
                                      k_sig[lo], v) == 0, "t%d kes batch rc\n", id);
      for (int k = 0; k < m; k++) CHECK(v[k] == k_ok[lo + k], "t%d kes batch %d\n", id, lo + k);
    }
    calls++;
  }
  g_calls[id] = calls;
  return NULL;
}

int main(int argc, char **argv) {
  const int threads = argc > 1 ? atoi(argv[1]) : 8;
  g_rounds = argc > 2 ? atoi(argv[2]) : 40;
  if (threads < 1 || threads > 64) return 2;
  uint64_t s = 12345;
  orc_synth_ed25519(NED, 777000, &ed_pk[0][0], &ed_sig[0][0], &ed_msg[0][0], 8);
  for (int i = 0; i < NED; i++) {
    if (rnd(&s) % 4 == 0) ed_sig[i][rnd(&s) % 64] ^= (uint8_t)(1u << (rnd(&s) % 8));
    ed_ok[i] = orc_ed25519_verify(ed_sig[i], ed_msg[i], 32, ed_pk[i]) == 0;
  }
  orc_synth_vrf(NVRF, 888000, &v_pk[0][0], &v_pi[0][0], &v_al[0][0], 8);
  for (int i = 0; i < NVRF; i++) {
    if (rnd(&s) % 4 == 0) v_pi[i][rnd(&s) % 80] ^= (uint8_t)(1u << (rnd(&s) % 8));
    v_ok[i] = orc_vrf03_verify(v_beta[i], v_pk[i], v_pi[i], v_al[i], 32) == 0;
  }
  for (int i = 0; i < NKES; i++) {
    uint8_t seed[32];
    orc_seed(seed, "kes", (uint64_t)(i % 8));
    orc_sum6kes_keygen(k_vk[i], seed);
    for (int b = 0; b < MLEN; b++) k_msg[i][b] = (uint8_t)rnd(&s);
    k_t[i] = (uint32_t)(rnd(&s) % 64);
    orc_sum6kes_sign(k_sig[i], seed, k_t[i], k_msg[i], MLEN);
    if (i % 5 == 1) k_t[i] = (k_t[i] + 1) % 64;
    if (i % 7 == 3) k_msg[i][0] ^= 1;
    k_ok[i] = orc_sum6kes_verify(k_vk[i], k_t[i], k_msg[i], MLEN, k_sig[i]) == 0;
  }
  pthread_t th[64];
  for (int t = 0; t < threads; t++) pthread_create(&th[t], NULL, worker, (void *)(long)t);
  long total = 0;
  for (int t = 0; t < threads; t++) {
    pthread_join(th[t], NULL);
    total += g_calls[t];
  }
  const int churn = argc > 3 ? atoi(argv[3]) : 0;
  size_t before = 0, after = 0, idle = 0;
  ouro_debug_contexts(0, &before, &idle);
  for (int t = 0; t < churn && !g_fail; t++) {
    pthread_t one;
    pthread_create(&one, NULL, short_lived, (void *)(long)(7 * t));
    pthread_join(one, NULL);
  }
  ouro_debug_contexts(0, &after, &idle);
  if (g_fail) {
    printf("FAIL %d\n", g_fail);
    return 1;
  }
  printf("ok %ld %zu\n", total, after - before);
  return 0;
}
