/*
 * batch.c -- threaded batch drivers over the oracle (the cpu_baseline leg of
 * bench.py) and threaded synthesis of test inputs.  TEST INFRASTRUCTURE ONLY.
 *
 * One item per work unit, dynamically scheduled over `threads` pthreads, the
 * CPU-baseline plan of BASELINE.md ("one item per std::thread x nproc").
 *
 * Synthetic-input seeds follow SURVEY.md §8(d):
 *   seed(tag, i) = SHA-512("ouro-mi355x/" || tag || LE64(i))[0:32]
 */
#include "internal.h"
#include <dlfcn.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdlib.h>
#include <string.h>

typedef void (*item_fn)(void *ctx, size_t i);

typedef struct {
  item_fn fn;
  void *ctx;
  size_t n;
  atomic_size_t next;
} pool_job;

#define CHUNK 16

static void *pool_worker(void *arg) {
  pool_job *j = (pool_job *)arg;
  for (;;) {
    size_t s = atomic_fetch_add(&j->next, CHUNK);
    if (s >= j->n) break;
    size_t e = s + CHUNK < j->n ? s + CHUNK : j->n;
    for (size_t i = s; i < e; i++) j->fn(j->ctx, i);
  }
  return NULL;
}

static void run_pool(item_fn fn, void *ctx, size_t n, int threads) {
  pool_job j;
  j.fn = fn;
  j.ctx = ctx;
  j.n = n;
  atomic_init(&j.next, 0);
  (void)cc(); /* build constants before fanning out */
  if (threads <= 1) {
    pool_worker(&j);
    return;
  }
  pthread_t *tid = (pthread_t *)malloc(sizeof(pthread_t) * (size_t)threads);
  int started = 0;
  for (int t = 0; t < threads; t++)
    if (pthread_create(&tid[t], NULL, pool_worker, &j) == 0) started++;
    else break;
  if (started == 0) pool_worker(&j);
  for (int t = 0; t < started; t++) pthread_join(tid[t], NULL);
  free(tid);
}

/* ---------------------------------------------------------- Ed25519 ---- */
typedef struct {
  const uint8_t *pk, *sig, *msg;
  const uint64_t *off;
  const uint32_t *len;
  uint8_t *verdict;
} ed_ctx;

static void ed_item(void *c, size_t i) {
  ed_ctx *x = (ed_ctx *)c;
  x->verdict[i] = orc_ed25519_verify(x->sig + 64 * i, x->msg + x->off[i], x->len[i],
                                     x->pk + 32 * i) == 0;
}

void orc_ed25519_verify_batch(size_t n, const uint8_t *pk, const uint8_t *sig,
                              const uint8_t *msg, const uint64_t *msg_off,
                              const uint32_t *msg_len, uint8_t *verdict, int threads) {
  ed_ctx c = {pk, sig, msg, msg_off, msg_len, verdict};
  run_pool(ed_item, &c, n, threads);
}

/* ---------------------------------------------------------- VRF ---- */
typedef struct {
  const uint8_t *pk, *proof, *alpha;
  size_t alpha_len;
  uint8_t *beta, *verdict;
} vrf_ctx;

static void vrf_item(void *c, size_t i) {
  vrf_ctx *x = (vrf_ctx *)c;
  uint8_t *b = x->beta + 64 * i;
  memset(b, 0, 64);
  x->verdict[i] = orc_vrf03_verify(b, x->pk + 32 * i, x->proof + 80 * i,
                                   x->alpha + x->alpha_len * i, x->alpha_len) == 0;
}

void orc_vrf03_verify_batch(size_t n, const uint8_t *pk, const uint8_t *proof,
                            const uint8_t *alpha, size_t alpha_len, uint8_t *beta,
                            uint8_t *verdict, int threads) {
  vrf_ctx c = {pk, proof, alpha, alpha_len, beta, verdict};
  run_pool(vrf_item, &c, n, threads);
}

/* ---------------------------------------------------------- KES ---- */
typedef struct {
  const uint8_t *vk;
  const uint32_t *t;
  const uint8_t *msg;
  const uint64_t *off;
  const uint32_t *len;
  const uint8_t *sig;
  uint8_t *verdict;
} kes_ctx;

static void kes_item(void *c, size_t i) {
  kes_ctx *x = (kes_ctx *)c;
  x->verdict[i] = orc_sum6kes_verify(x->vk + 32 * i, x->t[i], x->msg + x->off[i], x->len[i],
                                     x->sig + ORC_KES_SIGBYTES * i) == 0;
}

void orc_sum6kes_verify_batch(size_t n, const uint8_t *vk, const uint32_t *t,
                              const uint8_t *msg, const uint64_t *msg_off,
                              const uint32_t *msg_len, const uint8_t *sig, uint8_t *verdict,
                              int threads) {
  kes_ctx c = {vk, t, msg, msg_off, msg_len, sig, verdict};
  run_pool(kes_item, &c, n, threads);
}

/* ---------------------------------------------------------- headers ---- */
typedef struct {
  const orc_tpraos_batch *b;
  uint8_t *verdict, *be, *bl;
} hdr_ctx;

static void hdr_item(void *c, size_t i) {
  hdr_ctx *x = (hdr_ctx *)c;
  orc_tpraos_verify_one(x->b, i, x->verdict + i, x->be + 64 * i, x->bl + 64 * i);
}

void orc_tpraos_verify_batch(const orc_tpraos_batch *b, uint8_t *verdict, uint8_t *beta_eta,
                             uint8_t *beta_leader, int threads) {
  hdr_ctx c = {b, verdict, beta_eta, beta_leader};
  run_pool(hdr_item, &c, b->n, threads);
}

/* --------------------------------------- libsodium (the reference's) ---- */
/* bench.py's cpu_baseline for Ed25519: the function the
 * reference's Ed25519DSIGN binds, libsodium 1.0.18's
 * crypto_sign_ed25519_verify_detached, driven by the same pthread pool (no
 * Python per item).  `so_path` is dlopen()ed; returns -1 if it cannot be. */
typedef int (*sodium_verify_fn)(const unsigned char *, const unsigned char *,
                                unsigned long long, const unsigned char *);
typedef struct {
  sodium_verify_fn fn;
  const uint8_t *pk, *sig, *msg;
  uint8_t *verdict;
} sodium_ctx;

static void sodium_item(void *c, size_t i) {
  sodium_ctx *x = (sodium_ctx *)c;
  x->verdict[i] = x->fn(x->sig + 64 * i, x->msg + 32 * i, 32, x->pk + 32 * i) == 0;
}

int orc_sodium_ed25519_verify_batch(const char *so_path, size_t n, const uint8_t *pk,
                                    const uint8_t *sig, const uint8_t *msg32, uint8_t *verdict,
                                    int threads) {
  void *h = dlopen(so_path, RTLD_NOW | RTLD_LOCAL);
  if (!h) return -1;
  int (*init)(void) = (int (*)(void))dlsym(h, "sodium_init");
  sodium_verify_fn fn = (sodium_verify_fn)dlsym(h, "crypto_sign_ed25519_verify_detached");
  if (!init || !fn || init() < 0) return -1;
  sodium_ctx c = {fn, pk, sig, msg32, verdict};
  run_pool(sodium_item, &c, n, threads);
  return 0; /* the handle stays open: the library is process-wide */
}

/* ---------------------------------------------------------- synthesis ---- */
/* tag zero-padded to 12 bytes: every seed message is 32 bytes */
void orc_seed(uint8_t out[32], const char *tag, uint64_t i) {
  uint8_t buf[32];
  size_t tl = strlen(tag);
  if (tl > 12) tl = 12;
  memset(buf, 0, sizeof buf);
  memcpy(buf, "ouro-mi355x/", 12);
  memcpy(buf + 12, tag, tl);
  for (int k = 0; k < 8; k++) buf[24 + k] = (uint8_t)(i >> (8 * k));
  uint8_t h[64];
  orc_sha512(h, buf, 32);
  memcpy(out, h, 32);
}
#define seed_of orc_seed

typedef struct {
  uint64_t first;
  uint8_t *pk, *sig, *msg;
} synth_ed_ctx;

static void synth_ed_item(void *c, size_t i) {
  synth_ed_ctx *x = (synth_ed_ctx *)c;
  uint8_t seed[32], sk[64];
  seed_of(seed, "ed", x->first + i);
  seed_of(x->msg + 32 * i, "msg", x->first + i);
  orc_ed25519_seed_keypair(x->pk + 32 * i, sk, seed);
  orc_ed25519_sign(x->sig + 64 * i, x->msg + 32 * i, 32, sk);
}

void orc_synth_ed25519(size_t n, uint64_t first, uint8_t *pk, uint8_t *sig, uint8_t *msg32,
                       int threads) {
  synth_ed_ctx c = {first, pk, sig, msg32};
  run_pool(synth_ed_item, &c, n, threads);
}

typedef struct {
  uint64_t first;
  uint8_t *pk, *proof, *alpha;
} synth_vrf_ctx;

static void synth_vrf_item(void *c, size_t i) {
  synth_vrf_ctx *x = (synth_vrf_ctx *)c;
  uint8_t seed[32], sk[64];
  seed_of(seed, "vrf", x->first + i);
  seed_of(x->alpha + 32 * i, "alpha", x->first + i);
  orc_vrf03_keypair(x->pk + 32 * i, sk, seed);
  orc_vrf03_prove(x->proof + 80 * i, sk, x->alpha + 32 * i, 32);
}

void orc_synth_vrf(size_t n, uint64_t first, uint8_t *pk, uint8_t *proof, uint8_t *alpha32,
                   int threads) {
  synth_vrf_ctx c = {first, pk, proof, alpha32};
  run_pool(synth_vrf_item, &c, n, threads);
}
