/*
 * C callers of the one-call raw-CBOR entries (include/ouro_verify.h
 * ouro_tpraos_verify_cbor, ouro_integrity_verify_cbor)
 * and their multi-device forms (ouro_*_verify_cbor_multi; VERDICT r05 item
 * 2: threads with id % 4 == 2 pass devices {0}, id % 4 == 3 devices {0, 0}):
 * THREADS pthreads each call both entries ROUNDS times on the same raw
 * headers -- as a node's ChainDB / storage threads would through the FFI --
 * and compare status, verdicts and both VRF outputs with the expectations the
 * Python side computed from the pinned host slicer and the CPU oracle
 * (tests/test_gpu_cbor.py::test_c_callers writes INPUT).  Odd threads pass the
 * explicit VRF inputs, even threads the same arrays through a second
 * allocation, so every call owns its buffers.
 *
 * INPUT (little-endian): u64 n, u64 raw_bytes, u64 slots_per_kes_period,
 *   raw[raw_bytes], u64 off[n], u32 len[n], eta_alpha[32 n], leader_alpha[32 n],
 *   want_status[n], want_verdict[n], want_beta_eta[64 n], want_beta_leader[64 n],
 *   want_integrity[n]
 *
 * usage: cbor_callers INPUT THREADS ROUNDS  ->  "ok <calls>" or "FAIL ..."
 */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "ouro_verify.h"

static uint64_t n, raw_bytes, spkp;
static uint8_t *raw, *ea, *la, *w_st, *w_v, *w_be, *w_bl, *w_int;
static uint64_t *off;
static uint32_t *len;
static int rounds, g_fail;
static long g_calls[64];

static void *rd(FILE *f, size_t bytes) {
  void *p = malloc(bytes ? bytes : 1);
  if (!p || fread(p, 1, bytes, f) != bytes) {
    fprintf(stderr, "short input\n");
    exit(2);
  }
  return p;
}

#define CHECK(cond, ...)                \
  do {                                  \
    if (!(cond)) {                      \
      fprintf(stderr, __VA_ARGS__);     \
      __sync_fetch_and_add(&g_fail, 1); \
      goto done;                        \
    }                                   \
  } while (0)

static void *worker(void *arg) {
  const int id = (int)(long)arg;
  uint8_t *st = malloc(n), *v = malloc(n), *be = malloc(64 * n), *bl = malloc(64 * n);
  uint8_t *my_ea = malloc(32 * n), *my_la = malloc(32 * n);
  long calls = 0;
  memcpy(my_ea, ea, 32 * n);
  memcpy(my_la, la, 32 * n);
  static const int devs[2] = {0, 0};
  const int multi = id % 4 >= 2, ndev = id % 4 == 3 ? 2 : 1;
  for (int r = 0; r < rounds; r++) {
    memset(v, 0xEE, n);
    const uint8_t *a = (id & 1) ? ea : my_ea, *b = (id & 1) ? la : my_la;
    const int rc = multi ? ouro_tpraos_verify_cbor_multi(devs, ndev, raw, raw_bytes, off, len, n,
                                                         spkp, NULL, a, b, st, v, be, bl, NULL)
                         : ouro_tpraos_verify_cbor(raw, raw_bytes, off, len, n, spkp, NULL, a, b,
                                                   st, v, be, bl, NULL);
    CHECK(rc == OURO_OK, "t%d tpraos rc %d (%s)\n", id, rc, ouro_last_error());
    for (uint64_t i = 0; i < n; i++) {
      CHECK(st[i] == w_st[i], "t%d status %llu\n", id, (unsigned long long)i);
      CHECK(v[i] == w_v[i], "t%d verdict %llu: %d want %d\n", id, (unsigned long long)i, v[i],
            w_v[i]);
      if (st[i] == OURO_PACK_OK) {
        CHECK(memcmp(be + 64 * i, w_be + 64 * i, 64) == 0, "t%d beta_eta %llu\n", id,
              (unsigned long long)i);
        CHECK(memcmp(bl + 64 * i, w_bl + 64 * i, 64) == 0, "t%d beta_leader %llu\n", id,
              (unsigned long long)i);
      }
    }
    memset(v, 0xEE, n);
    const int ri = multi ? ouro_integrity_verify_cbor_multi(devs, ndev, raw, raw_bytes, off, len,
                                                            n, spkp, st, v)
                         : ouro_integrity_verify_cbor(raw, raw_bytes, off, len, n, spkp, st, v);
    CHECK(ri == OURO_OK, "t%d integrity rc %d (%s)\n", id, ri, ouro_last_error());
    for (uint64_t i = 0; i < n; i++)
      CHECK(v[i] == w_int[i], "t%d integrity %llu\n", id, (unsigned long long)i);
    calls += 2;
  }
done:
  g_calls[id] = calls;
  free(st); free(v); free(be); free(bl); free(my_ea); free(my_la);
  return NULL;
}

int main(int argc, char **argv) {
  if (argc < 4) return 2;
  FILE *f = fopen(argv[1], "rb");
  if (!f) return 2;
  const int threads = atoi(argv[2]);
  rounds = atoi(argv[3]);
  if (threads < 1 || threads > 64) return 2;
  uint64_t *h = rd(f, 24);
  n = h[0];
  raw_bytes = h[1];
  spkp = h[2];
  raw = rd(f, raw_bytes);
  off = rd(f, 8 * n);
  len = rd(f, 4 * n);
  ea = rd(f, 32 * n);
  la = rd(f, 32 * n);
  w_st = rd(f, n);
  w_v = rd(f, n);
  w_be = rd(f, 64 * n);
  w_bl = rd(f, 64 * n);
  w_int = rd(f, n);
  fclose(f);
  pthread_t th[64];
  for (int t = 0; t < threads; t++) pthread_create(&th[t], NULL, worker, (void *)(long)t);
  long total = 0;
  for (int t = 0; t < threads; t++) {
    pthread_join(th[t], NULL);
    total += g_calls[t];
  }
  if (g_fail) {
    printf("FAIL %d\n", g_fail);
    return 1;
  }
  printf("ok %ld\n", total);
  return 0;
}
