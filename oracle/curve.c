/*
 * curve.c -- GF(2^255-19), edwards25519 group and scalars mod L for the oracle.
 * TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Restates the behaviour of libsodium 1.0.18's ref10 internals that the
 * reference's Ed25519DSIGN / PraosVRF verify depend on (SURVEY.md App. B.1,
 * B.3): ge25519_frombytes / _negate_vartime (y read mod 2^255, x = 0 with sign
 * bit accepted), ge25519_is_canonical (y < p, sign bit ignored),
 * ge25519_has_small_order (7-entry y blocklist, sign bit masked),
 * sc25519_is_canonical (s < L), sc25519_reduce.  Group elements are only ever
 * compared through their canonical encodings, so the formulas used here
 * (add-2008-hwcd-3 / dbl-2008-hwcd) need not match ref10's.
 */
#include "internal.h"
#include <pthread.h>
#include <string.h>

typedef unsigned __int128 u128;
#define M51 0x7ffffffffffffULL

static inline uint64_t ld64(const uint8_t *p) {
  uint64_t v = 0;
  for (int i = 7; i >= 0; i--) v = (v << 8) | p[i];
  return v;
}
static inline void st64(uint8_t *p, uint64_t v) {
  for (int i = 0; i < 8; i++) { p[i] = (uint8_t)v; v >>= 8; }
}

/* ------------------------------------------------------------ field ---- */
void fe_0(fe *h) { memset(h, 0, sizeof *h); }
void fe_1(fe *h) { fe_0(h); h->v[0] = 1; }
void fe_from_u64(fe *h, uint64_t x) {
  fe_0(h);
  h->v[0] = x & M51;
  h->v[1] = x >> 51;
}

void fe_frombytes(fe *h, const uint8_t s[32]) {
  uint64_t w0 = ld64(s), w1 = ld64(s + 8), w2 = ld64(s + 16), w3 = ld64(s + 24);
  h->v[0] = w0 & M51;
  h->v[1] = ((w0 >> 51) | (w1 << 13)) & M51;
  h->v[2] = ((w1 >> 38) | (w2 << 26)) & M51;
  h->v[3] = ((w2 >> 25) | (w3 << 39)) & M51;
  h->v[4] = (w3 >> 12) & M51; /* bit 255 dropped */
}

static void fe_carry(fe *h) {
  uint64_t c;
  c = h->v[0] >> 51; h->v[0] &= M51; h->v[1] += c;
  c = h->v[1] >> 51; h->v[1] &= M51; h->v[2] += c;
  c = h->v[2] >> 51; h->v[2] &= M51; h->v[3] += c;
  c = h->v[3] >> 51; h->v[3] &= M51; h->v[4] += c;
  c = h->v[4] >> 51; h->v[4] &= M51; h->v[0] += 19 * c;
  c = h->v[0] >> 51; h->v[0] &= M51; h->v[1] += c;
}

void fe_tobytes(uint8_t s[32], const fe *f) {
  fe t = *f;
  fe_carry(&t);
  fe_carry(&t);
  /* q = floor((t + 19) / 2^255) in {0, 1}; t - q*p is canonical */
  uint64_t q = (t.v[0] + 19) >> 51;
  q = (t.v[1] + q) >> 51;
  q = (t.v[2] + q) >> 51;
  q = (t.v[3] + q) >> 51;
  q = (t.v[4] + q) >> 51;
  t.v[0] += 19 * q;
  uint64_t c;
  c = t.v[0] >> 51; t.v[0] &= M51; t.v[1] += c;
  c = t.v[1] >> 51; t.v[1] &= M51; t.v[2] += c;
  c = t.v[2] >> 51; t.v[2] &= M51; t.v[3] += c;
  c = t.v[3] >> 51; t.v[3] &= M51; t.v[4] += c;
  t.v[4] &= M51;
  st64(s, t.v[0] | (t.v[1] << 51));
  st64(s + 8, (t.v[1] >> 13) | (t.v[2] << 38));
  st64(s + 16, (t.v[2] >> 26) | (t.v[3] << 25));
  st64(s + 24, (t.v[3] >> 39) | (t.v[4] << 12));
}

void fe_add(fe *h, const fe *f, const fe *g) {
  for (int i = 0; i < 5; i++) h->v[i] = f->v[i] + g->v[i];
  fe_carry(h);
}

void fe_sub(fe *h, const fe *f, const fe *g) {
  /* f + 4p - g; 4p limbs = 2^53 - 76, 2^53 - 4 */
  h->v[0] = f->v[0] + 0x1fffffffffffb4ULL - g->v[0];
  for (int i = 1; i < 5; i++) h->v[i] = f->v[i] + 0x1ffffffffffffcULL - g->v[i];
  fe_carry(h);
}

void fe_neg(fe *h, const fe *f) {
  fe z;
  fe_0(&z);
  fe_sub(h, &z, f);
}

static void fe_reduce_wide(fe *h, u128 r0, u128 r1, u128 r2, u128 r3, u128 r4) {
  r1 += (uint64_t)(r0 >> 51);
  r2 += (uint64_t)(r1 >> 51);
  r3 += (uint64_t)(r2 >> 51);
  r4 += (uint64_t)(r3 >> 51);
  u128 t0 = (u128)((uint64_t)r0 & M51) + (u128)(uint64_t)(r4 >> 51) * 19;
  h->v[0] = (uint64_t)t0 & M51;
  h->v[1] = ((uint64_t)r1 & M51) + (uint64_t)(t0 >> 51);
  h->v[2] = (uint64_t)r2 & M51;
  h->v[3] = (uint64_t)r3 & M51;
  h->v[4] = (uint64_t)r4 & M51;
}

void fe_mul(fe *h, const fe *f, const fe *g) {
  uint64_t f0 = f->v[0], f1 = f->v[1], f2 = f->v[2], f3 = f->v[3], f4 = f->v[4];
  uint64_t g0 = g->v[0], g1 = g->v[1], g2 = g->v[2], g3 = g->v[3], g4 = g->v[4];
  uint64_t g1_19 = 19 * g1, g2_19 = 19 * g2, g3_19 = 19 * g3, g4_19 = 19 * g4;
  u128 r0 = (u128)f0 * g0 + (u128)f1 * g4_19 + (u128)f2 * g3_19 + (u128)f3 * g2_19 +
            (u128)f4 * g1_19;
  u128 r1 = (u128)f0 * g1 + (u128)f1 * g0 + (u128)f2 * g4_19 + (u128)f3 * g3_19 +
            (u128)f4 * g2_19;
  u128 r2 = (u128)f0 * g2 + (u128)f1 * g1 + (u128)f2 * g0 + (u128)f3 * g4_19 +
            (u128)f4 * g3_19;
  u128 r3 = (u128)f0 * g3 + (u128)f1 * g2 + (u128)f2 * g1 + (u128)f3 * g0 + (u128)f4 * g4_19;
  u128 r4 = (u128)f0 * g4 + (u128)f1 * g3 + (u128)f2 * g2 + (u128)f3 * g1 + (u128)f4 * g0;
  fe_reduce_wide(h, r0, r1, r2, r3, r4);
}

void fe_sq(fe *h, const fe *f) {
  uint64_t f0 = f->v[0], f1 = f->v[1], f2 = f->v[2], f3 = f->v[3], f4 = f->v[4];
  uint64_t f3_19 = 19 * f3, f4_19 = 19 * f4;
  u128 r0 = (u128)f0 * f0 + 2 * ((u128)f1 * f4_19 + (u128)f2 * f3_19);
  u128 r1 = 2 * ((u128)f0 * f1 + (u128)f2 * f4_19) + (u128)f3 * f3_19;
  u128 r2 = 2 * ((u128)f0 * f2 + (u128)f3 * f4_19) + (u128)f1 * f1;
  u128 r3 = 2 * ((u128)f0 * f3 + (u128)f1 * f2) + (u128)f4 * f4_19;
  u128 r4 = 2 * ((u128)f0 * f4 + (u128)f1 * f3) + (u128)f2 * f2;
  fe_reduce_wide(h, r0, r1, r2, r3, r4);
}

static void fe_sqn(fe *h, const fe *f, int n) {
  fe_sq(h, f);
  for (int i = 1; i < n; i++) fe_sq(h, h);
}

/* z^(2^250 - 1) and z^11, shared by invert and pow22523 */
static void fe_pow250(fe *z250, fe *z11, const fe *z) {
  fe z2, z9, t, z5, z10, z20, z50, z100;
  fe_sq(&z2, z);
  fe_sqn(&t, &z2, 2);
  fe_mul(&z9, &t, z);
  fe_mul(z11, &z9, &z2);
  fe_sq(&t, z11);
  fe_mul(&z5, &t, &z9); /* 2^5 - 1 */
  fe_sqn(&t, &z5, 5);
  fe_mul(&z10, &t, &z5); /* 2^10 - 1 */
  fe_sqn(&t, &z10, 10);
  fe_mul(&z20, &t, &z10);
  fe_sqn(&t, &z20, 20);
  fe_mul(&t, &t, &z20); /* 2^40 - 1 */
  fe_sqn(&t, &t, 10);
  fe_mul(&z50, &t, &z10);
  fe_sqn(&t, &z50, 50);
  fe_mul(&z100, &t, &z50);
  fe_sqn(&t, &z100, 100);
  fe_mul(&t, &t, &z100); /* 2^200 - 1 */
  fe_sqn(&t, &t, 50);
  fe_mul(z250, &t, &z50);
}

void fe_invert(fe *out, const fe *z) {
  fe z250, z11, t;
  fe_pow250(&z250, &z11, z);
  fe_sqn(&t, &z250, 5);
  fe_mul(out, &t, &z11); /* 2^255 - 21 = p - 2 */
}

void fe_pow22523(fe *out, const fe *z) {
  fe z250, z11, t;
  fe_pow250(&z250, &z11, z);
  fe_sqn(&t, &z250, 2);
  fe_mul(out, &t, z); /* 2^252 - 3 */
}

int fe_iszero(const fe *f) {
  uint8_t s[32];
  fe_tobytes(s, f);
  uint8_t acc = 0;
  for (int i = 0; i < 32; i++) acc |= s[i];
  return acc == 0;
}

int fe_isnegative(const fe *f) {
  uint8_t s[32];
  fe_tobytes(s, f);
  return s[0] & 1;
}

/* ------------------------------------------------------------ group ---- */
void ge_identity(ge *p) {
  fe_0(&p->X);
  fe_1(&p->Y);
  fe_1(&p->Z);
  fe_0(&p->T);
}

/* add-2008-hwcd-3 (a = -1), complete on edwards25519 */
void ge_add(ge *r, const ge *p, const ge *q) {
  const curve_consts *k = cc();
  fe a, b, c, d, e, f, g, h, t;
  fe_sub(&a, &p->Y, &p->X);
  fe_sub(&t, &q->Y, &q->X);
  fe_mul(&a, &a, &t);
  fe_add(&b, &p->Y, &p->X);
  fe_add(&t, &q->Y, &q->X);
  fe_mul(&b, &b, &t);
  fe_mul(&c, &p->T, &q->T);
  fe_mul(&c, &c, &k->d2);
  fe_mul(&d, &p->Z, &q->Z);
  fe_add(&d, &d, &d);
  fe_sub(&e, &b, &a);
  fe_sub(&f, &d, &c);
  fe_add(&g, &d, &c);
  fe_add(&h, &b, &a);
  fe_mul(&r->X, &e, &f);
  fe_mul(&r->Y, &g, &h);
  fe_mul(&r->T, &e, &h);
  fe_mul(&r->Z, &f, &g);
}

void ge_neg(ge *r, const ge *p) {
  fe_neg(&r->X, &p->X);
  r->Y = p->Y;
  r->Z = p->Z;
  fe_neg(&r->T, &p->T);
}

void ge_sub(ge *r, const ge *p, const ge *q) {
  ge nq;
  ge_neg(&nq, q);
  ge_add(r, p, &nq);
}

/* dbl-2008-hwcd (a = -1) */
void ge_dbl(ge *r, const ge *p) {
  fe a, b, c, e, g, f, h, t;
  fe_sq(&a, &p->X);
  fe_sq(&b, &p->Y);
  fe_sq(&c, &p->Z);
  fe_add(&c, &c, &c);
  fe_add(&t, &p->X, &p->Y);
  fe_sq(&t, &t);
  fe_sub(&e, &t, &a);
  fe_sub(&e, &e, &b);   /* E = (X+Y)^2 - A - B = 2XY */
  fe_sub(&g, &b, &a);   /* G = -A + B            */
  fe_sub(&f, &g, &c);   /* F = G - C             */
  fe_neg(&h, &a);
  fe_sub(&h, &h, &b);   /* H = -A - B            */
  fe_mul(&r->X, &e, &f);
  fe_mul(&r->Y, &g, &h);
  fe_mul(&r->T, &e, &h);
  fe_mul(&r->Z, &f, &g);
}

void ge_tobytes(uint8_t s[32], const ge *p) {
  fe zi, x, y;
  fe_invert(&zi, &p->Z);
  fe_mul(&x, &p->X, &zi);
  fe_mul(&y, &p->Y, &zi);
  fe_tobytes(s, &y);
  s[31] ^= (uint8_t)(fe_isnegative(&x) << 7);
}

/* shared decode: returns 0 and x with chosen parity, or -1 */
static int ge_decode(ge *p, const uint8_t s[32], int negate) {
  const curve_consts *k = cc();
  fe u, v, v3, vxx, chk, one;
  fe_frombytes(&p->Y, s);
  fe_1(&p->Z);
  fe_1(&one);
  fe_sq(&u, &p->Y);
  fe_mul(&v, &u, &k->d);
  fe_sub(&u, &u, &one); /* u = y^2 - 1   */
  fe_add(&v, &v, &one); /* v = d y^2 + 1 */
  fe_sq(&v3, &v);
  fe_mul(&v3, &v3, &v);       /* v^3 */
  fe_sq(&p->X, &v3);
  fe_mul(&p->X, &p->X, &v);
  fe_mul(&p->X, &p->X, &u);   /* u v^7 */
  fe_pow22523(&p->X, &p->X);
  fe_mul(&p->X, &p->X, &v3);
  fe_mul(&p->X, &p->X, &u);   /* u v^3 (u v^7)^((p-5)/8) */
  fe_sq(&vxx, &p->X);
  fe_mul(&vxx, &vxx, &v);
  fe_sub(&chk, &vxx, &u);
  if (!fe_iszero(&chk)) {
    fe_add(&chk, &vxx, &u);
    if (!fe_iszero(&chk)) return -1;
    fe_mul(&p->X, &p->X, &k->sqrtm1);
  }
  int sign = s[31] >> 7;
  int flip = negate ? (fe_isnegative(&p->X) == sign) : (fe_isnegative(&p->X) != sign);
  if (flip) fe_neg(&p->X, &p->X);
  fe_mul(&p->T, &p->X, &p->Y);
  return 0;
}

int ge_frombytes(ge *p, const uint8_t s[32]) { return ge_decode(p, s, 0); }
int ge_frombytes_negate(ge *p, const uint8_t s[32]) { return ge_decode(p, s, 1); }

int ge_is_canonical(const uint8_t s[32]) {
  /* y = s mod 2^255 must be < p = 2^255 - 19 */
  if ((s[31] & 0x7f) != 0x7f) return 1;
  for (int i = 30; i > 0; i--)
    if (s[i] != 0xff) return 1;
  return s[0] < 0xed;
}

/* y-coordinates of the small-order points (and their non-canonical aliases),
 * libsodium 1.0.18 ge25519_has_small_order's blocklist; built at init from
 * their definitions rather than typed in: 0, 1, +-y8 (order 8), p-1, p, p+1 */
static uint8_t small_order_y[7][32];

int ge_has_small_order(const uint8_t s[32]) {
  (void)cc();
  for (int i = 0; i < 7; i++) {
    int eq = 1;
    for (int j = 0; j < 31 && eq; j++) eq = (s[j] == small_order_y[i][j]);
    if (eq && (s[31] & 0x7f) == small_order_y[i][31]) return 1;
  }
  return 0;
}

/* width-5 signed sliding window recoding (odd digits in [-15, 15]) */
static void slide(int8_t r[256], const uint8_t a[32]) {
  for (int i = 0; i < 256; i++) r[i] = 1 & (a[i >> 3] >> (i & 7));
  for (int i = 0; i < 256; i++) {
    if (!r[i]) continue;
    for (int b = 1; b <= 6 && i + b < 256; b++) {
      if (!r[i + b]) continue;
      if (r[i] + (r[i + b] << b) <= 15) {
        r[i] += r[i + b] << b;
        r[i + b] = 0;
      } else if (r[i] - (r[i + b] << b) >= -15) {
        r[i] -= r[i + b] << b;
        for (int k = i + b; k < 256; k++) {
          if (!r[k]) { r[k] = 1; break; }
          r[k] = 0;
        }
      } else {
        break;
      }
    }
  }
}

static void odd_multiples(ge tab[8], const ge *P) {
  ge P2;
  tab[0] = *P;
  ge_dbl(&P2, P);
  for (int i = 1; i < 8; i++) ge_add(&tab[i], &tab[i - 1], &P2);
}

static void add_digit(ge *r, const ge tab[8], int8_t d) {
  if (d > 0) ge_add(r, r, &tab[d / 2]);
  else if (d < 0) ge_sub(r, r, &tab[(-d) / 2]);
}

void ge_double_scalarmult(ge *r, const uint8_t a[32], const ge *P, const uint8_t b[32],
                          const ge *Q) {
  int8_t as[256], bs[256];
  ge pt[8], qt[8];
  slide(as, a);
  slide(bs, b);
  odd_multiples(pt, P);
  odd_multiples(qt, Q);
  ge_identity(r);
  int i = 255;
  while (i >= 0 && !as[i] && !bs[i]) i--;
  for (; i >= 0; i--) {
    ge_dbl(r, r);
    add_digit(r, pt, as[i]);
    add_digit(r, qt, bs[i]);
  }
}

void ge_scalarmult(ge *r, const uint8_t a[32], const ge *P) {
  int8_t as[256];
  ge pt[8];
  slide(as, a);
  odd_multiples(pt, P);
  ge_identity(r);
  int i = 255;
  while (i >= 0 && !as[i]) i--;
  for (; i >= 0; i--) {
    ge_dbl(r, r);
    add_digit(r, pt, as[i]);
  }
}

void ge_scalarmult_base(ge *r, const uint8_t a[32]) {
  const curve_consts *k = cc();
  int8_t as[256];
  slide(as, a);
  ge_identity(r);
  int i = 255;
  while (i >= 0 && !as[i]) i--;
  for (; i >= 0; i--) {
    ge_dbl(r, r);
    add_digit(r, k->Btab, as[i]);
  }
}

/* ------------------------------------------------------------ constants ---- */
static curve_consts g_cc;
static pthread_once_t g_cc_once = PTHREAD_ONCE_INIT;
static __thread int g_cc_initialising; /* cc() re-entered from cc_init() */

static void cc_init(void) {
  fe t, u;
  g_cc_initialising = 1;
  /* d = -121665 / 121666 */
  fe_from_u64(&t, 121666);
  fe_invert(&t, &t);
  fe_from_u64(&u, 121665);
  fe_mul(&t, &t, &u);
  fe_neg(&g_cc.d, &t);
  fe_add(&g_cc.d2, &g_cc.d, &g_cc.d);
  /* sqrt(-1) = 2^((p-1)/4) = 2^(2^253 - 5) = 4^(2^252 - 3) * 2 */
  fe_from_u64(&t, 4);
  fe_pow22523(&u, &t);
  fe_from_u64(&t, 2);
  fe_mul(&g_cc.sqrtm1, &u, &t);
  fe_from_u64(&g_cc.mont_a, 486662);
  /* B: y = 4/5, x even (sign bit 0) */
  uint8_t by[32];
  fe_from_u64(&t, 5);
  fe_invert(&t, &t);
  fe_from_u64(&u, 4);
  fe_mul(&t, &t, &u);
  fe_tobytes(by, &t);
  ge_decode(&g_cc.B, by, 0);
  odd_multiples(g_cc.Btab, &g_cc.B);
  /* small-order y blocklist: 0 (order 4), 1 (identity), +-y8 (order 8),
   * then the non-canonical strings p-1 (order 2), p (= 0), p+1 (= 1) */
  memset(small_order_y, 0, sizeof small_order_y);
  small_order_y[1][0] = 1;
  {
    /* an order-8 point is [L]Q for any Q whose torsion part has order 8 */
    static const uint8_t L[32] = {0xed, 0xd3, 0xf5, 0x5c, 0x1a, 0x63, 0x12, 0x58,
                                  0xd6, 0x9c, 0xf7, 0xa2, 0xde, 0xf9, 0xde, 0x14,
                                  0,    0,    0,    0,    0,    0,    0,    0,
                                  0,    0,    0,    0,    0,    0,    0,    0x10};
    static const uint8_t id[32] = {1};
    for (uint64_t yy = 2;; yy++) {
      uint8_t ys[32], e4[32], ty[32];
      ge Q, T, T4;
      fe_from_u64(&t, yy);
      fe_tobytes(ys, &t);
      if (ge_decode(&Q, ys, 0) != 0) continue;
      ge_scalarmult(&T, L, &Q);
      ge_dbl(&T4, &T);
      ge_dbl(&T4, &T4);
      ge_tobytes(e4, &T4);
      if (memcmp(e4, id, 32) == 0) continue; /* order < 8 */
      ge_tobytes(ty, &T);
      ty[31] &= 0x7f;
      memcpy(small_order_y[2], ty, 32);
      fe_frombytes(&t, ty);
      fe_neg(&t, &t);
      fe_tobytes(small_order_y[3], &t);
      break;
    }
  }
  for (int j = 0; j < 3; j++) {
    memset(small_order_y[4 + j], 0xff, 32);
    small_order_y[4 + j][31] = 0x7f;
    small_order_y[4 + j][0] = (uint8_t)(0xec + j);
  }
  g_cc_initialising = 0;
}

const curve_consts *cc(void) {
  if (!g_cc_initialising) pthread_once(&g_cc_once, cc_init);
  return &g_cc;
}

/* ------------------------------------------------------------ scalars ---- */
static const uint64_t Lw[4] = {0x5812631a5cf5d3edULL, 0x14def9dea2f79cd6ULL, 0, 0x1000000000000000ULL};

static int geq_L(const uint64_t r[4]) {
  for (int i = 3; i >= 0; i--) {
    if (r[i] > Lw[i]) return 1;
    if (r[i] < Lw[i]) return 0;
  }
  return 1;
}

static void sub_L(uint64_t r[4]) {
  uint64_t borrow = 0;
  for (int i = 0; i < 4; i++) {
    u128 d = (u128)r[i] - Lw[i] - borrow;
    r[i] = (uint64_t)d;
    borrow = (uint64_t)(d >> 64) & 1;
  }
}

/* out = in mod L, in little-endian of nbytes; bit-serial (oracle: clarity first) */
void sc_reduce(uint8_t out[32], const uint8_t *in, size_t nbytes) {
  uint64_t r[4] = {0, 0, 0, 0};
  for (long bit = (long)nbytes * 8 - 1; bit >= 0; bit--) {
    r[3] = (r[3] << 1) | (r[2] >> 63);
    r[2] = (r[2] << 1) | (r[1] >> 63);
    r[1] = (r[1] << 1) | (r[0] >> 63);
    r[0] = (r[0] << 1) | ((in[bit >> 3] >> (bit & 7)) & 1);
    if (geq_L(r)) sub_L(r);
  }
  for (int i = 0; i < 4; i++) st64(out + 8 * i, r[i]);
}

void sc_muladd(uint8_t s[32], const uint8_t a[32], const uint8_t b[32], const uint8_t c[32]) {
  uint64_t aw[4], bw[4], prod[9] = {0};
  for (int i = 0; i < 4; i++) { aw[i] = ld64(a + 8 * i); bw[i] = ld64(b + 8 * i); }
  for (int i = 0; i < 4; i++) {
    uint64_t carry = 0;
    for (int j = 0; j < 4; j++) {
      u128 t = (u128)aw[i] * bw[j] + prod[i + j] + carry;
      prod[i + j] = (uint64_t)t;
      carry = (uint64_t)(t >> 64);
    }
    prod[i + 4] += carry;
  }
  uint64_t carry = 0;
  for (int i = 0; i < 9; i++) {
    u128 t = (u128)prod[i] + (i < 4 ? ld64(c + 8 * i) : 0) + carry;
    prod[i] = (uint64_t)t;
    carry = (uint64_t)(t >> 64);
  }
  uint8_t wide[72];
  for (int i = 0; i < 9; i++) st64(wide + 8 * i, prod[i]);
  sc_reduce(s, wide, 72);
}

int sc_is_canonical(const uint8_t s[32]) {
  uint64_t r[4];
  for (int i = 0; i < 4; i++) r[i] = ld64(s + 8 * i);
  return !geq_L(r);
}
