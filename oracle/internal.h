/* internal.h -- shared internals of the CPU oracle.  TEST INFRASTRUCTURE ONLY. */
#ifndef OURO_ORACLE_INTERNAL_H
#define OURO_ORACLE_INTERNAL_H
#include "oracle.h"

typedef struct {
  uint64_t H[8];
  uint8_t buf[128];
  size_t buflen;
  uint64_t total;
} orc_sha512_ctx;
void orc_sha512_init(orc_sha512_ctx *c);
void orc_sha512_update(orc_sha512_ctx *c, const uint8_t *in, size_t len);
void orc_sha512_final(orc_sha512_ctx *c, uint8_t out[64]);

/* GF(2^255-19), 5 x 51-bit limbs, weakly reduced (each limb < 2^52) */
typedef struct { uint64_t v[5]; } fe;
/* extended twisted-Edwards point (X:Y:Z:T), x = X/Z, y = Y/Z, xy = T/Z */
typedef struct { fe X, Y, Z, T; } ge;

void fe_frombytes(fe *h, const uint8_t s[32]);
void fe_tobytes(uint8_t s[32], const fe *f);
void fe_0(fe *h);
void fe_1(fe *h);
void fe_add(fe *h, const fe *f, const fe *g);
void fe_sub(fe *h, const fe *f, const fe *g);
void fe_neg(fe *h, const fe *f);
void fe_mul(fe *h, const fe *f, const fe *g);
void fe_sq(fe *h, const fe *f);
void fe_invert(fe *out, const fe *z);
void fe_pow22523(fe *out, const fe *z);
int fe_iszero(const fe *f);
int fe_isnegative(const fe *f);
void fe_from_u64(fe *h, uint64_t x);

/* curve constants, derived at first use */
typedef struct {
  fe d, d2, sqrtm1, mont_a;
  ge B;
  ge Btab[8]; /* odd multiples B, 3B, ..., 15B */
} curve_consts;
const curve_consts *cc(void);

void ge_identity(ge *p);
void ge_add(ge *r, const ge *p, const ge *q);
void ge_sub(ge *r, const ge *p, const ge *q);
void ge_dbl(ge *r, const ge *p);
void ge_neg(ge *r, const ge *p);
void ge_tobytes(uint8_t s[32], const ge *p);
/* libsodium ge25519_frombytes: 0 ok / -1 no square root; y read mod 2^255 */
int ge_frombytes(ge *p, const uint8_t s[32]);
/* libsodium ge25519_frombytes_negate_vartime: decodes -P */
int ge_frombytes_negate(ge *p, const uint8_t s[32]);
int ge_is_canonical(const uint8_t s[32]);
int ge_has_small_order(const uint8_t s[32]);
/* r = [a]P + [b]Q, vartime; a, b are 32-byte little-endian scalars < 2^256 */
void ge_double_scalarmult(ge *r, const uint8_t a[32], const ge *P, const uint8_t b[32],
                          const ge *Q);
void ge_scalarmult(ge *r, const uint8_t a[32], const ge *P);
void ge_scalarmult_base(ge *r, const uint8_t a[32]);

/* scalars mod L = 2^252 + 27742317777372353535851937790883648493 */
void sc_reduce(uint8_t out[32], const uint8_t *in, size_t nbytes);
void sc_muladd(uint8_t s[32], const uint8_t a[32], const uint8_t b[32], const uint8_t c[32]);
int sc_is_canonical(const uint8_t s[32]);

#endif
