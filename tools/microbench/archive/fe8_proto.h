// fe8_proto.h -- prototype GF(2^255-19) in 8 x 32-bit unsigned limbs (radix 2^32),
// for the field-multiply microbenchmark (fe_mul_variants.hip).  Values are kept
// in [0, 2^256) ("weakly reduced"); 2^256 = 38 (mod p).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fe8p {

struct fe8 {
  uint32_t v[8];
};

#define F8I __device__ __forceinline__

// acc = a*b + acc (64-bit), returns the carry-out lane mask
F8I uint64_t mad_cc(uint64_t& acc, uint32_t a, uint32_t b) {
  uint64_t cc;
  asm("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc), "=s"(cc) : "v"(a), "v"(b));
  return cc;
}
// x + carry(cc)
F8I uint32_t add_cc(uint32_t x, uint64_t cc) {
  uint32_t r;
  uint64_t dummy;
  asm("v_addc_co_u32_e64 %0, %1, %2, 0, %3" : "=v"(r), "=s"(dummy) : "v"(x), "s"(cc));
  return r;
}

// 512-bit product t[16] of two 256-bit values, product scanning, one chain
F8I void mul512_1chain(uint32_t t[16], const uint32_t a[8], const uint32_t b[8]) {
  uint64_t acc = 0;
  uint32_t hi = 0;
#pragma unroll
  for (int k = 0; k < 15; k++) {
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const int j = k - i;
      if (j < 0 || j > 7) continue;
      uint64_t cc = mad_cc(acc, a[i], b[j]);
      hi = add_cc(hi, cc);
    }
    t[k] = (uint32_t)acc;
    acc = (acc >> 32) | ((uint64_t)hi << 32);
    hi = 0;
  }
  t[15] = (uint32_t)acc;
}

// plain C version (compiler-scheduled)
F8I void mul512_c(uint32_t t[16], const uint32_t a[8], const uint32_t b[8]) {
  uint64_t acc = 0;
  uint32_t hi = 0;
#pragma unroll
  for (int k = 0; k < 15; k++) {
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const int j = k - i;
      if (j < 0 || j > 7) continue;
      uint64_t p = (uint64_t)a[i] * b[j];
      uint64_t s = acc + p;
      hi += (s < p) ? 1u : 0u;
      acc = s;
    }
    t[k] = (uint32_t)acc;
    acc = (acc >> 32) | ((uint64_t)hi << 32);
    hi = 0;
  }
  t[15] = (uint32_t)acc;
}

// lo(x) + hi(y) + carry-in -> (sum, carry-out)
F8I uint32_t addc3(uint32_t x, uint32_t y, uint64_t cin, uint64_t& cout) {
  uint32_t r;
  asm("v_addc_co_u32_e64 %0, %1, %2, %3, %4" : "=v"(r), "=s"(cout) : "v"(x), "v"(y), "s"(cin));
  return r;
}
F8I uint32_t add_co(uint32_t x, uint32_t y, uint64_t& cout) {
  uint32_t r;
  asm("v_add_co_u32_e64 %0, %1, %2, %3" : "=v"(r), "=s"(cout) : "v"(x), "v"(y));
  return r;
}
F8I uint64_t mad64(uint32_t a, uint32_t b, uint64_t c) {
  uint64_t r, cc;
  asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(r), "=s"(cc) : "v"(a), "v"(b), "v"(c));
  return r;
}

// operand scanning: row i adds a_i * b into t[i..i+8]; each product
// u_j = a_i b_j + t[i+j] (< 2^64), then t[i+j] = lo(u_j) + hi(u_{j-1}) + carry
F8I void mul512_os(uint32_t t[16], const uint32_t a[8], const uint32_t b[8]) {
  // row 0: plain products
  uint64_t u[8];
#pragma unroll
  for (int j = 0; j < 8; j++) u[j] = mad64(a[0], b[j], 0);
  t[0] = (uint32_t)u[0];
  uint64_t c;
  t[1] = add_co((uint32_t)u[1], (uint32_t)(u[0] >> 32), c);
#pragma unroll
  for (int j = 2; j < 8; j++) t[j] = addc3((uint32_t)u[j], (uint32_t)(u[j - 1] >> 32), c, c);
  t[8] = addc3((uint32_t)(u[7] >> 32), 0u, c, c);  // no carry out: row value < 2^288
#pragma unroll
  for (int i = 1; i < 8; i++) {
#pragma unroll
    for (int j = 0; j < 8; j++) u[j] = mad64(a[i], b[j], (uint64_t)t[i + j]);
    t[i] = (uint32_t)u[0];
    t[i + 1] = add_co((uint32_t)u[1], (uint32_t)(u[0] >> 32), c);
#pragma unroll
    for (int j = 2; j < 8; j++) t[i + j] = addc3((uint32_t)u[j], (uint32_t)(u[j - 1] >> 32), c, c);
    t[i + 8] = addc3((uint32_t)(u[7] >> 32), 0u, c, c);
  }
}

// operand scanning with compiler-visible ops (__builtin_addc chains)
F8I void mul512_osc(uint32_t t[16], const uint32_t a[8], const uint32_t b[8]) {
  uint64_t u[8];
  unsigned c;
#pragma unroll
  for (int j = 0; j < 8; j++) u[j] = (uint64_t)a[0] * b[j];
  t[0] = (uint32_t)u[0];
  c = 0;
#pragma unroll
  for (int j = 1; j < 8; j++) t[j] = __builtin_addc((uint32_t)u[j], (uint32_t)(u[j - 1] >> 32), c, &c);
  t[8] = (uint32_t)(u[7] >> 32) + c;
#pragma unroll
  for (int i = 1; i < 8; i++) {
#pragma unroll
    for (int j = 0; j < 8; j++) u[j] = (uint64_t)a[i] * b[j] + t[i + j] * (j < 8 - 0 ? 1ull : 1ull);
    t[i] = (uint32_t)u[0];
    c = 0;
#pragma unroll
    for (int j = 1; j < 8; j++)
      t[i + j] = __builtin_addc((uint32_t)u[j], (uint32_t)(u[j - 1] >> 32), c, &c);
    t[i + 8] = (uint32_t)(u[7] >> 32) + c;
  }
}

// r = t mod' p as 8 limbs in [0, 2^256): t_lo + 38 t_hi, folded twice
F8I fe8 reduce512(const uint32_t t[16]) {
  uint64_t w[8];
#pragma unroll
  for (int i = 0; i < 8; i++) w[i] = (uint64_t)t[8 + i] * 38u + t[i];  // < 2^38 + 2^32
  fe8 r;
  uint32_t c = 0;
  r.v[0] = (uint32_t)w[0];
#pragma unroll
  for (int i = 1; i < 8; i++) {
    uint64_t s = (uint64_t)(uint32_t)w[i] + (uint32_t)(w[i - 1] >> 32) + c;
    r.v[i] = (uint32_t)s;
    c = (uint32_t)(s >> 32);
  }
  uint32_t top = (uint32_t)(w[7] >> 32) + c;  // < 2^7
  uint64_t s = (uint64_t)top * 38u + r.v[0];
  r.v[0] = (uint32_t)s;
  c = (uint32_t)(s >> 32);
#pragma unroll
  for (int i = 1; i < 8; i++) {
    uint64_t s2 = (uint64_t)r.v[i] + c;
    r.v[i] = (uint32_t)s2;
    c = (uint32_t)(s2 >> 32);
  }
  r.v[0] += c * 38u;  // r < 2^13 here when c = 1: no carry
  return r;
}

F8I fe8 mul_1chain(const fe8& a, const fe8& b) {
  uint32_t t[16];
  mul512_1chain(t, a.v, b.v);
  return reduce512(t);
}
F8I fe8 mul_os(const fe8& a, const fe8& b) {
  uint32_t t[16];
  mul512_os(t, a.v, b.v);
  return reduce512(t);
}
F8I fe8 mul_osc(const fe8& a, const fe8& b) {
  uint32_t t[16];
  mul512_osc(t, a.v, b.v);
  return reduce512(t);
}
F8I fe8 mul_c(const fe8& a, const fe8& b) {
  uint32_t t[16];
  mul512_c(t, a.v, b.v);
  return reduce512(t);
}

// squaring: cross products once, doubled, plus the diagonal
F8I fe8 sq_1chain(const fe8& a) {
  uint32_t t[16];
  uint64_t acc = 0;
  uint32_t hi = 0;
  t[0] = 0;
#pragma unroll
  for (int k = 1; k < 14; k++) {
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const int j = k - i;
      if (j <= i || j > 7) continue;
      uint64_t cc = mad_cc(acc, a.v[i], a.v[j]);
      hi = add_cc(hi, cc);
    }
    t[k] = (uint32_t)acc;
    acc = (acc >> 32) | ((uint64_t)hi << 32);
    hi = 0;
  }
  t[14] = (uint32_t)acc;
  t[15] = (uint32_t)(acc >> 32);
  // double
#pragma unroll
  for (int k = 15; k > 0; k--) t[k] = (t[k] << 1) | (t[k - 1] >> 31);
  t[0] <<= 1;
  // add the diagonal a_i^2 at 2^(64 i)
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint64_t d = (uint64_t)a.v[i] * a.v[i];
    uint64_t s0 = (uint64_t)t[2 * i] + (uint32_t)d + c;
    t[2 * i] = (uint32_t)s0;
    uint64_t s1 = (uint64_t)t[2 * i + 1] + (uint32_t)(d >> 32) + (uint32_t)(s0 >> 32);
    t[2 * i + 1] = (uint32_t)s1;
    c = (uint32_t)(s1 >> 32);
  }
  return reduce512(t);
}

F8I fe8 from_words(const uint32_t w[8]) {
  fe8 r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = w[i];
  r.v[7] &= 0x7fffffffu;
  return r;
}

// canonical words: value < 2^256 -> subtract p at most twice
F8I void to_words(uint32_t w[8], const fe8& f) {
  uint32_t r[8];
#pragma unroll
  for (int i = 0; i < 8; i++) r[i] = f.v[i];
#pragma unroll
  for (int pass = 0; pass < 2; pass++) {
    // r >= p  <=>  r + 19 >= 2^255
    uint64_t s = (uint64_t)r[0] + 19u;
    uint32_t c = (uint32_t)(s >> 32);
#pragma unroll
    for (int i = 1; i < 7; i++) {
      uint64_t s2 = (uint64_t)r[i] + c;
      c = (uint32_t)(s2 >> 32);
    }
    const uint32_t ge = ((uint64_t)r[7] + c) >> 31 ? 1u : 0u;  // bit 255 of r + 19
    // r -= ge * p  ==  r + ge*19 - ge*2^255
    uint64_t t = (uint64_t)r[0] + 19u * ge;
    r[0] = (uint32_t)t;
    c = (uint32_t)(t >> 32);
#pragma unroll
    for (int i = 1; i < 8; i++) {
      uint64_t s2 = (uint64_t)r[i] + c;
      r[i] = (uint32_t)s2;
      c = (uint32_t)(s2 >> 32);
    }
    r[7] -= ge << 31;
  }
#pragma unroll
  for (int i = 0; i < 8; i++) w[i] = r[i];
}

// ---- radix 2^25.5, 10 UNSIGNED limbs, floor carries (prototype) ----------
struct fe10u {
  uint32_t v[10];
};

F8I fe10u carry64u(uint64_t t[10]) {
  uint64_t c;
#define CU(i, j, bits)            \
  c = t[i] >> bits;               \
  t[j] += c;                      \
  t[i] &= ((1ull << bits) - 1);
  CU(0, 1, 26)
  CU(4, 5, 26)
  CU(1, 2, 25)
  CU(5, 6, 25)
  CU(2, 3, 26)
  CU(6, 7, 26)
  CU(3, 4, 25)
  CU(7, 8, 25)
  CU(4, 5, 26)
  CU(8, 9, 26)
  c = t[9] >> 25;
  t[9] &= (1u << 25) - 1;
  t[0] += c * 19;
  CU(0, 1, 26)
#undef CU
  fe10u h;
#pragma unroll
  for (int i = 0; i < 10; i++) {
    h.v[i] = (uint32_t)t[i];
    asm("" : "+v"(h.v[i]));  // hide the limb ranges from known-bits narrowing
  }
  return h;
}

F8I fe10u mul10u(const fe10u& f, const fe10u& g) {
  uint32_t g19[10], f2[10];
#pragma unroll
  for (int i = 0; i < 10; i++) {
    g19[i] = 19u * g.v[i];
    f2[i] = (i & 1) ? 2u * f.v[i] : f.v[i];
  }
  uint64_t t[10];
#pragma unroll
  for (int k = 0; k < 10; k++) t[k] = 0;
#pragma unroll
  for (int i = 0; i < 10; i++) {
#pragma unroll
    for (int j = 0; j < 10; j++) {
      const int k = i + j;
      const uint32_t a = ((i & 1) && (j & 1)) ? f2[i] : f.v[i];
      const uint32_t b = (k >= 10) ? g19[j] : g.v[j];
      t[k >= 10 ? k - 10 : k] += (uint64_t)a * b;
    }
  }
  return carry64u(t);
}

F8I fe10u sq10u(const fe10u& f) {
  uint32_t f2[10], f4[10], f19[10];
#pragma unroll
  for (int i = 0; i < 10; i++) {
    f2[i] = 2u * f.v[i];
    f4[i] = 4u * f.v[i];
    f19[i] = 19u * f.v[i];
  }
  uint64_t t[10];
#pragma unroll
  for (int k = 0; k < 10; k++) t[k] = 0;
#pragma unroll
  for (int i = 0; i < 10; i++) {
    {
      const int k = 2 * i;
      const uint32_t a = (i & 1) ? f2[i] : f.v[i];
      const uint32_t b = (k >= 10) ? f19[i] : f.v[i];
      t[k >= 10 ? k - 10 : k] += (uint64_t)a * b;
    }
#pragma unroll
    for (int j = i + 1; j < 10; j++) {
      const int k = i + j;
      const uint32_t a = ((i & 1) && (j & 1)) ? f4[i] : f2[i];
      const uint32_t b = (k >= 10) ? f19[j] : f.v[j];
      t[k >= 10 ? k - 10 : k] += (uint64_t)a * b;
    }
  }
  return carry64u(t);
}

// Deferred-19 variants: wrapped columns (i + j >= 10) accumulate unscaled in
// hi[], then lo[k] += 19 hi[k] once per column.  No operand is pre-multiplied
// by 19, so the only input constraint is the column sum (< 2^64).
F8I fe10u mul10d(const fe10u& f, const fe10u& g) {
  uint32_t f2[10];
#pragma unroll
  for (int i = 0; i < 10; i++) f2[i] = (i & 1) ? 2u * f.v[i] : f.v[i];
  uint64_t lo[10], hi[10];
#pragma unroll
  for (int k = 0; k < 10; k++) lo[k] = hi[k] = 0;
#pragma unroll
  for (int i = 0; i < 10; i++) {
#pragma unroll
    for (int j = 0; j < 10; j++) {
      const int k = i + j;
      const uint32_t a = ((i & 1) && (j & 1)) ? f2[i] : f.v[i];
      if (k < 10) lo[k] += (uint64_t)a * g.v[j];
      else hi[k - 10] += (uint64_t)a * g.v[j];
    }
  }
#pragma unroll
  for (int k = 0; k < 9; k++) lo[k] += 19ull * hi[k];
  return carry64u(lo);
}

F8I fe10u sq10d(const fe10u& f) {
  uint32_t f2[10], f4[10];
#pragma unroll
  for (int i = 0; i < 10; i++) {
    f2[i] = 2u * f.v[i];
    f4[i] = 4u * f.v[i];
  }
  uint64_t lo[10], hi[10];
#pragma unroll
  for (int k = 0; k < 10; k++) lo[k] = hi[k] = 0;
#pragma unroll
  for (int i = 0; i < 10; i++) {
    {
      const int k = 2 * i;
      const uint32_t a = (i & 1) ? f2[i] : f.v[i];
      if (k < 10) lo[k] += (uint64_t)a * f.v[i];
      else hi[k - 10] += (uint64_t)a * f.v[i];
    }
#pragma unroll
    for (int j = i + 1; j < 10; j++) {
      const int k = i + j;
      const uint32_t a = ((i & 1) && (j & 1)) ? f4[i] : f2[i];
      if (k < 10) lo[k] += (uint64_t)a * f.v[j];
      else hi[k - 10] += (uint64_t)a * f.v[j];
    }
  }
#pragma unroll
  for (int k = 0; k < 9; k++) lo[k] += 19ull * hi[k];
  return carry64u(lo);
}

F8I fe10u from_words10u(const uint32_t w[8]) {
  ouro::fe s = ouro::fe_from_words(w);  // balanced -> carry to unsigned
  uint64_t t[10];
  // add 2p limbwise to make every limb positive, then floor-carry
  const uint32_t p2[10] = {0x7ffffda, 0x3fffffe, 0x7fffffe, 0x3fffffe, 0x7fffffe,
                           0x3fffffe, 0x7fffffe, 0x3fffffe, 0x7fffffe, 0x3fffffe};
#pragma unroll
  for (int i = 0; i < 10; i++) t[i] = (uint64_t)(int64_t)(s.v[i] + (int32_t)p2[i]);
  return carry64u(t);
}

F8I void to_words10u(uint32_t w[8], const fe10u& f) {
  ouro::fe s;
#pragma unroll
  for (int i = 0; i < 10; i++) s.v[i] = (int32_t)f.v[i];
  ouro::fe_to_words(w, s);
}

}  // namespace fe8p
