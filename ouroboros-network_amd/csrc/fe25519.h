// fe25519.h -- GF(2^255 - 19) for gfx950, one field element per lane.
//
// Representation: 10 signed 32-bit limbs, radix 2^25.5 (limb i weighs
// 2^ceil(25.5 i): 26-bit even limbs, 25-bit odd limbs).  Products accumulate
// in signed 64-bit, which hipcc lowers to v_mad_i64_i32 -- measured on MI355X
// at ~46.7 lane-ops/CU/clk, i.e. the 64-bit MAC path, see
// tools/microbench/int_rates.hip and DESIGN.md.  Signed limbs make subtraction
// free of 2p offsets.
//
// Bound discipline ("reduced" = what fe_mul/fe_sq/fe_carry return):
//   |even limb| <= 2^25, |odd limb| <= 2^24 (+ a few units).
// fe_mul / fe_sq inputs may be any sum/difference of at most three reduced
// elements (|limb| < 1.68 * 2^26 keeps 19*g in int32 and every column sum in
// int64).  The group formulas in ge25519.h respect this.
#pragma once
#include "common.h"

// Operation counting for the host test build only (tools/count_ops.py): the
// device code never defines OURO_COUNT_OPS.
// The same build also checks the bound discipline below on every multiplier
// input (tests assert zero violations over all vectors).
#if defined(OURO_COUNT_OPS) && !defined(__HIP_DEVICE_COMPILE__)
extern thread_local unsigned long long g_ouro_nmul, g_ouro_nsq, g_ouro_bound_violations;
#define OURO_COUNT_MUL() (++g_ouro_nmul)
#define OURO_COUNT_SQ() (++g_ouro_nsq)
#define OURO_CHECK_BOUNDS(f)                                                  \
  do {                                                                        \
    for (int i_ = 0; i_ < 10; i_++)                                           \
      if ((f).v[i_] > 113025455 || (f).v[i_] < -113025455) ++g_ouro_bound_violations; \
  } while (0)
#else
#define OURO_COUNT_MUL() ((void)0)
#define OURO_COUNT_SQ() ((void)0)
#define OURO_CHECK_BOUNDS(f) ((void)0)
#endif

namespace ouro {

struct fe {
  int32_t v[10];
};

// ---- constants (balanced limbs; generated from the integers) ----
#define OURO_FE(a0, a1, a2, a3, a4, a5, a6, a7, a8, a9) \
  { { a0, a1, a2, a3, a4, a5, a6, a7, a8, a9 } }
// d = -121665/121666
OURO_FI fe fe_d() {
  fe r = OURO_FE(-10913610, 13857413, -15372611, 6949391, 114729, -8787816, -6275908, -3247719,
                 -18696448, -12055116);
  return r;
}
OURO_FI fe fe_d2() {
  fe r = OURO_FE(-21827239, -5839606, -30745221, 13898782, 229458, 15978800, -12551817, -6495438,
                 29715968, 9444199);
  return r;
}
OURO_FI fe fe_sqrtm1() {
  fe r = OURO_FE(-32595792, -7943725, 9377950, 3500415, 12389472, -272473, -25146209, -2005654,
                 326686, 11406482);
  return r;
}
// Montgomery A = 486662 (curve25519), used by Elligator2
OURO_FI fe fe_mont_a() {
  fe r = OURO_FE(486662, 0, 0, 0, 0, 0, 0, 0, 0, 0);
  return r;
}

OURO_FI fe fe_zero() {
  fe r = OURO_FE(0, 0, 0, 0, 0, 0, 0, 0, 0, 0);
  return r;
}
OURO_FI fe fe_one() {
  fe r = OURO_FE(1, 0, 0, 0, 0, 0, 0, 0, 0, 0);
  return r;
}

OURO_FI fe fe_add(const fe& f, const fe& g) {
  fe h;
#pragma unroll
  for (int i = 0; i < 10; i++) h.v[i] = f.v[i] + g.v[i];
  return h;
}
OURO_FI fe fe_sub(const fe& f, const fe& g) {
  fe h;
#pragma unroll
  for (int i = 0; i < 10; i++) h.v[i] = f.v[i] - g.v[i];
  return h;
}
OURO_FI fe fe_neg(const fe& f) {
  fe h;
#pragma unroll
  for (int i = 0; i < 10; i++) h.v[i] = -f.v[i];
  return h;
}
// c ? a : b, per lane
OURO_FI fe fe_select(const fe& a, const fe& b, bool c) {
  fe h;
#pragma unroll
  for (int i = 0; i < 10; i++) h.v[i] = c ? a.v[i] : b.v[i];
  return h;
}

// signed bit-field extract of the low `bits` bits (v_bfe_i32)
OURO_FI int32_t sbfe(int32_t x, int bits) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_sbfe(x, 0, bits);
#else
  return (int32_t)((uint32_t)x << (32 - bits)) >> (32 - bits);
#endif
}

// Balanced (rounding) carry of a 10-column int64 accumulator into a reduced fe.
// Two interleaved chains (0..4 and 4..9) for ILP, then the 2^255 = 19 wrap.
// Per step: c = (t + 2^(b-1)) >> b, and the limb t - c 2^b is the b-bit
// signed field of t's low word (the representative of t mod 2^b in
// [-2^(b-1), 2^(b-1))), one v_bfe_i32.
OURO_FI fe fe_carry64(int64_t t[10]) {
  int64_t c;
#define OURO_CARRY(i, j, bits)                           \
  c = (t[i] + ((int64_t)1 << (bits - 1))) >> bits;        \
  t[j] += c;                                             \
  t[i] = sbfe((int32_t)t[i], bits);
  OURO_CARRY(0, 1, 26)
  OURO_CARRY(4, 5, 26)
  OURO_CARRY(1, 2, 25)
  OURO_CARRY(5, 6, 25)
  OURO_CARRY(2, 3, 26)
  OURO_CARRY(6, 7, 26)
  OURO_CARRY(3, 4, 25)
  OURO_CARRY(7, 8, 25)
  OURO_CARRY(4, 5, 26)
  OURO_CARRY(8, 9, 26)
  c = (t[9] + ((int64_t)1 << 24)) >> 25;
  t[0] += c * 19;
  t[9] = sbfe((int32_t)t[9], 25);
  OURO_CARRY(0, 1, 26)
#undef OURO_CARRY
  fe h;
#pragma unroll
  for (int i = 0; i < 10; i++) {
    h.v[i] = (int32_t)t[i];
#if defined(__HIP_DEVICE_COMPILE__)
    // hide the limb ranges: with them known, LLVM narrows the next multiply's
    // 64-bit MACs into 32-bit pieces and triples its instruction count
    asm("" : "+v"(h.v[i]));
#endif
  }
  return h;
}

// Re-balance an element whose limbs grew through additions.
OURO_FI fe fe_carry(const fe& f) {
  int64_t t[10];
#pragma unroll
  for (int i = 0; i < 10; i++) t[i] = f.v[i];
  return fe_carry64(t);
}

// h = f * g.  Column k collects f_i g_j with i + j = k (mod 10); odd*odd
// terms carry a factor 2 (2^ceil(25.5 i) 2^ceil(25.5 j) = 2 * 2^ceil(25.5 (i+j)))
// and wrapped terms a factor 19 (2^255 = 19).
OURO_FI fe fe_mul(const fe& f, const fe& g) {
  OURO_COUNT_MUL();
  OURO_CHECK_BOUNDS(f);
  OURO_CHECK_BOUNDS(g);
  int32_t g19[10], f2[10];
#pragma unroll
  for (int i = 0; i < 10; i++) {
    g19[i] = 19 * g.v[i];
    f2[i] = (i & 1) ? 2 * f.v[i] : f.v[i];
  }
  int64_t t[10];
#pragma unroll
  for (int k = 0; k < 10; k++) t[k] = 0;
#pragma unroll
  for (int i = 0; i < 10; i++) {
#pragma unroll
    for (int j = 0; j < 10; j++) {
      const int k = i + j;
      const int32_t a = ((i & 1) && (j & 1)) ? f2[i] : f.v[i];
      const int32_t b = (k >= 10) ? g19[j] : g.v[j];
      t[k >= 10 ? k - 10 : k] += (int64_t)a * b;
    }
  }
  return fe_carry64(t);
}

// Column sums of f^2 (before carry); shared by fe_sq and fe_sq2.
OURO_FI void fe_sq_cols(int64_t t[10], const fe& f) {
  OURO_COUNT_SQ();
  OURO_CHECK_BOUNDS(f);
  int32_t f2[10], f4[10], f19[10];
#pragma unroll
  for (int i = 0; i < 10; i++) {
    f2[i] = 2 * f.v[i];
    f4[i] = 4 * f.v[i];
    f19[i] = 19 * f.v[i];
  }
#pragma unroll
  for (int k = 0; k < 10; k++) t[k] = 0;
#pragma unroll
  for (int i = 0; i < 10; i++) {
    // diagonal: f_i^2 * (2 if i odd) * (19 if 2i >= 10)
    {
      const int k = 2 * i;
      const int32_t a = (i & 1) ? f2[i] : f.v[i];
      const int32_t b = (k >= 10) ? f19[i] : f.v[i];
      t[k >= 10 ? k - 10 : k] += (int64_t)a * b;
    }
#pragma unroll
    for (int j = i + 1; j < 10; j++) {
      // cross terms counted twice: 2 f_i f_j * (2 if both odd) * (19 if wrap)
      const int k = i + j;
      const int32_t a = ((i & 1) && (j & 1)) ? f4[i] : f2[i];
      const int32_t b = (k >= 10) ? f19[j] : f.v[j];
      t[k >= 10 ? k - 10 : k] += (int64_t)a * b;
    }
  }
}

OURO_FI fe fe_sq(const fe& f) {
  int64_t t[10];
  fe_sq_cols(t, f);
  return fe_carry64(t);
}

// 2 f^2
OURO_FI fe fe_sq2(const fe& f) {
  int64_t t[10];
  fe_sq_cols(t, f);
#pragma unroll
  for (int k = 0; k < 10; k++) t[k] += t[k];
  return fe_carry64(t);
}

// ---- encoding -------------------------------------------------------------
// 256-bit little-endian words -> fe (bit 255 ignored, like fe25519_frombytes)
OURO_FI fe fe_from_words(const uint32_t w[8]) {
  fe h;
  h.v[0] = (int32_t)(w[0] & 0x3ffffff);
  h.v[1] = (int32_t)(((w[0] >> 26) | (w[1] << 6)) & 0x1ffffff);
  h.v[2] = (int32_t)(((w[1] >> 19) | (w[2] << 13)) & 0x3ffffff);
  h.v[3] = (int32_t)(((w[2] >> 13) | (w[3] << 19)) & 0x1ffffff);
  h.v[4] = (int32_t)((w[3] >> 6) & 0x3ffffff);
  h.v[5] = (int32_t)(w[4] & 0x1ffffff);
  h.v[6] = (int32_t)(((w[4] >> 25) | (w[5] << 7)) & 0x3ffffff);
  h.v[7] = (int32_t)(((w[5] >> 19) | (w[6] << 13)) & 0x1ffffff);
  h.v[8] = (int32_t)(((w[6] >> 12) | (w[7] << 20)) & 0x3ffffff);
  h.v[9] = (int32_t)((w[7] >> 6) & 0x1ffffff);
  return fe_carry(h);  // unsigned 26-bit limbs -> balanced
}

// canonical little-endian encoding of f mod p as 8 words
OURO_FI void fe_to_words(uint32_t w[8], const fe& f) {
  int32_t h[10];
#pragma unroll
  for (int i = 0; i < 10; i++) h[i] = f.v[i];
  // three floor-carry passes leave every limb in [0, 2^bits) with the value
  // in [0, 2^255); the first pass absorbs any sign.
#pragma unroll
  for (int pass = 0; pass < 3; pass++) {
    int32_t c;
#pragma unroll
    for (int i = 0; i < 9; i++) {
      const int bits = (i & 1) ? 25 : 26;
      c = h[i] >> bits;
      h[i] -= c * (1 << bits);
      h[i + 1] += c;
    }
    c = h[9] >> 25;
    h[9] -= c * (1 << 25);
    h[0] += 19 * c;
  }
  // subtract p if value >= p: q = (value + 19) >> 255
  int32_t q = (h[0] + 19) >> 26;
#pragma unroll
  for (int i = 1; i < 10; i++) q = (h[i] + q) >> ((i & 1) ? 25 : 26);
  h[0] += 19 * q;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    const int bits = (i & 1) ? 25 : 26;
    int32_t c = h[i] >> bits;
    h[i] -= c * (1 << bits);
    h[i + 1] += c;
  }
  h[9] &= 0x1ffffff;
  const uint32_t* u = reinterpret_cast<const uint32_t*>(h);
  w[0] = u[0] | (u[1] << 26);
  w[1] = (u[1] >> 6) | (u[2] << 19);
  w[2] = (u[2] >> 13) | (u[3] << 13);
  w[3] = (u[3] >> 19) | (u[4] << 6);
  w[4] = u[5] | (u[6] << 25);
  w[5] = (u[6] >> 7) | (u[7] << 19);
  w[6] = (u[7] >> 13) | (u[8] << 12);
  w[7] = (u[8] >> 20) | (u[9] << 6);
}

OURO_FI bool fe_iszero(const fe& f) {
  uint32_t w[8];
  fe_to_words(w, f);
  uint32_t a = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) a |= w[i];
  return a == 0;
}

OURO_FI bool fe_isnegative(const fe& f) {
  uint32_t w[8];
  fe_to_words(w, f);
  return w[0] & 1;
}

// ---- exponentiations (kept out of line: code size) ----------
OURO_FI fe fe_sqn(fe t, int n) {
#pragma unroll 1
  for (int i = 0; i < n; i++) t = fe_sq(t);
  return t;
}

// z^(p-2) (mode 0, inversion) or z^(2^252-3) (mode 1, square-root helper):
// one out-of-line copy of the addition chain serves both.
OURO_NI fe fe_pow_chain(fe z, int mode) {
  fe z2 = fe_sq(z);
  fe t = fe_sqn(z2, 2);
  fe z9 = fe_mul(t, z);
  fe z11 = fe_mul(z9, z2);
  t = fe_sq(z11);
  fe z5 = fe_mul(t, z9);               // 2^5 - 1
  fe z10 = fe_mul(fe_sqn(z5, 5), z5);  // 2^10 - 1
  fe z20 = fe_mul(fe_sqn(z10, 10), z10);
  t = fe_mul(fe_sqn(z20, 20), z20);    // 2^40 - 1
  fe z50 = fe_mul(fe_sqn(t, 10), z10);
  fe z100 = fe_mul(fe_sqn(z50, 50), z50);
  t = fe_mul(fe_sqn(z100, 100), z100); // 2^200 - 1
  fe z250 = fe_mul(fe_sqn(t, 50), z50);
  t = fe_sqn(z250, mode ? 2 : 5);
  return fe_mul(t, mode ? z : z11);    // 2^252 - 3  |  2^255 - 21
}

OURO_FI fe fe_invert(const fe& z) { return fe_pow_chain(z, 0); }
OURO_FI fe fe_pow22523(const fe& z) { return fe_pow_chain(z, 1); }

}  // namespace ouro
