// lattice.h -- half-size scalars for the Ed25519 verification equation.
//
// libsodium 1.0.18 accepts iff encode([S]B - [h]A) == R_bytes (SURVEY.md App.
// B.1).  With R_bytes canonical and decodable to a point R (otherwise no
// encoding can equal it), that is Q = [S]B - [h]A - R == O.  For any odd c1
// with 0 < c1 < L and c0 = c1 h (mod 8L):
//   [c1]Q = [c1 S mod L]B - [c0]A - [c1]R,
// because B has order L and every curve point is killed by 8L; and
// [c1]Q == O  <=>  Q == O, because ord(Q) divides 8L, L does not divide c1 and
// no power of two divides an odd c1.  A short (c0, c1) -- about 2^127 each --
// halves the doubling chain of the double-scalar multiplication (Pornin,
// "Optimized lattice basis reduction in dimension 2, and fast Schnorr and
// EdDSA signature verification", 2020, whose equation this is, extended here
// to cofactorless verification of mixed-order keys by working modulo 8L).
//
// The short vector comes from a Lehmer-style half extended Euclid on
// (8L, h): rows (r, t) with r = t h (mod 8L) are combined by exact integer
// 2x2 steps, each derived from the leading 64 bits, so the lattice relation
// holds by construction whatever the approximation does.  Correctness needs
// nothing from the reduction but that relation and an odd c1, and both are
// re-checked at the end; a candidate that fails (never seen) or is not
// shorter than 2^250 is replaced by (h, 1), i.e. the classic full-length
// equation.
#pragma once
#include "sc25519.h"

namespace ouro {

// 288-bit two's complement integers, little-endian words
struct i288 {
  uint32_t w[9];
};

OURO_FI bool i288_is_neg(const i288& a) { return (a.w[8] >> 31) != 0; }

OURO_FI void i288_negate(i288& a) {
  uint32_t c = 1;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    const uint32_t x = ~a.w[i];
    a.w[i] = x + c;
    c = (a.w[i] < x) ? 1u : 0u;
  }
}

// a (signed 32-bit) * x  (mod 2^288)
OURO_FI i288 i288_mul_s32(const i288& x, int32_t a) {
  const uint32_t m = a < 0 ? (uint32_t)(-(int64_t)a) : (uint32_t)a;
  i288 r;
  uint64_t carry = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    const uint64_t t = (uint64_t)x.w[i] * m + carry;
    r.w[i] = (uint32_t)t;
    carry = t >> 32;
  }
  if (a < 0) i288_negate(r);
  return r;
}

OURO_FI i288 i288_add(const i288& x, const i288& y) {
  i288 r;
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    const uint64_t t = (uint64_t)x.w[i] + y.w[i] + c;
    r.w[i] = (uint32_t)t;
    c = (uint32_t)(t >> 32);
  }
  return r;
}

OURO_FI i288 i288_sub(const i288& x, const i288& y) {
  i288 r;
  uint32_t b = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    const uint64_t t = (uint64_t)x.w[i] - y.w[i] - b;
    r.w[i] = (uint32_t)t;
    b = (uint32_t)(t >> 63);
  }
  return r;
}

// bit length of a non-negative value
OURO_FI int i288_bitlen(const i288& a) {
  int len = 0;
#pragma unroll
  for (int i = 0; i < 9; i++)
    if (a.w[i]) len = 32 * i + 32 - __builtin_clz(a.w[i]);
  return len;
}

// bit length of |a|
OURO_FI int i288_abs_bitlen(const i288& a) {
  i288 m = a;
  if (i288_is_neg(m)) i288_negate(m);
  return i288_bitlen(m);
}

// word i (0 <= i, wave-divergent) of a non-negative value, 0 beyond the top
OURO_FI uint32_t i288_word(const i288& a, int i) {
  uint32_t r = 0;
#pragma unroll
  for (int k = 0; k < 9; k++) r = (i == k) ? a.w[k] : r;
  return r;
}

// bits [sh, sh + 64) of a non-negative value
OURO_FI uint64_t i288_bits64(const i288& a, int sh) {
  const int ws = sh >> 5, bs = sh & 31;
  const uint32_t w0 = i288_word(a, ws), w1 = i288_word(a, ws + 1), w2 = i288_word(a, ws + 2);
  const uint64_t lo = bs ? ((w0 >> bs) | (w1 << (32 - bs))) : w0;
  const uint64_t hi = bs ? ((w1 >> bs) | (w2 << (32 - bs))) : w1;
  return lo | (hi << 32);
}

OURO_FI int clz64(uint64_t x) { return __builtin_clzll(x); }

OURO_FI void i288_cswap(i288& a, i288& b, bool c) {
#pragma unroll
  for (int i = 0; i < 9; i++) {
    const uint32_t x = a.w[i], y = b.w[i];
    a.w[i] = c ? y : x;
    b.w[i] = c ? x : y;
  }
}

// a < b for non-negative a, b
OURO_FI bool i288_lt(const i288& a, const i288& b) { return i288_is_neg(i288_sub(a, b)); }

// 8L = 2^255 + 8 (L - 2^252)
OURO_FI i288 i288_8L() {
  i288 r;
  r.w[0] = 0xe7ae9f68u; r.w[1] = 0xc09318d2u; r.w[2] = 0x17bce6b2u; r.w[3] = 0xa6f7cef5u;
  r.w[4] = 0; r.w[5] = 0; r.w[6] = 0; r.w[7] = 0x80000000u; r.w[8] = 0;
  return r;
}

// Inner loop of the half Euclid on the leading 64 bits: 1 = one full
// quotient per step (q = floor(x / y) estimated in double precision and
// corrected exactly: one Euclid step each, ~0.6 steps per bit); 0 = binary
// subtract-and-shift steps (one per quotient bit, the round-2 form).  Both
// produce the exact remainder sequence while the matrix stays below 2^31.
#ifndef OURO_LATTICE_QUOT
#define OURO_LATTICE_QUOT 1
#endif

struct HalfScalars {
  uint32_t c0[8];  // |c0|
  uint32_t c1[8];  // c1 > 0, odd
  bool c0_neg;
  int bits;        // max(bitlen |c0|, bitlen c1)
};

// The common end of both reductions: from the rows (ru, tu), (rv, tv) with
// ru > rv around 2^128, the shortest candidate with odd t, re-checked.
OURO_HD inline void half_scalars_finish(HalfScalars& out, const uint32_t h[8], const i288& ru,
                                        const i288& rv, const i288& tu, const i288& tv) {
  // one Euclid step past v: w = u - q v, q from the leading bits (any integer
  // q keeps w in the lattice; the right one makes it the next remainder)
  i288 rw = rv, tw = tv;
  {
    const int lu = i288_bitlen(ru), lv = i288_bitlen(rv);
    if (lv > 0 && lu - lv < 30) {
      const int sh = lu > 64 ? lu - 64 : 0;
      const double x = (double)i288_bits64(ru, sh), y = (double)i288_bits64(rv, sh);
      const int32_t q = (int32_t)(x / y);
      rw = i288_add(ru, i288_mul_s32(rv, -q));
      tw = i288_add(tu, i288_mul_s32(tv, -q));
      if (i288_is_neg(rw)) { i288_negate(rw); i288_negate(tw); }
    }
  }
  // candidates with odd t among the remainders around 2^128 and their
  // neighbour sums: v, u, u + v, u - v, w, v + w, v - w; keep the shortest
  // (tests/test_devcode_host.py pins the size distribution)
  i288 best_r = rv, best_t = tv;
  int best = 1 << 20;
#pragma unroll 1
  for (int k = 0; k < 7; k++) {
    i288 r = k == 0 ? rv : ru, t = k == 0 ? tv : tu;
    if (k == 2) { r = i288_add(ru, rv); t = i288_add(tu, tv); }
    if (k == 3) { r = i288_sub(ru, rv); t = i288_sub(tu, tv); }
    if (k == 4) { r = rw; t = tw; }
    if (k == 5) { r = i288_add(rv, rw); t = i288_add(tv, tw); }
    if (k == 6) { r = i288_sub(rv, rw); t = i288_sub(tv, tw); }
    if ((t.w[0] & 1u) == 0) continue;
    const int br = i288_abs_bitlen(r), bt = i288_abs_bitlen(t);
    const int b = br > bt ? br : bt;
    if (b < best) { best = b; best_r = r; best_t = t; }
  }
  // c1 > 0
  if (i288_is_neg(best_t)) { i288_negate(best_t); i288_negate(best_r); }
  const bool c0_neg = i288_is_neg(best_r);
  if (c0_neg) i288_negate(best_r);
  // re-check c1 h = c0 (mod 8L): mod 8 on the low bits, mod L by reduction
  bool good = best <= 250;
  {
    uint32_t prod[16];
#pragma unroll
    for (int i = 0; i < 16; i++) prod[i] = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      uint64_t carry = 0;
#pragma unroll
      for (int j = 0; j < 8; j++) {
        const uint64_t t = (uint64_t)best_t.w[i] * h[j] + prod[i + j] + carry;
        prod[i + j] = (uint32_t)t;
        carry = t >> 32;
      }
      prod[i + 8] = (uint32_t)carry;
    }
    uint32_t a[8], b[8], c0w[8];
#pragma unroll
    for (int i = 0; i < 8; i++) c0w[i] = best_r.w[i];
    sc_reduce512(a, prod);
    sc_reduce256(b, c0w);
    if (c0_neg) {
      // b = L - b (or 0)
      uint32_t l[8];
      sc_L(l);
      bool z = true;
#pragma unroll
      for (int i = 0; i < 8; i++) z = z && b[i] == 0;
      uint32_t br = 0;
#pragma unroll
      for (int i = 0; i < 8; i++) {
        const uint64_t t = (uint64_t)l[i] - b[i] - br;
        b[i] = z ? 0u : (uint32_t)t;
        br = (uint32_t)(t >> 63);
      }
    }
    bool eq = true;
#pragma unroll
    for (int i = 0; i < 8; i++) eq = eq && a[i] == b[i];
    const uint32_t low = best_t.w[0] * h[0] - (c0_neg ? (0u - best_r.w[0]) : best_r.w[0]);
    good = good && eq && (low & 7u) == 0 && best_t.w[8] == 0 && best_r.w[8] == 0;
  }
#pragma unroll
  for (int i = 0; i < 8; i++) {
    out.c0[i] = good ? best_r.w[i] : h[i];
    out.c1[i] = good ? best_t.w[i] : (i == 0 ? 1u : 0u);
  }
  out.c0_neg = good && c0_neg;
  if (!good) {
    uint32_t hh[8];
#pragma unroll
    for (int i = 0; i < 8; i++) hh[i] = h[i];
    i288 hv;
#pragma unroll
    for (int i = 0; i < 9; i++) hv.w[i] = i < 8 ? hh[i] : 0u;
    best = i288_bitlen(hv);
  }
  out.bits = best;
}


// (c0, c1) for h < 2^253: c0 = c1 h (mod 8L), c1 odd, both short -- the
// round-1 form (int64 cofactors, an IEEE division per step; A/B and the
// equivalence test of tests/test_devcode_host.py).
OURO_HD inline void ed25519_half_scalars_v1(HalfScalars& out, const uint32_t h[8]) {
  i288 ru = i288_8L(), rv, tu, tv;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    rv.w[i] = i < 8 ? h[i] : 0u;
    tu.w[i] = 0;
    tv.w[i] = i == 0 ? 1u : 0u;
  }
  // invariant: ru >= rv >= 0, r = t h (mod 8L) for both rows
#pragma unroll 1
  for (int outer = 0; outer < 12; outer++) {
    if (i288_bitlen(rv) <= 128) break;
    const int len = i288_bitlen(ru);
    const int sh = len > 64 ? len - 64 : 0;
    uint64_t x = i288_bits64(ru, sh), y = i288_bits64(rv, sh);
    // rows of the step matrix: u' = m00 u + m01 v, v' = m10 u + m11 v
    int64_t m00 = 1, m01 = 0, m10 = 0, m11 = 1;
    bool moved = false;
    // stop when the leading bits are used up (y < 2^32) or when r_v crosses
    // 2^128 (y < 2^(128 - sh)), so that u stays the last remainder above it
    // (sh >= 65 here: r_u > r_v > 2^128)
    const int ybits = 128 - sh > 32 ? 128 - sh : 32;
#if OURO_LATTICE_QUOT
#pragma unroll 1
    for (int it = 0; it < 96; it++) {
      if (y < (1ull << ybits)) break;
      // q = floor(x / y) >= 1 (x >= y): the double quotient scaled down by
      // 2^-48 never exceeds it (x, y rounded to 53 bits: relative error
      // < 2^-51 in the ratio), and is at most 1 short -- fixed exactly below
      uint64_t q = (uint64_t)((double)x / (double)y * (1.0 - 0x1p-48));
      if (q == 0) q = 1;
      uint64_t r = x - q * y;  // q y <= x: no wrap
      if (r >= y) {
        q++;
        r -= y;
      }
      // keep |m| < 2^31: the modified row grows to |m0| + q |m1|
      if (q >= (1ull << 31)) break;
      const int64_t a10 = m10 < 0 ? -m10 : m10, a11 = m11 < 0 ? -m11 : m11;
      const int64_t a00 = m00 < 0 ? -m00 : m00, a01 = m01 < 0 ? -m01 : m01;
      if (a00 + (int64_t)q * a10 >= (1ll << 31) || a01 + (int64_t)q * a11 >= (1ll << 31)) break;
      m00 -= (int64_t)q * m10;
      m01 -= (int64_t)q * m11;
      moved = true;
      // r < y: swap the rows
      x = y;
      y = r;
      int64_t t = m00; m00 = m10; m10 = t;
      t = m01; m01 = m11; m11 = t;
    }
#else
#pragma unroll 1
    for (int it = 0; it < 96; it++) {
      if (y < (1ull << ybits)) break;
      int s = clz64(y) - clz64(x);
      if ((y << s) > x) s--;
      const int64_t a10 = m10 < 0 ? -m10 : m10, a11 = m11 < 0 ? -m11 : m11;
      const int64_t a00 = m00 < 0 ? -m00 : m00, a01 = m01 < 0 ? -m01 : m01;
      const int64_t big1 = a10 > a11 ? a10 : a11, big0 = a00 > a01 ? a00 : a01;
      if ((big1 << s) + big0 >= (1ll << 31)) break;  // keep |m| < 2^31
      x -= y << s;
      m00 -= m10 * ((int64_t)1 << s);
      m01 -= m11 * ((int64_t)1 << s);
      moved = true;
      if (x < y) {
        const uint64_t tx = x; x = y; y = tx;
        int64_t q = m00; m00 = m10; m10 = q;
        q = m01; m01 = m11; m11 = q;
      }
    }
#endif
    if (!moved) break;
    i288 nu = i288_add(i288_mul_s32(ru, (int32_t)m00), i288_mul_s32(rv, (int32_t)m01));
    i288 nv = i288_add(i288_mul_s32(ru, (int32_t)m10), i288_mul_s32(rv, (int32_t)m11));
    i288 ntu = i288_add(i288_mul_s32(tu, (int32_t)m00), i288_mul_s32(tv, (int32_t)m01));
    i288 ntv = i288_add(i288_mul_s32(tu, (int32_t)m10), i288_mul_s32(tv, (int32_t)m11));
    // the approximation may overshoot: (-r, -t) is the same lattice vector's negative
    if (i288_is_neg(nu)) { i288_negate(nu); i288_negate(ntu); }
    if (i288_is_neg(nv)) { i288_negate(nv); i288_negate(ntv); }
    const bool sw = i288_lt(nu, nv);
    i288_cswap(nu, nv, sw);
    i288_cswap(ntu, ntv, sw);
    ru = nu; rv = nv; tu = ntu; tv = ntv;
  }
  half_scalars_finish(out, h, ru, rv, tu, tv);
}

// a * x mod 2^288 for 0 <= a < 2^32 (two's complement x: the signed product)
OURO_FI i288 i288_mul_u32(const i288& x, uint32_t a) {
  i288 r;
  uint64_t carry = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    const uint64_t t = (uint64_t)x.w[i] * a + carry;
    r.w[i] = (uint32_t)t;
    carry = t >> 32;
  }
  return r;
}
OURO_FI double u64_to_f64(uint64_t v) {
  return (double)(uint32_t)(v >> 32) * 0x1p32 + (double)(uint32_t)v;
}
// 1 / d for 1 <= d < 2^64: the hardware reciprocal refined by two Newton
// steps (the refinement LLVM's f64 division uses before its final rounding
// fix-up, which the quotient estimate below does not need)
OURO_FI double recip_f64(double d) {
#if defined(__HIP_DEVICE_COMPILE__)
  double r = __builtin_amdgcn_rcp(d);
  double e = __builtin_fma(-d, r, 1.0);
  r = __builtin_fma(r, e, r);
  e = __builtin_fma(-d, r, 1.0);
  return __builtin_fma(r, e, r);
#else
  return 1.0 / d;
#endif
}

// The same reduction with a leaner Lehmer step (round 6): the inner loop
// keeps the cofactor rows as 32-bit MAGNITUDES -- an exact Euclid step's
// cofactors alternate in sign, so |m0'| = |m0| + q |m1| and the bound check
// is the update itself --, estimates q from a Newton-refined reciprocal
// instead of an IEEE division, converts only the new remainder, and applies
// the rows as a * r - b * r' (the overall sign is the one the normalisation
// below fixes anyway).  Same quotients, same breaks, so the same rows and
// the same (c0, c1) as ed25519_half_scalars_v1 bit for bit
// (tests/test_devcode_host.py::test_half_scalars_v2_equals_v1).
OURO_HD inline void ed25519_half_scalars_v2(HalfScalars& out, const uint32_t h[8]) {
  i288 ru = i288_8L(), rv, tu, tv;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    rv.w[i] = i < 8 ? h[i] : 0u;
    tu.w[i] = 0;
    tv.w[i] = i == 0 ? 1u : 0u;
  }
#pragma unroll 1
  for (int outer = 0; outer < 12; outer++) {
    if (i288_bitlen(rv) <= 128) break;
    const int len = i288_bitlen(ru);
    const int sh = len > 64 ? len - 64 : 0;
    uint64_t x = i288_bits64(ru, sh), y = i288_bits64(rv, sh);
    // |m00|, |m01| (row 0) and |m10|, |m11| (row 1), all < 2^31
    uint32_t a0 = 1, b0 = 0, a1 = 0, b1 = 1;
    bool moved = false;
    const int ybits = 128 - sh > 32 ? 128 - sh : 32;
    double xd = u64_to_f64(x), yd = u64_to_f64(y);
#pragma unroll 1
    for (int it = 0; it < 96; it++) {
      if (y < (1ull << ybits)) break;
      // q = floor(x / y) >= 1: the estimate never exceeds it (relative error
      // < 2^-51, scaled down by 2^-48) and is at most 1 short
      const double qd = xd * recip_f64(yd) * (1.0 - 0x1p-48);
      if (qd >= 0x1p31) break;  // a cofactor would reach 2^31
      uint32_t q = (uint32_t)qd;
      q = q ? q : 1u;
      uint64_t r = x - (uint64_t)q * y;
      if (r >= y) {
        q++;
        r -= y;
      }
      const uint64_t na = (uint64_t)q * a1 + a0, nb = (uint64_t)q * b1 + b0;
      if ((na | nb) >> 31) break;
      a0 = a1;
      b0 = b1;
      a1 = (uint32_t)na;
      b1 = (uint32_t)nb;
      moved = true;
      x = y;
      y = r;
      xd = yd;
      yd = u64_to_f64(r);
    }
    if (!moved) break;
    // u' = +-(a0 u - b0 v), v' = +-(b1 v - a1 u); the sign: the normalisation
    i288 nu = i288_sub(i288_mul_u32(ru, a0), i288_mul_u32(rv, b0));
    i288 ntu = i288_sub(i288_mul_u32(tu, a0), i288_mul_u32(tv, b0));
    i288 nv = i288_sub(i288_mul_u32(rv, b1), i288_mul_u32(ru, a1));
    i288 ntv = i288_sub(i288_mul_u32(tv, b1), i288_mul_u32(tu, a1));
    if (i288_is_neg(nu)) { i288_negate(nu); i288_negate(ntu); }
    if (i288_is_neg(nv)) { i288_negate(nv); i288_negate(ntv); }
    const bool sw = i288_lt(nu, nv);
    i288_cswap(nu, nv, sw);
    i288_cswap(ntu, ntv, sw);
    ru = nu; rv = nv; tu = ntu; tv = ntv;
  }
  half_scalars_finish(out, h, ru, rv, tu, tv);
}

#ifndef OURO_LATTICE_V2
#define OURO_LATTICE_V2 1  // 0: the round-1 step (A/B)
#endif
OURO_HD inline void ed25519_half_scalars(HalfScalars& out, const uint32_t h[8]) {
  if constexpr (OURO_LATTICE_V2) ed25519_half_scalars_v2(out, h);
  else ed25519_half_scalars_v1(out, h);
}

}  // namespace ouro
