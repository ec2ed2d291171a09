// host_fast.h -- the product's CPU implementation of the verifiers (host_path.hip).
//
// The kernels' lane routines are written for a 32-bit VALU: ten 25.5-bit limbs
// whose 64-bit products accumulate in v_mad_u64_u32.  Compiled for x86-64 they
// run at half libsodium's speed (62 us per Ed25519 against 31 us),
// so the host path -- single items, the *_host entries, and the recompute of a
// batch whose device run failed -- gets its own arithmetic here, shaped for a
// 64-bit CPU:
//   * GF(2^255 - 19) in five 51-bit limbs with 128-bit products (25 MULs per
//     multiply, the reduction by 19 folded into the operand);
//   * group operations in extended twisted-Edwards coordinates (a = -1), the
//     variable points of a verification as tables of odd multiples, width-5
//     wNAF digits; the base point B and 2^128 B as two affine tables of 64 odd
//     multiples (width-8 wNAF), built once per process;
//   * Ed25519 through the same half-size equation as the device
//     (lattice.h: [c1 S mod L]B + [c0](-A) + [c1](-R) = O, a ~128-bit chain
//     compared with the identity projectively, no inversion);
//   * the VRF's Elligator2 with one exponentiation (the algebra of verify.h
//     elligator2_pre/_post), U on a 128-bit chain (s split over B and 2^128 B),
//     one inversion for the four encodings.
// Everything that is not field or group arithmetic -- SHA-512, Blake2b, the
// scalar reductions, the lattice pair, the encoding predicates, the Merkle
// walk, the challenge and output hashes -- is the kernels' own code (word
// level, host-compiled), so the acceptance rules are the device's line for
// line: tests/test_host_path.py pins this path against the oracle on the same
// edge-case sets as the GPU tests.
#pragma once
#include <stdint.h>
#include <string.h>

#include "tpraos.h"

namespace ouro_cpu {

typedef unsigned __int128 u128;
constexpr uint64_t kM51 = (1ull << 51) - 1;

// ---- GF(2^255 - 19), radix 2^51 ----------------------------------------------
// Bounds: a "carried" element has limbs < 2^51 + 2^20; mul/sq take inputs with
// limbs < 2^54 (19 b_j < 2^59, a_i 19 b_j < 2^113, a column of five such terms
// < 2^116) and return carried elements; add of two carried elements stays
// below 2^53, so every product operand here is at most one add deep; sub adds
// 4p before subtracting (its subtrahend is always carried) and carries.
struct f51 {
  uint64_t v[5];
};

inline f51 f_c(uint64_t a, uint64_t b, uint64_t c, uint64_t d, uint64_t e) {
  return f51{{a, b, c, d, e}};
}
inline f51 f_zero() { return f_c(0, 0, 0, 0, 0); }
inline f51 f_one() { return f_c(1, 0, 0, 0, 0); }
inline f51 f_small(uint64_t x) { return f_c(x, 0, 0, 0, 0); }  // x < 2^51
inline f51 f_d() {
  return f_c(0x34dca135978a3ull, 0x1a8283b156ebdull, 0x5e7a26001c029ull, 0x739c663a03cbbull,
             0x52036cee2b6ffull);
}
inline f51 f_d2() {
  return f_c(0x69b9426b2f159ull, 0x35050762add7aull, 0x3cf44c0038052ull, 0x6738cc7407977ull,
             0x2406d9dc56dffull);
}
inline f51 f_sqrtm1() {
  return f_c(0x61b274a0ea0b0ull, 0xd5a5fc8f189dull, 0x7ef5e9cbd0c60ull, 0x78595a6804c9eull,
             0x2b8324804fc1dull);
}
inline f51 f_one_minus_i() {
  return f_c(0x1e4d8b5f15f3eull, 0x72a5a0370e762ull, 0x10a16342f39full, 0x7a6a597fb361ull,
             0x547cdb7fb03e2ull);
}
inline f51 f_one_plus_i() {
  return f_c(0x61b274a0ea0b1ull, 0xd5a5fc8f189dull, 0x7ef5e9cbd0c60ull, 0x78595a6804c9eull,
             0x2b8324804fc1dull);
}
constexpr uint64_t kMontA = 486662;

inline f51 f_carry(f51 h) {
  uint64_t c;
  c = h.v[0] >> 51; h.v[0] &= kM51; h.v[1] += c;
  c = h.v[1] >> 51; h.v[1] &= kM51; h.v[2] += c;
  c = h.v[2] >> 51; h.v[2] &= kM51; h.v[3] += c;
  c = h.v[3] >> 51; h.v[3] &= kM51; h.v[4] += c;
  c = h.v[4] >> 51; h.v[4] &= kM51; h.v[0] += 19 * c;
  return h;
}
inline f51 f_add(const f51& a, const f51& b) {
  return f_c(a.v[0] + b.v[0], a.v[1] + b.v[1], a.v[2] + b.v[2], a.v[3] + b.v[3], a.v[4] + b.v[4]);
}
// a - b + 4p, carried
inline f51 f_sub(const f51& a, const f51& b) {
  constexpr uint64_t k0 = 4 * ((1ull << 51) - 19), k = 4 * kM51;
  return f_carry(f_c(a.v[0] + k0 - b.v[0], a.v[1] + k - b.v[1], a.v[2] + k - b.v[2],
                     a.v[3] + k - b.v[3], a.v[4] + k - b.v[4]));
}
inline f51 f_neg(const f51& a) { return f_sub(f_zero(), a); }

// five column sums (each < 2^117) -> a carried element
inline f51 f_reduce_wide(u128 r0, u128 r1, u128 r2, u128 r3, u128 r4) {
  r1 += r0 >> 51;
  r2 += r1 >> 51;
  r3 += r2 >> 51;
  r4 += r3 >> 51;
  const u128 t = (u128)((uint64_t)r0 & kM51) + (r4 >> 51) * 19;
  f51 h;
  h.v[0] = (uint64_t)t & kM51;
  h.v[1] = ((uint64_t)r1 & kM51) + (uint64_t)(t >> 51);
  h.v[2] = (uint64_t)r2 & kM51;
  h.v[3] = (uint64_t)r3 & kM51;
  h.v[4] = (uint64_t)r4 & kM51;
  return h;
}

inline f51 f_mul(const f51& a, const f51& b) {
  const uint64_t b1 = 19 * b.v[1], b2 = 19 * b.v[2], b3 = 19 * b.v[3], b4 = 19 * b.v[4];
  const u128 r0 = (u128)a.v[0] * b.v[0] + (u128)a.v[1] * b4 + (u128)a.v[2] * b3 +
                  (u128)a.v[3] * b2 + (u128)a.v[4] * b1;
  const u128 r1 = (u128)a.v[0] * b.v[1] + (u128)a.v[1] * b.v[0] + (u128)a.v[2] * b4 +
                  (u128)a.v[3] * b3 + (u128)a.v[4] * b2;
  const u128 r2 = (u128)a.v[0] * b.v[2] + (u128)a.v[1] * b.v[1] + (u128)a.v[2] * b.v[0] +
                  (u128)a.v[3] * b4 + (u128)a.v[4] * b3;
  const u128 r3 = (u128)a.v[0] * b.v[3] + (u128)a.v[1] * b.v[2] + (u128)a.v[2] * b.v[1] +
                  (u128)a.v[3] * b.v[0] + (u128)a.v[4] * b4;
  const u128 r4 = (u128)a.v[0] * b.v[4] + (u128)a.v[1] * b.v[3] + (u128)a.v[2] * b.v[2] +
                  (u128)a.v[3] * b.v[1] + (u128)a.v[4] * b.v[0];
  return f_reduce_wide(r0, r1, r2, r3, r4);
}

inline f51 f_sq(const f51& a) {
  const uint64_t d0 = 2 * a.v[0], d1 = 2 * a.v[1];
  const uint64_t a3_19 = 19 * a.v[3], a4_19 = 19 * a.v[4];
  const u128 r0 = (u128)a.v[0] * a.v[0] + (u128)(2 * a.v[1]) * a4_19 + (u128)(2 * a.v[2]) * a3_19;
  const u128 r1 = (u128)d0 * a.v[1] + (u128)(2 * a.v[2]) * a4_19 + (u128)a.v[3] * a3_19;
  const u128 r2 = (u128)d0 * a.v[2] + (u128)a.v[1] * a.v[1] + (u128)(2 * a.v[3]) * a4_19;
  const u128 r3 = (u128)d0 * a.v[3] + (u128)d1 * a.v[2] + (u128)a.v[4] * a4_19;
  const u128 r4 = (u128)d0 * a.v[4] + (u128)d1 * a.v[3] + (u128)a.v[2] * a.v[2];
  return f_reduce_wide(r0, r1, r2, r3, r4);
}
inline f51 f_sqn(f51 a, int n) {
  for (int i = 0; i < n; i++) a = f_sq(a);
  return a;
}

// 255 bits of a little-endian 32-byte value (bit 255 ignored), not reduced mod p
inline f51 f_from_words(const uint32_t w[8]) {
  uint64_t q[4];
  for (int i = 0; i < 4; i++) q[i] = (uint64_t)w[2 * i] | ((uint64_t)w[2 * i + 1] << 32);
  return f_c(q[0] & kM51, ((q[0] >> 51) | (q[1] << 13)) & kM51, ((q[1] >> 38) | (q[2] << 26)) & kM51,
             ((q[2] >> 25) | (q[3] << 39)) & kM51, (q[3] >> 12) & kM51);
}
// canonical little-endian words
inline void f_to_words(uint32_t w[8], const f51& a) {
  f51 h = f_carry(f_carry(a));  // limbs < 2^51 + 19*small, then < 2^51 except limb 0
  // q = 1 iff h >= p: add 19 and look at bit 255
  uint64_t q = (h.v[0] + 19) >> 51;
  q = (h.v[1] + q) >> 51;
  q = (h.v[2] + q) >> 51;
  q = (h.v[3] + q) >> 51;
  q = (h.v[4] + q) >> 51;
  h.v[0] += 19 * q;
  uint64_t c;
  c = h.v[0] >> 51; h.v[0] &= kM51; h.v[1] += c;
  c = h.v[1] >> 51; h.v[1] &= kM51; h.v[2] += c;
  c = h.v[2] >> 51; h.v[2] &= kM51; h.v[3] += c;
  c = h.v[3] >> 51; h.v[3] &= kM51; h.v[4] += c;
  h.v[4] &= kM51;
  const uint64_t q0 = h.v[0] | (h.v[1] << 51), q1 = (h.v[1] >> 13) | (h.v[2] << 38),
                 q2 = (h.v[2] >> 26) | (h.v[3] << 25), q3 = (h.v[3] >> 39) | (h.v[4] << 12);
  const uint64_t q4[4] = {q0, q1, q2, q3};
  for (int i = 0; i < 4; i++) {
    w[2 * i] = (uint32_t)q4[i];
    w[2 * i + 1] = (uint32_t)(q4[i] >> 32);
  }
}
inline bool f_iszero(const f51& a) {
  uint32_t w[8];
  f_to_words(w, a);
  uint32_t o = 0;
  for (int i = 0; i < 8; i++) o |= w[i];
  return o == 0;
}
inline bool f_isneg(const f51& a) {
  uint32_t w[8];
  f_to_words(w, a);
  return (w[0] & 1u) != 0;
}
inline bool f_eq(const f51& a, const f51& b) { return f_iszero(f_sub(a, b)); }

// z^(2^252 - 3) and z^(p - 2)
inline f51 f_pow22523(const f51& z) {
  const f51 z2 = f_sq(z);                         // 2
  const f51 z9 = f_mul(f_sqn(z2, 2), z);          // 9
  const f51 z11 = f_mul(z9, z2);                  // 11
  const f51 z_5_0 = f_mul(f_sq(z11), z9);         // 2^5 - 1
  const f51 z_10_0 = f_mul(f_sqn(z_5_0, 5), z_5_0);
  const f51 z_20_0 = f_mul(f_sqn(z_10_0, 10), z_10_0);
  const f51 z_40_0 = f_mul(f_sqn(z_20_0, 20), z_20_0);
  const f51 z_50_0 = f_mul(f_sqn(z_40_0, 10), z_10_0);
  const f51 z_100_0 = f_mul(f_sqn(z_50_0, 50), z_50_0);
  const f51 z_200_0 = f_mul(f_sqn(z_100_0, 100), z_100_0);
  const f51 z_250_0 = f_mul(f_sqn(z_200_0, 50), z_50_0);
  return f_mul(f_sqn(z_250_0, 2), z);             // 2^252 - 3
}
inline f51 f_invert(const f51& z) {
  const f51 z2 = f_sq(z);
  const f51 z9 = f_mul(f_sqn(z2, 2), z);
  const f51 z11 = f_mul(z9, z2);
  const f51 z_5_0 = f_mul(f_sq(z11), z9);
  const f51 z_10_0 = f_mul(f_sqn(z_5_0, 5), z_5_0);
  const f51 z_20_0 = f_mul(f_sqn(z_10_0, 10), z_10_0);
  const f51 z_40_0 = f_mul(f_sqn(z_20_0, 20), z_20_0);
  const f51 z_50_0 = f_mul(f_sqn(z_40_0, 10), z_10_0);
  const f51 z_100_0 = f_mul(f_sqn(z_50_0, 50), z_50_0);
  const f51 z_200_0 = f_mul(f_sqn(z_100_0, 100), z_100_0);
  const f51 z_250_0 = f_mul(f_sqn(z_200_0, 50), z_50_0);
  return f_mul(f_sqn(z_250_0, 5), z11);           // 2^255 - 21
}

// ---- group: extended coordinates, a = -1 ---------------------------------------
struct P2 { f51 X, Y, Z; };
struct P3 { f51 X, Y, Z, T; };
struct P1 { f51 X, Y, Z, T; };          // completed: x = X/Z, y = Y/T
struct Cached { f51 YpX, YmX, Z, T2d; };
struct Niels { f51 ypx, ymx, xy2d; };    // affine, Z = 1

inline P2 to_p2(const P1& p) { return P2{f_mul(p.X, p.T), f_mul(p.Y, p.Z), f_mul(p.Z, p.T)}; }
inline P3 to_p3(const P1& p) {
  return P3{f_mul(p.X, p.T), f_mul(p.Y, p.Z), f_mul(p.Z, p.T), f_mul(p.X, p.Y)};
}
inline Cached to_cached(const P3& p) {
  return Cached{f_add(p.Y, p.X), f_sub(p.Y, p.X), p.Z, f_mul(p.T, f_d2())};
}
inline P3 p3_neg(const P3& p) { return P3{f_neg(p.X), p.Y, p.Z, f_neg(p.T)}; }
inline P3 p3_identity() { return P3{f_zero(), f_one(), f_one(), f_zero()}; }

// 2P: XX = X^2, YY = Y^2, B = 2 Z^2, S = (X + Y)^2
inline P1 dbl(const P2& p) {
  const f51 XX = f_sq(p.X), YY = f_sq(p.Y), ZZ = f_sq(p.Z), S = f_sq(f_add(p.X, p.Y));
  P1 r;
  r.Y = f_add(YY, XX);
  r.Z = f_sub(YY, XX);
  r.X = f_sub(S, r.Y);
  r.T = f_sub(f_add(ZZ, ZZ), r.Z);
  return r;
}
inline P1 dbl3(const P3& p) { return dbl(P2{p.X, p.Y, p.Z}); }

// P + Q / P - Q, Q cached
inline P1 add(const P3& p, const Cached& q) {
  const f51 A = f_mul(f_add(p.Y, p.X), q.YpX), B = f_mul(f_sub(p.Y, p.X), q.YmX);
  const f51 C = f_mul(p.T, q.T2d), ZZ = f_mul(p.Z, q.Z), D = f_add(ZZ, ZZ);
  return P1{f_sub(A, B), f_add(A, B), f_add(D, C), f_sub(D, C)};
}
inline P1 sub(const P3& p, const Cached& q) {
  const f51 A = f_mul(f_add(p.Y, p.X), q.YmX), B = f_mul(f_sub(p.Y, p.X), q.YpX);
  const f51 C = f_mul(p.T, q.T2d), ZZ = f_mul(p.Z, q.Z), D = f_add(ZZ, ZZ);
  return P1{f_sub(A, B), f_add(A, B), f_sub(D, C), f_add(D, C)};
}
inline P1 madd(const P3& p, const Niels& q) {
  const f51 A = f_mul(f_add(p.Y, p.X), q.ypx), B = f_mul(f_sub(p.Y, p.X), q.ymx);
  const f51 C = f_mul(p.T, q.xy2d), D = f_add(p.Z, p.Z);
  return P1{f_sub(A, B), f_add(A, B), f_add(D, C), f_sub(D, C)};
}
inline P1 msub(const P3& p, const Niels& q) {
  const f51 A = f_mul(f_add(p.Y, p.X), q.ymx), B = f_mul(f_sub(p.Y, p.X), q.ypx);
  const f51 C = f_mul(p.T, q.xy2d), D = f_add(p.Z, p.Z);
  return P1{f_sub(A, B), f_add(A, B), f_sub(D, C), f_add(D, C)};
}
inline P3 p3_add(const P3& p, const P3& q) { return to_p3(add(p, to_cached(q))); }
inline P3 mul8(const P3& p) {
  P2 t = to_p2(dbl3(p));
  t = to_p2(dbl(t));
  return to_p3(dbl(t));
}

// ge25519_frombytes (negate = false) / _negate_vartime (negate = true) exactly as
// the kernels' ge_decode (ge25519.h): y read mod 2^255, x = 0 with the sign
// bit set accepted; false when (y^2 - 1)/(d y^2 + 1) is not a square.
inline bool decode(P3* h, const uint32_t s[8], bool negate) {
  const f51 y = f_from_words(s);
  const f51 yy = f_sq(y);
  const f51 u = f_sub(yy, f_one());
  const f51 v = f_carry(f_add(f_mul(yy, f_d()), f_one()));
  const f51 v3 = f_mul(f_sq(v), v);
  f51 x = f_mul(f_mul(f_pow22523(f_mul(f_mul(f_sq(v3), v), u)), v3), u);
  const f51 vxx = f_mul(f_sq(x), v);
  const bool m_root = f_eq(vxx, u);
  const bool p_root = f_iszero(f_add(vxx, u));
  if (!m_root) x = f_mul(x, f_sqrtm1());
  const bool sign = (s[7] >> 31) != 0;
  const bool flip = negate ? (f_isneg(x) == sign) : (f_isneg(x) != sign);
  if (flip) x = f_neg(x);
  h->X = x;
  h->Y = f_carry(y);
  h->Z = f_one();
  h->T = f_mul(x, y);
  return m_root || p_root;
}

inline void encode_with_inv(uint32_t out[8], const f51& X, const f51& Y, const f51& zinv) {
  uint32_t xw[8];
  f_to_words(out, f_mul(Y, zinv));
  f_to_words(xw, f_mul(X, zinv));
  out[7] ^= (xw[0] & 1u) << 31;
}

// ---- scalars: width-w NAF ------------------------------------------------------
// digits[i] in {0, +-1, +-3, .., +-(2^(w-1) - 1)}, sum digits[i] 2^i = k (k given
// as 8 little-endian words, below 2^(32*8 - w)); returns the digit count (one
// past the top nonzero digit).  Variable time: every input is public.
inline int wnaf(int8_t* digits, const uint32_t k[8], int w, int maxbits) {
  memset(digits, 0, (size_t)maxbits + 1);
  auto bits_at = [&](int at, int n) -> uint32_t {  // n <= 9 bits from bit `at`
    const int q = at >> 5, r = at & 31;
    uint64_t x = k[q];
    if (q + 1 < 8) x |= (uint64_t)k[q + 1] << 32;
    return (uint32_t)(x >> r) & ((1u << n) - 1);
  };
  int carry = 0, top = 0;
  for (int bit = 0; bit < maxbits;) {
    if ((int)bits_at(bit, 1) == carry) {
      bit++;
      continue;
    }
    const int now = w < maxbits - bit ? w : maxbits - bit;
    int word = (int)bits_at(bit, now) + carry;
    carry = (word >> (w - 1)) & 1;
    word -= carry << w;
    digits[bit] = (int8_t)word;
    top = bit + 1;
    bit += now;
  }
  if (carry) {
    digits[maxbits] = 1;
    top = maxbits + 1;
  }
  return top;
}

// odd multiples [1, 3, .., 2 n - 1] P, cached
inline void odd_multiples(Cached* t, const P3& p, int n) {
  const P3 p2 = to_p3(dbl3(p));
  t[0] = to_cached(p);
  P3 acc = p;
  for (int i = 1; i < n; i++) {
    acc = to_p3(add(acc, to_cached(p2)));
    t[i] = to_cached(acc);
  }
}

// [1, 3, .., 127] B and the same of 2^128 B, affine (verify.h's base point and
// build order; built once per process from the encoding of B)
struct BaseTables {
  Niels b[64], b128[64];
};
const BaseTables& base_tables();

// The chain every verification here runs: sum of
//   [k_j] T_j     variable points, tables of 8 odd multiples (width 5),
//   [b] B         b < 2^256 split as b_lo + 2^128 b_hi over the two base tables
// with one shared doubling chain.  Digits of all terms at position i are added
// after the i-th doubling (Straus).
struct Term {
  const Cached* tab;
  int8_t naf[260];
  int len;
};
inline P3 straus(Term* terms, int nterms, const uint32_t* b /* 8 words or null */) {
  int8_t blo[136], bhi[136];
  int lb = 0, hb = 0;
  if (b) {
    const uint32_t lo[8] = {b[0], b[1], b[2], b[3], 0, 0, 0, 0};
    const uint32_t hi[8] = {b[4], b[5], b[6], b[7], 0, 0, 0, 0};
    lb = wnaf(blo, lo, 8, 128);
    hb = wnaf(bhi, hi, 8, 128);
  }
  int top = lb > hb ? lb : hb;
  for (int j = 0; j < nterms; j++) top = terms[j].len > top ? terms[j].len : top;
  const BaseTables& bt = base_tables();
  // the running sum in completed form; (0 : 1 : 1 : 1) is the identity
  P1 t{f_zero(), f_one(), f_one(), f_one()};
  for (int i = top - 1; i >= 0; i--) {
    t = dbl(to_p2(t));
    for (int j = 0; j < nterms; j++) {
      const int d = i < terms[j].len ? terms[j].naf[i] : 0;
      if (d > 0) t = add(to_p3(t), terms[j].tab[d >> 1]);
      else if (d < 0) t = sub(to_p3(t), terms[j].tab[(-d) >> 1]);
    }
    if (b) {
      const int dl = i < lb ? blo[i] : 0, dh = i < hb ? bhi[i] : 0;
      if (dl > 0) t = madd(to_p3(t), bt.b[dl >> 1]);
      else if (dl < 0) t = msub(to_p3(t), bt.b[(-dl) >> 1]);
      if (dh > 0) t = madd(to_p3(t), bt.b128[dh >> 1]);
      else if (dh < 0) t = msub(to_p3(t), bt.b128[(-dh) >> 1]);
    }
  }
  return to_p3(t);
}

inline void term_of(Term& t, const Cached* tab, const uint32_t k[8], int maxbits) {
  t.tab = tab;
  t.len = wnaf(t.naf, k, 5, maxbits);
}

// ---- Ed25519 (libsodium 1.0.18 / ByronDSIGN rules, verify.h) ---------------------
template <class Tail>
inline bool ed25519_verify(const uint32_t sig[16], const uint32_t pk[8], const Tail& msg,
                           uint32_t mlen, bool byron) {
  uint32_t R[8], S[8];
  for (int i = 0; i < 8; i++) {
    R[i] = sig[i];
    S[i] = sig[8 + i];
  }
  bool ok = ouro::ed25519_precheck(R, S, pk, byron);
  P3 negA, negR;
  ok = decode(&negA, pk, true) && ok;
  ok = ouro::ge_is_canonical(R) && ok;
  ok = decode(&negR, R, true) && ok;
  ok = ok && !(f_iszero(negR.X) && (R[7] >> 31) != 0);
  if (!ok) return false;  // (the scalars and the chain cannot change a rejection)
  ouro::HalfScalars hs;
  uint32_t b[8];
  ouro::ed25519_scalars(hs, b, R, S, pk, msg, mlen);
  // [b]B + [|c0|](+-A) + [c1](-R) == O
  Cached ta[8], tr[8];
  odd_multiples(ta, hs.c0_neg ? p3_neg(negA) : negA, 8);
  odd_multiples(tr, negR, 8);
  Term t[2];
  term_of(t[0], ta, hs.c0, 256);
  term_of(t[1], tr, hs.c1, 256);
  const P3 q = straus(t, 2, b);
  return f_iszero(q.X) && f_eq(q.Y, q.Z);
}

// ---- ECVRF-ED25519-SHA512-Elligator2 (draft-03), verify.h vrf03_verify_lane ----
// ge25519_from_uniform with x_sign = 0, then [8]: one (p-5)/8 power of
// num W^7 (verify.h elligator2_pre / elligator2_post derive the algebra).
inline P3 elligator2(const uint32_t r[8]) {
  const f51 rr = f_from_words(r);
  const f51 r2 = f_sq(rr);
  const f51 D = f_carry(f_add(f_add(r2, r2), f_one()));               // 1 + 2 r^2
  const f51 a2r2 = f_mul(f_small(kMontA * kMontA), r2);               // A^2 r^2
  const f51 W = f_sub(f_sq(D), f_add(a2r2, a2r2));                    // D^2 - 2 A^2 r^2
  const f51 num = f_mul(f_small((kMontA + 2) * kMontA), D);           // (A + 2) A D
  const f51 W3 = f_mul(f_sq(W), W), W7 = f_mul(f_sq(W3), W);
  const f51 beta = f_mul(f_mul(num, W3), f_pow22523(f_mul(num, W7)));
  const f51 vxx = f_mul(f_sq(beta), W);
  const bool lam_p1 = f_eq(vxx, num);
  const bool lam_m1 = f_iszero(f_add(vxx, num));
  const bool lam_pi = f_eq(vxx, f_mul(num, f_sqrtm1()));
  const bool nonsq = !(lam_p1 || lam_m1);
  const f51 F = nonsq ? (lam_pi ? f_one_minus_i() : f_one_plus_i())
                      : (lam_p1 ? f_one() : f_sqrtm1());
  f51 x = f_mul(beta, F);
  if (nonsq) x = f_mul(x, rr);
  if (f_isneg(x)) x = f_neg(x);
  const f51 Ar2 = f_mul(f_small(kMontA), r2);
  const f51 Xn = nonsq ? f_neg(f_add(Ar2, Ar2)) : f_neg(f_small(kMontA));
  const f51 n = f_sub(Xn, D), m = f_carry(f_add(Xn, D));
  return mul8(P3{f_mul(x, m), n, m, f_mul(x, n)});
}

// A decoded VRF key and its [1, 3, .., 15](-Y) table (shared by a header's two VRFs)
struct VrfKey {
  bool ok;
  Cached neg_y[8];
};
inline void vrf_key(VrfKey& k, const uint32_t pk[8]) {
  P3 Y;
  const bool okY = decode(&Y, pk, false);
  k.ok = !ouro::ge_has_small_order(pk) && ouro::ge_is_canonical(pk) && okY;
  odd_multiples(k.neg_y, p3_neg(Y), 8);
}

template <class Tail>
inline bool vrf03_verify(uint32_t beta[16], const VrfKey& key, const uint32_t pk[8],
                         const uint32_t pi[20], const Tail& alpha, uint32_t alen) {
  uint32_t G[8], c[8], s_raw[8], s[8];
  for (int i = 0; i < 8; i++) {
    G[i] = pi[i];
    s_raw[i] = pi[12 + i];
    c[i] = i < 4 ? pi[8 + i] : 0u;
  }
  P3 Gamma;
  bool ok = key.ok;
  ok = ouro::ge_is_canonical(G) && ok;
  ok = decode(&Gamma, G, false) && ok;
  ouro::sc_reduce256(s, s_raw);
  // H = hash_to_curve(Y, alpha): r = SHA-512(0x04 || 0x01 || Y || alpha)[0:32]
  uint32_t pre[9];
  pre[0] = 0x04u | (0x01u << 8) | (pk[0] << 16);
  for (int i = 1; i < 8; i++) pre[i] = (pk[i - 1] >> 16) | (pk[i] << 16);
  pre[8] = pk[7] >> 16;
  uint64_t Hs[8];
  ouro::sha512_prefixed<34>(Hs, pre, alpha, alen);
  uint32_t rw[16];
  ouro::sha512_digest_words(rw, Hs);
  rw[7] &= 0x7fffffffu;
  const P3 H = elligator2(rw);
  // U = [s]B - [c]Y (a 128-bit chain), V = [s]H - [c]Gamma
  Term tu;
  term_of(tu, key.neg_y, c, 128);
  const P3 U = straus(&tu, 1, s);
  Cached th[8], tg[8];
  odd_multiples(th, H, 8);
  odd_multiples(tg, p3_neg(Gamma), 8);
  Term tv[2];
  term_of(tv[0], th, s, 256);
  term_of(tv[1], tg, c, 128);
  const P3 V = straus(tv, 2, nullptr);
  const P3 G8 = mul8(Gamma);
  // one inversion for the four encodings
  const f51 a1 = f_mul(H.Z, U.Z), a2 = f_mul(a1, V.Z), a3 = f_mul(a2, G8.Z);
  f51 inv = f_invert(a3);
  const f51 i3 = f_mul(inv, a2);
  inv = f_mul(inv, G8.Z);
  const f51 i2 = f_mul(inv, a1);
  inv = f_mul(inv, V.Z);
  const f51 i1 = f_mul(inv, H.Z), i0 = f_mul(inv, U.Z);
  uint32_t Henc[8], Uenc[8], Venc[8], G8enc[8], Genc[8];
  encode_with_inv(Henc, H.X, H.Y, i0);
  encode_with_inv(Uenc, U.X, U.Y, i1);
  encode_with_inv(Venc, V.X, V.Y, i2);
  encode_with_inv(G8enc, G8.X, G8.Y, i3);
  // Gamma re-encoded: the input bytes, except x = 0 encodes with sign 0
  for (int i = 0; i < 8; i++) Genc[i] = G[i];
  if (f_iszero(Gamma.X)) Genc[7] &= 0x7fffffffu;
  uint32_t b[16];
  const bool ceq = ouro::vrf_finish(b, Henc, Genc, Uenc, Venc, G8enc, c);
  ok = ok && ceq;
  for (int i = 0; i < 16; i++) beta[i] = ok ? b[i] : 0u;
  return ok;
}

// ---- Sum6KES (verify.h sum6kes_verify_lane) -----------------------------------
template <class Tail>
inline bool sum6kes_verify(const uint32_t vk[8], uint32_t t, const uint32_t* sigw, const Tail& msg,
                           uint32_t mlen) {
  uint32_t cur[8], sig[16];
  const bool ok = ouro::sum6kes_walk(cur, sig, vk, t, sigw);
  return ed25519_verify(sig, cur, msg, mlen, false) && ok;
}

// proof_to_hash without verification (k_vrf03_proof_to_hash)
inline bool vrf03_proof_to_hash(uint32_t beta[16], const uint32_t pi[20]) {
  P3 Gamma;
  bool ok = ouro::ge_is_canonical(pi);
  ok = decode(&Gamma, pi, false) && ok;
  const P3 G8 = mul8(Gamma);
  uint32_t enc[8];
  encode_with_inv(enc, G8.X, G8.Y, f_invert(G8.Z));
  ouro::vrf_beta(beta, enc);
  return ok;
}

}  // namespace ouro_cpu
