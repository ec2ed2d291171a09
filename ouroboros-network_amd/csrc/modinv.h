// modinv.h -- variable-time inversion mod p = 2^255 - 19 by Bernstein-Yang
// divsteps ("safegcd", Bernstein & Yang 2019, "Fast constant-time gcd
// computation and modular inversion"; the variable-time batching of
// libsecp256k1's modinv32 as described in its safegcd_implementation notes).
//
// Every input on this path is public (signatures, keys, proofs), so the
// inversions of the finish -- the one Z^-1 batch per header, and per VRF in
// latency mode -- need not be constant time.  An exponentiation z^(p-2) costs
// 254 squarings + 11 multiplications (~33k VALU instructions per lane); the
// divsteps here work on 32-bit words (30 divsteps per batch, the 2x2
// transition matrix in int32, the 270-bit operands as nine signed 30-bit limbs
// updated with 32x32->64 multiply-adds), a few thousand instructions.
//
// Inside a batch the low bits of g are cancelled min(eta + 1, remaining) at a
// time with w = -g / f mod 2^limit (Newton inverse of the odd f), which is the
// composite of that many single divsteps: no swap can occur while eta >= 0.
// The result is the unique inverse (0 maps to 0, like z^(p-2)), so it is
// bit-identical to fe_invert after canonical encoding; tests/test_devcode_host.py
// compares the two on random and edge inputs.
#pragma once
#include "fe25519.h"

namespace ouro {

constexpr int32_t kM30 = 0x3fffffff;

// p in signed 30-bit limbs: 2^255 - 19 = (2^30 - 19) + (2^30 - 1)(2^30 + ... + 2^210) + (2^15 - 1) 2^240
OURO_FI int32_t sgcd_p_limb(int i) {
  return i == 0 ? 0x3fffffed : (i == 8 ? 0x7fff : 0x3fffffff);
}
// p^-1 mod 2^30
constexpr uint32_t sgcd_p_inv30() {
  uint32_t x = 0x3fffffedu;  // p = -19 (mod 2^30); p * p = 1 (mod 8)
  for (int k = 0; k < 5; k++) x *= 2u - 0x3fffffedu * x;
  return x & (uint32_t)kM30;
}
static_assert((sgcd_p_inv30() * 0x3fffffedu & (uint32_t)kM30) == 1u, "p^-1 mod 2^30");

// inverse of an odd f mod 2^32 (5 correct bits, then three Newton steps)
OURO_FI uint32_t sgcd_inv32(uint32_t f) {
  uint32_t x = (3u * f) ^ 2u;
  x *= 2u - f * x;
  x *= 2u - f * x;
  x *= 2u - f * x;
  return x;
}

struct SgcdMat { int32_t u, v, q, r; };

// -1 / f mod 2^kBits for an odd f: 5 correct bits, Newton steps to kBits
template <int kBits>
OURO_FI uint32_t sgcd_neg_inv(uint32_t f) {
  if (kBits > 10) return 0u - sgcd_inv32(f);
  uint32_t x = (3u * f) ^ 2u;
  x *= 2u - f * x;  // 10 bits
  return 0u - x;
}

// 30 divsteps on the low words of f (odd) and g; eta = -delta.  t maps
// (f, g) to (u f + v g, q f + r g) / 2^30.  kCap: at most that many low bits
// of g cancelled per step (<= 10: a one-Newton-step inverse of f, which is
// recomputed at nearly every step -- ~133 swaps in ~137 steps per inversion
// -- instead of three; the step count stays ~137 for random operands)
// kSpec (with kSel): the inverse of g computed ahead of the swap test, kept
// for f when the step swaps (off the step's dependent chain).
// kSel: the swap as selects and the inverse recomputed at every step, so a
// step has no branch but the loop's own (the wave inversion runs this on the
// scalar unit, where each taken branch costs an instruction refetch)
template <int kCap = 30, bool kSel = false, bool kSpec = false>
OURO_FI int32_t sgcd_divsteps30(int32_t eta, uint32_t f, uint32_t g, SgcdMat& t) {
  uint32_t u = 1, v = 0, q = 0, r = 1;
  uint32_t nfi = sgcd_neg_inv<kCap>(f);  // -1 / f mod 2^kCap, recomputed when f changes
  int i = 30;
  if (kSel) {
#pragma unroll 1
    for (;;) {
      const int zeros = __builtin_ctz(g | (0xffffffffu << i));
      g >>= zeros;
      u <<= zeros;
      v <<= zeros;
      eta -= zeros;
      i -= zeros;
      if (i == 0) break;
      // the inverse of g (f after a swap), computed before the swap test so
      // it overlaps it (kSpec), else of the new f after the swap
      const uint32_t nig = kSpec ? sgcd_neg_inv<kCap>(g) : 0u;
      const bool sw = eta < 0;
      const uint32_t f1 = sw ? g : f, g1 = sw ? 0u - f : g;
      const uint32_t u1 = sw ? q : u, q1 = sw ? 0u - u : q;
      const uint32_t v1 = sw ? r : v, r1 = sw ? 0u - v : r;
      eta = sw ? -eta : eta;
      f = f1;
      g = g1;
      u = u1;
      q = q1;
      v = v1;
      r = r1;
      if (kSpec) nfi = sw ? nig : nfi;
      const uint32_t ni = kSpec ? nfi : sgcd_neg_inv<kCap>(f);
      int limit = (eta + 1) > i ? i : (eta + 1);
      if (kCap < 30) limit = limit > kCap ? kCap : limit;
      const uint32_t w = (g * ni) & (0xffffffffu >> (32 - limit));
      g += f * w;
      q += u * w;
      r += v * w;
    }
    t.u = (int32_t)u;
    t.v = (int32_t)v;
    t.q = (int32_t)q;
    t.r = (int32_t)r;
    return eta;
  }
#pragma unroll 1
  for (;;) {
    // halvings of an even g, at most up to the batch end (sentinel bits)
    const int zeros = __builtin_ctz(g | (0xffffffffu << i));
    g >>= zeros;
    u <<= zeros;
    v <<= zeros;
    eta -= zeros;
    i -= zeros;
    if (i == 0) break;
    // g odd: with eta < 0 the divstep swaps (f, g) <- (g, -f)
    if (eta < 0) {
      uint32_t tmp;
      eta = -eta;
      tmp = f; f = g; g = 0u - tmp;
      tmp = u; u = q; q = 0u - tmp;
      tmp = v; v = r; r = 0u - tmp;
      nfi = sgcd_neg_inv<kCap>(f);
    }
    // then g <- (g + w f) / 2^k steps: cancel limit low bits of g at once
    int limit = (eta + 1) > i ? i : (eta + 1);
    if (kCap < 30) limit = limit > kCap ? kCap : limit;
    const uint32_t m = 0xffffffffu >> (32 - limit);
    const uint32_t w = (g * nfi) & m;
    g += f * w;
    q += u * w;
    r += v * w;
  }
  t.u = (int32_t)u;
  t.v = (int32_t)v;
  t.q = (int32_t)q;
  t.r = (int32_t)r;
  return eta;
}

// (f, g) <- t (f, g) / 2^30 (exact), nine limbs
OURO_FI void sgcd_update_fg(int32_t f[9], int32_t g[9], const SgcdMat& t) {
  const int64_t u = t.u, v = t.v, q = t.q, r = t.r;
  int64_t cf = u * f[0] + v * g[0], cg = q * f[0] + r * g[0];
  cf >>= 30;
  cg >>= 30;
#pragma unroll
  for (int i = 1; i < 9; i++) {
    cf += u * f[i] + v * g[i];
    cg += q * f[i] + r * g[i];
    f[i - 1] = (int32_t)cf & kM30;
    g[i - 1] = (int32_t)cg & kM30;
    cf >>= 30;
    cg >>= 30;
  }
  f[8] = (int32_t)cf;
  g[8] = (int32_t)cg;
}

// (d, e) <- t (d, e) / 2^30 mod p, keeping both in (-2p, p)
OURO_FI void sgcd_update_de(int32_t d[9], int32_t e[9], const SgcdMat& t) {
  const int32_t sd = d[8] >> 31, se = e[8] >> 31;
  int32_t md = (t.u & sd) + (t.v & se), me = (t.q & sd) + (t.r & se);
  const int64_t u = t.u, v = t.v, q = t.q, r = t.r;
  int64_t cd = u * d[0] + v * e[0], ce = q * d[0] + r * e[0];
  // md, me: multiples of p making the low 30 bits vanish
  md -= (int32_t)((sgcd_p_inv30() * (uint32_t)cd + (uint32_t)md) & (uint32_t)kM30);
  me -= (int32_t)((sgcd_p_inv30() * (uint32_t)ce + (uint32_t)me) & (uint32_t)kM30);
  cd += (int64_t)sgcd_p_limb(0) * md;
  ce += (int64_t)sgcd_p_limb(0) * me;
  cd >>= 30;
  ce >>= 30;
#pragma unroll
  for (int i = 1; i < 9; i++) {
    cd += u * d[i] + v * e[i] + (int64_t)sgcd_p_limb(i) * md;
    ce += q * d[i] + r * e[i] + (int64_t)sgcd_p_limb(i) * me;
    d[i - 1] = (int32_t)cd & kM30;
    e[i - 1] = (int32_t)ce & kM30;
    cd >>= 30;
    ce >>= 30;
  }
  d[8] = (int32_t)cd;
  e[8] = (int32_t)ce;
}

// limbs 0..7 into [0, 2^30), the sign in limb 8
OURO_FI void sgcd_propagate(int32_t d[9]) {
  int32_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const int32_t t = d[i] + c;
    d[i] = t & kM30;
    c = t >> 30;
  }
  d[8] += c;
}
OURO_FI void sgcd_add_p(int32_t d[9], int32_t sign) {  // d += p if sign (0 / -1)
#pragma unroll
  for (int i = 0; i < 9; i++) d[i] += sgcd_p_limb(i) & sign;
  sgcd_propagate(d);
}

// z^-1 mod p (0 for z = 0), variable time (kCap: sgcd_divsteps30)
template <int kCap = 30, bool kSel = false, bool kSpec = false>
OURO_HD inline fe fe_invert_vartime(const fe& z) {
  uint32_t zw[8];
  fe_to_words(zw, z);
  int32_t f[9], g[9], d[9], e[9];
#pragma unroll
  for (int i = 0; i < 9; i++) {
    f[i] = sgcd_p_limb(i);
    const int bit = 30 * i, w = bit >> 5, sh = bit & 31;
    uint64_t two = zw[w];
    if (w + 1 < 8) two |= (uint64_t)zw[w + 1] << 32;
    g[i] = (int32_t)(two >> sh) & kM30;
    d[i] = 0;
    e[i] = i == 0 ? 1 : 0;
  }
  int32_t eta = -1;
  // at most 724 divsteps for 255-bit operands (25 batches); the cap only
  // bounds the loop
#pragma unroll 1
  for (int it = 0; it < 32; it++) {
    SgcdMat t;
    eta = sgcd_divsteps30<kCap, kSel, kSpec>(eta, (uint32_t)f[0], (uint32_t)g[0], t);
    sgcd_update_de(d, e, t);
    sgcd_update_fg(f, g, t);
    int32_t nz = 0;
#pragma unroll
    for (int i = 0; i < 9; i++) nz |= g[i];
    if (nz == 0) break;
  }
  // f = +-1 (or p for z = 0, where d = 0): d * sign(f), reduced into [0, p)
  const int32_t fneg = f[8] >> 31;
  sgcd_propagate(d);
#pragma unroll
  for (int i = 0; i < 9; i++) d[i] = (d[i] ^ fneg) - fneg;
  sgcd_propagate(d);
  sgcd_add_p(d, d[8] >> 31);
  sgcd_add_p(d, d[8] >> 31);
  // subtract p once if d >= p
  int32_t s[9];
#pragma unroll
  for (int i = 0; i < 9; i++) s[i] = d[i] - sgcd_p_limb(i);
  sgcd_propagate(s);
  const int32_t keep = s[8] >> 31;  // -1: d < p
#pragma unroll
  for (int i = 0; i < 9; i++) d[i] = (d[i] & keep) | (s[i] & ~keep);
  // 255-bit value to words
  uint32_t w[8];
  uint64_t acc = 0;
  int bits = 0, wi = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    acc |= (uint64_t)(uint32_t)d[i] << bits;
    bits += 30;
    if (bits >= 32 && wi < 8) {
      w[wi++] = (uint32_t)acc;
      acc >>= 32;
      bits -= 32;
    }
  }
  return fe_from_words(w);
}

}  // namespace ouro
