// sc25519.h -- scalars mod L = 2^252 + 27742317777372353535851937790883648493.
//
// Barrett reduction (HAC 14.42, b = 2^32, k = 8) of a 512-bit (Ed25519 h) or
// 256-bit (VRF s) little-endian scalar, the canonicity test of libsodium
// sc25519_is_canonical, and the signed fixed-window recoding the
// double-scalar multiplication in verify.h consumes.
#pragma once
#include "common.h"

namespace ouro {

OURO_FI void sc_L(uint32_t l[8]) {
  l[0] = 0x5cf5d3edu; l[1] = 0x5812631au; l[2] = 0xa2f79cd6u; l[3] = 0x14def9deu;
  l[4] = 0; l[5] = 0; l[6] = 0; l[7] = 0x10000000u;
}

// a >= L ?
OURO_FI bool sc_geq_L(const uint32_t a[8]) {
  uint32_t l[8];
  sc_L(l);
  // lexicographic compare from the top word
  bool gt = false, eq = true;
#pragma unroll
  for (int i = 7; i >= 0; i--) {
    gt = gt || (eq && a[i] > l[i]);
    eq = eq && a[i] == l[i];
  }
  return gt || eq;
}

// sc25519_is_canonical: s < L
OURO_FI bool sc_is_canonical(const uint32_t s[8]) { return !sc_geq_L(s); }

OURO_FI void sc_sub_L(uint32_t a[8]) {
  uint32_t l[8];
  sc_L(l);
  uint64_t borrow = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint64_t d = (uint64_t)a[i] - l[i] - borrow;
    a[i] = (uint32_t)d;
    borrow = (d >> 63) & 1;
  }
}

// out = x mod L, x given as 16 little-endian words (zero-extend shorter input)
OURO_FI void sc_reduce512(uint32_t out[8], const uint32_t x[16]) {
  const uint32_t mu[9] = {0x0a2c131bu, 0xed9ce5a3u, 0x086329a7u, 0x2106215du, 0xffffffebu,
                          0xffffffffu, 0xffffffffu, 0xffffffffu, 0x0000000fu};
  uint32_t l[8];
  sc_L(l);
  // q2 = (x >> 224) * mu; keep words 9..17 (q3)
  uint32_t q2[18];
#pragma unroll
  for (int i = 0; i < 18; i++) q2[i] = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    uint64_t carry = 0;
#pragma unroll
    for (int j = 0; j < 9; j++) {
      uint64_t t = (uint64_t)x[7 + i] * mu[j] + q2[i + j] + carry;
      q2[i + j] = (uint32_t)t;
      carry = t >> 32;
    }
    q2[i + 9] = (uint32_t)carry;
  }
  // r2 = (q3 * L) mod 2^288
  uint32_t r2[9];
#pragma unroll
  for (int i = 0; i < 9; i++) r2[i] = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    uint64_t carry = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) {
      if (i + j < 9) {
        uint64_t t = (uint64_t)q2[9 + i] * l[j] + r2[i + j] + carry;
        r2[i + j] = (uint32_t)t;
        carry = t >> 32;
      }
    }
    if (i + 8 < 9) r2[i + 8] = (uint32_t)carry;
  }
  // r = (x mod 2^288) - r2  (mod 2^288), then r < 3L
  uint32_t r[9];
  uint64_t borrow = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    uint64_t d = (uint64_t)x[i] - r2[i] - borrow;
    r[i] = (uint32_t)d;
    borrow = (d >> 63) & 1;
  }
  // r < 3L < 2^255, so r[8] == 0 here
#pragma unroll
  for (int k = 0; k < 2; k++) {
    if (sc_geq_L(r)) sc_sub_L(r);
  }
#pragma unroll
  for (int i = 0; i < 8; i++) out[i] = r[i];
}

OURO_FI void sc_reduce256(uint32_t out[8], const uint32_t x[8]) {
  uint32_t w[16];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    w[i] = x[i];
    w[8 + i] = 0;
  }
  sc_reduce512(out, w);
}

// ---- signed fixed-window recoding ----------------------------------------
// Window j covers bits [W j, W j + W).  With c_0 = 0 and
//   t_j = bits_j + c_j,  c_{j+1} = (t_j > 2^(W-1)),  d_j = t_j - 2^W c_{j+1},
// every digit lies in [-(2^(W-1) - 1), 2^(W-1)].  The carries are packed in a
// mask (bit j = c_j) so the multiplication loop can form d_j from the scalar
// words and two mask bits without storing digits.
template <int W, int NWIN>
OURO_FI uint64_t sc_recode_carries(const uint32_t s[8]) {
  uint64_t mask = 0;
  uint32_t c = 0;
#pragma unroll
  for (int j = 0; j < NWIN; j++) {
    const int bit = W * j;
    static_assert(32 % W == 0, "windows must not straddle words");
    uint32_t v = (s[bit >> 5] >> (bit & 31)) & ((1u << W) - 1);
    mask |= (uint64_t)c << j;
    c = (v + c) > (1u << (W - 1)) ? 1u : 0u;
  }
  return mask;
}

// ---- digit streams for the double-scalar multiplication ---------------------
// A scalar consumed from its most significant window down: the next window
// sits in the top bits of w[N-1] and each step shifts the array left, so no
// register array is ever indexed dynamically (which the compiler would move
// to scratch memory).
template <int N>
OURO_FI void ss_shl(uint32_t w[N], int bits) {
#pragma unroll
  for (int i = N - 1; i > 0; i--) w[i] = (w[i] << bits) | (w[i - 1] >> (32 - bits));
  w[0] <<= bits;
}
// signed digit from the window value v (top bits of the stream) and the
// recoding carries into this window (cin) and out of it (cout)
template <int W>
OURO_FI int32_t sc_digit_from(uint32_t v, uint64_t carries, int j, int jmax) {
  const uint32_t cin = (uint32_t)(carries >> j) & 1u;
  const uint32_t cout = (j + 1 < jmax) ? (uint32_t)(carries >> (j + 1)) & 1u : 0u;
  return (int32_t)(v + cin) - (int32_t)(cout << W);
}

}  // namespace ouro
