// wide_inv.h -- one field inversion on one wave (latency mode), for the V2
// item's combination (encode2_wide; OURO_WIDE_INV=2).
//
// The wave-wide z^(p-2) (wide.h fw_invert) is 254 squarings + 11 products in
// a dependent chain, ~24 us on the configs[4] critical path; the lane's
// Bernstein-Yang inversion (modinv.h) ran ~12 us slower still, because one
// lane also does the 4 x 9-limb transition-matrix updates of every 30-divstep
// batch in series.  Here the batches' matrices are computed exactly as in
// modinv.h (sgcd_divsteps30, wave-uniform: every lane computes the same from
// the operands' low limbs, read out of lane 0), and the updates run across the
// lanes of each DPP row: lane k holds limb k (30 bits, signed) of f, g, d, e
// and forms u f_k + v g_k etc. with one multiply-add each; the exact division
// by 2^30 is two parallel carry rounds (row_shl / row_shr by one lane), after
// which limb 0 holds the exact low 30 bits the next batch needs and the other
// limbs stay in [-8, 2^30 + 8].  d and e are kept unreduced -- the multiple
// of p that clears their low bits is taken in [0, 2^30), so each batch adds
// at most p to their size and 25 batches stay below 2^260 (9 limbs) -- and
// reduced once at the end.  25 batches (750 divsteps) always: the variable-
// time bound for 255-bit operands is 724, and once g = 0 a batch leaves f, d,
// e as they are.  The result is the unique inverse (0 -> 0), so it equals
// z^(p-2) bit for bit; the latency parity tests compare the encodings with the
// oracle.  Since round 5 the loop ends at the first batch after which g is
// zero (OURO_INV_EARLY): the inputs are public points, so a data-dependent
// batch count leaks nothing.
#pragma once
#include "modinv.h"
#include "wide.h"

// leave the batch loop once g is zero (1) or always run all 25 batches (0, A/B)
#ifndef OURO_INV_EARLY
#define OURO_INV_EARLY 1
#endif
// bits of g cancelled per divstep step at most (modinv.h sgcd_divsteps30): 30
// (three Newton steps per inverse of f) or 10 (one step; A/B: no faster,
// profiles/r05j/inv_timing.json)
#ifndef OURO_INV_CAP
#define OURO_INV_CAP 30
#endif
// the divstep steps branch-free (modinv.h sgcd_divsteps30 kSel; A/B: the
// same time, profiles/r05j/inv_timing.json)
#ifndef OURO_INV_SEL
#define OURO_INV_SEL 0
#endif

namespace ouro {

// modinv.h sgcd_divsteps30 with its state in vector registers: the same
// steps (the swap as selects), issued by the VALU instead of the scalar unit,
// whose dependent instructions are the slower of the two (the 18 batches of an
// inversion's scalar loop take ~15 of its ~19 us, whatever the loop's
// instruction count: profiles/r05j/inv_timing.json).  Every lane computes the
// same; the loop's exit test reads lane 0.  A/B switch OURO_INV_VEC.
template <int kCap>
__device__ __forceinline__ int32_t sgcd_divsteps30_vec(int32_t eta, uint32_t f, uint32_t g,
                                                       SgcdMat& t) {
  uint32_t u = 1, v = 0, q = 0, r = 1;
  int32_t i = 30;
  asm volatile("" : "+v"(f), "+v"(g), "+v"(eta), "+v"(i), "+v"(u), "+v"(r));
#pragma unroll 1
  for (;;) {
    const uint32_t zeros = (uint32_t)__builtin_ctz(g | (0xffffffffu << i));
    g >>= zeros;
    u <<= zeros;
    v <<= zeros;
    eta -= (int32_t)zeros;
    i -= (int32_t)zeros;
    if (__builtin_amdgcn_readfirstlane(i) == 0) break;
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
    const uint32_t ni = sgcd_neg_inv<kCap>(f);
    int32_t limit = (eta + 1) > i ? i : (eta + 1);
    if (kCap < 30) limit = limit > kCap ? kCap : limit;
    const uint32_t w = (g * ni) & (0xffffffffu >> (32 - limit));
    g += f * w;
    q += u * w;
    r += v * w;
  }
  t.u = __builtin_amdgcn_readfirstlane((int32_t)u);
  t.v = __builtin_amdgcn_readfirstlane((int32_t)v);
  t.q = __builtin_amdgcn_readfirstlane((int32_t)q);
  t.r = __builtin_amdgcn_readfirstlane((int32_t)r);
  return __builtin_amdgcn_readfirstlane(eta);
}
#ifndef OURO_INV_VEC
#define OURO_INV_VEC 0
#endif

// lane j <- lane j + 1 / lane j - 1 of the same row (0 past the row's end)
__device__ __forceinline__ int32_t row_from_next(int32_t x) {
  return __builtin_amdgcn_mov_dpp(x, 0x101, 0xf, 0xf, true);  // row_shl:1
}
__device__ __forceinline__ int32_t row_from_prev(int32_t x) {
  return __builtin_amdgcn_mov_dpp(x, 0x111, 0xf, 0xf, true);  // row_shr:1
}

// (sum_k c_k 2^(30 k)) / 2^30 with c_0 = 0 (mod 2^30), limb k on lane k of
// the row (k <= kTopLimb; lanes above hold 0): new_k = lo30(c_(k+1)) +
// (c_k >> 30), then one more carry round.  The top limb keeps its whole signed
// value (a negative number's borrow stops there instead of creeping up the
// row one lane per batch).
constexpr int kTopLimb = 9;
__device__ __forceinline__ int32_t sgcd_div30_rows(int64_t c, bool top) {
  const int32_t lo = (int32_t)((uint32_t)c & (uint32_t)kM30);
  const int64_t r1 = (c >> 30) + (int64_t)(uint32_t)row_from_next(lo);
  const int32_t r1lo = top ? (int32_t)r1 : (int32_t)((uint32_t)r1 & (uint32_t)kM30);
  const int32_t r1hi = top ? 0 : (int32_t)(r1 >> 30);  // |r1| < 2^33: a small carry
  return r1lo + row_from_prev(r1hi);
}

// z^-1 mod p (0 for z = 0); z the same in every lane.  kEarly: leave the
// batch loop once g is zero (OURO_INV_EARLY; both forms for the timing probe)
template <bool kEarly = (OURO_INV_EARLY != 0), int kCap = OURO_INV_CAP,
          bool kSel = (OURO_INV_SEL != 0), bool kVec = (OURO_INV_VEC != 0)>
__device__ __noinline__ fe fe_invert_wave(fe z) {
  const int k = (int)(threadIdx.x & 15u);  // limb index: the four rows alike
  uint32_t zw[8];
  fe_to_words(zw, z);
  // limb k of z: bits 30 k .. 30 k + 29
  uint64_t two = 0;
#pragma unroll
  for (int w = 0; w < 8; w++) {
    const uint64_t pair = (uint64_t)zw[w] | (w + 1 < 8 ? (uint64_t)zw[w + 1] << 32 : 0ull);
    two = ((30 * k) >> 5) == w ? pair : two;
  }
  int32_t g = k < 9 ? (int32_t)((two >> ((30 * k) & 31)) & (uint64_t)kM30) : 0;
  const int32_t pk = k == 0 ? 0x3fffffed : (k == 8 ? 0x7fff : (k < 8 ? 0x3fffffff : 0));
  int32_t f = pk, d = 0, e = k == 0 ? 1 : 0;
  const bool top = k == kTopLimb;
  int32_t eta = -1;
#pragma unroll 1
  for (int it = 0; it < 25; it++) {
    const uint32_t f0 = (uint32_t)__builtin_amdgcn_readfirstlane(f);
    const uint32_t g0 = (uint32_t)__builtin_amdgcn_readfirstlane(g);
    const uint32_t d0 = (uint32_t)__builtin_amdgcn_readfirstlane(d);
    const uint32_t e0 = (uint32_t)__builtin_amdgcn_readfirstlane(e);
    SgcdMat t;
    if (kVec) eta = sgcd_divsteps30_vec<kCap>(eta, f0, g0, t);
    else eta = sgcd_divsteps30<kCap, kSel>(eta, f0, g0, t);
    // the multiples of p clearing the low 30 bits of t (d, e), in [0, 2^30)
    const uint32_t md = (0u - ((uint32_t)t.u * d0 + (uint32_t)t.v * e0) * sgcd_p_inv30()) &
                        (uint32_t)kM30;
    const uint32_t me = (0u - ((uint32_t)t.q * d0 + (uint32_t)t.r * e0) * sgcd_p_inv30()) &
                        (uint32_t)kM30;
    const int64_t cf = (int64_t)t.u * f + (int64_t)t.v * g;
    const int64_t cg = (int64_t)t.q * f + (int64_t)t.r * g;
    const int64_t cd = (int64_t)t.u * d + (int64_t)t.v * e + (int64_t)pk * (int64_t)md;
    const int64_t ce = (int64_t)t.q * d + (int64_t)t.r * e + (int64_t)pk * (int64_t)me;
    f = sgcd_div30_rows(cf, top);
    g = sgcd_div30_rows(cg, top);
    d = sgcd_div30_rows(cd, top);
    e = sgcd_div30_rows(ce, top);
    // g = 0: done (17--19 batches for random operands, against the 25 of the
    // bound).  Its limbs need not all be 0 (the carry rounds leave e.g.
    // (0, 2^30, -1, ...)), but its low limb is 0 mod 2^30, which a nonzero g
    // shows with probability 2^-30: only then is the value checked exactly,
    // wave-uniformly from the row's limbs.
    if (kEarly && ((uint32_t)__builtin_amdgcn_readfirstlane(g) & (uint32_t)kM30) == 0) {
      int64_t c = 0;
      bool zero = true;
#pragma unroll
      for (int i = 0; i < kTopLimb; i++) {
        c += (int64_t)__builtin_amdgcn_readlane(g, i);
        zero = zero && (c & kM30) == 0;
        c >>= 30;
      }
      c += (int64_t)__builtin_amdgcn_readlane(g, kTopLimb);
      if (zero && c == 0) break;
    }
  }
  // f = +-1 (p for z = 0, where d = 0): its low limb says which
  const bool fneg = (uint32_t)__builtin_amdgcn_readfirstlane(f) == (uint32_t)kM30;
  // d's limbs to every lane, then d mod p: + 32 p (|d| < 26 p), carried into
  // [0, 2^30) limbs, 2^255 = 19 folded, and at most two subtractions of p
  int64_t L[kTopLimb + 1];
#pragma unroll
  for (int i = 0; i <= kTopLimb; i++)
    L[i] = (int64_t)__builtin_amdgcn_readlane(d, i) + (i < 9 ? 32 * (int64_t)sgcd_p_limb(i) : 0);
#pragma unroll
  for (int i = 0; i < kTopLimb; i++) {
    L[i + 1] += L[i] >> 30;
    L[i] &= kM30;
  }
  // value in (6 p, 58 p): bits 255.. are limb 8's above 15 and limb 9
  const int64_t hi = (L[8] >> 15) + (L[9] << 15);
  L[8] &= 0x7fff;
  L[0] += 19 * hi;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    L[i + 1] += L[i] >> 30;
    L[i] &= kM30;
  }
  // now < 2^255 + 2^12 (limb 8 at most 0x7fff + 1): subtract p while >= p
#pragma unroll
  for (int pass = 0; pass < 2; pass++) {
    int64_t s[9], c = 0;
#pragma unroll
    for (int i = 0; i < 9; i++) {
      const int64_t v = L[i] - sgcd_p_limb(i) + c;
      s[i] = v & kM30;
      c = v >> 30;
    }
    const bool ge = c >= 0;  // no borrow out of the top: value >= p
#pragma unroll
    for (int i = 0; i < 9; i++) L[i] = ge ? s[i] : L[i];
  }
  uint32_t w[8];
  uint64_t acc = 0;
  int bits = 0, wi = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    acc |= (uint64_t)L[i] << bits;
    bits += 30;
    if (bits >= 32 && wi < 8) {
      w[wi++] = (uint32_t)acc;
      acc >>= 32;
      bits -= 32;
    }
  }
  fe r = fe_from_words(w);
  if (fneg) r = fe_carry(fe_neg(r));
  return r;
}

}  // namespace ouro
