// leader.h -- TPraos leader-threshold check on the leader VRF output
// (SURVEY.md §8(f) rank 3): ledger-specs `checkLeaderValue`, called from
// ouroboros-consensus-shelley/src/Ouroboros/Consensus/Shelley/Protocol.hs:473-491
// (`meetsLeaderThreshold`), restated bit for bit in exact integer arithmetic.
//
// The reference (shelley-spec-ledger BlockChain.hs + shelley-spec-non-integral,
// un-vendored; PARITY UNPINNED) decides
//     p < 1 - (1 - f)^sigma  <=>  1 / (1 - p) < exp(-sigma ln(1 - f))
// with p = certNat / 2^512 and everything in FixedPoint = Data.Fixed E34
// (integers scaled by res = 10^34; x * y = floor(x y / res), x / y =
// floor(x res / y), fromRational r = floor(r res)):
//     recip_q = fromRational (2^512 % (2^512 - certNat))
//     c       = activeSlotLog f      -- an integer mantissa L, given
//     x       = - fromRational sigma * c
//     taylorExpCmp 3 recip_q x:  ABOVE -> False, BELOW -> True,
//                                MaxReached (1000 terms) -> False
// with taylorExpCmp boundX cmp x = go 1000 0 x 1 1 and, per step,
//     acc' = acc + err, err' = (err * x) / (divisor + 1),
//     errorTerm = |err' * boundX|,
//     cmp >= acc' + errorTerm -> ABOVE;  cmp < acc' - errorTerm -> BELOW.
// Because res divides the scale, (err * x) / k = floor(floor(err x / res) / k)
// and errorTerm = 3 |err'| exactly, so every quantity is an integer here.
//
// Domain (checked, else OURO_LEADER_BADARG): 0 <= sigma <= 1 (num <= den,
// den > 0, both < 2^64) and -8 res <= L <= 0 (f <= 1 - e^-8); then x <= 8,
// every accumulator stays below 2^127 and 4-word arithmetic is exact.  A
// recip_q of 2^128 or more is capped: it exceeds acc' + errorTerm < 2^127 on
// the first step, which is the reference's ABOVE as well.
#pragma once
#include "common.h"

namespace ouro {

constexpr int32_t kLeaderNo = 0;
constexpr int32_t kLeaderYes = 1;
constexpr int32_t kLeaderBadArg = -1;

// res = 10^34 as 4 little-endian words
OURO_FI void fp_res(uint32_t r[4]) {
  r[0] = 0x00000000u; r[1] = 0x378d8e64u; r[2] = 0xbead87c0u; r[3] = 0x0001ed09u;
}

// a >= b over N words
template <int N>
OURO_FI bool mw_ge(const uint32_t* a, const uint32_t* b) {
  bool gt = false, eq = true;
#pragma unroll
  for (int i = N - 1; i >= 0; i--) {
    gt = gt || (eq && a[i] > b[i]);
    eq = eq && a[i] == b[i];
  }
  return gt || eq;
}

template <int N>
OURO_FI void mw_add(uint32_t* r, const uint32_t* a, const uint32_t* b) {
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < N; i++) {
    const uint64_t t = (uint64_t)a[i] + b[i] + c;
    r[i] = (uint32_t)t;
    c = (uint32_t)(t >> 32);
  }
}

// r = a - b, returns the borrow out
template <int N>
OURO_FI uint32_t mw_sub(uint32_t* r, const uint32_t* a, const uint32_t* b) {
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < N; i++) {
    const uint64_t t = (uint64_t)a[i] - b[i] - br;
    r[i] = (uint32_t)t;
    br = (uint32_t)(t >> 63);
  }
  return br;
}

// r (NA + NB words) = a * b
template <int NA, int NB>
OURO_FI void mw_mul(uint32_t* r, const uint32_t* a, const uint32_t* b) {
#pragma unroll
  for (int i = 0; i < NA + NB; i++) r[i] = 0;
#pragma unroll
  for (int i = 0; i < NA; i++) {
    uint64_t carry = 0;
#pragma unroll
    for (int j = 0; j < NB; j++) {
      const uint64_t t = (uint64_t)a[i] * b[j] + r[i + j] + carry;
      r[i + j] = (uint32_t)t;
      carry = t >> 32;
    }
    r[i + NB] = (uint32_t)carry;
  }
}

// Restoring division with a bounded quotient: q (QW words) = floor(a / d),
// rem (ND words) = a mod d, valid when floor(a / 2^(32 QW)) < d -- the caller
// guarantees it (or checks it with mw_div_fits).  a has NA >= QW words.
template <int NA, int ND, int QW>
OURO_HD inline void mw_divq(uint32_t* q, uint32_t* rem, const uint32_t* a, const uint32_t* d) {
  uint32_t r[ND + 1];
#pragma unroll
  for (int i = 0; i <= ND; i++) r[i] = (i < ND && i + QW < NA) ? a[i + QW] : 0u;
  uint32_t dd[ND + 1];
#pragma unroll
  for (int i = 0; i <= ND; i++) dd[i] = i < ND ? d[i] : 0u;
#pragma unroll
  for (int w = QW - 1; w >= 0; w--) {
    const uint32_t word = a[w];
    uint32_t qw = 0;
#pragma unroll 1
    for (int b = 31; b >= 0; b--) {
      // r = 2 r + bit (r < d, so 2 r + 1 < 2 d fits ND words and one bit)
#pragma unroll
      for (int i = ND; i > 0; i--) r[i] = (r[i] << 1) | (r[i - 1] >> 31);
      r[0] = (r[0] << 1) | ((word >> b) & 1u);
      uint32_t t[ND + 1];
      const uint32_t br = mw_sub<ND + 1>(t, r, dd);
#pragma unroll
      for (int i = 0; i <= ND; i++) r[i] = br ? r[i] : t[i];
      qw |= (br ^ 1u) << b;
    }
    q[w] = qw;
  }
#pragma unroll
  for (int i = 0; i < ND; i++) rem[i] = r[i];
}

// floor(a / 2^(32 QW)) < d ?
template <int NA, int ND, int QW>
OURO_FI bool mw_div_fits(const uint32_t* a, const uint32_t* d) {
  uint32_t hi[ND + 1], dd[ND + 1];
#pragma unroll
  for (int i = 0; i <= ND; i++) {
    hi[i] = (i + QW < NA) ? a[i + QW] : 0u;
    dd[i] = i < ND ? d[i] : 0u;
  }
  // words of a above ND + QW must be zero too
  bool high_zero = true;
#pragma unroll
  for (int i = ND + 1 + QW; i < NA; i++) high_zero = high_zero && a[i] == 0;
  return high_zero && !mw_ge<ND + 1>(hi, dd);
}

// r (4 words) = floor(a / k) for a 32-bit k > 0
OURO_FI void mw_div_small4(uint32_t r[4], const uint32_t a[4], uint32_t k) {
  uint64_t rem = 0;
#pragma unroll
  for (int i = 3; i >= 0; i--) {
    const uint64_t cur = (rem << 32) | a[i];
    r[i] = (uint32_t)(cur / k);
    rem = cur % k;
  }
}

// beta: the 64-byte leader VRF output (big-endian natural, as
// getOutputVRFNatural); sigma = num / den; act_log = the ActiveSlotCoeff's
// unActiveSlotLog as a signed 128-bit integer (lo, hi words).
OURO_HD inline int32_t leader_check_lane(const uint8_t* beta, uint64_t num, uint64_t den,
                                         uint64_t act_log_lo, int64_t act_log_hi) {
  uint32_t res[4];
  fp_res(res);
  // domain: 0 <= num <= den, den > 0, -8 res <= L <= 0
  if (den == 0 || num > den) return kLeaderBadArg;
  uint32_t L[4] = {(uint32_t)act_log_lo, (uint32_t)(act_log_lo >> 32), (uint32_t)act_log_hi,
                   (uint32_t)((uint64_t)act_log_hi >> 32)};
  if (act_log_hi > 0 || (act_log_hi == 0 && act_log_lo != 0)) return kLeaderBadArg;
  uint32_t absL[4], zero[4] = {0, 0, 0, 0};
  mw_sub<4>(absL, zero, L);  // -L
  uint32_t eight_res[4];
  {
    uint32_t e[1] = {8u}, t[5];
    mw_mul<4, 1>(t, res, e);
#pragma unroll
    for (int i = 0; i < 4; i++) eight_res[i] = t[i];
  }
  if (!mw_ge<4>(eight_res, absL)) return kLeaderBadArg;

  // recip_q = floor(2^512 res / (2^512 - certNat)), capped below 2^128
  uint32_t cn[16];
#pragma unroll
  for (int i = 0; i < 16; i++) {
    const uint8_t* p = beta + 60 - 4 * i;  // big-endian bytes -> little-endian words
    cn[i] = ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
  }
  uint32_t D[17];
  {
    uint32_t two512[17];
#pragma unroll
    for (int i = 0; i < 17; i++) two512[i] = i == 16 ? 1u : 0u;
    uint32_t cn17[17];
#pragma unroll
    for (int i = 0; i < 17; i++) cn17[i] = i < 16 ? cn[i] : 0u;
    mw_sub<17>(D, two512, cn17);  // >= 1
  }
  uint32_t N[20];
#pragma unroll
  for (int i = 0; i < 20; i++) N[i] = i >= 16 ? res[i - 16] : 0u;  // res << 512
  uint32_t cmp[4];
  if (mw_div_fits<20, 17, 4>(N, D)) {
    uint32_t rem[17];
    mw_divq<20, 17, 4>(cmp, rem, N, D);
  } else {
#pragma unroll
    for (int i = 0; i < 4; i++) cmp[i] = 0xffffffffu;
  }

  // sigma_m = floor(num res / den)  (<= res, so 4 words)
  uint32_t sigma_m[4];
  {
    uint32_t n2[2] = {(uint32_t)num, (uint32_t)(num >> 32)};
    uint32_t d2[2] = {(uint32_t)den, (uint32_t)(den >> 32)};
    uint32_t prod[6], rem[2];
    mw_mul<4, 2>(prod, res, n2);
    // floor(prod / 2^128) <= num res / 2^128 < num <= den
    mw_divq<6, 2, 4>(sigma_m, rem, prod, d2);
  }
  // x_m = -floor(sigma_m L / res) = ceil(sigma_m |L| / res)  (<= 8 res)
  uint32_t x[4];
  {
    uint32_t prod[8], rem[4];
    mw_mul<4, 4>(prod, sigma_m, absL);
    // prod <= res * 8 res, so floor(prod / 2^128) < res
    mw_divq<8, 4, 4>(x, rem, prod, res);
    const bool nz = (rem[0] | rem[1] | rem[2] | rem[3]) != 0;
    uint32_t one[4] = {nz ? 1u : 0u, 0, 0, 0};
    mw_add<4>(x, x, one);
  }

  // taylorExpCmp 3 recip_q x = go 1000 0 x 1 1
  uint32_t err[4], acc[4];
#pragma unroll
  for (int i = 0; i < 4; i++) {
    err[i] = x[i];
    acc[i] = res[i];
  }
#pragma unroll 1
  for (uint32_t n = 0; n < 1000; n++) {
    uint32_t acc1[4];
    mw_add<4>(acc1, acc, err);  // acc' = acc + err
    // err' = floor(floor(err x / res) / (n + 2))   (err x < 2^226)
    uint32_t prod[8], t[4], rem[4], err1[4];
    mw_mul<4, 4>(prod, err, x);
    mw_divq<8, 4, 4>(t, rem, prod, res);
    mw_div_small4(err1, t, n + 2);
    // errorTerm = 3 err'
    uint32_t e3[4], et[5], three[1] = {3u};
    mw_mul<4, 1>(et, err1, three);
#pragma unroll
    for (int i = 0; i < 4; i++) e3[i] = et[i];
    uint32_t hi[4];
    mw_add<4>(hi, acc1, e3);
    if (mw_ge<4>(cmp, hi)) return kLeaderNo;  // ABOVE
    uint32_t lo[4];
    const uint32_t neg = mw_sub<4>(lo, acc1, e3);
    if (!neg && !mw_ge<4>(cmp, lo)) return kLeaderYes;  // BELOW: cmp < acc' - errorTerm
#pragma unroll
    for (int i = 0; i < 4; i++) {
      err[i] = err1[i];
      acc[i] = acc1[i];
    }
  }
  return kLeaderNo;  // MaxReached
}

}  // namespace ouro
