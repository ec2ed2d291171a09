// fe25519.h -- GF(2^255 - 19) for gfx950, one field element per lane.
//
// Representation: 10 UNSIGNED 32-bit limbs, radix 2^25.5 (limb i weighs
// 2^ceil(25.5 i): 26-bit even limbs, 25-bit odd limbs).  Products accumulate
// in unsigned 64-bit, which hipcc lowers to v_mad_u64_u32.  The signed form
// (v_mad_i64_i32) issues slower on MI355X: the same multiply runs 14 % faster
// unsigned although it executes more instructions (profiles/r01c/
// fe_mul_variants.json; tools/microbench/fe_mul_variants.hip).
//
// Unsigned limbs mean subtraction adds a multiple of p first:
//   fe_sub(f, g)  = f + 2p - g      (g <= 2p limbwise)
//   fe_sub4(f, g) = f + 4p - g      (g <= 4p limbwise)
// and every operand of a multiplication must keep its column sums below 2^64
// and 19 * (its second operand) below 2^32.  The group formulas in ge25519.h
// are arranged for that.  Rather than a hand proof per formula, the host test
// build (OURO_COUNT_OPS) carries a worst-case upper bound for every limb next
// to its value -- constants exact, loads/stores through a shadow table,
// add/sub/select/mul/carry propagating maxima independent of the data -- and
// counts every operation whose worst case could overflow
// (tests/test_devcode_host.py::test_zero_bound_violations).  Because the
// arithmetic's control flow does not depend on the values, one pass through a
// routine covers all of its inputs.
//
// "Reduced" = what fe_mul/fe_sq/fe_carry64 return: limb i <= mask_i (2^26 - 1
// even, 2^25 - 1 odd), except limb 1 <= 2^25 + 2^18 and (two-chain scanned
// multiply) limb 6 <= 2^26 + 2^12; the host tracker carries the exact bounds.
#pragma once
#include "common.h"

#if defined(OURO_COUNT_OPS) && !defined(__HIP_DEVICE_COMPILE__)
#define OURO_TRACK_BOUNDS 1
extern thread_local unsigned long long g_ouro_nmul, g_ouro_nsq, g_ouro_bound_violations;
#define OURO_COUNT_MUL() (++g_ouro_nmul)
#define OURO_COUNT_SQ() (++g_ouro_nsq)
#define OURO_TRK(...) __VA_ARGS__
// shadow table for bounds of elements kept in memory (devhost_test.hip)
void ouro_trk_store(const void* p, const uint64_t b[10]);
void ouro_trk_load(const void* p, uint64_t b[10]);
void ouro_trk_violation();  // counts; aborts under OURO_TRK_ABORT=1 (for gdb)
#else
#define OURO_COUNT_MUL() ((void)0)
#define OURO_COUNT_SQ() ((void)0)
#define OURO_TRK(...)
#endif

namespace ouro {

struct fe {
  uint32_t v[10];
#if defined(OURO_TRACK_BOUNDS)
  uint64_t b[10];  // host bound tracker: worst-case value of each limb
#endif
};

OURO_FI constexpr uint32_t limb_bits(int i) { return (i & 1) ? 25u : 26u; }
OURO_FI constexpr uint32_t limb_mask(int i) { return (1u << limb_bits(i)) - 1u; }
// limb i of K*p in the canonical split (limb 0 = K (2^26 - 19))
OURO_FI constexpr uint32_t kp_limb(uint32_t K, int i) {
  return i == 0 ? K * ((1u << 26) - 19u) : K * limb_mask(i);
}

#if defined(OURO_TRACK_BOUNDS)
inline void trk_check(bool ok) {
  if (!ok) ouro_trk_violation();
}
inline void trk_exact(fe& f) {
  for (int i = 0; i < 10; i++) f.b[i] = f.v[i];
}
// upper bounds after a floor carry chain over column bounds T (checked < 2^64)
inline void trk_carry(fe& h, const unsigned __int128 T[10], unsigned __int128 lim) {
  unsigned __int128 t[10];
  for (int i = 0; i < 10; i++) {
    t[i] = T[i];
    trk_check(t[i] < lim);
  }
  auto step = [&](int i, int j) {
    t[j] += t[i] >> limb_bits(i);
    if (t[i] > limb_mask(i)) t[i] = limb_mask(i);
    trk_check(t[j] < lim);
  };
  step(0, 1); step(4, 5); step(1, 2); step(5, 6); step(2, 3);
  step(6, 7); step(3, 4); step(7, 8); step(4, 5); step(8, 9);
  t[0] += 19 * (t[9] >> 25);
  if (t[9] > limb_mask(9)) t[9] = limb_mask(9);
  trk_check(t[0] < lim);
  step(0, 1);
  for (int i = 0; i < 10; i++) h.b[i] = (uint64_t)t[i];
}
#endif

OURO_FI fe fe_make(uint32_t a0, uint32_t a1, uint32_t a2, uint32_t a3, uint32_t a4, uint32_t a5,
                   uint32_t a6, uint32_t a7, uint32_t a8, uint32_t a9) {
  fe r;
  r.v[0] = a0; r.v[1] = a1; r.v[2] = a2; r.v[3] = a3; r.v[4] = a4;
  r.v[5] = a5; r.v[6] = a6; r.v[7] = a7; r.v[8] = a8; r.v[9] = a9;
  OURO_TRK(trk_exact(r));
  return r;
}

// ---- constants (canonical limbs; tools/check_fe_constants.py) ---------------
// d = -121665/121666
OURO_FI fe fe_d() {
  return fe_make(56195235, 13857412, 51736253, 6949390, 114729, 24766616, 60832955, 30306712,
                 48412415, 21499315);
}
OURO_FI fe fe_d2() {
  return fe_make(45281625, 27714825, 36363642, 13898781, 229458, 15978800, 54557047, 27058993,
                 29715967, 9444199);
}
// sqrt(-1) = 2^((p-1)/4), libsodium's fe25519_sqrtm1
OURO_FI fe fe_sqrtm1() {
  return fe_make(34513072, 25610706, 9377949, 3500415, 12389472, 33281959, 41962654, 31548777,
                 326685, 11406482);
}
// Montgomery A = 486662 (curve25519), used by Elligator2
OURO_FI fe fe_mont_a() { return fe_make(486662, 0, 0, 0, 0, 0, 0, 0, 0, 0); }
// A^2 and (A + 2) A (Elligator2's sqrt-ratio numerator), 1 + sqrt(-1), 1 - sqrt(-1)
OURO_FI fe fe_mont_a2() { return fe_make(12721188, 3529, 0, 0, 0, 0, 0, 0, 0, 0); }
OURO_FI fe fe_mont_a2a() { return fe_make(13694512, 3529, 0, 0, 0, 0, 0, 0, 0, 0); }
OURO_FI fe fe_one_plus_i() {
  return fe_make(34513073, 25610706, 9377949, 3500415, 12389472, 33281959, 41962654, 31548777,
                 326685, 11406482);
}
OURO_FI fe fe_one_minus_i() {
  return fe_make(32595774, 7943725, 57730914, 30054016, 54719391, 272472, 25146209, 2005654,
                 66782178, 22147949);
}
OURO_FI fe fe_zero() { return fe_make(0, 0, 0, 0, 0, 0, 0, 0, 0, 0); }
OURO_FI fe fe_one() { return fe_make(1, 0, 0, 0, 0, 0, 0, 0, 0, 0); }
OURO_FI fe fe_two() { return fe_make(2, 0, 0, 0, 0, 0, 0, 0, 0, 0); }

OURO_FI fe fe_add(const fe& f, const fe& g) {
  fe h;
#pragma unroll
  for (int i = 0; i < 10; i++) h.v[i] = f.v[i] + g.v[i];
  OURO_TRK(for (int i = 0; i < 10; i++) {
    h.b[i] = f.b[i] + g.b[i];
    trk_check(h.b[i] < (1ull << 32));
  })
  return h;
}
// f + K p - g
template <uint32_t K>
OURO_FI fe fe_subk(const fe& f, const fe& g) {
  fe h;
#pragma unroll
  for (int i = 0; i < 10; i++) h.v[i] = (f.v[i] + kp_limb(K, i)) - g.v[i];
  OURO_TRK(for (int i = 0; i < 10; i++) {
    trk_check(g.b[i] <= kp_limb(K, i));
    h.b[i] = f.b[i] + kp_limb(K, i);
    trk_check(h.b[i] < (1ull << 32));
  })
  return h;
}
OURO_FI fe fe_sub(const fe& f, const fe& g) { return fe_subk<2>(f, g); }
OURO_FI fe fe_sub4(const fe& f, const fe& g) { return fe_subk<4>(f, g); }
OURO_FI fe fe_neg(const fe& f) { return fe_subk<2>(fe_zero(), f); }
OURO_FI fe fe_neg4(const fe& f) { return fe_subk<4>(fe_zero(), f); }

// c ? a : b, per lane
OURO_FI fe fe_select(const fe& a, const fe& b, bool c) {
  fe h;
#pragma unroll
  for (int i = 0; i < 10; i++) h.v[i] = c ? a.v[i] : b.v[i];
  OURO_TRK(for (int i = 0; i < 10; i++) h.b[i] = a.b[i] > b.b[i] ? a.b[i] : b.b[i];)
  return h;
}

// Floor carry of a 10-column accumulator into a reduced element.  Two
// interleaved chains (0..4 and 4..9) for ILP, then the 2^255 = 19 wrap.
OURO_FI fe fe_carry64(uint64_t t[10]) {
  uint64_t c;
#define OURO_CARRY(i, j)          \
  c = t[i] >> limb_bits(i);       \
  t[j] += c;                      \
  t[i] &= limb_mask(i);
  OURO_CARRY(0, 1)
  OURO_CARRY(4, 5)
  OURO_CARRY(1, 2)
  OURO_CARRY(5, 6)
  OURO_CARRY(2, 3)
  OURO_CARRY(6, 7)
  OURO_CARRY(3, 4)
  OURO_CARRY(7, 8)
  OURO_CARRY(4, 5)
  OURO_CARRY(8, 9)
  c = t[9] >> 25;
  t[9] &= limb_mask(9);
  t[0] += c * 19;
  OURO_CARRY(0, 1)
#undef OURO_CARRY
  fe h;
#pragma unroll
  for (int i = 0; i < 10; i++) {
    h.v[i] = (uint32_t)t[i];
#if defined(__HIP_DEVICE_COMPILE__)
    // hide the limb ranges: with them known, LLVM narrows the next multiply's
    // 64-bit MACs into 32-bit pieces and triples its instruction count
    asm("" : "+v"(h.v[i]));
#endif
  }
  return h;
}

// Cheap 32-bit re-normalisation of an element whose limbs grew through
// additions (one sequential pass; limb 0 may keep a small excess).
OURO_FI fe fe_carry(const fe& f) {
  fe h;
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 10; i++) {
    const uint32_t t = f.v[i] + c;
    c = t >> limb_bits(i);
    h.v[i] = t & limb_mask(i);
  }
  h.v[0] += 19 * c;
  OURO_TRK({
    uint64_t cb = 0;
    for (int i = 0; i < 10; i++) {
      const uint64_t t = f.b[i] + cb;
      trk_check(t < (1ull << 32));
      cb = t >> limb_bits(i);
      h.b[i] = t < limb_mask(i) ? t : limb_mask(i);
    }
    h.b[0] += 19 * cb;
  })
  return h;
}

// ---- column-scan products ---------------------------------------------------
// The carry out of column k is the FIRST addend of column k + 1's chain of
// multiply-adds (v_mad_u64_u32 adds a 64-bit value for free), so a product
// needs one shift and one mask per column instead of the separate 64-bit
// carry additions of fe_carry64.  The accumulator is made opaque after each
// multiply-add: LLVM would otherwise reassociate the column sum and add the
// carry last.  Squarings scan the ten columns in one chain; multiplies in two
// independent chains (columns 0..4 and 5..9, whose dependent multiply-adds the
// scheduler interleaves), joined by carrying column 4 into limb 5.  Either way
// column 9's carry wraps into limb 0 (x 19) and limb 0 carries into limb 1.
// tools/microbench/fe_cs.hip (profiles/r02c/fe_cs.json): squaring 344 -> 368 G/s,
// multiply 239 -> 245 G/s on MI355X, canonical outputs identical.
#ifndef OURO_FE_SCAN
#define OURO_FE_SCAN 1
#endif
// 2 v: v_add_u32 v, v on the device.  LLVM writes 2v / 4v as v_lshlrev_b32,
// which issues at 3.46 SIMD cycles per wave-instruction at two waves per SIMD
// against 2.52 for v_add_u32 (profiles/r04/valu_costs.json); non-volatile asm,
// so equal inputs still CSE.  OURO_ADD_SCALE=0: the shifts (A/B).
#ifndef OURO_ADD_SCALE
#define OURO_ADD_SCALE 1
#endif
OURO_FI uint32_t u32_x2(uint32_t v) {
#if defined(__HIP_DEVICE_COMPILE__) && OURO_ADD_SCALE
  uint32_t r;
  asm("v_add_u32 %0, %1, %1" : "=v"(r) : "v"(v));
  return r;
#else
  return 2u * v;
#endif
}
// OURO_MAD_BARRIER=0 (A/B only): no barrier; LLVM then adds each column's
// carry last and drops most s_nop (profiles/r06p)
#ifndef OURO_MAD_BARRIER
#define OURO_MAD_BARRIER 1
#endif
OURO_FI uint64_t mad_acc(uint32_t a, uint32_t b, uint64_t c) {
  uint64_t r = (uint64_t)a * b + c;
#if defined(__HIP_DEVICE_COMPILE__) && OURO_MAD_BARRIER
  asm("" : "+v"(r));
#endif
  return r;
}
// limbs of a scanned product, carry c9 out of column 9 still to wrap
OURO_FI fe scan_finish(uint32_t h[10], uint64_t c9) {
  const uint64_t t = (uint64_t)h[0] + 19ull * c9;
  h[0] = (uint32_t)t & limb_mask(0);
  h[1] += (uint32_t)(t >> 26);
  fe r;
#pragma unroll
  for (int i = 0; i < 10; i++) {
    r.v[i] = h[i];
#if defined(__HIP_DEVICE_COMPILE__)
    asm("" : "+v"(r.v[i]));  // hide the limb ranges (see fe_carry64)
#endif
  }
  return r;
}
#if defined(OURO_TRACK_BOUNDS)
// bounds of a scanned product from its column bounds T: chains starting at
// columns starts[0] = 0 < starts[1] < ... scanned with the carry as first
// addend, each chain's carry-out joined into the next chain's first limb,
// then the wrap of column 9's carry
inline void trk_scan(fe& h, const unsigned __int128 T[10], int nchains) {
  const int starts3[3] = {0, 4, 7}, starts2[2] = {0, 5}, starts1[1] = {0};
  const int* st = nchains == 3 ? starts3 : (nchains == 2 ? starts2 : starts1);
  const unsigned __int128 lim = (unsigned __int128)1 << 64;
  unsigned __int128 b[10], cout[3] = {0, 0, 0};
  for (int c = 0; c < nchains; c++) {
    const int end = c + 1 < nchains ? st[c + 1] : 10;
    unsigned __int128 carry = 0;
    for (int k = st[c]; k < end; k++) {
      const unsigned __int128 t = T[k] + carry;
      trk_check(t < lim);
      b[k] = t > limb_mask(k) ? limb_mask(k) : t;
      carry = t >> limb_bits(k);
    }
    cout[c] = carry;
  }
  for (int c = 0; c + 1 < nchains; c++) {  // join into the next chain's first limb
    const int k = st[c + 1];
    const unsigned __int128 t = b[k] + cout[c];
    trk_check(t < lim);
    b[k] = t > limb_mask(k) ? limb_mask(k) : t;
    b[k + 1] += t >> limb_bits(k);
  }
  const unsigned __int128 t0 = b[0] + 19 * cout[nchains - 1];
  trk_check(t0 < lim);
  b[0] = t0 > limb_mask(0) ? limb_mask(0) : t0;
  b[1] += t0 >> 26;
  for (int i = 0; i < 10; i++) {
    trk_check(b[i] < ((unsigned __int128)1 << 32));
    h.b[i] = (uint64_t)b[i];
  }
}
#endif

// h = f * g.  Column k collects f_i g_j with i + j = k (mod 10); odd*odd
// terms carry a factor 2 (2^ceil(25.5 i) 2^ceil(25.5 j) = 2 * 2^ceil(25.5 (i+j)))
// and wrapped terms a factor 19 (2^255 = 19), applied to g.  Needs
// 19 g_j < 2^32: g is the operand with the smaller bound.
OURO_FI fe fe_mul_scan(const fe& f, const fe& g) {
  uint32_t g19[10], f2[10];
#pragma unroll
  for (int i = 0; i < 10; i++) {
    g19[i] = 19u * g.v[i];
    f2[i] = (i & 1) ? u32_x2(f.v[i]) : f.v[i];
  }
  uint32_t h[10];
  uint64_t cA = 0, cB = 0;
#pragma unroll
  for (int s = 0; s < 5; s++) {
    uint64_t tA = cA, tB = cB;
#pragma unroll
    for (int i = 0; i < 10; i++) {
#pragma unroll
      for (int half = 0; half < 2; half++) {
        const int k = s + 5 * half;
        const int j = (k - i + 10) % 10;
        const uint32_t a = ((i & 1) && (j & 1)) ? f2[i] : f.v[i];
        const uint32_t b = (i + j >= 10) ? g19[j] : g.v[j];
        if (half) tB = mad_acc(a, b, tB);
        else tA = mad_acc(a, b, tA);
      }
    }
    h[s] = (uint32_t)tA & limb_mask(s);
    cA = tA >> limb_bits(s);
    h[s + 5] = (uint32_t)tB & limb_mask(s + 5);
    cB = tB >> limb_bits(s + 5);
  }
  const uint64_t t5 = (uint64_t)h[5] + cA;
  h[5] = (uint32_t)t5 & limb_mask(5);
  h[6] += (uint32_t)(t5 >> 25);
  return scan_finish(h, cB);
}

// the row-order form (A/B: OURO_FE_SCAN=0)
OURO_FI fe fe_mul_rows(const fe& f, const fe& g) {
  OURO_COUNT_MUL();
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
  fe h = fe_carry64(t);
  OURO_TRK({
    unsigned __int128 T[10] = {0};
    for (int i = 0; i < 10; i++) {
      if (i & 1) trk_check(2 * f.b[i] < (1ull << 32));
      if (i >= 1) trk_check(19 * g.b[i] < (1ull << 32));
      for (int j = 0; j < 10; j++) {
        const int k = i + j;
        unsigned __int128 x = (unsigned __int128)f.b[i] * g.b[j];
        if ((i & 1) && (j & 1)) x *= 2;
        if (k >= 10) x *= 19;
        T[k % 10] += x;
      }
    }
    trk_carry(h, T, (unsigned __int128)1 << 64);
  })
  return h;
}

// three chains (columns 0..3, 4..6, 7..9): a chain's dependent multiply-adds
// are two instructions apart, which the MI355X issues without the s_nop the
// two-chain form needs between each pair
OURO_FI fe fe_mul_scan3(const fe& f, const fe& g) {
  uint32_t g19[10], f2[10];
#pragma unroll
  for (int i = 0; i < 10; i++) {
    g19[i] = 19u * g.v[i];
    f2[i] = (i & 1) ? 2u * f.v[i] : f.v[i];
  }
  constexpr int kStart[3] = {0, 4, 7}, kLen[3] = {4, 3, 3};
  uint32_t h[10];
  uint64_t c[3] = {0, 0, 0};
#pragma unroll
  for (int s = 0; s < 4; s++) {
    uint64_t t[3] = {c[0], c[1], c[2]};
#pragma unroll
    for (int i = 0; i < 10; i++) {
#pragma unroll
      for (int ch = 0; ch < 3; ch++) {
        if (s >= kLen[ch]) continue;
        const int k = kStart[ch] + s;
        const int j = (k - i + 10) % 10;
        const uint32_t a = ((i & 1) && (j & 1)) ? f2[i] : f.v[i];
        const uint32_t b = (i + j >= 10) ? g19[j] : g.v[j];
        t[ch] = mad_acc(a, b, t[ch]);
      }
    }
#pragma unroll
    for (int ch = 0; ch < 3; ch++) {
      if (s >= kLen[ch]) continue;
      const int k = kStart[ch] + s;
      h[k] = (uint32_t)t[ch] & limb_mask(k);
      c[ch] = t[ch] >> limb_bits(k);
    }
  }
  // joins: column 3's carry into limb 4, column 6's into limb 7
  const uint64_t t4 = (uint64_t)h[4] + c[0];
  h[4] = (uint32_t)t4 & limb_mask(4);
  h[5] += (uint32_t)(t4 >> 26);
  const uint64_t t7 = (uint64_t)h[7] + c[1];
  h[7] = (uint32_t)t7 & limb_mask(7);
  h[8] += (uint32_t)(t7 >> 25);
  return scan_finish(h, c[2]);
}
#ifndef OURO_MUL_X2
#define OURO_MUL_X2 0  // 1: paired products, fewer s_nop but spills: no gain (profiles/r02c/ab_mul_x2.json)
#endif
#ifndef OURO_MUL_CHAINS
#define OURO_MUL_CHAINS 2  // 3: profiles/r02c/ab_mul_chains.json, 2.0 % slower
#endif

OURO_FI fe fe_mul(const fe& f, const fe& g) {
#if OURO_FE_SCAN
  OURO_COUNT_MUL();
  fe h = OURO_MUL_CHAINS == 3 ? fe_mul_scan3(f, g) : fe_mul_scan(f, g);
  OURO_TRK({
    unsigned __int128 T[10] = {0};
    for (int i = 0; i < 10; i++) {
      if (i & 1) trk_check(2 * f.b[i] < (1ull << 32));
      if (i >= 1) trk_check(19 * g.b[i] < (1ull << 32));
      for (int j = 0; j < 10; j++) {
        const int k = i + j;
        unsigned __int128 x = (unsigned __int128)f.b[i] * g.b[j];
        if ((i & 1) && (j & 1)) x *= 2;
        if (k >= 10) x *= 19;
        T[k % 10] += x;
      }
    }
    trk_scan(h, T, OURO_MUL_CHAINS);
  })
  return h;
#else
  return fe_mul_rows(f, g);
#endif
}

// Two independent products with their four scan chains interleaved (a
// chain's dependent multiply-adds then sit four instructions apart, the
// distance the MI355X needs between a 64-bit multiply-add result and its use
// without s_nop); the group formulas pair their independent products.
OURO_FI void fe_mul_x2(fe& h1, fe& h2, const fe& f1, const fe& g1, const fe& f2, const fe& g2) {
#if OURO_FE_SCAN && OURO_MUL_X2
  const fe* F[2] = {&f1, &f2};
  const fe* G[2] = {&g1, &g2};
  uint32_t g19[2][10], fd[2][10];
#pragma unroll
  for (int p = 0; p < 2; p++)
#pragma unroll
    for (int i = 0; i < 10; i++) {
      g19[p][i] = 19u * G[p]->v[i];
      fd[p][i] = (i & 1) ? 2u * F[p]->v[i] : F[p]->v[i];
    }
  uint32_t h[2][10];
  uint64_t c[2][2] = {{0, 0}, {0, 0}};
#pragma unroll
  for (int s = 0; s < 5; s++) {
    uint64_t t[2][2] = {{c[0][0], c[0][1]}, {c[1][0], c[1][1]}};
#pragma unroll
    for (int i = 0; i < 10; i++) {
#pragma unroll
      for (int half = 0; half < 2; half++) {
#pragma unroll
        for (int p = 0; p < 2; p++) {
          const int k = s + 5 * half;
          const int j = (k - i + 10) % 10;
          const uint32_t a = ((i & 1) && (j & 1)) ? fd[p][i] : F[p]->v[i];
          const uint32_t b = (i + j >= 10) ? g19[p][j] : G[p]->v[j];
          t[p][half] = mad_acc(a, b, t[p][half]);
        }
      }
    }
#pragma unroll
    for (int p = 0; p < 2; p++) {
      h[p][s] = (uint32_t)t[p][0] & limb_mask(s);
      c[p][0] = t[p][0] >> limb_bits(s);
      h[p][s + 5] = (uint32_t)t[p][1] & limb_mask(s + 5);
      c[p][1] = t[p][1] >> limb_bits(s + 5);
    }
  }
  fe r[2];
#pragma unroll
  for (int p = 0; p < 2; p++) {
    const uint64_t t5 = (uint64_t)h[p][5] + c[p][0];
    h[p][5] = (uint32_t)t5 & limb_mask(5);
    h[p][6] += (uint32_t)(t5 >> 25);
    r[p] = scan_finish(h[p], c[p][1]);
  }
  h1 = r[0];
  h2 = r[1];
  OURO_TRK({
    fe t1 = fe_mul(f1, g1), t2 = fe_mul(f2, g2);  // bounds (and counts) of the pair
    for (int i = 0; i < 10; i++) {
      h1.b[i] = t1.b[i];
      h2.b[i] = t2.b[i];
    }
  })
#else
  h1 = fe_mul(f1, g1);
  h2 = fe_mul(f2, g2);
#endif
}

// f * g with the factor 19 applied per column after accumulation: no bound on
// 19 g, for the few products whose operands are both wide (slower: ~9 % per
// multiply on MI355X, profiles/r01c/fe_mul_variants.json "fe10d_mul").
OURO_FI fe fe_mul_wide(const fe& f, const fe& g) {
  OURO_COUNT_MUL();
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
  fe h = fe_carry64(lo);
  OURO_TRK({
    unsigned __int128 T[10] = {0};
    for (int i = 0; i < 10; i++) {
      if (i & 1) trk_check(2 * f.b[i] < (1ull << 32));
      for (int j = 0; j < 10; j++) {
        const int k = i + j;
        unsigned __int128 x = (unsigned __int128)f.b[i] * g.b[j];
        if ((i & 1) && (j & 1)) x *= 2;
        if (k >= 10) x *= 19;
        T[k % 10] += x;
      }
    }
    trk_carry(h, T, (unsigned __int128)1 << 64);
  })
  return h;
}

// Column sums of f^2 (before carry); shared by fe_sq and fe_sq2.
OURO_FI void fe_sq_cols(uint64_t t[10], const fe& f) {
  OURO_COUNT_SQ();
  uint32_t f2[10], f4[10], f19[10];
#pragma unroll
  for (int i = 0; i < 10; i++) {
    f2[i] = 2u * f.v[i];
    f4[i] = 4u * f.v[i];
    f19[i] = 19u * f.v[i];
  }
#pragma unroll
  for (int k = 0; k < 10; k++) t[k] = 0;
#pragma unroll
  for (int i = 0; i < 10; i++) {
    // diagonal: f_i^2 * (2 if i odd) * (19 if 2i >= 10)
    {
      const int k = 2 * i;
      const uint32_t a = (i & 1) ? f2[i] : f.v[i];
      const uint32_t b = (k >= 10) ? f19[i] : f.v[i];
      t[k >= 10 ? k - 10 : k] += (uint64_t)a * b;
    }
#pragma unroll
    for (int j = i + 1; j < 10; j++) {
      // cross terms counted twice: 2 f_i f_j * (2 if both odd) * (19 if wrap)
      const int k = i + j;
      const uint32_t a = ((i & 1) && (j & 1)) ? f4[i] : f2[i];
      const uint32_t b = (k >= 10) ? f19[j] : f.v[j];
      t[k >= 10 ? k - 10 : k] += (uint64_t)a * b;
    }
  }
}

#if defined(OURO_TRACK_BOUNDS)
inline void trk_sq(fe& h, const fe& f, unsigned scale) {
  unsigned __int128 T[10] = {0};
  for (int i = 0; i < 10; i++) {
    trk_check(((i & 1) ? 4 : 2) * f.b[i] < (1ull << 32));
    if (i >= 5) trk_check(19 * f.b[i] < (1ull << 32));
    for (int j = 0; j < 10; j++) {
      const int k = i + j;
      unsigned __int128 x = (unsigned __int128)f.b[i] * f.b[j];
      if ((i & 1) && (j & 1)) x *= 2;
      if (k >= 10) x *= 19;
      T[k % 10] += x * scale;
    }
  }
  trk_carry(h, T, (unsigned __int128)1 << 64);
}
#endif

// f^2 (scale 1) or 2 f^2 (scale 2) scanned in one chain: column k's terms
// are the diagonal f_i^2 (x2 if i odd) and the cross terms 2 f_i f_j (x2 if
// both odd), x19 when wrapped; scale 2 doubles the left operands
template <int kScale>
OURO_FI fe fe_sq_scan(const fe& f) {
  uint32_t fs[10], f2s[10], f4s[10], f19[10];
#pragma unroll
  for (int i = 0; i < 10; i++) {
    fs[i] = kScale == 1 ? f.v[i] : u32_x2(f.v[i]);
    f2s[i] = u32_x2(fs[i]);
    f4s[i] = u32_x2(f2s[i]);
    f19[i] = 19u * f.v[i];
  }
  uint32_t h[10];
  uint64_t c = 0;
#pragma unroll
  for (int k = 0; k < 10; k++) {
    uint64_t t = c;
#pragma unroll
    for (int i = 0; i < 10; i++) {
#pragma unroll
      for (int j = i; j < 10; j++) {
        if ((i + j) % 10 != k) continue;
        uint32_t a, b;
        if (i == j) {
          a = (i & 1) ? f2s[i] : fs[i];
          b = (2 * i >= 10) ? f19[i] : f.v[i];
        } else {
          a = ((i & 1) && (j & 1)) ? f4s[i] : f2s[i];
          b = (i + j >= 10) ? f19[j] : f.v[j];
        }
        t = mad_acc(a, b, t);
      }
    }
    h[k] = (uint32_t)t & limb_mask(k);
    c = t >> limb_bits(k);
  }
  return scan_finish(h, c);
}
// The same squaring in two interleaved chains (columns 0..4 and 5..9, joined
// like fe_mul_scan's): a chain's dependent multiply-adds then alternate with
// the other chain's instead of waiting a cycle each (the one-chain form needs
// an s_nop between consecutive v_mad_u64_u32 of its chain).
#ifndef OURO_SQ_CHAINS
#define OURO_SQ_CHAINS 1
#endif
template <int kScale>
OURO_FI fe fe_sq_scan2(const fe& f) {
  uint32_t fs[10], f2s[10], f4s[10], f19[10];
#pragma unroll
  for (int i = 0; i < 10; i++) {
    fs[i] = kScale * f.v[i];
    f2s[i] = 2u * kScale * f.v[i];
    f4s[i] = 4u * kScale * f.v[i];
    f19[i] = 19u * f.v[i];
  }
  uint32_t h[10];
  uint64_t cA = 0, cB = 0;
#pragma unroll
  for (int s = 0; s < 5; s++) {
    uint64_t t[2] = {cA, cB};
    // the terms of column s (chain 0) and s + 5 (chain 1), alternated
    int ti[2][6], tj[2][6], nt[2] = {0, 0};
#pragma unroll
    for (int half = 0; half < 2; half++) {
      const int k = s + 5 * half;
#pragma unroll
      for (int i = 0; i < 10; i++)
#pragma unroll
        for (int j = i; j < 10; j++)
          if ((i + j) % 10 == k) {
            ti[half][nt[half]] = i;
            tj[half][nt[half]] = j;
            nt[half]++;
          }
    }
#pragma unroll
    for (int q = 0; q < 6; q++) {
#pragma unroll
      for (int half = 0; half < 2; half++) {
        if (q >= nt[half]) continue;
        const int i = ti[half][q], j = tj[half][q];
        uint32_t a, b;
        if (i == j) {
          a = (i & 1) ? f2s[i] : fs[i];
          b = (2 * i >= 10) ? f19[i] : f.v[i];
        } else {
          a = ((i & 1) && (j & 1)) ? f4s[i] : f2s[i];
          b = (i + j >= 10) ? f19[j] : f.v[j];
        }
        t[half] = mad_acc(a, b, t[half]);
      }
    }
    h[s] = (uint32_t)t[0] & limb_mask(s);
    cA = t[0] >> limb_bits(s);
    h[s + 5] = (uint32_t)t[1] & limb_mask(s + 5);
    cB = t[1] >> limb_bits(s + 5);
  }
  const uint64_t t5 = (uint64_t)h[5] + cA;
  h[5] = (uint32_t)t5 & limb_mask(5);
  h[6] += (uint32_t)(t5 >> 25);
  return scan_finish(h, cB);
}

#if defined(OURO_TRACK_BOUNDS)
inline void trk_sq_scan(fe& h, const fe& f, unsigned scale, int nchains = 1) {
  unsigned __int128 T[10] = {0};
  for (int i = 0; i < 10; i++) {
    trk_check(((i & 1) ? 4 : 2) * scale * f.b[i] < (1ull << 32));
    if (i >= 5) trk_check(19 * f.b[i] < (1ull << 32));
    for (int j = 0; j < 10; j++) {
      const int k = i + j;
      unsigned __int128 x = (unsigned __int128)f.b[i] * f.b[j];
      if ((i & 1) && (j & 1)) x *= 2;
      if (k >= 10) x *= 19;
      T[k % 10] += x * scale;
    }
  }
  trk_scan(h, T, nchains);
}
#endif

OURO_FI fe fe_sq(const fe& f) {
#if OURO_FE_SCAN
  OURO_COUNT_SQ();
  fe h = OURO_SQ_CHAINS == 2 ? fe_sq_scan2<1>(f) : fe_sq_scan<1>(f);
  OURO_TRK(trk_sq_scan(h, f, 1, OURO_SQ_CHAINS));
  return h;
#else
  uint64_t t[10];
  fe_sq_cols(t, f);
  fe h = fe_carry64(t);
  OURO_TRK(trk_sq(h, f, 1));
  return h;
#endif
}

// Two independent squarings scanned in lockstep: one chain each, their
// multiply-adds alternating, so neither waits on its own previous result
// (the paired exponentiations below).
OURO_FI void fe_sq_x2(fe& f, fe& g) {
#if OURO_FE_SCAN
  OURO_COUNT_SQ();
  OURO_COUNT_SQ();
  const fe* in[2] = {&f, &g};
  uint32_t fs[2][10], f2s[2][10], f4s[2][10], f19[2][10];
#pragma unroll
  for (int e = 0; e < 2; e++)
#pragma unroll
    for (int i = 0; i < 10; i++) {
      fs[e][i] = in[e]->v[i];
      f2s[e][i] = 2u * in[e]->v[i];
      f4s[e][i] = 4u * in[e]->v[i];
      f19[e][i] = 19u * in[e]->v[i];
    }
  uint32_t h[2][10];
  uint64_t c[2] = {0, 0};
#pragma unroll
  for (int k = 0; k < 10; k++) {
    uint64_t t[2] = {c[0], c[1]};
#pragma unroll
    for (int i = 0; i < 10; i++) {
#pragma unroll
      for (int j = i; j < 10; j++) {
        if ((i + j) % 10 != k) continue;
#pragma unroll
        for (int e = 0; e < 2; e++) {
          uint32_t a, b;
          if (i == j) {
            a = (i & 1) ? f2s[e][i] : fs[e][i];
            b = (2 * i >= 10) ? f19[e][i] : fs[e][i];
          } else {
            a = ((i & 1) && (j & 1)) ? f4s[e][i] : f2s[e][i];
            b = (i + j >= 10) ? f19[e][j] : fs[e][j];
          }
          t[e] = mad_acc(a, b, t[e]);
        }
      }
    }
#pragma unroll
    for (int e = 0; e < 2; e++) {
      h[e][k] = (uint32_t)t[e] & limb_mask(k);
      c[e] = t[e] >> limb_bits(k);
    }
  }
  fe rf = scan_finish(h[0], c[0]), rg = scan_finish(h[1], c[1]);
  OURO_TRK(trk_sq_scan(rf, f, 1); trk_sq_scan(rg, g, 1);)
  f = rf;
  g = rg;
#else
  f = fe_sq(f);
  g = fe_sq(g);
#endif
}

// 2 f^2
OURO_FI fe fe_sq2(const fe& f) {
#if OURO_FE_SCAN
  OURO_COUNT_SQ();
  fe h = OURO_SQ_CHAINS == 2 ? fe_sq_scan2<2>(f) : fe_sq_scan<2>(f);
  OURO_TRK(trk_sq_scan(h, f, 2, OURO_SQ_CHAINS));
  return h;
#else
  uint64_t t[10];
  fe_sq_cols(t, f);
#pragma unroll
  for (int k = 0; k < 10; k++) t[k] += t[k];
  fe h = fe_carry64(t);
  OURO_TRK(trk_sq(h, f, 2));
  return h;
#endif
}

// ---- independent products in lockstep (round 4) ------------------------------
// N independent products, each scanned in ONE chain (column k's carry the
// first addend of column k + 1), their multiply-adds interleaved so a chain's
// dependent v_mad_u64_u32 sit N instructions apart.  A MAD's result is ready
// ~14 cycles after it issues while a wave issues one every ~7
// (tools/microbench/valu_costs.hip, profiles/r04/valu_costs.json), so at two
// waves per SIMD a chain whose MADs depend back to back stalls; three or four
// chains in lockstep do not.  The doubling built from these (ge25519.h
// ge_dbl_lockstep) runs 25.9 vs 29.3 ps per chip-wide doubling
// (tools/microbench/occupancy.hip, profiles/r04/occupancy_lockstep.json);
// the same instruction count.
template <int N>
OURO_FI void fe_mul_xn(fe* h, const fe* f, const fe* g) {
  uint32_t g19[N][10], f2[N][10];
#pragma unroll
  for (int e = 0; e < N; e++)
#pragma unroll
    for (int i = 0; i < 10; i++) {
      g19[e][i] = 19u * g[e].v[i];
      f2[e][i] = (i & 1) ? u32_x2(f[e].v[i]) : f[e].v[i];
    }
  uint32_t hv[N][10];
  uint64_t c[N];
#pragma unroll
  for (int e = 0; e < N; e++) c[e] = 0;
#pragma unroll
  for (int k = 0; k < 10; k++) {
    uint64_t t[N];
#pragma unroll
    for (int e = 0; e < N; e++) t[e] = c[e];
#pragma unroll
    for (int i = 0; i < 10; i++) {
      const int j = (k - i + 10) % 10;
#pragma unroll
      for (int e = 0; e < N; e++) {
        const uint32_t a = ((i & 1) && (j & 1)) ? f2[e][i] : f[e].v[i];
        const uint32_t b = (i + j >= 10) ? g19[e][j] : g[e].v[j];
        t[e] = mad_acc(a, b, t[e]);
      }
    }
#pragma unroll
    for (int e = 0; e < N; e++) {
      hv[e][k] = (uint32_t)t[e] & limb_mask(k);
      c[e] = t[e] >> limb_bits(k);
    }
  }
#pragma unroll
  for (int e = 0; e < N; e++) {
    OURO_COUNT_MUL();
    h[e] = scan_finish(hv[e], c[e]);
    OURO_TRK({
      unsigned __int128 T[10] = {0};
      for (int i = 0; i < 10; i++) {
        if (i & 1) trk_check(2 * f[e].b[i] < (1ull << 32));
        if (i >= 1) trk_check(19 * g[e].b[i] < (1ull << 32));
        for (int j = 0; j < 10; j++) {
          const int k = i + j;
          unsigned __int128 x = (unsigned __int128)f[e].b[i] * g[e].b[j];
          if ((i & 1) && (j & 1)) x *= 2;
          if (k >= 10) x *= 19;
          T[k % 10] += x;
        }
      }
      trk_scan(h[e], T, 1);
    })
  }
}
// N independent squarings in lockstep; element e is scaled by kScale[e]
// (1: f^2, 2: 2 f^2), one chain each as fe_sq_scan.  kComp (device only):
// the elements whose bit is set are returned COMPLEMENTED, limb k as
// mask_k - h_k -- the same single instruction per limb as the mask
// ((~t) & mask), limb 1 with its carry subtracted instead of added -- so a
// caller's Y - h becomes Y + (mask - h) + (2p - mask): one three-input add per
// limb instead of an add and a subtract (ge25519.h ge_dbl_lockstep).
template <int N, unsigned kComp = 0>
OURO_FI void fe_sq_xn(fe* h, const fe* f, const int (&scale)[N]) {
  uint32_t fs[N][10], f2s[N][10], f4s[N][10], f19[N][10];
#pragma unroll
  for (int e = 0; e < N; e++)
#pragma unroll
    for (int i = 0; i < 10; i++) {
      fs[e][i] = scale[e] == 1 ? f[e].v[i] : u32_x2(f[e].v[i]);
      f2s[e][i] = u32_x2(fs[e][i]);
      f4s[e][i] = u32_x2(f2s[e][i]);
      f19[e][i] = 19u * f[e].v[i];
    }
  uint32_t hv[N][10];
  uint64_t c[N];
#pragma unroll
  for (int e = 0; e < N; e++) c[e] = 0;
#pragma unroll
  for (int k = 0; k < 10; k++) {
    uint64_t t[N];
#pragma unroll
    for (int e = 0; e < N; e++) t[e] = c[e];
#pragma unroll
    for (int i = 0; i < 10; i++)
#pragma unroll
      for (int j = i; j < 10; j++) {
        if ((i + j) % 10 != k) continue;
#pragma unroll
        for (int e = 0; e < N; e++) {
          uint32_t a, b;
          if (i == j) {
            a = (i & 1) ? f2s[e][i] : fs[e][i];
            b = (2 * i >= 10) ? f19[e][i] : f[e].v[i];
          } else {
            a = ((i & 1) && (j & 1)) ? f4s[e][i] : f2s[e][i];
            b = (i + j >= 10) ? f19[e][j] : f[e].v[j];
          }
          t[e] = mad_acc(a, b, t[e]);
        }
      }
#pragma unroll
    for (int e = 0; e < N; e++) {
      // (limb 0 stays plain: scan_finish adds the wrap to it first)
      const bool comp = ((kComp >> e) & 1u) && k > 0;
      hv[e][k] = comp ? ~(uint32_t)t[e] & limb_mask(k) : (uint32_t)t[e] & limb_mask(k);
      c[e] = t[e] >> limb_bits(k);
    }
  }
#pragma unroll
  for (int e = 0; e < N; e++) {
    OURO_COUNT_SQ();
    if ((kComp >> e) & 1u) {
      // scan_finish with the complement: limb 0 = mask_0 - (t0 & mask_0),
      // limb 1 = (mask_1 - h_1) - (t0 >> 26)
      const uint64_t t0 = (uint64_t)hv[e][0] + 19ull * c[e];
      hv[e][0] = ~(uint32_t)t0 & limb_mask(0);
      hv[e][1] -= (uint32_t)(t0 >> 26);
#pragma unroll
      for (int i = 0; i < 10; i++) {
        h[e].v[i] = hv[e][i];
#if defined(__HIP_DEVICE_COMPILE__)
        asm("" : "+v"(h[e].v[i]));  // hide the limb ranges (see fe_carry64)
#endif
      }
    } else {
      h[e] = scan_finish(hv[e], c[e]);
    }
    OURO_TRK(trk_sq_scan(h[e], f[e], (unsigned)scale[e], 1));
  }
}

// ---- encoding -------------------------------------------------------------
// 256-bit little-endian words -> fe (bit 255 ignored, like fe25519_frombytes)
OURO_FI fe fe_from_words(const uint32_t w[8]) {
  fe h;
  h.v[0] = w[0] & 0x3ffffff;
  h.v[1] = ((w[0] >> 26) | (w[1] << 6)) & 0x1ffffff;
  h.v[2] = ((w[1] >> 19) | (w[2] << 13)) & 0x3ffffff;
  h.v[3] = ((w[2] >> 13) | (w[3] << 19)) & 0x1ffffff;
  h.v[4] = (w[3] >> 6) & 0x3ffffff;
  h.v[5] = w[4] & 0x1ffffff;
  h.v[6] = ((w[4] >> 25) | (w[5] << 7)) & 0x3ffffff;
  h.v[7] = ((w[5] >> 19) | (w[6] << 13)) & 0x1ffffff;
  h.v[8] = ((w[6] >> 12) | (w[7] << 20)) & 0x3ffffff;
  h.v[9] = (w[7] >> 6) & 0x1ffffff;
  OURO_TRK(for (int i = 0; i < 10; i++) h.b[i] = limb_mask(i);)
  return h;
}

// canonical little-endian encoding of f mod p as 8 words (limbs < 2^31)
OURO_FI void fe_to_words(uint32_t w[8], const fe& f) {
  OURO_TRK(for (int i = 0; i < 10; i++) trk_check(f.b[i] < (1ull << 31));)
  uint32_t h[10];
#pragma unroll
  for (int i = 0; i < 10; i++) h[i] = f.v[i];
  // three floor-carry passes leave limbs 1..9 within their masks and the
  // value below 2^255 + 2^26
#pragma unroll
  for (int pass = 0; pass < 3; pass++) {
    uint32_t c;
#pragma unroll
    for (int i = 0; i < 9; i++) {
      c = h[i] >> limb_bits(i);
      h[i] &= limb_mask(i);
      h[i + 1] += c;
    }
    c = h[9] >> 25;
    h[9] &= limb_mask(9);
    h[0] += 19 * c;
  }
  // subtract p if value >= p: q = (value + 19) >> 255 (exact carry chain)
  uint32_t q = (h[0] + 19) >> 26;
#pragma unroll
  for (int i = 1; i < 10; i++) q = (h[i] + q) >> limb_bits(i);
  h[0] += 19 * q;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    const uint32_t c = h[i] >> limb_bits(i);
    h[i] &= limb_mask(i);
    h[i + 1] += c;
  }
  h[9] &= limb_mask(9);
  w[0] = h[0] | (h[1] << 26);
  w[1] = (h[1] >> 6) | (h[2] << 19);
  w[2] = (h[2] >> 13) | (h[3] << 13);
  w[3] = (h[3] >> 19) | (h[4] << 6);
  w[4] = h[5] | (h[6] << 25);
  w[5] = (h[6] >> 7) | (h[7] << 19);
  w[6] = (h[7] >> 13) | (h[8] << 12);
  w[7] = (h[8] >> 20) | (h[9] << 6);
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
#ifndef OURO_SQN_UNROLL
#define OURO_SQN_UNROLL 1  // A/B switch: squarings per loop trip in the chains
#endif
// The squarings of the exponentiation chains in one scan chain (1) or two
// interleaved ones (2, fe_sq_scan2): a chain's squarings depend on each
// other, so the one-chain form issues dependent multiply-adds back to back
// (6.9 SIMD cycles each at 2 waves against 4.4 for two chains,
// profiles/r04/valu_costs.json).  A/B switch for the chains only (the
// doublings' squarings are already interleaved, ge_dbl_lockstep).  Two
// since round 5: with the additions in lockstep it took the header kernel
// -1.25 / -0.55 % in two A/Bs (profiles/r05y, r05z; mixed in round 4).
#ifndef OURO_POW_SQ_CHAINS
#define OURO_POW_SQ_CHAINS 2
#endif
OURO_FI fe fe_sq_pow(const fe& f) {
  if constexpr (OURO_POW_SQ_CHAINS == 2) {
    OURO_COUNT_SQ();
    fe h = fe_sq_scan2<1>(f);
    OURO_TRK(trk_sq_scan(h, f, 1, 2));
    return h;
  } else {
    return fe_sq(f);
  }
}
OURO_FI fe fe_sqn(fe t, int n) {
#pragma unroll OURO_SQN_UNROLL
  for (int i = 0; i < n; i++) t = fe_sq_pow(t);
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

// Two independent z^(2^252 - 3) at once: the same addition chain on both,
// every squaring of the pair scanned in lockstep (fe_sq_x2), so the two
// dependency chains fill each other's wait states -- the decodes of an
// Ed25519 check (A, R), of a VRF's key and Gamma, and Gamma's decode beside
// Elligator2's root.
struct fe_pair {
  fe a, b;
};
OURO_FI void fe_sqn_x2(fe& a, fe& b, int n) {
#pragma unroll 1
  for (int i = 0; i < n; i++) fe_sq_x2(a, b);
}
OURO_NI fe_pair fe_pow22523_x2(fe za, fe zb) {
  fe a = za, b = zb;
  fe_sq_x2(a, b);                      // z^2
  fe a2 = a, b2 = b;
  fe_sqn_x2(a, b, 2);                  // z^8
  fe a9 = fe_mul(a, za), b9 = fe_mul(b, zb);
  fe a11 = fe_mul(a9, a2), b11 = fe_mul(b9, b2);
  a = a11;
  b = b11;
  fe_sq_x2(a, b);
  fe a5 = fe_mul(a, a9), b5 = fe_mul(b, b9);  // 2^5 - 1
  a = a5;
  b = b5;
  fe_sqn_x2(a, b, 5);
  fe a10 = fe_mul(a, a5), b10 = fe_mul(b, b5);  // 2^10 - 1
  a = a10;
  b = b10;
  fe_sqn_x2(a, b, 10);
  fe a20 = fe_mul(a, a10), b20 = fe_mul(b, b10);
  a = a20;
  b = b20;
  fe_sqn_x2(a, b, 20);
  a = fe_mul(a, a20);                  // 2^40 - 1
  b = fe_mul(b, b20);
  fe_sqn_x2(a, b, 10);
  fe a50 = fe_mul(a, a10), b50 = fe_mul(b, b10);
  a = a50;
  b = b50;
  fe_sqn_x2(a, b, 50);
  fe a100 = fe_mul(a, a50), b100 = fe_mul(b, b50);
  a = a100;
  b = b100;
  fe_sqn_x2(a, b, 100);
  a = fe_mul(a, a100);                 // 2^200 - 1
  b = fe_mul(b, b100);
  fe_sqn_x2(a, b, 50);
  a = fe_mul(a, a50);                  // 2^250 - 1
  b = fe_mul(b, b50);
  fe_sqn_x2(a, b, 2);
  return fe_pair{fe_mul(a, za), fe_mul(b, zb)};  // 2^252 - 3
}

}  // namespace ouro
