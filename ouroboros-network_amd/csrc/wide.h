// wide.h -- wave-wide field and group arithmetic for the latency mode.
//
// configs[4] (a 64-header ChainSync window) is latency-bound on its longest
// item: the [s]H half of a VRF's V = [s]H - [c]Gamma, a 252-bit variable-base
// chain after Elligator2's exponentiation.
// A lane quad (ge25519.h) splits each group operation's four products over
// four lanes, but every product still runs on one lane: ~480 instructions per
// doubling.  Here ONE WAVE runs one item and every product is spread over the
// 16 lanes of a DPP row:
//
//   field element ("fw"): lane j of a row holds limb j (signed, radix 2^16,
//   16 limbs, 2^256 = 38 mod p); the four rows of the wave hold four
//   independent elements, so a group operation's four products run at once.
//
//   product f * g: 16 steps; step i broadcasts f_i along the row
//   (row_newbcast:i) and rotates g one lane (row_ror:1; the limb that wraps
//   from lane 15 to lane 0 is multiplied by 38 there), one v_mad_i64_i32 per
//   step, then three carry rounds (shift, row_ror:1, x38 at lane 0).  ~75
//   instructions for all four rows' products.
//
//   point ("pw"): X, Y, Z, T each REPLICATED in all four rows.  A group
//   operation is two layers of four products: each row forms its own two
//   operands from the replicated coordinates (row selects), multiplies, and
//   the four rows' results are exchanged with v_permlane16_swap /
//   v_permlane32_swap (gfx950) so every row holds all four again.
//
// Limb bounds (signed): a carried element has |limb| <= 65,535 + 38*16 <
// 2^16.01.  The rotated operand g of a product passes through v_mul_i32_i24
// (x38 at lane 0, x1 elsewhere) after it wrapped, so |38 g| < 2^23, i.e. |g|
// <= 3 carried elements summed (<= 196,833 < 220,752); the broadcast operand
// f is a full 32-bit input of v_mad_i64_i32 and takes the 4-term sums.  The
// accumulator is then below 16 * 2^18.01 * 2^23 < 2^45.1, so its >> 16 fits
// an int32, and the carry rounds stay inside the i24 ranges they use.  Every
// formula below puts its narrow (<= 3-term) operand second.
//
// Device-only: every routine here is wave-collective (DPP, permlane).
#pragma once
#include "verify.h"

namespace ouro {
#if defined(__HIP_DEVICE_COMPILE__)
namespace wide {

// lane constants of one wave
struct Lanes {
  int j;          // limb index (lane & 15)
  int32_t fac;    // 38 at limb 0 (the wrap 2^256 = 38), 1 elsewhere
  bool odd, high; // row 1 or 3; row 2 or 3
  int32_t fac2;   // 38 at limbs 0 and 1 (a rotation by two lanes), 1 elsewhere
  int32_t facr;   // 38 at limbs below 4 r in row r (a rotation by 4 r lanes), 1 elsewhere
};
__device__ __forceinline__ Lanes lanes() {
  const int j = (int)(threadIdx.x & 15u);
  const int r = (int)((threadIdx.x >> 4) & 3u);
  return Lanes{j, j == 0 ? 38 : 1, (threadIdx.x & 16u) != 0, (threadIdx.x & 32u) != 0,
               j < 2 ? 38 : 1, j < 4 * r ? 38 : 1};
}

__device__ __forceinline__ int32_t s24(int32_t x) { return (x << 8) >> 8; }
template <int C>
__device__ __forceinline__ int32_t dpp(int32_t x) {
  return __builtin_amdgcn_mov_dpp(x, C, 0xf, 0xf, true);  // bound_ctrl: DPP-combinable
}
__device__ __forceinline__ int32_t ror1(int32_t x) { return dpp<0x121>(x); }  // lane j <- j-1
template <int I>
__device__ __forceinline__ int32_t bcast(int32_t x) { return dpp<0x150 + I>(x); }  // row_newbcast:I

// carry an accumulator (|acc| < 2^46) into limbs |l| < 2^16.01
#ifndef OURO_FW_CARRY2
#define OURO_FW_CARRY2 1  // A/B switch: 1 = two rounds (below), 0 = three rounds
#endif
// Two rounds: acc = a0 + a1 2^16 + a2 2^32 with a0, a1 in [0, 2^16) and
// |a2| < 2^13.1; limb j takes a0_j + a1_(j-1) + a2_(j-2) (x 38 where the
// rotation wrapped): below 2^16 + 38 (2^16 + 2^13.1) < 2^21.4, then one
// shift-and-rotate round leaves it below 2^16 + 38 * 2^5.4 < 2^16.03.  Three
// DPP reads in two dependent levels instead of three rounds in series.
__device__ __forceinline__ int32_t fw_carry2(int64_t acc, const int32_t fac, const int32_t fac2) {
  const uint32_t lo32 = (uint32_t)acc;
  const int32_t a0 = (int32_t)(lo32 & 0xffffu);
  const int32_t a1 = (int32_t)(lo32 >> 16);
  const int32_t a2 = (int32_t)(acc >> 32);
  const int32_t s = a0 + s24(dpp<0x121>(a1)) * s24(fac) + s24(dpp<0x122>(a2)) * s24(fac2);
  return (s & 0xffff) + s24(ror1(s >> 16)) * s24(fac);
}
__device__ __forceinline__ int32_t fw_carry(int64_t acc, int32_t fac) {
  int32_t lo = (int32_t)acc & 0xffff;
  int32_t hi = (int32_t)(acc >> 16);
  const int64_t t = (int64_t)ror1(hi) * fac + lo;  // lane 0: < 2^36
  lo = (int32_t)t & 0xffff;
  hi = (int32_t)(t >> 16);                         // < 2^20.6
  int32_t u = s24(ror1(hi)) * s24(fac) + lo;       // < 2^26
  lo = u & 0xffff;
  hi = u >> 16;                                    // < 2^10
  return s24(ror1(hi)) * s24(fac) + lo;
}

#ifndef OURO_FW_ACC2
#define OURO_FW_ACC2 1  // A/B switch: even and odd steps in two accumulators
#endif
template <int I>
__device__ __forceinline__ void fw_mul_steps(int64_t& acc0, int64_t& acc1, int32_t& G, int32_t f,
                                             int32_t fac) {
  if constexpr (I > 0) G = s24(ror1(G)) * s24(fac);
  const int64_t p = (int64_t)bcast<I>(f) * G;
  int64_t& acc = (OURO_FW_ACC2 && (I & 1)) ? acc1 : acc0;
  if constexpr (I == 0 || (OURO_FW_ACC2 && I == 1)) acc = p; else acc += p;
  if constexpr (I < 15) fw_mul_steps<I + 1>(acc0, acc1, G, f, fac);
}

__device__ __forceinline__ int32_t fw_carry_l(int64_t acc, const Lanes& L) {
  return OURO_FW_CARRY2 ? fw_carry2(acc, L.fac, L.fac2) : fw_carry(acc, L.fac);
}

// f * g per row (g: the narrow operand, |g| <= 196,833 per limb)
__device__ __forceinline__ int32_t fw_mul(int32_t f, int32_t g, const Lanes& L) {
  // (two independent rotation chains of eight steps, interleaved: issue-bound
  // all the same, configs[4] p50 0.2279 / 0.2302 ms, dropped)
  int64_t acc0, acc1 = 0;
  int32_t G = g;
  fw_mul_steps<0>(acc0, acc1, G, f, L.fac);
  return fw_carry_l(OURO_FW_ACC2 ? acc0 + acc1 : acc0, L);
}
__device__ __forceinline__ int32_t fw_sq(int32_t f, const Lanes& L) { return fw_mul(f, f, L); }

// the four rows' values of x, each replicated in every row
struct fw4 { int32_t r0, r1, r2, r3; };
__device__ __forceinline__ fw4 fw_gather(int32_t x) {
  // odd rows of the first operand <-> even rows of the second (per 32-lane half)
  const auto p = __builtin_amdgcn_permlane16_swap(x, x, false, false);  // [0,0,2,2] / [1,1,3,3]
  const auto q = __builtin_amdgcn_permlane32_swap(p[0], p[0], false, false);  // [0]x4 / [2]x4
  const auto r = __builtin_amdgcn_permlane32_swap(p[1], p[1], false, false);  // [1]x4 / [3]x4
  return fw4{(int32_t)q[0], (int32_t)r[0], (int32_t)q[1], (int32_t)r[1]};
}

// row r takes a_r (row bits of the lane id, so LLVM's hazard recognizer sees
// every select: a v_cndmask in inline asm followed by a DPP read of its
// result would miss the 2 wait states DPP needs)
__device__ __forceinline__ int32_t sel4(int32_t a0, int32_t a1, int32_t a2, int32_t a3,
                                        const Lanes& L) {
  const int32_t lo = L.odd ? a1 : a0, hi = L.odd ? a3 : a2;
  return L.high ? hi : lo;
}

// f * g for REPLICATED f, g (every row the same element): the sixteen steps
// split over the four rows (row r takes steps 4r..4r+3, its operands rotated
// into place by 4r lanes first), the rows' accumulators summed across rows
// with permlane swaps, one carry: ~43 instructions instead of ~62 -- for the
// exponentiation chains, whose operands are replicated.
__device__ __forceinline__ int64_t add_rows_u64(int64_t a) {
  const uint32_t lo = (uint32_t)a, hi = (uint32_t)((uint64_t)a >> 32);
  const auto l1 = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
  const auto h1 = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
  const uint64_t s = ((uint64_t)h1[0] << 32 | l1[0]) + ((uint64_t)h1[1] << 32 | l1[1]);
  const uint32_t slo = (uint32_t)s, shi = (uint32_t)(s >> 32);
  const auto l2 = __builtin_amdgcn_permlane32_swap(slo, slo, false, false);
  const auto h2 = __builtin_amdgcn_permlane32_swap(shi, shi, false, false);
  return (int64_t)(((uint64_t)h2[0] << 32 | l2[0]) + ((uint64_t)h2[1] << 32 | l2[1]));
}
// The replicated products' carry: each row's partial accumulator (four
// steps: |acc_r| < 2^43.1) goes through the first carry round by itself
// (a0 + a1 + a2 of fw_carry2, below 2^21.4), the four rows' 32-bit results
// are summed across rows (below 2^23.4), then the last shift-and-rotate
// round: limbs below 2^16 + 38 * 2^7.4 < 2^16.13 (3 of them sum below
// 220,752, the narrow operand's limit).  Two 32-bit permlane sums instead of
// two 64-bit ones before the carry.
#ifndef OURO_FW_ROWSUM32
#define OURO_FW_ROWSUM32 1  // A/B switch: 0 = 64-bit cross-row sum, then fw_carry_l
#endif
__device__ __forceinline__ int32_t add_rows_i32(int32_t x) {
  const auto p = __builtin_amdgcn_permlane16_swap(x, x, false, false);
  const int32_t s = (int32_t)p[0] + (int32_t)p[1];
  const auto q = __builtin_amdgcn_permlane32_swap(s, s, false, false);
  return (int32_t)q[0] + (int32_t)q[1];
}
__device__ __forceinline__ int32_t fw_carry_rows(int64_t acc, const Lanes& L) {
  if (!OURO_FW_ROWSUM32) return fw_carry_l(add_rows_u64(acc), L);
  const uint32_t lo32 = (uint32_t)acc;
  const int32_t a2 = (int32_t)(acc >> 32);
  const int32_t sr = (int32_t)(lo32 & 0xffffu) + s24(dpp<0x121>((int32_t)(lo32 >> 16))) * s24(L.fac) +
                     s24(dpp<0x122>(a2)) * s24(L.fac2);
  const int32_t s = add_rows_i32(sr);
  return (s & 0xffff) + s24(ror1(s >> 16)) * s24(L.fac);
}

__device__ __forceinline__ int32_t fw_mul_rep(int32_t f, int32_t g, const Lanes& L) {
  const int j = L.j;
  // f' lane k = f_(4r + k); G lane j = g_(j - 4r) (x 38 where it wrapped)
  const int32_t fr = sel4(f, dpp<0x12c>(f), dpp<0x128>(f), dpp<0x124>(f), L);  // ror 12 / 8 / 4
  const int32_t g4 = s24(dpp<0x124>(g)) * (j < 4 ? 38 : 1);
  const int32_t g8 = s24(dpp<0x128>(g)) * (j < 8 ? 38 : 1);
  const int32_t g12 = s24(dpp<0x12c>(g)) * (j < 12 ? 38 : 1);
  int32_t G = sel4(g, g4, g8, g12, L);
  int64_t acc = (int64_t)bcast<0>(fr) * G;
  G = s24(ror1(G)) * s24(L.fac);
  acc += (int64_t)bcast<1>(fr) * G;
  G = s24(ror1(G)) * s24(L.fac);
  acc += (int64_t)bcast<2>(fr) * G;
  G = s24(ror1(G)) * s24(L.fac);
  acc += (int64_t)bcast<3>(fr) * G;
  return fw_carry_rows(acc, L);
}

// f^2 for a REPLICATED f: fw_mul_rep with g = f, the three row rotations
// shared by both operands (the broadcast one is rotated left by 4 r, the
// other right by 4 r: rows 1 and 3 swap them) and one multiply by the row's
// wrap factors instead of three
#ifndef OURO_FW_SQ_FAC
#define OURO_FW_SQ_FAC 1  // A/B switch: 0 = fw_mul_rep(f, f)
#endif
__device__ __forceinline__ int32_t fw_sq_rep(int32_t f, const Lanes& L) {
  if (!OURO_FW_SQ_FAC) return fw_mul_rep(f, f, L);
  const int32_t d12 = dpp<0x12c>(f), d8 = dpp<0x128>(f), d4 = dpp<0x124>(f);  // ror 12 / 8 / 4
  const int32_t fr = sel4(f, d12, d8, d4, L);
  int32_t G = s24(sel4(f, d4, d8, d12, L)) * s24(L.facr);
  int64_t acc = (int64_t)bcast<0>(fr) * G;
  G = s24(ror1(G)) * s24(L.fac);
  acc += (int64_t)bcast<1>(fr) * G;
  G = s24(ror1(G)) * s24(L.fac);
  acc += (int64_t)bcast<2>(fr) * G;
  G = s24(ror1(G)) * s24(L.fac);
  acc += (int64_t)bcast<3>(fr) * G;
  return fw_carry_rows(acc, L);
}

// ---- conversions -------------------------------------------------------------
// lane-local fe (same value in every lane) -> replicated fw
__device__ __forceinline__ int32_t fe_to_fw(const fe& f, const Lanes& L) {
  uint32_t w[8];
  fe_to_words(w, f);
  uint32_t x = w[0];
#pragma unroll
  for (int k = 1; k < 8; k++) x = (L.j >> 1) == k ? w[k] : x;
  return (int32_t)((x >> ((L.j & 1) << 4)) & 0xffffu);
}

// fw -> lane-local fe in every lane (limbs within fe's reduced profile,
// limb 0 up to 2^26 + 18): row `row`'s limbs read out with v_readlane
__device__ __forceinline__ fe fw_to_fe(int32_t x, int row = 0) {
  // + 4p first (limbs 4 * (0xffed, 0xffff x 14, 0x7fff) >= 2^17 > |negative limb|)
  uint32_t h[16];
  int32_t c = 0;
#pragma unroll
  for (int k = 0; k < 16; k++) {
    const int32_t pk = k == 0 ? 0xffed : (k == 15 ? 0x7fff : 0xffff);
    const int32_t t = __builtin_amdgcn_readlane(x, 16 * row + k) + 4 * pk + c;
    h[k] = (uint32_t)t & 0xffffu;
    c = t >> 16;
  }
  // value = sum h 2^16k + c 2^256, c >= 0 small: fold 38 c twice
#pragma unroll
  for (int pass = 0; pass < 2; pass++) {
    uint32_t cc = (uint32_t)c * 38u;
#pragma unroll
    for (int k = 0; k < 16; k++) {
      const uint32_t t = h[k] + cc;
      h[k] = t & 0xffffu;
      cc = t >> 16;
    }
    c = (int32_t)cc;
  }
  uint32_t w[8];
#pragma unroll
  for (int k = 0; k < 8; k++) w[k] = h[2 * k] | (h[2 * k + 1] << 16);
  const uint32_t top = w[7] >> 31;  // 2^255 = 19
  w[7] &= 0x7fffffffu;
  fe f = fe_from_words(w);
  f.v[0] += 19u * top;
  return f;
}

// fw_to_fe of the element in this lane's own row, on every lane at once: the
// row's sixteen limbs gathered with ds_bpermute, then fw_to_fe's arithmetic
// in vector registers, so the four rows convert in one pass instead of four
// scalar ones (encode2_wide, OURO_ENC_ROWS)
__device__ __forceinline__ fe fw_to_fe_own_row(int32_t x) {
  const int base = (int)(threadIdx.x & 48u);
  uint32_t h[16];
  int32_t c = 0;
#pragma unroll
  for (int k = 0; k < 16; k++) {
    const int32_t pk = k == 0 ? 0xffed : (k == 15 ? 0x7fff : 0xffff);
    const int32_t t = __builtin_amdgcn_ds_bpermute((base + k) << 2, x) + 4 * pk + c;
    h[k] = (uint32_t)t & 0xffffu;
    c = t >> 16;
  }
#pragma unroll
  for (int pass = 0; pass < 2; pass++) {
    uint32_t cc = (uint32_t)c * 38u;
#pragma unroll
    for (int k = 0; k < 16; k++) {
      const uint32_t t = h[k] + cc;
      h[k] = t & 0xffffu;
      cc = t >> 16;
    }
    c = (int32_t)cc;
  }
  uint32_t w[8];
#pragma unroll
  for (int k = 0; k < 8; k++) w[k] = h[2 * k] | (h[2 * k + 1] << 16);
  const uint32_t top = w[7] >> 31;  // 2^255 = 19
  w[7] &= 0x7fffffffu;
  fe f = fe_from_words(w);
  f.v[0] += 19u * top;
  return f;
}

__device__ __forceinline__ int32_t fw_one(const Lanes& L) { return L.j == 0 ? 1 : 0; }

// ---- exponentiations -------------------------------------------------------------
#ifndef OURO_FW_REP
#define OURO_FW_REP 1  // A/B switch: replicated chains with the row-split product
#endif
template <bool kRep>
__device__ __forceinline__ int32_t fw_mul_t(int32_t f, int32_t g, const Lanes& L) {
  return (kRep && OURO_FW_REP) ? fw_mul_rep(f, g, L) : fw_mul(f, g, L);
}
template <bool kRep>
__device__ __forceinline__ int32_t fw_sq_t(int32_t f, const Lanes& L) {
  return (kRep && OURO_FW_REP) ? fw_sq_rep(f, L) : fw_mul(f, f, L);
}
template <bool kRep>
__device__ __forceinline__ int32_t fw_sqn(int32_t t, int n, const Lanes& L) {
#pragma unroll 1
  for (int i = 0; i < n; i++) t = fw_sq_t<kRep>(t, L);
  return t;
}
// z^(2^252 - 3) (mode 1: the square-root helper) or z^(p - 2) (mode 0: the
// inversion), fe25519.h fe_pow_chain's addition chain.  kRep: z replicated
// (one chain on the wave, row-split products); else each row its own chain.
template <bool kRep>
__device__ __noinline__ int32_t fw_pow_chain(int32_t z, int mode) {
  const Lanes L = lanes();
#define fw_mul(a, b, l) fw_mul_t<kRep>(a, b, l)
#define fw_sq(a, l) fw_sq_t<kRep>(a, l)
#define fw_sqn fw_sqn<kRep>
  const int32_t z2 = fw_sq(z, L);
  int32_t t = fw_sqn(z2, 2, L);
  const int32_t z9 = fw_mul(t, z, L);
  const int32_t z11 = fw_mul(z9, z2, L);
  t = fw_sq(z11, L);
  const int32_t z5 = fw_mul(t, z9, L);                    // 2^5 - 1
  const int32_t z10 = fw_mul(fw_sqn(z5, 5, L), z5, L);    // 2^10 - 1
  const int32_t z20 = fw_mul(fw_sqn(z10, 10, L), z10, L);
  t = fw_mul(fw_sqn(z20, 20, L), z20, L);                 // 2^40 - 1
  const int32_t z50 = fw_mul(fw_sqn(t, 10, L), z10, L);
  const int32_t z100 = fw_mul(fw_sqn(z50, 50, L), z50, L);
  t = fw_mul(fw_sqn(z100, 100, L), z100, L);              // 2^200 - 1
  const int32_t z250 = fw_mul(fw_sqn(t, 50, L), z50, L);
  return fw_mul(fw_sqn(z250, mode ? 2 : 5, L), mode ? z : z11, L);  // 2^252 - 3 | 2^255 - 21
#undef fw_mul
#undef fw_sq
#undef fw_sqn
}
// rows independent (e.g. two decodes at once)
__device__ __forceinline__ int32_t fw_pow22523_rows(int32_t z) { return fw_pow_chain<false>(z, 1); }
// z replicated in every row
__device__ __forceinline__ int32_t fw_pow22523(int32_t z) { return fw_pow_chain<true>(z, 1); }
__device__ __forceinline__ int32_t fw_invert(int32_t z) { return fw_pow_chain<true>(z, 0); }

// ---- group operations ----------------------------------------------------------
struct pw { int32_t X, Y, Z, T; };  // extended point, coordinates replicated

__device__ __forceinline__ pw pw_identity(const Lanes& L) {
  const int32_t one = fw_one(L);
  return pw{0, one, one, 0};
}
__device__ __forceinline__ pw pw_from_p3(const ge_p3& P, const Lanes& L) {
  return pw{fe_to_fw(P.X, L), fe_to_fw(P.Y, L), fe_to_fw(P.Z, L), fe_to_fw(P.T, L)};
}

// 2P (T of the input unused).  Layer 1: rows square X, Y, Z, X + Y; then
// Y3 = YY + XX, Z3 = YY - XX, X3 = AA - Y3, T3 = 2 ZZ - Z3 and layer 2 forms
// X = X3 T3, Y = Y3 Z3, Z = Z3 T3, T = X3 Y3 (ref10 ge_p2_dbl + p1p1 -> p3).
__device__ __forceinline__ pw pw_dbl(const pw& p, const Lanes& L) {
  const int32_t op = sel4(p.X, p.Y, p.Z, p.X + p.Y, L);
  const fw4 s = fw_gather(fw_sq(op, L));
  const int32_t Y3 = s.r1 + s.r0, Z3 = s.r1 - s.r0;
  const int32_t X3 = s.r3 - Y3, T3 = 2 * s.r2 - Z3;
  // narrow (<= 3-term) operand second: X3, Z3, Z3, Y3
  const int32_t a = sel4(T3, Y3, T3, X3, L), b = sel4(X3, Z3, Z3, Y3, L);
  const fw4 m = fw_gather(fw_mul(a, b, L));
  return pw{m.r0, m.r1, m.r2, m.r3};
}

// P + Q with Q given as this row's cached operand q (row 0: Y2 - X2, row 1:
// Y2 + X2, row 2: 2d T2, row 3: 2 Z2; -Q swaps rows 0/1 and negates row 2).
// Layer 1: A = (Y1 - X1) q0, B = (Y1 + X1) q1, C = T1 q2, D = Z1 q3; then
// E = B - A, H = B + A, F = D - C, G = D + C and X = E F, Y = G H, Z = F G,
// T = E H (ref10 ge_add + p1p1 -> p3).
__device__ __forceinline__ pw pw_add(const pw& p, int32_t q, const Lanes& L) {
  const int32_t a = sel4(p.Y - p.X, p.Y + p.X, p.T, p.Z, L);
  const fw4 s = fw_gather(fw_mul(a, q, L));
  const int32_t E = s.r1 - s.r0, H = s.r1 + s.r0, F = s.r3 - s.r2, G = s.r3 + s.r2;
  const int32_t a2 = sel4(E, G, F, E, L), b2 = sel4(F, H, G, H, L);
  const fw4 m = fw_gather(fw_mul(a2, b2, L));
  return pw{m.r0, m.r1, m.r2, m.r3};
}

// cached operands of P for this row: +P and -P
struct cw { int32_t pos, neg; };
__device__ __forceinline__ cw pw_cached(const pw& P, int32_t d2, const Lanes& L) {
  const int32_t T2d = fw_mul(P.T, d2, L);  // every row the same product
  const int32_t ypx = P.Y + P.X, ymx = P.Y - P.X, z2 = P.Z + P.Z;
  return cw{sel4(ymx, ypx, T2d, z2, L), sel4(ypx, ymx, -T2d, z2, L)};
}

// [1..8]P in this row's cached operands (VGPRs; the index is wave-uniform)
struct TabW { int32_t pos[8], neg[8]; };
__device__ __forceinline__ void tab_build(TabW& t, const pw& P, int32_t d2, const Lanes& L) {
  const cw c1 = pw_cached(P, d2, L);
  t.pos[0] = c1.pos;
  t.neg[0] = c1.neg;
  pw Pk = pw_dbl(P, L);
#pragma unroll
  for (int k = 1; k < 8; k++) {
    if (k > 1) Pk = pw_add(Pk, c1.pos, L);
    const cw ck = pw_cached(Pk, d2, L);
    t.pos[k] = ck.pos;
    t.neg[k] = ck.neg;
  }
}

// this row's operand of table entry d (wave-uniform, d != 0), by a chain of
// selects on the index (indexed, the register table becomes a scratch array,
// which LLVM also got wrong inside an out-of-line function here)
__device__ __forceinline__ int32_t tab_pick(const TabW& tab, int32_t d) {
  const int idx = d == 0 ? 0 : (d < 0 ? -d : d) - 1;
  int32_t qp = tab.pos[0], qn = tab.neg[0];
#pragma unroll
  for (int k = 1; k < 8; k++) {
    qp = idx == k ? tab.pos[k] : qp;
    qn = idx == k ? tab.neg[k] : qn;
  }
  return d < 0 ? qn : qp;
}

// ---- the fixed base B in wide form -----------------------------------------
// Stored after the niels B tables (verify.h build_btab_wide, kBTabWords int32
// words in): for every entry [k]B (k = 1..2^15), then [k](2^128 B), the
// canonical 16-bit limbs of y - x, y + x and 2dxy (kBWideU16 uint16 each).
static_assert(kBW == 16 && !kBSplitRecode, "the wide chain reads 16-bit B digits");

// this row's operand of [d]G (G = B for half 0, 2^128 B for half 1), d != 0:
// rows 0 / 1 take y - x / y + x (swapped for -G), row 2 2dxy (negated for
// -G), row 3 2Z = 2 (affine)
__device__ __forceinline__ int32_t bw_operand(const uint16_t* bw, int half, int32_t d,
                                              const Lanes& L) {
  const bool neg = d < 0;
  const int idx = d == 0 ? 0 : (neg ? -d : d) - 1;
  const int coord = L.high ? 2 : ((L.odd != neg) ? 1 : 0);
  const int32_t v = (int32_t)ldg_u16(bw + ((size_t)half * kBTabEntries + idx) * kBWideU16 +
                                     coord * 16 + L.j);
  const int32_t v2 = (L.high && !L.odd && neg) ? -v : v;
  return (L.high && L.odd) ? (L.j == 0 ? 2 : 0) : v2;
}

// [a1]T1 + [a2]T2 + [b]B on one doubling chain: signed width-4 windows for
// the register tables (nw1 / nw2 windows), b's 16-bit digits from the wide B
// tables every fourth window (b split at bit 128, as verify.h dsm_body), all
// digits wave-uniform (scalars read out of the first lane).  Result in p3 form.
// kBMask: which halves of b's digits are added -- 1 the low eight (with B), 2
// the high eight (with 2^128 B), 3 both.  Both recode b as one number, so a
// chain taking the low half and another taking the high half of the same b
// sum to [b]B exactly (the carry out of digit 7 is digit 8's carry in).
// Likewise only the windows below nw1 of a1 are added, their digits recoded
// from the whole a1: the top one carries out what the windows above take in.
template <bool kT2, bool kB, int kBMask = 3>
__device__ __forceinline__ pw pw_dsm(const TabW& t1, const uint32_t a1_in[8], int nw1_in,
                                     const TabW& t2, const uint32_t a2_in[8], int nw2_in,
                                     const uint32_t b_in[8], const uint16_t* bw,
                                     const Lanes& L) {
  uint32_t a1[8], a2[8], b[8];
#pragma unroll
  for (int k = 0; k < 8; k++) {
    a1[k] = __builtin_amdgcn_readfirstlane(a1_in[k]);
    a2[k] = kT2 ? __builtin_amdgcn_readfirstlane(a2_in[k]) : 0u;
    b[k] = kB ? __builtin_amdgcn_readfirstlane(b_in[k]) : 0u;
  }
  const int nw1 = __builtin_amdgcn_readfirstlane(nw1_in);
  const int nw2 = kT2 ? __builtin_amdgcn_readfirstlane(nw2_in) : 0;
  const uint64_t c1 = sc_recode_carries<4, 64>(a1);
  const uint64_t c2 = kT2 ? sc_recode_carries<4, 64>(a2) : 0ull;
  const uint64_t cb = kB ? sc_recode_b(b) : 0ull;
  constexpr int kBWin = kBStride * kBDigitsHalf;  // windows the B digits span
  int top = nw1 > nw2 ? nw1 : nw2;
  if (kB && top < kBWin) top = kBWin;
  pw acc = pw_identity(L);
#pragma unroll 1
  for (int j = top - 1; j >= 0; j--) {
    // digits and operands first: the B loads then overlap the doublings
    const int32_t d1 = j < nw1 ? sc_digit_from<4>((a1[j >> 3] >> (4 * (j & 7))) & 15u, c1, j, 64) : 0;
    const int32_t q1 = tab_pick(t1, d1);
    int32_t d2 = 0, q2 = 0, d3 = 0, q3 = 0, d4 = 0, q4 = 0;
    if (kT2 && j < nw2) {
      d2 = sc_digit_from<4>((a2[j >> 3] >> (4 * (j & 7))) & 15u, c2, j, 64);
      q2 = tab_pick(t2, d2);
    }
    if (kB && (j % kBStride) == 0 && j < kBWin) {
      const int k = j / kBStride, kh = k + kBDigitsHalf;
      d3 = sc_digit_from<kBW>((b[k >> 1] >> (16 * (k & 1))) & 0xffffu, cb, k, 2 * kBDigitsHalf);
      d4 = sc_digit_from<kBW>((b[kh >> 1] >> (16 * (kh & 1))) & 0xffffu, cb, kh,
                              2 * kBDigitsHalf);
      if (!(kBMask & 1)) d3 = 0;
      if (!(kBMask & 2)) d4 = 0;
      q3 = (kBMask & 1) ? bw_operand(bw, 0, d3, L) : 0;
      q4 = (kBMask & 2) ? bw_operand(bw, 1, d4, L) : 0;
    }
    if (j != top - 1) {
#pragma unroll
      for (int k = 0; k < 4; k++) acc = pw_dbl(acc, L);
    }
    if (d1 != 0) acc = pw_add(acc, q1, L);
    if (d2 != 0) acc = pw_add(acc, q2, L);
    if (d3 != 0) acc = pw_add(acc, q3, L);
    if (d4 != 0) acc = pw_add(acc, q4, L);
  }
  return acc;
}

// a wave-wide point in a record (kPwWords = 64 words): lanes 0..15 store their
// limb of X, Y, Z, T (the rows hold copies); every lane loads its limb back
__device__ __forceinline__ void st_pw(Slot p, const pw& P) {
  const int j = (int)(threadIdx.x & 63u);
  if (j < 16) {
    *p.word(j) = P.X;
    *p.word(16 + j) = P.Y;
    *p.word(32 + j) = P.Z;
    *p.word(48 + j) = P.T;
  }
}
__device__ __forceinline__ pw ld_pw(Slot p) {
  const int j = (int)(threadIdx.x & 15u);
  return pw{ldg1(p.word(j)), ldg1(p.word(16 + j)), ldg1(p.word(32 + j)), ldg1(p.word(48 + j))};
}

// P + Q for two wave-wide points in p3 form (complete: a = -1, d non-square)
__device__ __forceinline__ pw pw_add_p3(const pw& P, const pw& Q, int32_t d2, const Lanes& L) {
  return pw_add(P, pw_cached(Q, d2, L).pos, L);
}

// [s]P for a 253-bit s (signed width-4 windows), result in p3 form
__device__ __forceinline__ pw pw_scalarmult(const TabW& tab, const uint32_t s[8], const Lanes& L) {
  return pw_dsm<false, false>(tab, s, 64, tab, s, 0, s, nullptr, L);
}

}  // namespace wide
#endif
}  // namespace ouro
