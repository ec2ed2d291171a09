// wide_cores.h -- the latency mode's cores on one wave each (wide.h): the
// eight work items of a header (tpraos.h hdr_core with split V) with every
// exponentiation and scalar multiplication as wave-wide arithmetic.  The
// scalar work around them (hashes, scalar reduction, the lattice pair,
// encoding checks, lane-local decode algebra) runs on every lane alike; lane
// 0 stores the header record's fields exactly as the lane routines do, so
// the finish (k_tpraos_finish) is shared.
#pragma once
#include "tpraos.h"
#include "wide.h"
#include "wide_inv.h"

namespace ouro {
// the latency probe's stamp table (lstamp below; host and device passes both
// see it, so the host reads it with hipMemcpyFromSymbol)
#ifndef OURO_LAT_STAMPS
#define OURO_LAT_STAMPS 0
#endif
constexpr int kStampItems = 16, kStampTags = 24;
#if OURO_LAT_STAMPS
__device__ unsigned long long g_lat_stamps[kStampItems][kStampTags];
#endif
#if defined(__HIP_DEVICE_COMPILE__)
namespace wide {

// timing probe (a build with -DOURO_LAT_STAMPS=1, tools/lat_stamps.py): the
// eta V item of header 0 in a fused launch (block 4) prints phase times
#ifndef OURO_LAT_STAMPS
#define OURO_LAT_STAMPS 0
#endif
#if OURO_LAT_STAMPS
__device__ unsigned long long g_vstamps[8];
__device__ unsigned long long g_kstamps[2][8];  // header 0's KES points / scalars items
#endif
// phase k of that item (0 start, 1 sha, 2 elligator, 3 table, 4 chain,
// 5 combine-add, 6 encoded), kept in device memory: printed once at the end
__device__ __forceinline__ void vstamp(int k) {
#if OURO_LAT_STAMPS
  if (blockIdx.x == 4 && threadIdx.x == 0) g_vstamps[k] = __builtin_amdgcn_s_memrealtime();
#else
  (void)k;
#endif
}
// phase k of header 0's KES points (block 1) / scalars (block 9) item:
// 0 start, 1 Merkle walk, 2 decodes / SHA + lattice, 3 arrival, 4 chain
__device__ __forceinline__ void kstamp(int k) {
#if OURO_LAT_STAMPS
  if ((blockIdx.x == 1 || blockIdx.x == 9) && threadIdx.x == 0) {
    unsigned long long* s = g_kstamps[blockIdx.x == 9];
    if (k == 0)
      for (int j = 1; j < 8; j++) s[j] = 0;
    s[k] = __builtin_amdgcn_s_memrealtime();
  }
#else
  (void)k;
#endif
}
__device__ __forceinline__ void kstamp_print() {
#if OURO_LAT_STAMPS
  if ((blockIdx.x == 1 || blockIdx.x == 9) && threadIdx.x == 0) {
    const unsigned long long* s = g_kstamps[blockIdx.x == 9];
    printf("kstamp %d %llu %llu %llu %llu %llu %llu %llu %llu\n", blockIdx.x == 9 ? 9 : 1, s[0],
           s[1], s[2], s[3], s[4], s[5], s[6], s[7]);
  }
#endif
}
// printf-free probe of the fused launch (split form): the lead lane of header
// 0's items (blocks 0..kStampItems-1 with 64-thread workgroups) records
// s_memrealtime at tagged points into g_lat_stamps[item][tag]; the host reads
// them after the launch (kernels.hip ouro_debug_lat_stamps, tools/lat_stamps.py)
__device__ __forceinline__ void lstamp(int tag) {
#if OURO_LAT_STAMPS
  if (blockIdx.x < (unsigned)kStampItems && (threadIdx.x & 63u) == 0 && tag < kStampTags)
    g_lat_stamps[blockIdx.x][tag] = __builtin_amdgcn_s_memrealtime();
#else
  (void)tag;
#endif
}
__device__ __forceinline__ void vstamp_print() {
#if OURO_LAT_STAMPS
  if (blockIdx.x == 4 && threadIdx.x == 0)
    printf("vstamp %llu %llu %llu %llu %llu %llu %llu\n", g_vstamps[0], g_vstamps[1],
           g_vstamps[2], g_vstamps[3], g_vstamps[4], g_vstamps[5], g_vstamps[6]);
#endif
}

// Row elements made canonical in one vector pass, every row its own element
// (wide.h fw_to_fe_own_row): the encodings' coordinates and Elligator2's
// three zero tests (1, since round 5: the V2 item's encodings 3.1 -> 1.3 us,
// profiles/r05af), or one after another on the scalar path (0, A/B)
#ifndef OURO_ENC_ROWS
#define OURO_ENC_ROWS 1
#endif

// z^(2^252 - 3) of a lane-local element on the wave
__device__ __forceinline__ fe pow22523_wide(const fe& z) {
  return fw_to_fe(fw_pow22523(fe_to_fw(z, lanes())));
}

// ge_decode with its exponentiation on the wave
__device__ __forceinline__ bool ge_decode_wide(ge_p3* h, const uint32_t s[8], bool negate) {
  DecodePre d;
  const fe t = ge_decode_pre(d, s);
  return ge_decode_post(h, d, pow22523_wide(t), s, negate);
}

// two decodes, both exponentiations at once: a's on rows 0/2, b's on rows 1/3
__device__ __forceinline__ void ge_decode_pair_wide(ge_p3* a, bool* oka, ge_p3* b, bool* okb,
                                                    const uint32_t sa[8], const uint32_t sb[8],
                                                    bool negate) {
  const Lanes L = lanes();
  DecodePre da, db;
  const fe ta = ge_decode_pre(da, sa), tb = ge_decode_pre(db, sb);
  const int32_t x = L.odd ? fe_to_fw(tb, L) : fe_to_fw(ta, L);
  const int32_t y = fw_pow22523_rows(x);
  *oka = ge_decode_post(a, da, fw_to_fe(y, 0), sa, negate);
  *okb = ge_decode_post(b, db, fw_to_fe(y, 1), sb, negate);
}

__device__ __forceinline__ int32_t d2_wide(const Lanes& L) { return fe_to_fw(fe_d2(), L); }

__device__ __forceinline__ bool pw_is_identity(const pw& Q) {
  return fe_iszero(fw_to_fe(Q.X)) && fe_iszero(fw_to_fe(Q.Y - Q.Z));
}
__device__ __forceinline__ ge_p2 pw_to_p2(const pw& Q) {
  return ge_p2{fw_to_fe(Q.X), fw_to_fe(Q.Y), fw_to_fe(Q.Z)};
}

// ---- Elligator2 on the wave ------------------------------------------------------
// verify.h elligator2_pre / elligator2_post (the one-exponentiation form of
// libsodium's ge25519_from_uniform) with every product on the wave instead of
// a lane (each lane-local product is one wave's dependent chain of ~200
// instructions; a replicated wave product ~45): the same point, then the
// cofactor cleared by three wave-wide doublings.  A/B switch OURO_ELL2_WIDE.
// Bounds (wide.h): carried elements have limbs below 2^16.13; D and Xn are
// 2-term sums and W a 3-term one (narrow operands: at most 3 terms); n and m
// (4 terms) are renormalised by one shift-and-rotate round (fw_norm) before
// they enter a product or the point.
#ifndef OURO_ELL2_WIDE
#define OURO_ELL2_WIDE 1
#endif
// one carry round of a limb vector below 2^20: limbs below 2^16 + 38 * 16
__device__ __forceinline__ int32_t fw_norm(int32_t x, const Lanes& L) {
  return (x & 0xffff) + s24(ror1(x >> 16)) * s24(L.fac);
}
// whether the replicated element in `row` of x is 0 mod p
__device__ __forceinline__ bool fw_row_iszero(int32_t x, int row) {
  return fe_iszero(fw_to_fe(x, row));
}
__device__ __forceinline__ pw elligator2_wide(const uint32_t r[8], const Lanes& L) {
  const int32_t one = fw_one(L);
  const int32_t rr = fe_to_fw(fe_from_words(r), L);
  const int32_t r2 = fw_sq_rep(rr, L);
  const int32_t D = r2 + r2 + one;                               // 1 + 2 r^2 (2 terms)
  // A^2 r^2 (rows 0/2) and D^2 (rows 1/3) at once
  const fw4 a = fw_gather(fw_mul(L.odd ? D : fe_to_fw(fe_mont_a2(), L), L.odd ? D : r2, L));
  const int32_t W = a.r1 - a.r0 - a.r0;                          // D^2 - 2 A^2 r^2 (3 terms)
  // (A + 2) A D (rows 0/2) and W^2 (rows 1/3)
  const fw4 b = fw_gather(fw_mul(L.odd ? W : fe_to_fw(fe_mont_a2a(), L), L.odd ? W : D, L));
  const int32_t num = b.r0;
  const int32_t W3 = fw_mul_rep(b.r1, W, L);
  const int32_t W7 = fw_mul_rep(fw_sq_rep(W3, L), W, L);
  // num W3 and num sqrt(-1) (needed after the root) beside num W7 (its base)
  const fw4 c = fw_gather(fw_mul(num, sel4(W7, W3, fe_to_fw(fe_sqrtm1(), L), W7, L), L));
  const int32_t root = fw_pow22523(c.r0);                        // (num W^7)^((p-5)/8)
  const int32_t beta = fw_mul_rep(c.r1, root, L);                // num W^3 (num W^7)^((p-5)/8)
  const int32_t vxx = fw_mul_rep(fw_sq_rep(beta, L), W, L);      // beta^2 W
  // the root's 4th root of unity: vxx = num (1), -num (-1), num i (i) or -num i
  const int32_t d = sel4(vxx - num, vxx + num, vxx - c.r2, vxx - num, L);
  bool lam_p1, lam_m1, lam_pi;
  if (OURO_ENC_ROWS) {  // the three tests in one vector pass, each row its own
    const uint32_t z = fe_iszero(fw_to_fe_own_row(d)) ? 1u : 0u;
    lam_p1 = __builtin_amdgcn_readlane((int)z, 0) != 0;
    lam_m1 = __builtin_amdgcn_readlane((int)z, 16) != 0;
    lam_pi = __builtin_amdgcn_readlane((int)z, 32) != 0;
  } else {
    lam_p1 = fw_row_iszero(d, 0);
    lam_m1 = fw_row_iszero(d, 1);
    lam_pi = fw_row_iszero(d, 2);
  }
  const bool nonsq = !(lam_p1 || lam_m1);
  const fe Ff = fe_select(fe_select(fe_one_minus_i(), fe_one_plus_i(), lam_pi),
                          fe_select(fe_one(), fe_sqrtm1(), lam_p1), nonsq);
  int32_t x = fw_mul_rep(beta, fe_to_fw(Ff, L), L);
  if (nonsq) x = fw_mul_rep(x, rr, L);
  if (fe_isnegative(fw_to_fe(x))) x = -x;                       // sign bit 0: even x
  const int32_t Ar2 = fw_mul_rep(fe_to_fw(fe_mont_a(), L), r2, L);
  const int32_t Xn = nonsq ? -(Ar2 + Ar2) : -fe_to_fw(fe_mont_a(), L);  // 2 terms
  const int32_t n = fw_norm(Xn - D, L), m = fw_norm(Xn + D, L);
  // P = (x m, n, m, x n): rows 0/2 x m, rows 1/3 x n
  const fw4 e = fw_gather(fw_mul(x, L.odd ? n : m, L));
  const pw P{e.r0, n, m, e.r1};
  return pw_dbl(pw_dbl(pw_dbl(P, L), L), L);
}

// verify.h ed25519_verify_lane (libsodium 1.0.18 rules through the half-size
// equation) on one wave
template <class Tail>
__device__ __forceinline__ bool ed25519_verify_wide(const uint32_t sig[16], const uint32_t pk[8],
                                                    const Tail& msg, uint32_t mlen,
                                                    const uint16_t* bw, bool byron = false) {
  const Lanes L = lanes();
  uint32_t R[8], S[8];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    R[i] = sig[i];
    S[i] = sig[8 + i];
  }
  bool ok = ed25519_precheck(R, S, pk, byron);
  ge_p3 negA, negR;
  bool okA, okR;
  ge_decode_pair_wide(&negA, &okA, &negR, &okR, pk, R, true);
  ok = okA && ok;
  ok = ge_is_canonical(R) && ok;
  ok = okR && ok;
  ok = ok && !(fe_iszero(negR.X) && (R[7] >> 31) != 0);
  HalfScalars hs;
  uint32_t b[8];
  ed25519_scalars(hs, b, R, S, pk, msg, mlen);
  const int32_t d2 = d2_wide(L);
  TabW t1, t2;
  tab_build(t1, pw_from_p3(hs.c0_neg ? ge_p3_neg(negA) : negA, L), d2, L);
  tab_build(t2, pw_from_p3(negR, L), d2, L);
  int nw = (hs.bits + 4) >> 2;
  nw = nw < 1 ? 1 : (nw > 64 ? 64 : nw);
  const pw Q = pw_dsm<true, true>(t1, hs.c0, nw, t2, hs.c1, nw, b, bw, L);
  return ok && pw_is_identity(Q);
}

// verify.h sum6kes_walk with the six Blake2b hashes at once: lane k hashes
// the (vk0, vk1) pair of level k + 1 (lanes 6.. repeat them), then the walk
// reads each level's digest out of its lane
__device__ __forceinline__ bool sum6kes_walk_wide(uint32_t cur[8], uint32_t sig[16],
                                                  const uint32_t vk[8], uint32_t t,
                                                  const uint32_t* sigw) {
  const int mine = (int)((threadIdx.x & 63u) % 6u);
  uint32_t pw[16], h[8];
  ld_words(pw, reinterpret_cast<const uint8_t*>(sigw + 16 + 16 * mine), 4);
  blake2b256_64(h, pw);
#pragma unroll
  for (int i = 0; i < 8; i++) cur[i] = vk[i];
  bool ok = true;
#pragma unroll
  for (int k = 6; k >= 1; k--) {
    uint32_t pk[16];
    ld_words(pk, reinterpret_cast<const uint8_t*>(sigw + 16 + 16 * (k - 1)), 4);
#pragma unroll
    for (int i = 0; i < 8; i++) ok = ok && (uint32_t)__builtin_amdgcn_readlane((int)h[i], k - 1) == cur[i];
    const uint32_t half = 1u << (k - 1);
    const bool right = t >= half;
    t = right ? t - half : t;
#pragma unroll
    for (int i = 0; i < 8; i++) cur[i] = right ? pk[8 + i] : pk[i];
  }
  ld_words(sig, reinterpret_cast<const uint8_t*>(sigw), 4);
  return ok;
}

template <class Tail>
__device__ __forceinline__ bool sum6kes_verify_wide(const uint32_t vk[8], uint32_t t,
                                                    const uint32_t* sigw, const Tail& msg,
                                                    uint32_t mlen, const uint16_t* bw) {
  uint32_t cur[8], sig[16];
  const bool ok = sum6kes_walk_wide(cur, sig, vk, t, sigw);
  const bool leaf = ed25519_verify_wide(sig, cur, msg, mlen, bw);
  return ok && leaf;
}

// tpraos.h vrf_u_core: U = [s]B - [c]Y (Y decoded and checked here)
__device__ __forceinline__ bool vrf_u_wide_pw(pw& U, const uint32_t pk[8], const uint32_t pi[20],
                                              const uint16_t* bw) {
  const Lanes L = lanes();
  ge_p3 Y;
  bool ok = !ge_has_small_order(pk) && ge_is_canonical(pk);
  ok = ge_decode_wide(&Y, pk, false) && ok;
  uint32_t c[8], s_raw[8], s[8];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    s_raw[i] = pi[12 + i];
    c[i] = i < 4 ? pi[8 + i] : 0u;
  }
  sc_reduce256(s, s_raw);
  TabW t;
  tab_build(t, pw_from_p3(ge_p3_neg(Y), L), d2_wide(L), L);
  U = pw_dsm<false, true>(t, c, 33, t, c, 0, s, bw, L);
  return ok;
}
__device__ __forceinline__ bool vrf_u_wide(ge_p2& U, const uint32_t pk[8], const uint32_t pi[20],
                                           const uint16_t* bw) {
  pw Uw;
  const bool ok = vrf_u_wide_pw(Uw, pk, pi, bw);
  U = pw_to_p2(Uw);
  return ok;
}

// tpraos.h vrf_v_core part 2: the Gamma checks, -[c]Gamma (to `partial`) and
// [8]Gamma; returns the flag word
__device__ __forceinline__ int32_t vrf_gamma_wide(ge_p2& partial, ge_p3& G8,
                                                  const uint32_t pi[20]) {
  const Lanes L = lanes();
  uint32_t G[8], c[8];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    G[i] = pi[i];
    c[i] = i < 4 ? pi[8 + i] : 0u;
  }
  ge_p3 Gamma;
  bool ok = ge_is_canonical(G);
  ok = ge_decode_wide(&Gamma, G, false) && ok;
  TabW t;
  const pw Gw = pw_from_p3(Gamma, L);
  tab_build(t, pw_from_p3(ge_p3_neg(Gamma), L), d2_wide(L), L);
  partial = pw_to_p2(pw_dsm<false, false>(t, c, 33, t, c, 0, c, nullptr, L));
  const pw G8w = pw_dbl(pw_dbl(pw_dbl(Gw, L), L), L);
  G8 = ge_p3{fw_to_fe(G8w.X), fw_to_fe(G8w.Y), fw_to_fe(G8w.Z), fw_to_fe(G8w.T)};
  return (ok ? kFlagOk : 0) | (fe_iszero(Gamma.X) ? kFlagGammaX0 : 0);
}

// tpraos.h vrf_v_core part 1: H = hash_to_curve(pk, alpha) (Elligator2 with
// its exponentiation on the wave) and V = [s mod L]H, both in every lane.
template <class Tail>
__device__ __forceinline__ void vrf_sh(ge_p3& H, ge_p2& V, const uint32_t pk[8],
                                       const uint32_t pi[20], const Tail& alpha) {
  const Lanes L = lanes();
  uint32_t s_raw[8], s[8];
#pragma unroll
  for (int k = 0; k < 8; k++) s_raw[k] = pi[12 + k];
  sc_reduce256(s, s_raw);
  uint32_t pre[9];
  pre[0] = 0x04u | (0x01u << 8) | (pk[0] << 16);
#pragma unroll
  for (int k = 1; k < 8; k++) pre[k] = (pk[k - 1] >> 16) | (pk[k] << 16);
  pre[8] = pk[7] >> 16;
  uint64_t Hs[8];
  vstamp(0);
  sha512_prefixed<34>(Hs, pre, alpha, 32);
  uint32_t rw[16];
  sha512_digest_words(rw, Hs);
  rw[7] &= 0x7fffffffu;
  vstamp(1);
  // the Elligator2 point, its cofactor cleared by three doublings on the wave
  auto pw22523 = [](const fe& z) { return pow22523_wide(z); };
  const ge_p3 P = elligator2_h_with<decltype(pw22523), false>(rw, pw22523);
  const pw Hw = pw_dbl(pw_dbl(pw_dbl(pw_from_p3(P, L), L), L), L);
  H = ge_p3{fw_to_fe(Hw.X), fw_to_fe(Hw.Y), fw_to_fe(Hw.Z), fw_to_fe(Hw.T)};
  vstamp(2);
  TabW tab;
  tab_build(tab, Hw, d2_wide(L), L);
  vstamp(3);
  V = pw_to_p2(pw_scalarmult(tab, s, L));
  vstamp(4);
}

// ---- a whole draft-03 VRF verification on one wave (small batches) ---------------
// verify.h vrf03_verify_lane with the wave-wide arithmetic: Y's and Gamma's
// decodes on alternate rows at once, Elligator2, U = [s]B - [c]Y, V = [s]H -
// [c]Gamma, [8]Gamma, one inversion for the four encodings, the challenge
// and beta.  beta is zeroed unless the proof verifies.
__device__ __forceinline__ fe invert_wide(const fe& z);
template <class Tail>
__device__ __forceinline__ bool vrf03_verify_wide(uint32_t beta[16], const uint32_t pk[8],
                                                  const uint32_t pi[20], const Tail& alpha,
                                                  uint32_t alen, const uint16_t* bw) {
  const Lanes L = lanes();
  uint32_t G[8], c[8], s_raw[8], s[8];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    G[i] = pi[i];
    c[i] = i < 4 ? pi[8 + i] : 0u;
    s_raw[i] = pi[12 + i];
  }
  ge_p3 Y, Gamma;
  bool okY, okG;
  ge_decode_pair_wide(&Y, &okY, &Gamma, &okG, pk, G, false);
  bool ok = !ge_has_small_order(pk) && ge_is_canonical(pk) && okY;
  ok = ge_is_canonical(G) && okG && ok;
  sc_reduce256(s, s_raw);
  uint32_t pre[9];
  pre[0] = 0x04u | (0x01u << 8) | (pk[0] << 16);
#pragma unroll
  for (int i = 1; i < 8; i++) pre[i] = (pk[i - 1] >> 16) | (pk[i] << 16);
  pre[8] = pk[7] >> 16;
  uint64_t Hs[8];
  sha512_prefixed<34>(Hs, pre, alpha, alen);
  uint32_t rw[16];
  sha512_digest_words(rw, Hs);
  rw[7] &= 0x7fffffffu;
  ge_p3 Hp;
  if (OURO_ELL2_WIDE) {
    const pw Hw = elligator2_wide(rw, L);
    Hp = ge_p3{fw_to_fe(Hw.X), fw_to_fe(Hw.Y), fw_to_fe(Hw.Z), fw_to_fe(Hw.T)};
  } else {
    Hp = elligator2_h_with(rw, [](const fe& z) { return pow22523_wide(z); });
  }
  const int32_t d2 = d2_wide(L);
  TabW tY, tH, tG;
  tab_build(tY, pw_from_p3(ge_p3_neg(Y), L), d2, L);
  const ge_p2 U = pw_to_p2(pw_dsm<false, true>(tY, c, 33, tY, c, 0, s, bw, L));
  tab_build(tH, pw_from_p3(Hp, L), d2, L);
  const pw Gw = pw_from_p3(Gamma, L);
  tab_build(tG, pw_from_p3(ge_p3_neg(Gamma), L), d2, L);
  const ge_p2 V = pw_to_p2(pw_dsm<true, false>(tH, s, 64, tG, c, 33, s, nullptr, L));
  const ge_p2 G8 = pw_to_p2(pw_dbl(pw_dbl(pw_dbl(Gw, L), L), L));
  // one inversion for the four encodings
  const fe a1 = fe_mul(Hp.Z, U.Z), a2 = fe_mul(a1, V.Z), a3 = fe_mul(a2, G8.Z);
  fe inv = invert_wide(a3);
  const fe z3 = fe_mul(inv, a2);
  inv = fe_mul(inv, G8.Z);
  const fe z2 = fe_mul(inv, a1);
  inv = fe_mul(inv, V.Z);
  const fe z1 = fe_mul(inv, Hp.Z), z0 = fe_mul(inv, U.Z);
  uint32_t Henc[8], Uenc[8], Venc[8], G8enc[8], Genc[8], cc[4], b[16];
  ge_encode_with_inv(Henc, Hp.X, Hp.Y, z0);
  ge_encode_with_inv(Uenc, U.X, U.Y, z1);
  ge_encode_with_inv(Venc, V.X, V.Y, z2);
  ge_encode_with_inv(G8enc, G8.X, G8.Y, z3);
#pragma unroll
  for (int i = 0; i < 8; i++) Genc[i] = G[i];
  if (fe_iszero(Gamma.X)) Genc[7] &= 0x7fffffffu;
#pragma unroll
  for (int i = 0; i < 4; i++) cc[i] = c[i];
  ok = vrf_finish(b, Henc, Genc, Uenc, Venc, G8enc, cc) && ok;
#pragma unroll
  for (int i = 0; i < 16; i++) beta[i] = ok ? b[i] : 0u;
  return ok;
}

// ---- fused mode: each core encodes the points it makes ----------------------
// Z^-1 on the wave: 2 (the default since round 4) = the divsteps with the
// operand updates spread over the lanes (wide_inv.h fe_invert_wave): configs[4]
// p50 0.2137 -> 0.2060 ms against 1 = z^(p-2) (~265 wave-wide products,
// profiles/r04k/ablat_wave_inversion.json), which was itself 12 us faster
// than the lane's divsteps inversion (0)
#ifndef OURO_WIDE_INV
#define OURO_WIDE_INV 2
#endif
__device__ __forceinline__ fe invert_wide(const fe& z) {
  if (OURO_WIDE_INV == 2) return fe_invert_wave(z);
  if (OURO_WIDE_INV) return fw_to_fe(fw_invert(fe_to_fw(z, lanes())));
  return fe_invert_vartime(z);
}
// the same for a wave-wide element (replicated rows)
__device__ __forceinline__ int32_t fw_invert_sel(int32_t z, const Lanes& L) {
  if (OURO_WIDE_INV == 2) return fe_to_fw(fe_invert_wave(fw_to_fe(z)), L);
  return fw_invert(z);
}
// canonical encoding of a p2 point (one inversion)
__device__ __forceinline__ void encode_p2(uint32_t enc[8], const ge_p2& P) {
  ge_encode_with_inv(enc, P.X, P.Y, invert_wide(P.Z));
}

// The whole V = [s]H - [c]Gamma on one wave: Elligator2's exponentiation on
// rows 0/2 and Gamma's decode on rows 1/3 at once, then one chain over the
// tables of H and -Gamma (s: 64 windows, c: 33).  H and V encoded with one
// inversion.  (Gamma's acceptance checks are the Gamma core's.)
template <class Tail>
__device__ __forceinline__ void vrf_v_full_wide(uint32_t Henc[8], uint32_t Venc[8],
                                                const uint32_t pk[8], const uint32_t pi[20],
                                                const Tail& alpha) {
  const Lanes L = lanes();
  uint32_t G[8], c[8], s_raw[8], s[8];
#pragma unroll
  for (int k = 0; k < 8; k++) {
    G[k] = pi[k];
    c[k] = k < 4 ? pi[8 + k] : 0u;
    s_raw[k] = pi[12 + k];
  }
  sc_reduce256(s, s_raw);
  uint32_t pre[9];
  pre[0] = 0x04u | (0x01u << 8) | (pk[0] << 16);
#pragma unroll
  for (int k = 1; k < 8; k++) pre[k] = (pk[k - 1] >> 16) | (pk[k] << 16);
  pre[8] = pk[7] >> 16;
  uint64_t Hs[8];
  sha512_prefixed<34>(Hs, pre, alpha, 32);
  uint32_t rw[16];
  sha512_digest_words(rw, Hs);
  rw[7] &= 0x7fffffffu;
  DecodePre dg;
  const fe tg = ge_decode_pre(dg, G);
  fe gpow;
  const ge_p3 H = elligator2_h_with(rw, [&](const fe& z) {
    const int32_t x = L.odd ? fe_to_fw(tg, L) : fe_to_fw(z, L);
    const int32_t y = fw_pow22523_rows(x);
    gpow = fw_to_fe(y, 1);
    return fw_to_fe(y, 0);
  });
  ge_p3 Gamma;
  ge_decode_post(&Gamma, dg, gpow, G, false);
  const int32_t d2 = d2_wide(L);
  TabW tH, tG;
  tab_build(tH, pw_from_p3(H, L), d2, L);
  tab_build(tG, pw_from_p3(ge_p3_neg(Gamma), L), d2, L);
  const ge_p2 V = pw_to_p2(pw_dsm<true, false>(tH, s, 64, tG, c, 33, s, nullptr, L));
  const fe zz = fe_mul(H.Z, V.Z);
  const fe inv = invert_wide(zz);
  ge_encode_with_inv(Henc, H.X, H.Y, fe_mul(inv, V.Z));
  ge_encode_with_inv(Venc, V.X, V.Y, fe_mul(inv, H.Z));
}

// canonical encodings from this row's affine coordinate of x and y (rows
// rx / ry of c): y with x's parity in bit 255 (ge25519.h ge_encode_with_inv)
__device__ __forceinline__ void enc_from_rows(uint32_t out[8], int32_t c, int rx, int ry) {
  uint32_t xw[8];
  fe_to_words(out, fw_to_fe(c, ry));
  fe_to_words(xw, fw_to_fe(c, rx));
  out[7] ^= (xw[0] & 1u) << 31;
}
// encode(P) for a wave-wide point: Z^-1 on the wave, then x and y as one
// layer of row products (rows 0 / 1)
__device__ __forceinline__ void encode1_wide(uint32_t enc[8], const pw& P) {
  const Lanes L = lanes();
  const int32_t zi = fw_invert_sel(P.Z, L);
  const int32_t c = fw_mul(L.odd ? P.Y : P.X, zi, L);
  if (OURO_ENC_ROWS) {  // x and y canonical in one vector pass (encode2_wide)
    uint32_t w[8];
    fe_to_words(w, fw_to_fe_own_row(c));
#pragma unroll
    for (int k = 0; k < 8; k++) enc[k] = (uint32_t)__builtin_amdgcn_readlane((int)w[k], 16);
    enc[7] ^= ((uint32_t)__builtin_amdgcn_readlane((int)w[0], 0) & 1u) << 31;
  } else {
    enc_from_rows(enc, c, 0, 1);
  }
}
// encode(H) and encode(V) with one inversion: 1 / (ZH ZV), then 1 / ZH and
// 1 / ZV (rows 0 / 1), then xH, yH, xV, yV (rows 0..3), all on the wave
__device__ __forceinline__ void encode2_wide(uint32_t Henc[8], uint32_t Venc[8], const pw& H,
                                             const pw& V) {
  const Lanes L = lanes();
  const int32_t inv = fw_invert_sel(fw_mul_rep(H.Z, V.Z, L), L);
  lstamp(6);
  const fw4 zi = fw_gather(fw_mul(inv, L.odd ? H.Z : V.Z, L));  // r0 = 1/ZH, r1 = 1/ZV
  const int32_t c = fw_mul(sel4(H.X, H.Y, V.X, V.Y, L), L.high ? zi.r1 : zi.r0, L);
  if (OURO_ENC_ROWS) {
    // all four coordinates canonical at once (each row its own), then read out
    uint32_t w[8];
    fe_to_words(w, fw_to_fe_own_row(c));
#pragma unroll
    for (int k = 0; k < 8; k++) {
      Henc[k] = (uint32_t)__builtin_amdgcn_readlane((int)w[k], 16);  // row 1: yH
      Venc[k] = (uint32_t)__builtin_amdgcn_readlane((int)w[k], 48);  // row 3: yV
    }
    Henc[7] ^= ((uint32_t)__builtin_amdgcn_readlane((int)w[0], 0) & 1u) << 31;   // xH's sign
    Venc[7] ^= ((uint32_t)__builtin_amdgcn_readlane((int)w[0], 32) & 1u) << 31;  // xV's sign
  } else {
    enc_from_rows(Henc, c, 0, 1);
    enc_from_rows(Venc, c, 2, 3);
  }
}

// The Gamma core of the split form in two parts: the acceptance checks and
// the V part -[c]Gamma (stored at `part`, a wave-wide point) first -- a VRF's
// combination waits for it -- then [8]Gamma and beta, which only the header's
// tail reads.  Returns the flag word; Gw keeps the decoded Gamma.
__device__ __forceinline__ int32_t vrf_gamma_part_wide(Slot part, pw& Gw, const uint32_t pi[20]) {
  const Lanes L = lanes();
  uint32_t G[8], c[8];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    G[i] = pi[i];
    c[i] = i < 4 ? pi[8 + i] : 0u;
  }
  ge_p3 Gamma;
  bool ok = ge_is_canonical(G);
  ok = ge_decode_wide(&Gamma, G, false) && ok;
  Gw = pw_from_p3(Gamma, L);
  TabW t;
  tab_build(t, pw_from_p3(ge_p3_neg(Gamma), L), d2_wide(L), L);
  st_pw(part, pw_dsm<false, false>(t, c, 33, t, c, 0, c, nullptr, L));
  return (ok ? kFlagOk : 0) | (fe_iszero(Gamma.X) ? kFlagGammaX0 : 0);
}
__device__ __forceinline__ void vrf_gamma_beta_part_wide(uint32_t beta[16], const pw& Gw) {
  const Lanes L = lanes();
  uint32_t enc[8];
  encode1_wide(enc, pw_dbl(pw_dbl(pw_dbl(Gw, L), L), L));
  vrf_beta(beta, enc);
}

// The Gamma core: acceptance checks, [8]Gamma, beta = SHA-512(suite || 0x03
// || encode([8]Gamma)) and the V half -[c]Gamma (`partial`); returns the flag
// word (with kFlagGammaX0)
// (split form: -[c]Gamma stored as a wave-wide point at `split` instead)
__device__ __forceinline__ int32_t vrf_gamma_beta_wide(uint32_t beta[16], ge_p2& partial,
                                                       const uint32_t pi[20],
                                                       const Slot* split = nullptr) {
  const Lanes L = lanes();
  uint32_t G[8], c[8];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    G[i] = pi[i];
    c[i] = i < 4 ? pi[8 + i] : 0u;
  }
  ge_p3 Gamma;
  bool ok = ge_is_canonical(G);
  ok = ge_decode_wide(&Gamma, G, false) && ok;
  const pw Gw = pw_from_p3(Gamma, L);
  const pw G8w = pw_dbl(pw_dbl(pw_dbl(Gw, L), L), L);
  uint32_t enc[8];
  encode_p2(enc, pw_to_p2(G8w));
  vrf_beta(beta, enc);
  TabW t;
  tab_build(t, pw_from_p3(ge_p3_neg(Gamma), L), d2_wide(L), L);
  const pw part = pw_dsm<false, false>(t, c, 33, t, c, 0, c, nullptr, L);
  if (split) st_pw(*split, part);
  else partial = pw_to_p2(part);
  return (ok ? kFlagOk : 0) | (fe_iszero(Gamma.X) ? kFlagGammaX0 : 0);
}

// The second of a VRF's V and Gamma cores to arrive: V = [s]H + (-[c]Gamma)
// from the record, H and V encoded with one inversion
__device__ __forceinline__ void vrf_combine_encode(Slot res, int which) {
  const int ptH = which ? kPtHl : kPtHe, ptV = which ? kPtVl : kPtVe;
  const ge_p2 H = ld_point_at(res + ptH * kPtWords);
  const ge_p2 V = ge_p2_add(ld_point_at(res + ptV * kPtWords),
                            ld_point_at(res + kLatPart + which * kPtWords));
  vstamp(5);
  const fe inv = invert_wide(fe_mul(H.Z, V.Z));
  uint32_t Henc[8], Venc[8];
  ge_encode_with_inv(Henc, H.X, H.Y, fe_mul(inv, V.Z));
  ge_encode_with_inv(Venc, V.X, V.Y, fe_mul(inv, H.Z));
  vstamp(6);
  if ((threadIdx.x & 63u) == 0) {
    st_words8(res + kLatEnc + 8 * (3 * which + 0), Henc);
    st_words8(res + kLatEnc + 8 * (3 * which + 2), Venc);
  }
}

// Arrival at a counter of `parties` waves: this wave's record stores are
// released, the counter bumped; true for the last party (then acquired).
// The counter word is tagged with the launch's generation (gen, 28 bits,
// never 0: bits 4..31; the arrivals in bits 0..3): an arrival that finds
// another generation's tag starts the count afresh, so a counter left
// mid-count by an earlier launch that never completed (or a zeroed one) can
// never make a header finish early with that launch's record contents --
// every core rewrites its record fields before it arrives.
// (A/B switch OURO_ARRIVE_RA: 1 = a release fence before the count and an
// acquire fence after it for the last party only, 0 = two full fences)
#ifndef OURO_ARRIVE_RA
#define OURO_ARRIVE_RA 1
#endif
__device__ __forceinline__ bool arrive_last(int32_t* ctr, uint32_t gen,
                                            uint32_t parties = kLatCores) {
  if (OURO_ARRIVE_RA) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  else __threadfence();
  uint32_t mine = 0;
  if ((threadIdx.x & 63u) == 0) {
    unsigned int* c = reinterpret_cast<unsigned int*>(ctr);
    const uint32_t tag = (gen & 0x0fffffffu) << 4;
    uint32_t cur = __hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (;;) {
      const uint32_t want = (cur & ~0xfu) == tag ? cur + 1u : (tag | 1u);
      const uint32_t prev = atomicCAS(c, cur, want);
      if (prev == cur) {
        mine = want & 0xfu;
        break;
      }
      cur = prev;
    }
  }
  mine = (uint32_t)__builtin_amdgcn_readlane((int)mine, 0);
  if (mine != parties) return false;
  if (OURO_ARRIVE_RA) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  else __threadfence();
  return true;
}

// Whether every other party of a `parties` counter has arrived in this
// launch (then acquired): the caller is the last without arriving, so it
// need not publish what it holds in registers -- no release of its own
// stores, no count (the counter is tagged, so the next launch starts it
// afresh).  A false answer changes nothing: the caller publishes and arrives.
// (A/B switch OURO_LAST_PEEK: 0 = always publish and arrive)
#ifndef OURO_LAST_PEEK
#define OURO_LAST_PEEK 1
#endif
__device__ __forceinline__ bool others_arrived(int32_t* ctr, uint32_t gen, uint32_t parties) {
  if (!OURO_LAST_PEEK) return false;
  uint32_t seen = 0;
  if ((threadIdx.x & 63u) == 0)
    seen = __hip_atomic_load(reinterpret_cast<unsigned int*>(ctr), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
  seen = (uint32_t)__builtin_amdgcn_readlane((int)seen, 0);
  if (seen != (((gen & 0x0fffffffu) << 4) | (parties - 1u))) return false;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  return true;
}

// ---- fused mode: an Ed25519 check over two waves ------------------------------
// The points item (encoding checks, both decodes: one exponentiation time) and
// the scalars item (SHA-512 of R || A || M -- five blocks for a KES body --,
// reduction, the lattice pair, b = c1 S) run at once; the second to arrive
// builds the tables and runs the chain (ed_chain).  Record words (Slot e):
// c0 0, c1 8, b 16, nw 24, c0_neg 25 | -A 28 (X, Y, Z, T at 12-word stride),
// -R 76, points ok 124, counter 125.
__device__ __forceinline__ void ed_points_item(Slot e, const uint32_t sig[16],
                                               const uint32_t pk[8], bool extra_ok) {
  uint32_t R[8], S[8];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    R[i] = sig[i];
    S[i] = sig[8 + i];
  }
  bool ok = ed25519_precheck(R, S, pk, false) && extra_ok;
  ge_p3 negA, negR;
  bool okA, okR;
  ge_decode_pair_wide(&negA, &okA, &negR, &okR, pk, R, true);
  ok = okA && ok;
  ok = ge_is_canonical(R) && ok;
  ok = okR && ok;
  ok = ok && !(fe_iszero(negR.X) && (R[7] >> 31) != 0);
  if ((threadIdx.x & 63u) == 0) {
    st_fe(e + 28, negA.X); st_fe(e + 40, negA.Y); st_fe(e + 52, negA.Z); st_fe(e + 64, negA.T);
    st_fe(e + 76, negR.X); st_fe(e + 88, negR.Y); st_fe(e + 100, negR.Z); st_fe(e + 112, negR.T);
    stg1(e.word(124), ok ? 1 : 0);
  }
}
// verify.h ed25519_scalars with SHA-512(R || A || M) on the whole wave
// (sha512.h sha512_prefixed_wave; messages beyond its block capacity hash on
// the lane).  A/B switch OURO_SHA_WAVE=0: the lane hash.
#ifndef OURO_SHA_WAVE
#define OURO_SHA_WAVE 1
#endif
template <class Tail>
__device__ __forceinline__ void ed25519_scalars_wave(HalfScalars& hs, uint32_t b[8],
                                                     const uint32_t R[8], const uint32_t S[8],
                                                     const uint32_t pk[8], const Tail& msg,
                                                     uint32_t mlen) {
  uint32_t pre[16];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    pre[i] = R[i];
    pre[8 + i] = pk[i];
  }
  uint64_t H[8];
  if (OURO_SHA_WAVE && ((64 + mlen + 17 + 127) >> 7) <= sha_wave_max_blocks<64>())
    sha512_prefixed_wave<64, 64>(H, pre, msg, mlen);
  else
    sha512_prefixed<64>(H, pre, msg, mlen);
  ed25519_scalars_from_digest(hs, b, H, S);
}

// tpraos.h vrf_challenge_ok for the two VRFs of a header at once, one per
// half-wave (sha512_prefixed_wave, two messages per wave)
__device__ __forceinline__ bool vrf_challenge_ok_wave(const uint32_t Henc[8], const uint32_t Genc[8],
                                                      const uint32_t Uenc[8], const uint32_t Venc[8],
                                                      const uint32_t c[4]) {
  if (!OURO_SHA_WAVE) return vrf_challenge_ok(Henc, Genc, Uenc, Venc, c);
  uint32_t hp[33];
  hp[0] = 0x04u | (0x02u << 8);
  pack_shifted(hp, 1, Henc);
  pack_shifted(hp, 9, Genc);
  pack_shifted(hp, 17, Uenc);
  pack_shifted(hp, 25, Venc);
  uint64_t Hc[8];
  sha512_prefixed_wave<130, 32>(Hc, hp, ShaNoTail{}, 0);
  uint32_t cw[16];
  sha512_digest_words(cw, Hc);
  bool ceq = true;
#pragma unroll
  for (int i = 0; i < 4; i++) ceq = ceq && cw[i] == c[i];
  return ceq;
}

template <class Tail>
__device__ __forceinline__ void ed_scalars_item(Slot e, const uint32_t sig[16], const uint32_t pk[8],
                                                const Tail& msg, uint32_t mlen) {
  uint32_t R[8], S[8], b[8];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    R[i] = sig[i];
    S[i] = sig[8 + i];
  }
  HalfScalars hs;
#if OURO_LAT_STAMPS
  {  // ed25519_scalars with phase stamps (5 SHA-512, 6 reduction, 7 lattice)
    uint32_t pre[16];
    for (int i = 0; i < 8; i++) {
      pre[i] = R[i];
      pre[8 + i] = pk[i];
    }
    uint64_t H[8];
    sha512_prefixed<64>(H, pre, msg, mlen);
    kstamp(5);
    uint32_t hw[16], h[8];
    sha512_digest_words(hw, H);
    sc_reduce512(h, hw);
    kstamp(6);
    ed25519_half_scalars(hs, h);
    kstamp(7);
    uint32_t prod[16];
    for (int i = 0; i < 16; i++) prod[i] = 0;
    for (int i = 0; i < 8; i++) {
      uint64_t carry = 0;
      for (int j = 0; j < 8; j++) {
        const uint64_t t = (uint64_t)hs.c1[i] * S[j] + prod[i + j] + carry;
        prod[i + j] = (uint32_t)t;
        carry = t >> 32;
      }
      prod[i + 8] = (uint32_t)carry;
    }
    sc_reduce512(b, prod);
  }
#else
  ed25519_scalars_wave(hs, b, R, S, pk, msg, mlen);
#endif
  int nw = (hs.bits + 4) >> 2;
  nw = nw < 1 ? 1 : (nw > 64 ? 64 : nw);
  if ((threadIdx.x & 63u) == 0) {
    st_words8(e + 0, hs.c0);
    st_words8(e + 8, hs.c1);
    st_words8(e + 16, b);
    stg1(e.word(24), nw);
    stg1(e.word(25), hs.c0_neg ? 1 : 0);
  }
}
// [|c0|](+-A) + [c1](-R) + [b]B == O from the record (the ed25519_verify_wide
// equation)
__device__ __forceinline__ bool ed_chain(Slot e, const uint16_t* bw) {
  const Lanes L = lanes();
  uint32_t c0[8], c1[8], b[8];
  ld_words8(c0, e + 0);
  ld_words8(c1, e + 8);
  ld_words8(b, e + 16);
  const int nw = ldg1(e.word(24));
  const bool c0_neg = ldg1(e.word(25)) != 0;
  const ge_p3 negA{ld_fe(e + 28), ld_fe(e + 40), ld_fe(e + 52), ld_fe(e + 64)};
  const ge_p3 negR{ld_fe(e + 76), ld_fe(e + 88), ld_fe(e + 100), ld_fe(e + 112)};
  const bool ok = ldg1(e.word(124)) != 0;
  const int32_t d2 = d2_wide(L);
  TabW t1, t2;
  tab_build(t1, pw_from_p3(c0_neg ? ge_p3_neg(negA) : negA, L), d2, L);
  tab_build(t2, pw_from_p3(negR, L), d2, L);
  const pw Q = pw_dsm<true, true>(t1, c0, nw, t2, c1, nw, b, bw, L);
  return ok && pw_is_identity(Q);
}

// ---- fused mode, split form (kernels_lat.hip OURO_LAT_SPLIT) -------------------
// Each Ed25519 check over THREE waves and without the lattice pair: libsodium
// accepts iff Q = [S]B - [h]A - R == O (R_bytes canonical and decodable, x = 0
// only with sign 0; h = SHA-512(R || A || M) mod L; the same precondition as
// the half-size equation), and with h's signed width-4 windows 0..31 / 32..63
// and S's 16-bit digits 0..7 / 8..15 (each recoded as one number)
//   X = [h windows 0..31](-A) + [S digits 0..7]B           (128-bit chain)
//   Y = [h windows 32..63](-A128) + [S digits 8..15]B'     (A128 = 2^128 A, B' = 2^128 B)
//   Q = X + Y + (-R).
// The points item P (checks, A and R decoded), the scalars item S (the hash)
// and the doubling item D (A decoded again, 128 doublings to -A128) start
// together; X runs on the second of P and S to arrive, Y on the second of D
// and S, and the second chain to finish adds the three points and compares
// with the identity.  No wave ever waits: whoever completes a pair runs what
// the pair enables.  Record (Slot e, kEdWords): h 0, S 8, points ok 16,
// counters 17 (X), 18 (Y), 19 (both chains done), wave-wide points -A 32,
// -R 96, -A128 160, X 224, Y 288.
constexpr int kEsH = 0, kEsS = 8, kEsOk = 16, kEsCx = 17, kEsCy = 18, kEsCd = 19;
constexpr int kEsA = 32, kEsR = kEsA + kPwWords, kEsA128 = kEsR + kPwWords;
constexpr int kEsX = kEsA128 + kPwWords, kEsY = kEsX + kPwWords;
static_assert(kEsY + kPwWords <= kEdWords, "Ed record");

__device__ __forceinline__ void eds_points(Slot e, const uint32_t sig[16], const uint32_t pk[8],
                                           bool extra_ok) {
  const Lanes L = lanes();
  uint32_t R[8], S[8];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    R[i] = sig[i];
    S[i] = sig[8 + i];
  }
  bool ok = ed25519_precheck(R, S, pk, false) && extra_ok;
  ge_p3 negA, negR;
  bool okA, okR;
  ge_decode_pair_wide(&negA, &okA, &negR, &okR, pk, R, true);
  ok = okA && ok;
  ok = ge_is_canonical(R) && ok;
  ok = okR && ok;
  ok = ok && !(fe_iszero(negR.X) && (R[7] >> 31) != 0);
  st_pw(e + kEsA, pw_from_p3(negA, L));
  st_pw(e + kEsR, pw_from_p3(negR, L));
  if ((threadIdx.x & 63u) == 0) stg1(e.word(kEsOk), ok ? 1 : 0);
}

template <class Tail>
__device__ __forceinline__ void eds_scalars(Slot e, const uint32_t sig[16], const uint32_t pk[8],
                                            const Tail& msg, uint32_t mlen) {
  uint32_t pre[16];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    pre[i] = sig[i];
    pre[8 + i] = pk[i];
  }
  uint64_t H[8];
  if (OURO_SHA_WAVE && ((64 + mlen + 17 + 127) >> 7) <= sha_wave_max_blocks<64>())
    sha512_prefixed_wave<64, 64>(H, pre, msg, mlen);
  else
    sha512_prefixed<64>(H, pre, msg, mlen);
  uint32_t hw[16], h[8];
  sha512_digest_words(hw, H);
  sc_reduce512(h, hw);
  if ((threadIdx.x & 63u) == 0) {
    st_words8(e + kEsH, h);
    st_words8(e + kEsS, sig + 8);
  }
}

// -A128 = [2^128](-A), A decoded once more on this wave
__device__ __forceinline__ void eds_double(Slot e, const uint32_t pk[8]) {
  const Lanes L = lanes();
  ge_p3 negA;
  ge_decode_wide(&negA, pk, true);
  pw P = pw_from_p3(negA, L);
#pragma unroll 1
  for (int k = 0; k < 128; k++) P = pw_dbl(P, L);
  st_pw(e + kEsA128, P);
}

// h >> 128 plus the carry h's signed windows 0..31 hand to window 32
OURO_FI void sc_high_half_with_carry(uint32_t hh[8], const uint32_t h[8]) {
  const uint32_t cin = (uint32_t)(sc_recode_carries<4, 64>(h) >> 32) & 1u;
  uint64_t c = cin;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    c += h[4 + i];
    hh[i] = (uint32_t)c;
    c >>= 32;
    hh[4 + i] = 0;
  }
}

__device__ __forceinline__ void eds_chain(Slot e, const uint16_t* bw, bool high) {
  const Lanes L = lanes();
  uint32_t h[8], S[8], a[8];
  ld_words8(h, e + kEsH);
  ld_words8(S, e + kEsS);
  TabW t;
  tab_build(t, ld_pw(e + (high ? kEsA128 : kEsA)), d2_wide(L), L);
  if (high) {
    sc_high_half_with_carry(a, h);
    st_pw(e + kEsY, pw_dsm<false, true, 2>(t, a, 32, t, a, 0, S, bw, L));
  } else {
    st_pw(e + kEsX, pw_dsm<false, true, 1>(t, h, 32, t, h, 0, S, bw, L));
  }
}

__device__ __forceinline__ bool eds_combine(Slot e) {
  const Lanes L = lanes();
  const int32_t d2 = d2_wide(L);
  const pw Q = pw_add_p3(pw_add_p3(ld_pw(e + kEsX), ld_pw(e + kEsY), d2, L), ld_pw(e + kEsR), d2, L);
  return ldg1(e.word(kEsOk)) != 0 && pw_is_identity(Q);
}

// The windows at which the split form cuts s between its V items.  V2 pays
// 4 K doublings to 2^(4K) H before its chain over windows K..63, so its time
// is ~253 doublings plus the additions of its windows whatever K, while V's
// chain grows with K: K = 32 (bit 128, rounds 3--4) left V2 32 additions
// that V did not wait for; 48 ends the two chains together (profiles/r05d).
// OURO_LAT_V3 = 1 cuts once more, at K2: V2 then takes windows K..K2-1 and a
// V3 item (H again, 4 K2 doublings) windows K2..63, which takes all but a few
// additions off the item that does the ~253 doublings.
#ifndef OURO_LAT_VWIN
#define OURO_LAT_VWIN (OURO_LAT_V3 ? 49 : 48)
#endif
#ifndef OURO_LAT_VWIN2
#define OURO_LAT_VWIN2 61
#endif
static_assert(OURO_LAT_VWIN >= 8 && OURO_LAT_VWIN <= 60, "V / V2 split window");
static_assert(!OURO_LAT_V3 || (OURO_LAT_VWIN2 > OURO_LAT_VWIN && OURO_LAT_VWIN2 <= 63),
              "V2 / V3 split window");

// (s >> 4K) plus the carry s's signed windows 0..K-1 hand to window K: the
// windows below K recoded from the whole s plus [that]·16^K are s exactly
// (pw_dsm recodes its scalar whole and adds only the windows it is given)
template <int K>
OURO_FI void sc_high_from_window(uint32_t hh[8], const uint32_t s[8]) {
  const uint32_t cin = (uint32_t)(sc_recode_carries<4, 64>(s) >> K) & 1u;
  constexpr int kW = (4 * K) >> 5, kB = (4 * K) & 31;
  uint64_t c = cin;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint32_t w = i + kW < 8 ? s[i + kW] >> kB : 0u;
    if (kB != 0 && i + kW + 1 < 8) w |= s[i + kW + 1] << ((32 - kB) & 31);
    c += w;
    hh[i] = (uint32_t)c;
    c >>= 32;
  }
}

// V = [s]H - [c]Gamma over THREE waves: [s windows 0..K-1]H (the V item,
// part 0), [s windows K..63](2^(4K) H) (the V2 item, part 1: H again, then 4K
// doublings; K = OURO_LAT_VWIN) and -[c]Gamma (the Gamma item); the last of
// the three adds them and encodes H and V.  With OURO_LAT_V3 part 1 stops at
// window K2 and part 2 (the V3 item) does [(s >> 4K) windows K2-K..](2^(4 K2) H).
// Record per VRF (kLatVsplit + 4 kPwWords which): H, the parts 0 and 1,
// -[c]Gamma, as wave-wide points; part 2 at kLatV3 + kPwWords which.
template <class Tail>
__device__ __forceinline__ pw vrf_sh_split(Slot v, Slot v3, const uint32_t pk[8],
                                           const uint32_t pi[20], const Tail& alpha, int part,
                                           bool store = true) {
  const Lanes L = lanes();
  uint32_t s_raw[8], s[8];
#pragma unroll
  for (int k = 0; k < 8; k++) s_raw[k] = pi[12 + k];
  sc_reduce256(s, s_raw);
  uint32_t pre[9];
  pre[0] = 0x04u | (0x01u << 8) | (pk[0] << 16);
#pragma unroll
  for (int k = 1; k < 8; k++) pre[k] = (pk[k - 1] >> 16) | (pk[k] << 16);
  pre[8] = pk[7] >> 16;
  uint64_t Hs[8];
  sha512_prefixed<34>(Hs, pre, alpha, 32);
  uint32_t rw[16];
  sha512_digest_words(rw, Hs);
  rw[7] &= 0x7fffffffu;
  lstamp(12);
  pw Hw;
  if (OURO_ELL2_WIDE) {
    Hw = elligator2_wide(rw, L);
  } else {
    auto pw22523 = [](const fe& z) {
      lstamp(13);
      const fe r = pow22523_wide(z);
      lstamp(14);
      return r;
    };
    const ge_p3 P = elligator2_h_with<decltype(pw22523), false>(rw, pw22523);
    Hw = pw_dbl(pw_dbl(pw_dbl(pw_from_p3(P, L), L), L), L);
  }
  lstamp(15);
  constexpr int K = OURO_LAT_VWIN, K2 = OURO_LAT_V3 ? OURO_LAT_VWIN2 : 64;
  int nw = K;
  if (part == 0) {
    st_pw(v, Hw);
  } else {
    const int dbl = 4 * (part == 1 ? K : K2);
#pragma unroll 1
    for (int k = 0; k < dbl; k++) Hw = pw_dbl(Hw, L);
    uint32_t hh[8];
    sc_high_from_window<K>(hh, s);
    if (OURO_LAT_V3 && part == 2) {
      sc_high_from_window<(K2 - K) & 63>(s, hh);
      nw = 64 - K2;
    } else {
#pragma unroll
      for (int k = 0; k < 8; k++) s[k] = hh[k];
      nw = K2 - K;
    }
  }
  lstamp(16);
  TabW tab;
  tab_build(tab, Hw, d2_wide(L), L);
  lstamp(17);
  const pw R = pw_dsm<false, false>(tab, s, nw, tab, s, 0, s, nullptr, L);
  if (store) st_pw(part == 2 ? v3 : v + (part + 1) * kPwWords, R);
  lstamp(18);
  return R;
}

// the last of a VRF's V, V2 (V3) and Gamma items: V = the parts, H and V
// encoded with one inversion
// (hi: the V2 part in registers when the V2 item combines without having
// stored it, else read from the record)
__device__ __forceinline__ void vrf_split_combine_encode(Slot res, int which,
                                                         const pw* hi = nullptr) {
  const Lanes L = lanes();
  const Slot v = res + kLatVsplit + 4 * kPwWords * which;
  const int32_t d2 = d2_wide(L);
  lstamp(4);
  pw Vw = pw_add_p3(pw_add_p3(ld_pw(v + kPwWords), hi ? *hi : ld_pw(v + 2 * kPwWords), d2, L),
                    ld_pw(v + 3 * kPwWords), d2, L);
  if (OURO_LAT_V3) Vw = pw_add_p3(Vw, ld_pw(res + kLatV3 + kPwWords * which), d2, L);
  lstamp(5);
  uint32_t Henc[8], Venc[8];
  encode2_wide(Henc, Venc, ld_pw(v), Vw);
  lstamp(7);
  if ((threadIdx.x & 63u) == 0) {
    st_words8(res + kLatEnc + 8 * (3 * which + 0), Henc);
    st_words8(res + kLatEnc + 8 * (3 * which + 2), Venc);
  }
}

// The eta nonce's candidates (tpraos.h hdr_eta_nonce): Blake2b-256 of the
// claimed eta output when the batch carries it, else of this core's beta --
// the nonce if the VRF verifies -- and of 64 zero bytes (if it does not).
// Lanes 0 / 1 hash one each; stored for the tail to pick.
__device__ __forceinline__ void eta_nonce_candidates(const ouro_tpraos_batch& b, size_t i,
                                                     uint32_t opts, Slot res,
                                                     const uint32_t beta[16]) {
  const uint32_t lane = threadIdx.x & 63u;
  uint32_t in[16], h[8];
  if (opts & kOptEtaClaim) {
    ld_words(in, b.eta_output + 64 * i, 4);
  } else {
#pragma unroll
    for (int k = 0; k < 16; k++) in[k] = beta[k];
  }
#pragma unroll
  for (int k = 0; k < 16; k++) in[k] = lane == 1 ? 0u : in[k];
  blake2b256_64(h, in);
  if (lane < 2) st_words8(res + kLatNonce + 8 * (int)lane, h);
}

// The tail of header i on the last core's wave: both VRFs at once (lanes
// 0..31 the eta VRF, 32..63 the leader VRF) -- challenge check from the
// record's encodings, beta, claimed-output bits, the eta nonce -- and the
// verdict.  Same bits and outputs
// as k_tpraos_finish (tpraos.h vrf_finish_split).
#ifndef OURO_TAIL_PRELOAD
#define OURO_TAIL_PRELOAD 1
#endif
__device__ __forceinline__ void hdr_tail_wide(const ouro_tpraos_batch& b, size_t i, uint32_t opts,
                                              Slot res, uint8_t* verdict, uint8_t* beta_eta,
                                              uint8_t* beta_leader) {
  const uint32_t lane = threadIdx.x & 63u;
  const int which = (int)(lane >> 5);
  auto fl = [&](int core) { return ldg1(res.word(kResFlags + core)); };
  const int32_t fu = fl(which ? kCoreUl : kCoreUe), fv = fl(which ? kCoreVl : kCoreVe);
  const int32_t fg = fl(which ? kCoreGl : kCoreGe);
  uint32_t pi[20], Henc[8], Uenc[8], Venc[8], Genc[8], c[4], beta[16];
  ld_words(pi, (which ? b.leader_proof : b.eta_proof) + 80 * i, 5);
  ld_words8(Henc, res + kLatEnc + 8 * (3 * which + 0));
  ld_words8(Uenc, res + kLatEnc + 8 * (3 * which + 1));
  ld_words8(Venc, res + kLatEnc + 8 * (3 * which + 2));
#pragma unroll
  for (int k = 0; k < 8; k++) Genc[k] = pi[k];
  if (fg & kFlagGammaX0) Genc[7] &= 0x7fffffffu;
#pragma unroll
  for (int k = 0; k < 4; k++) c[k] = pi[8 + k];
  // everything the verdict needs besides the challenge, loaded before it so
  // the loads' latency hides behind the hash (OURO_TAIL_PRELOAD; A/B)
  uint32_t cl[16];
  int32_t focert = 0, fkes = 0;
  const bool claim = (opts & (which ? kOptLeaderClaim : kOptEtaClaim)) != 0;
  if (OURO_TAIL_PRELOAD) {
    ld_words8(beta, res + kLatBeta + 16 * which);
    ld_words8(beta + 8, res + kLatBeta + 16 * which + 8);
    if (claim) ld_words(cl, (which ? b.leader_output : b.eta_output) + 64 * i, 4);
    focert = fl(kCoreOcert);
    fkes = fl(kCoreKes);
  }
  // the eta nonce's two candidates (the eta Gamma core's, wide_cores.h
  // eta_nonce_candidates): which one depends on ok
  uint32_t n0[8], n1[8];
  if (OURO_TAIL_PRELOAD && (opts & kOptEtaNonce)) {
    ld_words8(n0, res + kLatNonce);
    ld_words8(n1, res + kLatNonce + 8);
  }
  lstamp(9);
  const bool ceq = vrf_challenge_ok_wave(Henc, Genc, Uenc, Venc, c);
  lstamp(10);
  const bool ok = (fu & fv & fg & kFlagOk) && ceq;
  if (!OURO_TAIL_PRELOAD) {
    ld_words8(beta, res + kLatBeta + 16 * which);
    ld_words8(beta + 8, res + kLatBeta + 16 * which + 8);
  }
#pragma unroll
  for (int k = 0; k < 16; k++) beta[k] = ok ? beta[k] : 0u;
  uint32_t bit = ok ? (which ? 0x08u : 0x04u) : 0u;
  if (OURO_TAIL_PRELOAD) {
    if (ok && claim) {
      uint32_t diff = 0;
#pragma unroll
      for (int k = 0; k < 16; k++) diff |= cl[k] ^ beta[k];
      if (!diff) bit |= which ? 0x20u : 0x10u;
    }
  } else {
    bit |= hdr_claim_bit(b, i, opts, which, ok, beta);
  }
  if (!sc_is_canonical(pi + 12)) bit |= which ? OURO_HDR_LEADER_S_UNREDUCED : OURO_HDR_ETA_S_UNREDUCED;
  uint8_t* dst = which ? beta_leader : beta_eta;
  if ((lane & 31u) == 0 && dst) st_words(dst + 64 * i, beta, 4);
  // the eta nonce: the candidate the eta Gamma core hashed (claimed output, or
  // beta when the proof verified; Blake2b of zeros when it did not)
  if (lane == 0 && (opts & kOptEtaNonce)) {
    const bool pick0 = (opts & kOptEtaClaim) || ok;
    uint32_t h[8];
    if (OURO_TAIL_PRELOAD) {
#pragma unroll
      for (int k = 0; k < 8; k++) h[k] = pick0 ? n0[k] : n1[k];
    } else {
      ld_words8(h, res + kLatNonce + (pick0 ? 0 : 8));
    }
    st_words(b.eta_nonce + 32 * i, h, 2);
  }
  const uint32_t other = (uint32_t)__builtin_amdgcn_readlane((int)bit, 32);
  if (lane == 0) {
    uint32_t v = bit | other;
    if ((OURO_TAIL_PRELOAD ? focert : fl(kCoreOcert)) & kFlagOk) v |= 0x01u;
    if ((OURO_TAIL_PRELOAD ? fkes : fl(kCoreKes)) & kFlagOk) v |= 0x02u;
    verdict[i] = (uint8_t)v;
  }
}

}  // namespace wide
#endif
}  // namespace ouro
