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

namespace ouro {
#if defined(__HIP_DEVICE_COMPILE__)
namespace wide {

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
  const int32_t y = fw_pow22523(x);
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

// verify.h ed25519_verify_lane (libsodium 1.0.18 rules through the half-size
// equation) on one wave
template <class Tail>
__device__ __forceinline__ bool ed25519_verify_wide(const uint32_t sig[16], const uint32_t pk[8],
                                                    const Tail& msg, uint32_t mlen,
                                                    const uint16_t* bw) {
  const Lanes L = lanes();
  uint32_t R[8], S[8];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    R[i] = sig[i];
    S[i] = sig[8 + i];
  }
  bool ok = ed25519_precheck(R, S, pk, false);
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

template <class Tail>
__device__ __forceinline__ bool sum6kes_verify_wide(const uint32_t vk[8], uint32_t t,
                                                    const uint32_t* sigw, const Tail& msg,
                                                    uint32_t mlen, const uint16_t* bw) {
  uint32_t cur[8], sig[16];
  const bool ok = sum6kes_walk(cur, sig, vk, t, sigw);
  const bool leaf = ed25519_verify_wide(sig, cur, msg, mlen, bw);
  return ok && leaf;
}

// tpraos.h vrf_u_core: U = [s]B - [c]Y (Y decoded and checked here)
__device__ __forceinline__ bool vrf_u_wide(ge_p2& U, const uint32_t pk[8], const uint32_t pi[20],
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
  U = pw_to_p2(pw_dsm<false, true>(t, c, 33, t, c, 0, s, bw, L));
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
  sha512_prefixed<34>(Hs, pre, alpha, 32);
  uint32_t rw[16];
  sha512_digest_words(rw, Hs);
  rw[7] &= 0x7fffffffu;
  H = elligator2_h_with(rw, [](const fe& z) { return pow22523_wide(z); });
  TabW tab;
  tab_build(tab, pw_from_p3(H, L), d2_wide(L), L);
  V = pw_to_p2(pw_scalarmult(tab, s, L));
}

}  // namespace wide
#endif
}  // namespace ouro
