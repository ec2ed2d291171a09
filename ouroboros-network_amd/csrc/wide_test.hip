// wide_test.hip -- TEST-ONLY: the wave-wide arithmetic of wide.h checked
// against the lane-local routines it replaces (fe25519.h / ge25519.h), on the
// device, one wave per case.  tests/test_gpu_wide.py drives it; the product
// library does not contain this file.
#include <hip/hip_runtime.h>

#include <vector>

#include "verify.h"
#include "wide_cores.h"

using namespace ouro;

namespace {

__device__ uint64_t mix64(uint64_t z) {
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
__device__ void rand_words(uint32_t w[8], uint64_t seed, uint64_t tag) {
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const uint64_t v = mix64(seed * 0x100000001b3ull + tag * 131 + k);
    w[2 * k] = (uint32_t)v;
    w[2 * k + 1] = (uint32_t)(v >> 32);
  }
}
__device__ bool same_fe(const fe& a, const fe& b) {
  uint32_t x[8], y[8];
  fe_to_words(x, a);
  fe_to_words(y, b);
  uint32_t d = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) d |= x[k] ^ y[k];
  return d == 0;
}
__device__ void enc_p3(uint32_t e[8], const fe& X, const fe& Y, const fe& Z) {
  ge_encode_with_inv(e, X, Y, fe_invert(Z));
}
#if defined(__HIP_DEVICE_COMPILE__)
__device__ bool same_point(const ge_p3& P, const wide::pw& W) {
  uint32_t a[8], b[8];
  enc_p3(a, P.X, P.Y, P.Z);
  enc_p3(b, wide::fw_to_fe(W.X), wide::fw_to_fe(W.Y), wide::fw_to_fe(W.Z));
  uint32_t d = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) d |= a[k] ^ b[k];
  // T consistent: X Y = Z T
  const fe xy = fe_mul(wide::fw_to_fe(W.X), wide::fw_to_fe(W.Y));
  const fe zt = fe_mul(wide::fw_to_fe(W.Z), wide::fw_to_fe(W.T));
  return d == 0 && same_fe(xy, zt);
}
#endif

constexpr int kTests = 10;

// out[wave * kTests + t] = 1 when test t passed; dbg (wave 0): fw_mul's
// sixteen row-0 limbs, then the expected canonical words
#ifndef WT_BOUNDS
#define WT_BOUNDS 64
#endif
__global__ void __launch_bounds__(WT_BOUNDS) k_wide_selftest(uint64_t seed, int32_t* out, int32_t* dbg) {
#if defined(__HIP_DEVICE_COMPILE__)
  using namespace wide;
  const Lanes L = lanes();
  const uint64_t wv = blockIdx.x;
  const uint64_t sd = seed ^ (wv << 20);
  uint32_t wa[8], wb[8], wr[8];
  rand_words(wa, sd, 1);
  rand_words(wb, sd, 2);
  rand_words(wr, sd, 3);
  wa[7] &= 0x7fffffffu;
  wb[7] &= 0x7fffffffu;
  wr[7] &= 0x7fffffffu;
  if (wv == 1) {  // edge: p - 1 and 0
    for (int k = 0; k < 8; k++) { wa[k] = 0xffffffffu; wb[k] = 0u; }
    wa[0] = 0xffffffecu;
    wa[7] = 0x7fffffffu;
  }
  if (wv == 2) {  // edge: p - 1 squared, 2^255 - 20 times 2^255 - 20
    for (int k = 0; k < 8; k++) wa[k] = wb[k] = 0xffffffffu;
    wa[0] = wb[0] = 0xffffffecu;
    wa[7] = wb[7] = 0x7fffffffu;
  }
  const fe a = fe_from_words(wa), b = fe_from_words(wb);
  int32_t res[kTests];
  // 0: conversion round trip
  res[0] = same_fe(fw_to_fe(fe_to_fw(a, L)), a) && same_fe(fw_to_fe(fe_to_fw(b, L)), b);
  // 1: product
  const int32_t m = fw_mul(fe_to_fw(a, L), fe_to_fw(b, L), L);
  res[1] = same_fe(fw_to_fe(m), fe_mul(a, b));
  if (wv == 0 && threadIdx.x < 16) {
    dbg[threadIdx.x] = m;
    uint32_t e[8];
    fe_to_words(e, fe_mul(a, b));
    if (threadIdx.x < 8) dbg[16 + threadIdx.x] = (int32_t)e[threadIdx.x];
  }
  // 2: square, and a chain of 20 squarings (bounds stay closed)
  int32_t sq = fw_sq(fe_to_fw(a, L), L);
  fe sq_ref = fe_sq(a);
  bool ok = same_fe(fw_to_fe(sq), sq_ref);
  for (int k = 0; k < 20; k++) {
    sq = fw_sq(sq, L);
    sq_ref = fe_sq(sq_ref);
  }
  res[2] = ok && same_fe(fw_to_fe(sq), sq_ref);
  // 3: z^(2^252 - 3)
  // (and z^(p - 2), the wave-wide inversion)
  // (and the inversion by divsteps with lane-parallel updates, wide_inv.h,
  // on a, b and the edges 0, 1, p - 1 and 2^255 - 1 = p + 18, unreduced)
  uint32_t ew[4][8] = {{0}, {1}, {0xffffffecu}, {0xffffffffu}};
#pragma unroll
  for (int k = 1; k < 8; k++) {
    ew[2][k] = k == 7 ? 0x7fffffffu : 0xffffffffu;
    ew[3][k] = k == 7 ? 0x7fffffffu : 0xffffffffu;
  }
  bool inv_ok = same_fe(fe_invert_wave(a), fe_invert(a)) && same_fe(fe_invert_wave(b), fe_invert(b));
#pragma unroll 1
  for (int k = 0; k < 4; k++) {
    const fe z = fe_from_words(ew[k]);
    inv_ok = inv_ok && same_fe(fe_invert_wave(z), fe_invert(z));
  }
  res[3] = same_fe(fw_to_fe(fw_pow22523(fe_to_fw(a, L))), fe_pow22523(a)) &&
           same_fe(fw_to_fe(fw_invert(fe_to_fw(b, L))), fe_invert(b)) && inv_ok;
  // points: Elligator2 images
  const ge_p3 P = elligator2_h(wa), Q = elligator2_h(wb);
  const pw Pw = pw_from_p3(P, L), Qw = pw_from_p3(Q, L);
  const int32_t d2 = fe_to_fw(fe_d2(), L);
  // 4: doubling (twice, the second from a wide result)
  const ge_p3 P2 = ge_p1p1_to_p3(ge_p3_dbl(P));
  const ge_p3 P4 = ge_p1p1_to_p3(ge_p3_dbl(P2));
  const pw P2w = pw_dbl(Pw, L);
  res[4] = same_point(P2, P2w) && same_point(P4, pw_dbl(P2w, L));
  // 5: P + Q and P - Q, then (P + Q) + (P + Q) via add
  const ge_cached Qc = ge_p3_to_cached(Q);
  const cw qw = pw_cached(Qw, d2, L);
  const ge_p3 S = ge_p1p1_to_p3(ge_add_cached(P, Qc, false));
  const ge_p3 D = ge_p1p1_to_p3(ge_add_cached(P, Qc, true));
  const pw Sw = pw_add(Pw, qw.pos, L);
  const pw Dw = pw_add(Pw, qw.neg, L);
  const cw sw = pw_cached(Sw, d2, L);
  const ge_p3 SS = ge_p1p1_to_p3(ge_add_cached(S, ge_p3_to_cached(S), false));
  res[5] = same_point(S, Sw) && same_point(D, Dw) && same_point(SS, pw_add(Sw, sw.pos, L));
  // 6: [s]P, s reduced mod L, against double-and-add on the lane
  uint32_t s[8];
  sc_reduce256(s, wr);
  TabW tab;
  tab_build(tab, Pw, d2, L);
  const pw R = pw_scalarmult(tab, s, L);
  ge_p3 acc = ge_p3_identity();
  const ge_cached Pc = ge_p3_to_cached(P);
  for (int bit = 252; bit >= 0; bit--) {
    acc = ge_p1p1_to_p3(ge_p3_dbl(acc));
    if ((s[bit >> 5] >> (bit & 31)) & 1u) acc = ge_p1p1_to_p3(ge_add_cached(acc, Pc, false));
  }
  res[6] = same_point(acc, R);
  // 7: the identity through an addition and a doubling
  const pw I = pw_identity(L);
  res[7] = same_point(P, pw_add(I, pw_cached(Pw, d2, L).pos, L)) &&
           same_point(ge_p3_identity(), pw_dbl(I, L));
  // 8, 9: the latency mode's [s]H item (wide_vrf.h) against the lane
  // routines: H = Elligator2(SHA-512(suite || 0x01 || pk || alpha)), [s]H
  {
    uint32_t pk[8], pi[20];
    rand_words(pk, sd, 4);
    rand_words(pi, sd, 5);
    rand_words(pi + 8, sd, 6);
    rand_words(pi + 12, sd, 7);
    SeedMsg alpha;
    rand_words(alpha.w, sd, 8);
    ge_p3 Hw;
    ge_p2 Vw;
    vrf_sh(Hw, Vw, pk, pi, alpha);
    uint32_t pre[9];
    pre[0] = 0x04u | (0x01u << 8) | (pk[0] << 16);
    for (int k = 1; k < 8; k++) pre[k] = (pk[k - 1] >> 16) | (pk[k] << 16);
    pre[8] = pk[7] >> 16;
    uint64_t Hs[8];
    sha512_prefixed<34>(Hs, pre, alpha, 32);
    uint32_t rw[16];
    sha512_digest_words(rw, Hs);
    rw[7] &= 0x7fffffffu;
    const ge_p3 Href = elligator2_h(rw);
    uint32_t e1[8], e2[8];
    enc_p3(e1, Href.X, Href.Y, Href.Z);
    enc_p3(e2, Hw.X, Hw.Y, Hw.Z);
    uint32_t dd = 0;
    for (int k = 0; k < 8; k++) dd |= e1[k] ^ e2[k];
    res[8] = dd == 0;
    uint32_t sv[8];
    sc_reduce256(sv, pi + 12);
    ge_p3 acc2 = ge_p3_identity();
    const ge_cached Hc = ge_p3_to_cached(Href);
    for (int bit = 252; bit >= 0; bit--) {
      acc2 = ge_p1p1_to_p3(ge_p3_dbl(acc2));
      if ((sv[bit >> 5] >> (bit & 31)) & 1u) acc2 = ge_p1p1_to_p3(ge_add_cached(acc2, Hc, false));
    }
    enc_p3(e1, acc2.X, acc2.Y, acc2.Z);
    enc_p3(e2, Vw.X, Vw.Y, Vw.Z);
    dd = 0;
    for (int k = 0; k < 8; k++) dd |= e1[k] ^ e2[k];
    res[9] = dd == 0;
  }
  if (threadIdx.x == 0)
    for (int t = 0; t < kTests; t++) out[wv * kTests + t] = res[t];
#endif
}

// timing probe of the wave inversion (wide_inv.h): each wave inverts a
// chain of `iters` elements (z <- 1 / z + 1) with or without the early exit;
// out[2 wave] = s_memrealtime ticks (100 MHz) for the chain, out[2 wave + 1]
// = the last result's low word (keeps the chain live)
template <bool kEarly, int kCap, bool kSel, bool kVec = false>
__global__ void __launch_bounds__(64) k_inv_timing(uint64_t seed, int iters,
                                                  unsigned long long* out) {
#if defined(__HIP_DEVICE_COMPILE__)
  uint32_t w[8];
  rand_words(w, seed ^ ((uint64_t)blockIdx.x << 20), 7);
  w[7] &= 0x7fffffffu;
  fe z = fe_from_words(w);
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
#pragma unroll 1
  for (int k = 0; k < iters; k++)
    z = fe_carry(fe_add(fe_invert_wave<kEarly, kCap, kSel, kVec>(z), fe_one()));
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  uint32_t e[8];
  fe_to_words(e, z);
  if (threadIdx.x == 0) {
    out[2 * blockIdx.x] = t1 - t0;
    out[2 * blockIdx.x + 1] = e[0];
  }
#endif
}

// the same chain with only the batches' 30-divstep matrices (modinv.h
// sgcd_divsteps30 on the low words, f / g advanced by the matrix mod 2^32):
// what the wave inversion's scalar part costs without the limb updates
template <int kCap, bool kSel, bool kVec = false, bool kSpec = false>
__global__ void __launch_bounds__(64) k_divsteps_timing(uint64_t seed, int iters,
                                                       unsigned long long* out) {
#if defined(__HIP_DEVICE_COMPILE__)
  uint32_t w[8];
  rand_words(w, seed ^ ((uint64_t)blockIdx.x << 20), 9);
  uint32_t f = 0x3fffffedu, g = (uint32_t)__builtin_amdgcn_readfirstlane(w[0]);
  uint32_t acc = 0;
  int32_t eta = -1;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
#pragma unroll 1
  for (int k = 0; k < iters * 18; k++) {
    SgcdMat t;
    if (kVec) eta = sgcd_divsteps30_vec<kCap>(eta, f, g, t);
    else eta = sgcd_divsteps30<kCap, kSel, kSpec>(eta, f, g, t);
    const uint32_t nf = (uint32_t)t.u * f + (uint32_t)t.v * g;
    const uint32_t ng = (uint32_t)t.q * f + (uint32_t)t.r * g;
    f = (nf >> 30 | 1u) ^ (uint32_t)k;  // keep f odd, vary the words
    f |= 1u;
    g = ng ^ (uint32_t)(k * 0x9e3779b9u);
    acc += (uint32_t)t.u ^ (uint32_t)t.r;
    if (eta > 100 || eta < -100) eta = -1;
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) {
    out[2 * blockIdx.x] = t1 - t0;
    out[2 * blockIdx.x + 1] = acc;
  }
#endif
}

// One wave per input: the latency mode's Elligator2 (hash-to-curve with the
// cofactor cleared) and its one-point encoding, exactly as the V / V2 items
// run them (wide_cores.h elligator2_wide, encode1_wide), for the oracle
// comparison in tests/test_gpu_wide.py.  r: 32 bytes per input, top bit clear.
__global__ void __launch_bounds__(64) k_wide_elligator2(int n, const uint8_t* r, uint8_t* out) {
#if defined(__HIP_DEVICE_COMPILE__)
  using namespace wide;
  const int i = (int)blockIdx.x;
  if (i >= n) return;
  const Lanes L = lanes();
  uint32_t rw[8], enc[8];
#pragma unroll
  for (int k = 0; k < 8; k++) rw[k] = reinterpret_cast<const uint32_t*>(r + 32 * (size_t)i)[k];
  rw[7] &= 0x7fffffffu;
  encode1_wide(enc, elligator2_wide(rw, L));
  if (threadIdx.x == 0) {
#pragma unroll
    for (int k = 0; k < 8; k++) reinterpret_cast<uint32_t*>(out + 32 * (size_t)i)[k] = enc[k];
  }
#endif
}

// One wave per input: the latency encodings' inversion (wide_inv.h
// fe_invert_wave, the divsteps with the operand updates over the lanes) on a
// 256-bit input reduced as fe_from_words reads it; canonical output words.
__global__ void __launch_bounds__(64) k_wide_invert(int n, const uint32_t* z, uint32_t* out) {
#if defined(__HIP_DEVICE_COMPILE__)
  const int i = (int)blockIdx.x;
  if (i >= n) return;
  uint32_t w[8];
#pragma unroll
  for (int k = 0; k < 8; k++) w[k] = z[8 * (size_t)i + k];
  const fe r = fe_invert_wave(fe_from_words(w));
  fe_to_words(w, r);
  if (threadIdx.x == 0) {
#pragma unroll
    for (int k = 0; k < 8; k++) out[8 * (size_t)i + k] = w[k];
  }
#endif
}

// One wave per input: [s mod L]P on the wave (wide.h pw_scalarmult: the
// latency chains' table, windows and additions) and its encoding
// (encode1_wide), P decoded on the lane; ok[i] = 0 when P does not decode.
__global__ void __launch_bounds__(64) k_wide_scalarmult(int n, const uint32_t* pe, const uint32_t* sc,
                                                        uint32_t* out, int32_t* ok) {
#if defined(__HIP_DEVICE_COMPILE__)
  using namespace wide;
  const int i = (int)blockIdx.x;
  if (i >= n) return;
  const Lanes L = lanes();
  uint32_t w[8], sr[8], s[8], enc[8];
#pragma unroll
  for (int k = 0; k < 8; k++) {
    w[k] = pe[8 * (size_t)i + k];
    sr[k] = sc[8 * (size_t)i + k];
  }
  ge_p3 P;
  const bool dec = ge_decode(&P, w, false);
  sc_reduce256(s, sr);
  TabW tab;
  tab_build(tab, pw_from_p3(dec ? P : ge_p3_identity(), L), d2_wide(L), L);
  encode1_wide(enc, pw_scalarmult(tab, s, L));
  if (threadIdx.x == 0) {
#pragma unroll
    for (int k = 0; k < 8; k++) out[8 * (size_t)i + k] = enc[k];
    ok[i] = dec ? 1 : 0;
  }
#endif
}

// One wave per message: the latency items' wave SHA-512 (sha512.h
// sha512_prefixed_wave) over a 64-byte prefix (R || A) and a global-memory
// tail of len[i] bytes (stride 1024), as the Ed25519 scalars items hash.
__global__ void __launch_bounds__(64) k_wide_sha_prefixed(int n, const uint32_t* pre, const uint8_t* msg,
                                                          const uint32_t* len, uint32_t* out) {
#if defined(__HIP_DEVICE_COMPILE__)
  const int i = (int)blockIdx.x;
  if (i >= n) return;
  uint32_t p[16], d[16];
#pragma unroll
  for (int k = 0; k < 16; k++) p[k] = pre[16 * (size_t)i + k];
  uint64_t H[8];
  sha512_prefixed_wave<64, 64>(H, p, ShaGlobalTail{msg + 1024 * (size_t)i}, len[i]);
  sha512_digest_words(d, H);
  if (threadIdx.x == 0) {
#pragma unroll
    for (int k = 0; k < 16; k++) out[16 * (size_t)i + k] = d[k];
  }
#endif
}
// Two 130-byte messages per wave, one per half (the tail's challenge form,
// sha512_prefixed_wave<130, 32>); msg: 33 words per message (last 2 bytes used)
__global__ void __launch_bounds__(64) k_wide_sha130_pairs(int pairs, const uint32_t* msg, uint32_t* out) {
#if defined(__HIP_DEVICE_COMPILE__)
  const int i = (int)blockIdx.x;
  if (i >= pairs) return;
  const size_t m = 2 * (size_t)i + (threadIdx.x >> 5);
  uint32_t hp[33], d[16];
#pragma unroll
  for (int k = 0; k < 33; k++) hp[k] = msg[33 * m + k];
  uint64_t H[8];
  sha512_prefixed_wave<130, 32>(H, hp, ShaNoTail{}, 0);
  sha512_digest_words(d, H);
  if ((threadIdx.x & 31u) == 0) {
#pragma unroll
    for (int k = 0; k < 16; k++) out[16 * m + k] = d[k];
  }
#endif
}

}  // namespace

extern "C" {
// SHA-512(pre_i || msg_i[0..len_i)) for n messages on the device, one wave
// each (pre: 64 B each; msg: 1024-B stride, len_i <= 943); 0 / -1 / -2
int ouro_wide_sha512_prefixed(int n, const uint8_t* pre, const uint8_t* msg, const uint32_t* len,
                              uint8_t* out) {
  if (n <= 0 || !pre || !msg || !len || !out) return -1;
  for (int i = 0; i < n; i++)
    if (len[i] > 943) return -1;  // the wave form's 8 blocks
  uint32_t *d_p = nullptr, *d_l = nullptr, *d_o = nullptr;
  uint8_t* d_m = nullptr;
  int rc = 0;
  if (hipMalloc(&d_p, 64 * (size_t)n) != hipSuccess || hipMalloc(&d_m, 1024 * (size_t)n) != hipSuccess ||
      hipMalloc(&d_l, 4 * (size_t)n) != hipSuccess || hipMalloc(&d_o, 64 * (size_t)n) != hipSuccess)
    rc = -2;
  if (!rc && (hipMemcpy(d_p, pre, 64 * (size_t)n, hipMemcpyHostToDevice) != hipSuccess ||
              hipMemcpy(d_m, msg, 1024 * (size_t)n, hipMemcpyHostToDevice) != hipSuccess ||
              hipMemcpy(d_l, len, 4 * (size_t)n, hipMemcpyHostToDevice) != hipSuccess))
    rc = -2;
  if (!rc) {
    hipLaunchKernelGGL(k_wide_sha_prefixed, dim3(n), dim3(64), 0, 0, n, d_p, d_m, d_l, d_o);
    if (hipDeviceSynchronize() != hipSuccess || hipGetLastError() != hipSuccess) rc = -2;
  }
  if (!rc && hipMemcpy(out, d_o, 64 * (size_t)n, hipMemcpyDeviceToHost) != hipSuccess) rc = -2;
  if (d_p) (void)hipFree(d_p);
  if (d_m) (void)hipFree(d_m);
  if (d_l) (void)hipFree(d_l);
  if (d_o) (void)hipFree(d_o);
  return rc;
}
// SHA-512 of 2 * pairs 130-byte messages (33 words each), two per wave; 0 / -1 / -2
int ouro_wide_sha512_130_pairs(int pairs, const uint8_t* msg, uint8_t* out) {
  if (pairs <= 0 || !msg || !out) return -1;
  uint32_t *d_m = nullptr, *d_o = nullptr;
  const size_t nm = 2 * (size_t)pairs;
  int rc = 0;
  if (hipMalloc(&d_m, 132 * nm) != hipSuccess || hipMalloc(&d_o, 64 * nm) != hipSuccess) rc = -2;
  if (!rc && hipMemcpy(d_m, msg, 132 * nm, hipMemcpyHostToDevice) != hipSuccess) rc = -2;
  if (!rc) {
    hipLaunchKernelGGL(k_wide_sha130_pairs, dim3(pairs), dim3(64), 0, 0, pairs, d_m, d_o);
    if (hipDeviceSynchronize() != hipSuccess || hipGetLastError() != hipSuccess) rc = -2;
  }
  if (!rc && hipMemcpy(out, d_o, 64 * nm, hipMemcpyDeviceToHost) != hipSuccess) rc = -2;
  if (d_m) (void)hipFree(d_m);
  if (d_o) (void)hipFree(d_o);
  return rc;
}
// [s mod L]P for n host (P encoding, s) pairs on the device, one wave each;
// 0, -1 on bad arguments, -2 on a HIP error
int ouro_wide_scalarmult(int n, const uint8_t* pe, const uint8_t* sc, uint8_t* out, int32_t* ok) {
  if (n <= 0 || !pe || !sc || !out || !ok) return -1;
  uint32_t *d_p = nullptr, *d_s = nullptr, *d_o = nullptr;
  int32_t* d_ok = nullptr;
  const size_t bytes = 32 * (size_t)n;
  int rc = 0;
  if (hipMalloc(&d_p, bytes) != hipSuccess || hipMalloc(&d_s, bytes) != hipSuccess ||
      hipMalloc(&d_o, bytes) != hipSuccess || hipMalloc(&d_ok, sizeof(int32_t) * n) != hipSuccess)
    rc = -2;
  if (!rc && (hipMemcpy(d_p, pe, bytes, hipMemcpyHostToDevice) != hipSuccess ||
              hipMemcpy(d_s, sc, bytes, hipMemcpyHostToDevice) != hipSuccess))
    rc = -2;
  if (!rc) {
    hipLaunchKernelGGL(k_wide_scalarmult, dim3(n), dim3(64), 0, 0, n, d_p, d_s, d_o, d_ok);
    if (hipDeviceSynchronize() != hipSuccess || hipGetLastError() != hipSuccess) rc = -2;
  }
  if (!rc && (hipMemcpy(out, d_o, bytes, hipMemcpyDeviceToHost) != hipSuccess ||
              hipMemcpy(ok, d_ok, sizeof(int32_t) * n, hipMemcpyDeviceToHost) != hipSuccess))
    rc = -2;
  if (d_p) (void)hipFree(d_p);
  if (d_s) (void)hipFree(d_s);
  if (d_o) (void)hipFree(d_o);
  if (d_ok) (void)hipFree(d_ok);
  return rc;
}
// z^-1 mod p of n host inputs (32 bytes each) on the device, one wave each;
// 0, -1 on bad arguments, -2 on a HIP error
int ouro_wide_invert(int n, const uint8_t* z, uint8_t* out) {
  if (n <= 0 || !z || !out) return -1;
  uint32_t *d_z = nullptr, *d_o = nullptr;
  const size_t bytes = 32 * (size_t)n;
  int rc = 0;
  if (hipMalloc(&d_z, bytes) != hipSuccess || hipMalloc(&d_o, bytes) != hipSuccess) rc = -2;
  if (!rc && hipMemcpy(d_z, z, bytes, hipMemcpyHostToDevice) != hipSuccess) rc = -2;
  if (!rc) {
    hipLaunchKernelGGL(k_wide_invert, dim3(n), dim3(64), 0, 0, n, d_z, d_o);
    if (hipDeviceSynchronize() != hipSuccess || hipGetLastError() != hipSuccess) rc = -2;
  }
  if (!rc && hipMemcpy(out, d_o, bytes, hipMemcpyDeviceToHost) != hipSuccess) rc = -2;
  if (d_z) (void)hipFree(d_z);
  if (d_o) (void)hipFree(d_o);
  return rc;
}
// Elligator2 + encoding of n host inputs on the device (one wave each);
// 0, -1 on bad arguments, -2 on a HIP error
int ouro_wide_elligator2(int n, const uint8_t* r, uint8_t* out) {
  if (n <= 0 || !r || !out) return -1;
  uint8_t *d_r = nullptr, *d_o = nullptr;
  const size_t bytes = 32 * (size_t)n;
  int rc = 0;
  if (hipMalloc(&d_r, bytes) != hipSuccess || hipMalloc(&d_o, bytes) != hipSuccess) rc = -2;
  if (!rc && hipMemcpy(d_r, r, bytes, hipMemcpyHostToDevice) != hipSuccess) rc = -2;
  if (!rc) {
    hipLaunchKernelGGL(k_wide_elligator2, dim3(n), dim3(64), 0, 0, n, d_r, d_o);
    if (hipDeviceSynchronize() != hipSuccess || hipGetLastError() != hipSuccess) rc = -2;
  }
  if (!rc && hipMemcpy(out, d_o, bytes, hipMemcpyDeviceToHost) != hipSuccess) rc = -2;
  if (d_r) (void)hipFree(d_r);
  if (d_o) (void)hipFree(d_o);
  return rc;
}

// us per 18 batches of divsteps matrices (one inversion's worth); mode 0 cap
// 30, 1 cap 10, 2 cap 10 branch-free, 3 cap 30 branch-free, 4 cap 30 on the
// VALU, 5 cap 10 on the VALU, 6 cap 30 branch-free with the speculative inverse
double ouro_wide_divsteps_us(int waves, int iters, int mode, uint64_t seed) {
  unsigned long long* d = nullptr;
  if (hipMalloc(&d, sizeof(unsigned long long) * 2 * waves) != hipSuccess) return -1;
  const dim3 gr(waves), bl(64);
  switch (mode) {
    case 0: hipLaunchKernelGGL((k_divsteps_timing<30, false>), gr, bl, 0, 0, seed, iters, d); break;
    case 1: hipLaunchKernelGGL((k_divsteps_timing<10, false>), gr, bl, 0, 0, seed, iters, d); break;
    case 2: hipLaunchKernelGGL((k_divsteps_timing<10, true>), gr, bl, 0, 0, seed, iters, d); break;
    case 3: hipLaunchKernelGGL((k_divsteps_timing<30, true>), gr, bl, 0, 0, seed, iters, d); break;
    case 4: hipLaunchKernelGGL((k_divsteps_timing<30, false, true>), gr, bl, 0, 0, seed, iters, d); break;
    case 5: hipLaunchKernelGGL((k_divsteps_timing<10, false, true>), gr, bl, 0, 0, seed, iters, d); break;
    default: hipLaunchKernelGGL((k_divsteps_timing<30, true, false, true>), gr, bl, 0, 0, seed, iters, d); break;
  }
  std::vector<unsigned long long> h(2 * (size_t)waves);
  double r = -1;
  if (hipDeviceSynchronize() == hipSuccess &&
      hipMemcpy(h.data(), d, sizeof(unsigned long long) * 2 * waves, hipMemcpyDeviceToHost) ==
          hipSuccess) {
    double t = 0;
    for (int i = 0; i < waves; i++) t += (double)h[2 * i];
    r = t / waves / iters / 100.0;
  }
  (void)hipFree(d);
  return r;
}
// us per inversion averaged over `waves` waves x `iters` inversions; mode:
// 0 all 25 batches, cap 30, branching steps (round 4); 1 early exit; 2 early,
// cap 10; 3 early, cap 10, branch-free steps; 4 early, cap 30, branch-free;
// 5 early, cap 30, steps on the VALU; 6 the same with cap 10; -1 on a HIP error
double ouro_wide_invert_us(int waves, int iters, int mode, uint64_t seed) {
  unsigned long long* d = nullptr;
  if (hipMalloc(&d, sizeof(unsigned long long) * 2 * waves) != hipSuccess) return -1;
  const dim3 gr(waves), bl(64);
  switch (mode) {
    case 0: hipLaunchKernelGGL((k_inv_timing<false, 30, false>), gr, bl, 0, 0, seed, iters, d); break;
    case 1: hipLaunchKernelGGL((k_inv_timing<true, 30, false>), gr, bl, 0, 0, seed, iters, d); break;
    case 2: hipLaunchKernelGGL((k_inv_timing<true, 10, false>), gr, bl, 0, 0, seed, iters, d); break;
    case 3: hipLaunchKernelGGL((k_inv_timing<true, 10, true>), gr, bl, 0, 0, seed, iters, d); break;
    case 4: hipLaunchKernelGGL((k_inv_timing<true, 30, true>), gr, bl, 0, 0, seed, iters, d); break;
    case 5: hipLaunchKernelGGL((k_inv_timing<true, 30, false, true>), gr, bl, 0, 0, seed, iters, d); break;
    default: hipLaunchKernelGGL((k_inv_timing<true, 10, false, true>), gr, bl, 0, 0, seed, iters, d); break;
  }
  std::vector<unsigned long long> h(2 * (size_t)waves);
  double r = -1;
  if (hipDeviceSynchronize() == hipSuccess &&
      hipMemcpy(h.data(), d, sizeof(unsigned long long) * 2 * waves, hipMemcpyDeviceToHost) ==
          hipSuccess) {
    double t = 0;
    for (int i = 0; i < waves; i++) t += (double)h[2 * i];
    r = t / waves / iters / 100.0;
  }
  (void)hipFree(d);
  return r;
}

// waves cases from seed; out: waves * 10 int32 (1 = pass), dbg: 24 int32.
// Returns 0, or -2 on a HIP error.
int ouro_wide_selftest(int waves, uint64_t seed, int32_t* out, int32_t* dbg) {
  int32_t *d_out = nullptr, *d_dbg = nullptr;
  if (hipMalloc(&d_out, sizeof(int32_t) * waves * kTests) != hipSuccess) return -2;
  if (hipMalloc(&d_dbg, sizeof(int32_t) * 24) != hipSuccess) return -2;
  (void)hipMemset(d_out, 0xff, sizeof(int32_t) * waves * kTests);
  hipLaunchKernelGGL(k_wide_selftest, dim3(waves), dim3(64), 0, 0, seed, d_out, d_dbg);
  int rc = hipDeviceSynchronize() == hipSuccess && hipGetLastError() == hipSuccess ? 0 : -2;
  if (!rc) {
    rc |= hipMemcpy(out, d_out, sizeof(int32_t) * waves * kTests, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -2;
    rc |= hipMemcpy(dbg, d_dbg, sizeof(int32_t) * 24, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -2;
  }
  (void)hipFree(d_out);
  (void)hipFree(d_dbg);
  return rc;
}
}
