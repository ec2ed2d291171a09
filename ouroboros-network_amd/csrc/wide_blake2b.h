// wide_blake2b.h -- Blake2b-256 of one short message on the four lanes of a
// DPP quad (latency mode), for mkSeed on the V and V2 items' critical path
// (the node configuration derives the VRF inputs from (slot, eta0) on the
// device: Shelley/Protocol.hs:409-410).
//
// A round of Blake2b is four column G functions, then four diagonal ones,
// each four independent.  Lane c of a quad holds column c of the state (v[c],
// v[4 + c], v[8 + c], v[12 + c]) and runs column G c; for the diagonal step
// it takes rows 1 / 2 / 3 from lanes c + 1 / c + 2 / c + 3 of the quad
// (quad_perm rotations), runs diagonal G c, and rotates them back.  One G per
// lane per step instead of eight in series: ~70 instructions a round against
// ~175 on one lane (blake2b.h).  Every quad of the wave computes the same;
// the digest is broadcast from the quad's lanes.  Same bytes as
// blake2b256_short (the latency parity tests run the node configuration).
#pragma once
#include <utility>

#include "tpraos.h"

namespace ouro {

// this lane's value from lane (c + k) mod 4 of its quad, 64-bit
template <int kCtrl>
__device__ __forceinline__ uint64_t quad_perm64(uint64_t x) {
  const int lo = __builtin_amdgcn_mov_dpp((int)(uint32_t)x, kCtrl, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_mov_dpp((int)(uint32_t)(x >> 32), kCtrl, 0xf, 0xf, false);
  return ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo;
}
constexpr int kQuadFrom1 = 0x39;  // quad_perm [1, 2, 3, 0]: lane c <- c + 1
constexpr int kQuadFrom2 = 0x4e;  // [2, 3, 0, 1]
constexpr int kQuadFrom3 = 0x93;  // [3, 0, 1, 2]

__device__ __forceinline__ void b2b_g(uint64_t& a, uint64_t& b, uint64_t& c, uint64_t& d,
                                      uint64_t x, uint64_t y) {
  a = a + b + x;
  d = b2b_rotr(d ^ a, 32);
  c = c + d;
  b = b2b_rotr(b ^ c, 24);
  a = a + b + y;
  d = b2b_rotr(d ^ a, 16);
  c = c + d;
  b = b2b_rotr(b ^ c, 63);
}

// message word k of the 64-byte block (in: 16 little-endian 32-bit words)
__device__ __forceinline__ uint64_t b2b_word(const uint32_t in[16], int k) {
  return (uint64_t)in[2 * k] | ((uint64_t)in[2 * k + 1] << 32);
}

// this lane's pick of four values by its quad position (selects, no branch)
__device__ __forceinline__ uint64_t quad_sel(uint64_t v0, uint64_t v1, uint64_t v2, uint64_t v3,
                                             bool q1, bool q2) {
  const uint64_t lo = q1 ? v1 : v0, hi = q1 ? v3 : v2;
  return q2 ? hi : lo;
}
// round R (compile-time sigma): column G q, then diagonal G q
template <int R>
__device__ __forceinline__ void b2b_round_quad(uint64_t& a, uint64_t& b, uint64_t& c, uint64_t& d,
                                               const uint64_t m[16], bool q1, bool q2) {
  constexpr const uint8_t* s = kB2bSigma[R];
  b2b_g(a, b, c, d, quad_sel(m[s[0]], m[s[2]], m[s[4]], m[s[6]], q1, q2),
        quad_sel(m[s[1]], m[s[3]], m[s[5]], m[s[7]], q1, q2));
  b = quad_perm64<kQuadFrom1>(b);
  c = quad_perm64<kQuadFrom2>(c);
  d = quad_perm64<kQuadFrom3>(d);
  b2b_g(a, b, c, d, quad_sel(m[s[8]], m[s[10]], m[s[12]], m[s[14]], q1, q2),
        quad_sel(m[s[9]], m[s[11]], m[s[13]], m[s[15]], q1, q2));
  b = quad_perm64<kQuadFrom3>(b);
  c = quad_perm64<kQuadFrom2>(c);
  d = quad_perm64<kQuadFrom1>(d);
}
template <int... R>
__device__ __forceinline__ void b2b_rounds_quad(uint64_t& a, uint64_t& b, uint64_t& c,
                                                uint64_t& d, const uint64_t m[16], bool q1,
                                                bool q2, std::integer_sequence<int, R...>) {
  (b2b_round_quad<R>(a, b, c, d, m, q1, q2), ...);
}

// out = Blake2b-256 of the first len <= 64 bytes of in (bytes past len zero),
// as blake2b.h blake2b256_short; the whole wave in quads, all lanes alike
__device__ __noinline__ void blake2b256_short_quad(uint32_t out[8], const uint32_t in[16],
                                                   uint32_t len) {
  const uint32_t q = threadIdx.x & 3u;
  const bool q1 = (q & 1u) != 0, q2 = (q & 2u) != 0;
  constexpr uint64_t IV[8] = {0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL,
                              0xa54ff53a5f1d36f1ULL, 0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL,
                              0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};
  uint64_t m[16];
#pragma unroll
  for (int k = 0; k < 16; k++) m[k] = k < 8 ? b2b_word(in, k) : 0ull;
  // column q of the initial state: h = IV ^ params, then IV with t0 = len and f0
  const uint64_t hq = quad_sel(IV[0] ^ (0x01010000ULL ^ 32), IV[1], IV[2], IV[3], q1, q2);
  uint64_t a = hq;
  uint64_t b = quad_sel(IV[4], IV[5], IV[6], IV[7], q1, q2);
  uint64_t c = quad_sel(IV[0], IV[1], IV[2], IV[3], q1, q2);
  uint64_t d = quad_sel(IV[4] ^ len, IV[5], ~IV[6], IV[7], q1, q2);
  b2b_rounds_quad(a, b, c, d, m, q1, q2, std::make_integer_sequence<int, 12>{});
  // digest words 2q, 2q + 1 = h[q] ^ v[q] ^ v[8 + q], broadcast from lane q
  const uint64_t x = hq ^ a ^ c;
  const uint64_t w[4] = {quad_perm64<0x00>(x), quad_perm64<0x55>(x), quad_perm64<0xaa>(x),
                         quad_perm64<0xff>(x)};  // quad_perm [k, k, k, k]
#pragma unroll
  for (int k = 0; k < 4; k++) {
    out[2 * k] = (uint32_t)w[k];
    out[2 * k + 1] = (uint32_t)(w[k] >> 32);
  }
}

// hdr_seed (tpraos.h) with mkSeed's Blake2b on the quads
__device__ __forceinline__ void hdr_seed_wave(SeedMsg& a, const ouro_tpraos_batch& b, size_t i,
                                              bool leader, uint32_t opts) {
  if (!(opts & kOptSeeds)) {
    ld_words(a.w, (leader ? b.leader_alpha : b.eta_alpha) + 32 * i, 2);
    return;
  }
  const uint64_t slot = b.slot[i];
  uint32_t in[16];
#pragma unroll
  for (int k = 0; k < 16; k++) in[k] = 0;
  in[0] = bswap32_b2((uint32_t)(slot >> 32));
  in[1] = bswap32_b2((uint32_t)slot);
  const bool eta0 = (opts & kOptEpochNonce) != 0;
  if (eta0) {
    uint32_t e0[8];
    ld_words(e0, b.epoch_nonce, 2);
#pragma unroll
    for (int k = 0; k < 8; k++) in[2 + k] = e0[k];
  }
  blake2b256_short_quad(a.w, in, eta0 ? 40u : 8u);
#pragma unroll
  for (int k = 0; k < 8; k++) a.w[k] ^= leader ? kSeedL[k] : kSeedEta[k];
}

}  // namespace ouro
