// blake2b.h -- per-lane unkeyed Blake2b-256 of one 64-byte input (RFC 7693).
//
// The Sum6KES Merkle hash: hashPairOfVKeys (vk0, vk1) = Blake2b_256(vk0 || vk1),
// SURVEY.md App. B.2.  A 64-byte input is a single final compression with
// counter t = 64, so the 12 rounds are unrolled with compile-time sigma.
#pragma once
#include "common.h"

namespace ouro {

constexpr uint8_t kB2bSigma[12][16] = {
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15},
    {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
    {11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4},
    {7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8},
    {9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13},
    {2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9},
    {12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11},
    {13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10},
    {6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5},
    {10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0},
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15},
    {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3}};

// G's rotations (32, 24, 16, 63; compile-time n).  On the device two
// v_alignbit_b32 per rotation (a half swap for 32): LLVM writes the shift form
// as a 64-bit shift pair and two ORs, four instructions (OURO_B2B_ALIGNBIT=0:
// that form, for A/B)
#ifndef OURO_B2B_ALIGNBIT
#define OURO_B2B_ALIGNBIT 1
#endif
OURO_FI uint64_t b2b_rotr(uint64_t x, int n) {
#if defined(__HIP_DEVICE_COMPILE__) && OURO_B2B_ALIGNBIT
  const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  if (n == 32) return ((uint64_t)lo << 32) | hi;
  uint32_t rl, rh;
  if (n < 32) {
    rl = __builtin_amdgcn_alignbit(hi, lo, n);
    rh = __builtin_amdgcn_alignbit(lo, hi, n);
  } else {
    rl = __builtin_amdgcn_alignbit(lo, hi, n - 32);
    rh = __builtin_amdgcn_alignbit(hi, lo, n - 32);
  }
  return ((uint64_t)rh << 32) | rl;
#else
  return (x >> n) | (x << (64 - n));
#endif
}

// out = Blake2b-256 of the first `len` <= 64 bytes of in (16 little-endian
// 32-bit words; bytes past len must be zero).  One final compression with
// counter t = len: the KES Merkle pairs (64 B), mkSeed's BE64(slot) || eta0
// (40 B, or 8 B for NeutralNonce), mkNonceFromOutputVRF (64 B).
OURO_FI void blake2b256_short(uint32_t out[8], const uint32_t in[16], uint32_t len) {
  const uint64_t IV[8] = {0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL,
                          0xa54ff53a5f1d36f1ULL, 0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL,
                          0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};
  uint64_t m[16];
#pragma unroll
  for (int i = 0; i < 8; i++) m[i] = (uint64_t)in[2 * i] | ((uint64_t)in[2 * i + 1] << 32);
#pragma unroll
  for (int i = 8; i < 16; i++) m[i] = 0;
  uint64_t h[8];
#pragma unroll
  for (int i = 0; i < 8; i++) h[i] = IV[i];
  h[0] ^= 0x01010000ULL ^ 32;  // digest length 32, key length 0, fanout 1, depth 1
  uint64_t v[16];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    v[i] = h[i];
    v[i + 8] = IV[i];
  }
  v[12] ^= len;   // t0 = bytes hashed
  v[14] = ~v[14]; // final block
#define OURO_B2G(a, b, c, d, x, y)                     \
  v[a] = v[a] + v[b] + (x);                            \
  v[d] = b2b_rotr(v[d] ^ v[a], 32);                    \
  v[c] = v[c] + v[d];                                  \
  v[b] = b2b_rotr(v[b] ^ v[c], 24);                    \
  v[a] = v[a] + v[b] + (y);                            \
  v[d] = b2b_rotr(v[d] ^ v[a], 16);                    \
  v[c] = v[c] + v[d];                                  \
  v[b] = b2b_rotr(v[b] ^ v[c], 63);
#pragma unroll
  for (int r = 0; r < 12; r++) {
    const uint8_t* s = kB2bSigma[r];
    OURO_B2G(0, 4, 8, 12, m[s[0]], m[s[1]])
    OURO_B2G(1, 5, 9, 13, m[s[2]], m[s[3]])
    OURO_B2G(2, 6, 10, 14, m[s[4]], m[s[5]])
    OURO_B2G(3, 7, 11, 15, m[s[6]], m[s[7]])
    OURO_B2G(0, 5, 10, 15, m[s[8]], m[s[9]])
    OURO_B2G(1, 6, 11, 12, m[s[10]], m[s[11]])
    OURO_B2G(2, 7, 8, 13, m[s[12]], m[s[13]])
    OURO_B2G(3, 4, 9, 14, m[s[14]], m[s[15]])
  }
#undef OURO_B2G
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const uint64_t x = h[i] ^ v[i] ^ v[i + 8];
    out[2 * i] = (uint32_t)x;
    out[2 * i + 1] = (uint32_t)(x >> 32);
  }
}

OURO_FI void blake2b256_64(uint32_t out[8], const uint32_t in[16]) { blake2b256_short(out, in, 64); }

// ---- mkSeed / mkNonceFromNumber ----------------------
// seedEta = mkNonceFromNumber 0, seedL = mkNonceFromNumber 1, i.e.
// Blake2b-256(BE64(0 / 1)) as little-endian words.  Pinned by
// tests/test_nonce.py: seedL against the Nonce values of the reference's golden
// ChainDepState (ouroboros-consensus-shelley-test/test/golden/disk/ChainDepState,
// built from SL.mkNonceFromNumber 1 at Examples.hs:531-537), both against the
// device routine below compiled for the host.
constexpr uint32_t kSeedEta[8] = {0x197ae481u, 0x0a9bb2e6u, 0x1759b965u, 0x4351ce62u,
                                  0x26d030edu, 0xa3245d1eu, 0x50521720u, 0x5cf1206bu};
constexpr uint32_t kSeedL[8] = {0x6a0add12u, 0x2a220e7du, 0xa06d9297u, 0x775adb3au,
                                0xc71cd368u, 0x68bdc2c5u, 0x7d4ae128u, 0x603afa25u};

OURO_FI uint32_t bswap32_b2(uint32_t x) {
  return (x >> 24) | ((x >> 8) & 0xff00u) | ((x << 8) & 0xff0000u) | (x << 24);
}

// The hash half of ledger-specs mkSeed (called at
// ouroboros-consensus-shelley/src/Ouroboros/Consensus/Shelley/Protocol.hs:409-410):
// Blake2b-256(BE64(slot) || eta0), eta0 = 8 words or NULL (NeutralNonce: the
// slot bytes alone).  The caller XORs seedEta / seedL.
OURO_FI void mkseed_hash(uint32_t out[8], uint64_t slot, const uint32_t* eta0) {
  uint32_t in[16];
#pragma unroll
  for (int i = 0; i < 16; i++) in[i] = 0;
  in[0] = bswap32_b2((uint32_t)(slot >> 32));
  in[1] = bswap32_b2((uint32_t)slot);
  if (eta0) {
#pragma unroll
    for (int i = 0; i < 8; i++) in[2 + i] = eta0[i];
  }
  blake2b256_short(out, in, eta0 ? 40u : 8u);
}

}  // namespace ouro
