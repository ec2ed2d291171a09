// sha512.h -- per-lane SHA-512 (FIPS 180-4) for gfx950.
//
// The inner hash of Ed25519 (h = H(R || A || M)) and of the draft-03 VRF
// (hash-to-curve, challenge, proof_to_hash).  Messages are assembled on the
// fly from a byte source: a wave-uniform register prefix followed by bytes
// fetched from global memory, so nothing is staged per lane.
#pragma once
#include <type_traits>
#include <utility>

#include "common.h"

namespace ouro {

constexpr uint64_t kSha512K[80] = {
    0x428a2f98d728ae22ULL, 0x7137449123ef65cdULL, 0xb5c0fbcfec4d3b2fULL, 0xe9b5dba58189dbbcULL,
    0x3956c25bf348b538ULL, 0x59f111f1b605d019ULL, 0x923f82a4af194f9bULL, 0xab1c5ed5da6d8118ULL,
    0xd807aa98a3030242ULL, 0x12835b0145706fbeULL, 0x243185be4ee4b28cULL, 0x550c7dc3d5ffb4e2ULL,
    0x72be5d74f27b896fULL, 0x80deb1fe3b1696b1ULL, 0x9bdc06a725c71235ULL, 0xc19bf174cf692694ULL,
    0xe49b69c19ef14ad2ULL, 0xefbe4786384f25e3ULL, 0x0fc19dc68b8cd5b5ULL, 0x240ca1cc77ac9c65ULL,
    0x2de92c6f592b0275ULL, 0x4a7484aa6ea6e483ULL, 0x5cb0a9dcbd41fbd4ULL, 0x76f988da831153b5ULL,
    0x983e5152ee66dfabULL, 0xa831c66d2db43210ULL, 0xb00327c898fb213fULL, 0xbf597fc7beef0ee4ULL,
    0xc6e00bf33da88fc2ULL, 0xd5a79147930aa725ULL, 0x06ca6351e003826fULL, 0x142929670a0e6e70ULL,
    0x27b70a8546d22ffcULL, 0x2e1b21385c26c926ULL, 0x4d2c6dfc5ac42aedULL, 0x53380d139d95b3dfULL,
    0x650a73548baf63deULL, 0x766a0abb3c77b2a8ULL, 0x81c2c92e47edaee6ULL, 0x92722c851482353bULL,
    0xa2bfe8a14cf10364ULL, 0xa81a664bbc423001ULL, 0xc24b8b70d0f89791ULL, 0xc76c51a30654be30ULL,
    0xd192e819d6ef5218ULL, 0xd69906245565a910ULL, 0xf40e35855771202aULL, 0x106aa07032bbd1b8ULL,
    0x19a4c116b8d2d0c8ULL, 0x1e376c085141ab53ULL, 0x2748774cdf8eeb99ULL, 0x34b0bcb5e19b48a8ULL,
    0x391c0cb3c5c95a63ULL, 0x4ed8aa4ae3418acbULL, 0x5b9cca4f7763e373ULL, 0x682e6ff3d6b2b8a3ULL,
    0x748f82ee5defb2fcULL, 0x78a5636f43172f60ULL, 0x84c87814a1f0ab72ULL, 0x8cc702081a6439ecULL,
    0x90befffa23631e28ULL, 0xa4506cebde82bde9ULL, 0xbef9a3f7b2c67915ULL, 0xc67178f2e372532bULL,
    0xca273eceea26619cULL, 0xd186b8c721c0c207ULL, 0xeada7dd6cde0eb1eULL, 0xf57d4f7fee6ed178ULL,
    0x06f067aa72176fbaULL, 0x0a637dc5a2c898a6ULL, 0x113f9804bef90daeULL, 0x1b710b35131c471bULL,
    0x28db77f523047d84ULL, 0x32caab7b40c72493ULL, 0x3c9ebe0a15c9bebcULL, 0x431d67c49c100d4cULL,
    0x4cc5d4becb3e42b6ULL, 0x597f299cfc657e2aULL, 0x5fcb6fab3ad6faecULL, 0x6c44198c4a475817ULL};

// 64-bit rotate / shift by a compile-time amount on 32-bit halves: two
// v_alignbit_b32 per rotate (the generic form costs three instructions)
OURO_FI uint64_t rotr64(uint64_t x, int n) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
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
OURO_FI uint64_t shr64(uint64_t x, int n) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  return ((uint64_t)(hi >> n) << 32) | __builtin_amdgcn_alignbit(hi, lo, n);
#else
  return x >> n;
#endif
}

// three-input XOR and majority per 32-bit half: one gfx950 v_bitop3_b32 each
// (truth tables 0x96 / 0xE8, both symmetric in their inputs) instead of two
// XORs, or an AND-XOR chain
#if defined(__HIP_DEVICE_COMPILE__)
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
template <int kTable>
OURO_FI uint64_t bitop3_64(uint64_t a, uint64_t b, uint64_t c) {
  const u32x2 x = __builtin_bit_cast(u32x2, a), y = __builtin_bit_cast(u32x2, b),
              z = __builtin_bit_cast(u32x2, c);
  const u32x2 r = {(uint32_t)__builtin_amdgcn_bitop3_b32(x.x, y.x, z.x, kTable),
                   (uint32_t)__builtin_amdgcn_bitop3_b32(x.y, y.y, z.y, kTable)};
  return __builtin_bit_cast(uint64_t, r);
}
#endif
OURO_FI uint64_t xor3_64(uint64_t a, uint64_t b, uint64_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
  return bitop3_64<0x96>(a, b, c);
#else
  return a ^ b ^ c;
#endif
}
OURO_FI uint64_t maj64(uint64_t a, uint64_t b, uint64_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
  return bitop3_64<0xE8>(a, b, c);
#else
  return (a & b) ^ (a & c) ^ (b & c);
#endif
}

OURO_FI void sha512_init(uint64_t H[8]) {
  H[0] = 0x6a09e667f3bcc908ULL; H[1] = 0xbb67ae8584caa73bULL;
  H[2] = 0x3c6ef372fe94f82bULL; H[3] = 0xa54ff53a5f1d36f1ULL;
  H[4] = 0x510e527fade682d1ULL; H[5] = 0x9b05688c2b3e6c1fULL;
  H[6] = 0x1f83d9abfb41bd6bULL; H[7] = 0x5be0cd19137e2179ULL;
}

OURO_FI void sha512_round(uint64_t& a, uint64_t& b, uint64_t& c, uint64_t& d, uint64_t& e,
                          uint64_t& f, uint64_t& g, uint64_t& h, uint64_t k, uint64_t w) {
  const uint64_t S1 = xor3_64(rotr64(e, 14), rotr64(e, 18), rotr64(e, 41));
  const uint64_t ch = (e & f) ^ (~e & g);
  const uint64_t T1 = h + S1 + ch + k + w;
  const uint64_t S0 = xor3_64(rotr64(a, 28), rotr64(a, 34), rotr64(a, 39));
  const uint64_t mj = maj64(a, b, c);
  h = g; g = f; f = e; e = d + T1; d = c; c = b; b = a; a = T1 + S0 + mj;
}

// 80 rounds: 16 on the block's words, then 4 passes of 16 that extend the
// schedule in a 16-word ring (no per-round branch; out of line so the
// several hash call sites share one copy of the round code)
OURO_NI void sha512_compress(uint64_t H[8], uint64_t W[16]) {
  uint64_t a = H[0], b = H[1], c = H[2], d = H[3], e = H[4], f = H[5], g = H[6], h = H[7];
#pragma unroll
  for (int i = 0; i < 16; i++) sha512_round(a, b, c, d, e, f, g, h, kSha512K[i], W[i]);
#pragma unroll 1
  for (int r0 = 16; r0 < 80; r0 += 16) {
#pragma unroll
    for (int i = 0; i < 16; i++) {
      const uint64_t w15 = W[(i + 1) & 15], w2 = W[(i + 14) & 15];
      const uint64_t s0 = xor3_64(rotr64(w15, 1), rotr64(w15, 8), shr64(w15, 7));
      const uint64_t s1 = xor3_64(rotr64(w2, 19), rotr64(w2, 61), shr64(w2, 6));
      W[i] += s0 + W[(i + 9) & 15] + s1;
      sha512_round(a, b, c, d, e, f, g, h, kSha512K[r0 + i], W[i]);
    }
  }
  H[0] += a; H[1] += b; H[2] += c; H[3] += d; H[4] += e; H[5] += f; H[6] += g; H[7] += h;
}

// Byte sources.  `prefix(p)` is only ever asked for a compile-time p < PL in
// the first block; `tail(q)` reads message byte q.  A source may also offer
// word_be(q, tl): bytes q..q+7 as one big-endian word (bytes at or beyond tl
// arbitrary); the others are assembled byte by byte (sha_tail_word).
struct ShaNoTail {
  OURO_FI uint32_t tail(uint32_t) const { return 0; }
};
// bytes in global memory at any alignment: the dwords covering q..q+7 (only
// those that start before the message end: never a load past the buffer),
// funnel-shifted into place (v_alignbit) and byte-swapped -- three dword loads
// per eight bytes instead of eight byte loads with their shifts and ORs
struct ShaGlobalTail {
  const uint8_t* msg;
  OURO_FI uint32_t tail(uint32_t q) const { return ldg_u8(msg + q); }
#if defined(__HIP_DEVICE_COMPILE__)
  OURO_FI uint64_t word_be(uint32_t q, uint32_t tl) const {
    const uintptr_t a = reinterpret_cast<uintptr_t>(msg) + q;
    const uintptr_t end = reinterpret_cast<uintptr_t>(msg) + tl;
    const uintptr_t w = a & ~uintptr_t(3);
    const uint32_t sh = (uint32_t)(a & 3) * 8;
    const uint32_t d0 = w < end ? (uint32_t)ldg1(reinterpret_cast<const void*>(w)) : 0u;
    const uint32_t d1 = w + 4 < end ? (uint32_t)ldg1(reinterpret_cast<const void*>(w + 4)) : 0u;
    const uint32_t d2 = w + 8 < end ? (uint32_t)ldg1(reinterpret_cast<const void*>(w + 8)) : 0u;
    const uint32_t lo = __builtin_amdgcn_alignbit(d1, d0, sh);  // bytes q..q+3, little-endian
    const uint32_t hi = __builtin_amdgcn_alignbit(d2, d1, sh);  // bytes q+4..q+7
    return ((uint64_t)__builtin_bswap32(lo) << 32) | __builtin_bswap32(hi);
  }
  // the sixteen words at q0, q0 + 8, ..., q0 + 120 (one tail block) from
  // eight dwordx4 loads and one dword at dword alignment instead of 33 dword
  // loads; a dwordx4 is issued only when its last dword starts before the
  // end, else its dwords one by one under word_be's rule, so it never reads
  // further past the end than word_be does (OURO_SHA_BLOCK_LOAD)
  OURO_FI void block_be(uint64_t W[16], uint32_t q0, uint32_t tl) const {
    const uintptr_t a = reinterpret_cast<uintptr_t>(msg) + q0;
    const uintptr_t end = reinterpret_cast<uintptr_t>(msg) + tl;
    const uintptr_t base = a & ~uintptr_t(3);
    const uint32_t sh = (uint32_t)(a & 3) * 8;
    uint32_t d[33];
#pragma unroll
    for (int j = 0; j < 8; j++) {
      const uintptr_t p = base + 16 * (uintptr_t)j;
      if (p + 12 < end) {
        const int4 v = ldg4(reinterpret_cast<const void*>(p));
        d[4 * j] = (uint32_t)v.x;
        d[4 * j + 1] = (uint32_t)v.y;
        d[4 * j + 2] = (uint32_t)v.z;
        d[4 * j + 3] = (uint32_t)v.w;
      } else {
#pragma unroll
        for (int k = 0; k < 4; k++)
          d[4 * j + k] = p + 4 * k < end ? (uint32_t)ldg1(reinterpret_cast<const void*>(p + 4 * k)) : 0u;
      }
    }
    d[32] = base + 128 < end ? (uint32_t)ldg1(reinterpret_cast<const void*>(base + 128)) : 0u;
#pragma unroll
    for (int k = 0; k < 16; k++) {
      const uint32_t lo = __builtin_amdgcn_alignbit(d[2 * k + 1], d[2 * k], sh);
      const uint32_t hi = __builtin_amdgcn_alignbit(d[2 * k + 2], d[2 * k + 1], sh);
      W[k] = ((uint64_t)__builtin_bswap32(lo) << 32) | __builtin_bswap32(hi);
    }
  }
#endif
};
#ifndef OURO_SHA_BLOCK_LOAD
#define OURO_SHA_BLOCK_LOAD 1
#endif
template <class T, class = void>
struct has_block_be : std::false_type {};
#if defined(__HIP_DEVICE_COMPILE__)
template <class T>
struct has_block_be<T, decltype((void)std::declval<const T&>().block_be(nullptr, 0u, 0u))>
    : std::true_type {};
#endif

// A tail in global memory that the WAVE stages into LDS with coalesced loads
// (round 5, OURO_KES_STAGE; the throughput Sum6KES kernel's leaf message).
// Each lane's message sits at its own address, so the per-lane loads of
// ShaGlobalTail touch 64 cache lines per wave instruction; here the wave loads
// lane k's next 256 bytes with all 64 lanes at once (one dword each: four
// lines per instruction), k = 0..63, into row k of the wave's LDS block, and
// each lane then builds its message words from its own row.  Stage s covers
// tail bytes [t0, t0 + 256), t0 = 0 (blocks 0, 1 of an R || A || M hash:
// prefix 64 bytes) or 256 s - 64 (blocks 2s, 2s + 1).  Loads stop at the
// message end exactly as ShaGlobalTail's do (only dwords that start before
// it).  Needs every lane of the wave active (the kernel keeps EXEC full).
constexpr int kStageRowDw = 65;                       // odd: conflict-free row reads
constexpr int kStageWaveDw = 64 * kStageRowDw;        // 16,640 B per wave
struct ShaStagedTail {
  const uint8_t* msg;
  uint32_t* rows;  // this wave's kStageWaveDw dwords of LDS
  OURO_FI uint32_t tail(uint32_t q) const { return ldg_u8(msg + q); }
};
template <class T>
struct is_staged_tail : std::false_type {};
template <>
struct is_staged_tail<ShaStagedTail> : std::true_type {};

template <class T, class = void>
struct has_word_be : std::false_type {};
template <class T>
struct has_word_be<T, decltype((void)std::declval<const T&>().word_be(0u, 0u))> : std::true_type {};

// bytes q..q+7 of a tail as a big-endian word (bytes at or beyond tl arbitrary)
template <class Tail>
OURO_FI uint64_t sha_tail_word(const Tail& t, uint32_t q, uint32_t tl) {
  if constexpr (has_word_be<Tail>::value) {
    return t.word_be(q, tl);
  } else {
    uint64_t r = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) r = (r << 8) | (q + k < tl ? t.tail(q + k) : 0u);
    return r;
  }
}

// the padded message word at byte position p (>= PL) from its raw tail bytes:
// data before `total`, the 0x80 terminator at `total`, zeros after
OURO_FI uint64_t sha_pad_word(uint64_t raw, uint32_t p, uint32_t total) {
  if (p + 8 <= total) return raw;
  if (p >= total) return p == total ? (0x80ull << 56) : 0ull;
  const uint32_t v = total - p;  // 1..7 message bytes in this word
  const uint64_t keep = ~0ull << (64 - 8 * v);
  return (raw & keep) | (0x80ull << (56 - 8 * v));
}

#if defined(__HIP_DEVICE_COMPILE__)
// largest lane value over the wave (every lane active)
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t x) {
  uint32_t m = 0;
#pragma unroll 1
  for (int b = 31; b >= 0; b--) {
    const uint32_t t = m | (1u << b);
    if (__ballot(x >= t) != 0) m = t;
  }
  return m;
}
// tail bytes [t0, t0 + 256) of every lane's message into its LDS row: iteration
// k loads 64 consecutive dwords of lane k's message, one per lane; then each
// lane its own 65th dword
__device__ __forceinline__ void sha_stage(const ShaStagedTail& t, uint32_t t0, uint32_t tl) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t base = (uint64_t)(uintptr_t)t.msg;
  const uint64_t w0 = (base + t0) & ~3ull, end = base + tl;
  const int wlo = (int)(uint32_t)w0, whi = (int)(uint32_t)(w0 >> 32);
  const int elo = (int)(uint32_t)end, ehi = (int)(uint32_t)(end >> 32);
#pragma unroll 8
  for (int k = 0; k < 64; k++) {
    const uint64_t bk = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane(whi, k) << 32) |
                        (uint32_t)__builtin_amdgcn_readlane(wlo, k);
    const uint64_t ek = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane(ehi, k) << 32) |
                        (uint32_t)__builtin_amdgcn_readlane(elo, k);
    const uint64_t ad = bk + 4ull * lane;
    t.rows[k * kStageRowDw + lane] =
        ad < ek ? (uint32_t)ldg1(reinterpret_cast<const void*>((uintptr_t)ad)) : 0u;
  }
  const uint64_t ad = w0 + 256;
  t.rows[lane * kStageRowDw + 64] =
      ad < end ? (uint32_t)ldg1(reinterpret_cast<const void*>((uintptr_t)ad)) : 0u;
}
// sha512_prefixed over a 64-byte register prefix and a staged tail: the block
// loop runs to the wave's largest block count (staging needs the whole wave),
// each lane compressing only its own blocks
template <int PL>
__device__ __forceinline__ void sha512_prefixed_staged(uint64_t out[8], const uint32_t* prefix,
                                                       const ShaStagedTail& tail, uint32_t tl) {
  static_assert(PL == 64, "staged tails follow a 64-byte prefix (R || A)");
  const uint32_t total = PL + tl;
  const uint32_t nb = (total + 17 + 127) >> 7;
  const uint32_t nbmax = wave_max_u32(nb);
  const uint32_t r8 = (uint32_t)((uintptr_t)tail.msg & 3u) * 8u;
  const uint32_t* row = tail.rows + (threadIdx.x & 63u) * kStageRowDw;
  uint32_t t0 = 0;
  auto word = [&](uint32_t q) -> uint64_t {  // tail bytes q..q+7, big-endian
    const uint32_t di = (q - t0) >> 2;
    const uint32_t d0 = row[di], d1 = row[di + 1], d2 = row[di + 2];
    const uint32_t lo = __builtin_amdgcn_alignbit(d1, d0, r8);
    const uint32_t hi = __builtin_amdgcn_alignbit(d2, d1, r8);
    return ((uint64_t)__builtin_bswap32(lo) << 32) | __builtin_bswap32(hi);
  };
  auto len_words = [&](uint32_t widx, uint64_t r) -> uint64_t {
    if (widx == nb * 16 - 1) return (uint64_t)total << 3;
    if (widx == nb * 16 - 2) return 0;
    return r;
  };
  uint64_t H[8];
  sha512_init(H);
  sha_stage(tail, 0, tl);
  {
    uint64_t W[16];
#pragma unroll
    for (int w = 0; w < 16; w++) {
      const uint32_t p0 = (uint32_t)(w * 8);
      uint64_t r;
      if (w < 8) {
        r = ((uint64_t)__builtin_bswap32(prefix[2 * w]) << 32) | __builtin_bswap32(prefix[2 * w + 1]);
      } else {
        r = sha_pad_word(word(p0 - PL), p0, total);
      }
      W[w] = len_words((uint32_t)w, r);
    }
    sha512_compress(H, W);
  }
#pragma unroll 1
  for (uint32_t b = 1; b < nbmax; b++) {
    if (b >= 2 && (b & 1u) == 0) {
      t0 = 256u * (b >> 1) - 64u;
      sha_stage(tail, t0, tl);
    }
    if (b < nb) {
      uint64_t W[16];
#pragma unroll
      for (int w = 0; w < 16; w++) {
        const uint32_t p0 = b * 128 + (uint32_t)w * 8;
        W[w] = len_words(b * 16 + (uint32_t)w, sha_pad_word(word(p0 - PL), p0, total));
      }
      sha512_compress(H, W);
    }
  }
#pragma unroll
  for (int i = 0; i < 8; i++) out[i] = H[i];
}
#endif

// SHA-512 over prefix (PL bytes, as little-endian packed words) || tail (tl
// bytes).  PL <= 128 - 17 is not required: the prefix may spill into block 1
// only for all-register inputs (tail length 0), which stay fully unrolled.
template <int PL, class Tail>
OURO_FI void sha512_prefixed(uint64_t out[8], const uint32_t* prefix, const Tail& tail,
                             uint32_t tl) {
#if defined(__HIP_DEVICE_COMPILE__)
  if constexpr (is_staged_tail<Tail>::value) {
    sha512_prefixed_staged<PL>(out, prefix, tail, tl);
    return;
  }
#endif
  const uint32_t total = PL + tl;
  const uint32_t nb = (total + 17 + 127) >> 7;
  uint64_t H[8];
  sha512_init(H);
  // blocks that may touch the prefix: static byte positions
  constexpr int kStaticBlocks = (PL + 127) / 128 > 0 ? (PL + 127) / 128 : 1;
#pragma unroll
  for (int b = 0; b < kStaticBlocks; b++) {
    if (b > 0 && (uint32_t)b >= nb) break;
    uint64_t W[16];
#pragma unroll
    for (int w = 0; w < 16; w++) {
      const uint32_t p0 = (uint32_t)(b * 128 + w * 8);
      uint64_t r = 0;
      if (p0 >= (uint32_t)PL) {
        r = sha_pad_word(sha_tail_word(tail, p0 - PL, tl), p0, total);
      } else {
#pragma unroll
        for (int k = 0; k < 8; k++) {
          const uint32_t p = p0 + k;
          uint32_t byte;
          if (p < (uint32_t)PL) byte = byte_of(prefix, (int)p);
          else byte = (p < total) ? tail.tail(p - PL) : (p == total ? 0x80u : 0u);
          r = (r << 8) | byte;
        }
      }
      const uint32_t widx = (uint32_t)(b * 16 + w);
      if (widx == nb * 16 - 1) r = (uint64_t)total << 3;
      else if (widx == nb * 16 - 2) r = 0;
      W[w] = r;
    }
    sha512_compress(H, W);
  }
  // remaining blocks read only the tail
#pragma unroll 1
  for (uint32_t b = kStaticBlocks; b < nb; b++) {
    uint64_t W[16], raw[16];
    if constexpr (OURO_SHA_BLOCK_LOAD && has_block_be<Tail>::value) tail.block_be(raw, b * 128 - PL, tl);
#pragma unroll
    for (int w = 0; w < 16; w++) {
      const uint32_t p0 = b * 128 + w * 8;
      uint64_t r;
      if constexpr (OURO_SHA_BLOCK_LOAD && has_block_be<Tail>::value) r = sha_pad_word(raw[w], p0, total);
      else r = sha_pad_word(sha_tail_word(tail, p0 - PL, tl), p0, total);
      const uint32_t widx = b * 16 + w;
      if (widx == nb * 16 - 1) r = (uint64_t)total << 3;
      else if (widx == nb * 16 - 2) r = 0;
      W[w] = r;
    }
    sha512_compress(H, W);
  }
#pragma unroll
  for (int i = 0; i < 8; i++) out[i] = H[i];
}

#if defined(__HIP_DEVICE_COMPILE__)
// ---- wave-cooperative SHA-512 (latency mode: one message per wave) ----------
// A latency-mode work item runs on a whole wave with every lane holding the
// same values, so a hash is one dependent chain issued by 64 lanes alike.  The
// message schedule does not depend on the chaining state: lane b builds block
// b's sixteen words and extends its schedule while the other lanes do the
// same for theirs, all blocks at once, and stores K[t] + W[t] of every round
// in LDS; the compression then runs the 80 rounds of each block with one LDS
// broadcast read per round and no schedule.  A 5-block Sum6KES leaf message
// (R || A || 544-B body) thus pays one schedule's latency instead of five.
// kGroup = 32 hashes two messages per wave (one per half; same length).
constexpr int kShaWaveMaxBlocks = 8;  // per wave (all groups together)
constexpr int kShaWaveMaxWaves = 4;   // waves per workgroup (latency blocks <= 256 threads)
__device__ __forceinline__ uint64_t* sha_wave_lds() {
  __shared__ uint64_t s_kw[kShaWaveMaxWaves * kShaWaveMaxBlocks * 80];
  return s_kw + (threadIdx.x >> 6) * (kShaWaveMaxBlocks * 80);
}
// blocks a group of kGroup lanes can hash (the caller falls back above it)
template <int kGroup>
constexpr uint32_t sha_wave_max_blocks() { return kShaWaveMaxBlocks * kGroup / 64; }

// word w (compile-time) of static block b (compile-time: a block the prefix
// reaches), padded, with the length words of an nb-block message
template <int PL, class Tail>
OURO_FI uint64_t sha_static_word(int b, int w, const uint32_t* prefix, const Tail& tail,
                                 uint32_t tl, uint32_t total, uint32_t nb) {
  const uint32_t p0 = (uint32_t)(b * 128 + w * 8);
  uint64_t r = 0;
  if (p0 >= (uint32_t)PL) {
    r = sha_pad_word(sha_tail_word(tail, p0 - PL, tl), p0, total);
  } else {
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const uint32_t p = p0 + k;
      uint32_t byte;
      if (p < (uint32_t)PL) byte = byte_of(prefix, (int)p);
      else byte = (p < total) ? tail.tail(p - PL) : (p == total ? 0x80u : 0u);
      r = (r << 8) | byte;
    }
  }
  const uint32_t widx = (uint32_t)(b * 16 + w);
  if (widx == nb * 16 - 1) r = (uint64_t)total << 3;
  else if (widx == nb * 16 - 2) r = 0;
  return r;
}

template <int PL, int kGroup, class Tail>
__device__ __forceinline__ void sha512_prefixed_wave(uint64_t out[8], const uint32_t* prefix,
                                                     const Tail& tail, uint32_t tl) {
  static_assert(kGroup == 64 || kGroup == 32, "one or two messages per wave");
  constexpr uint32_t kMaxB = sha_wave_max_blocks<kGroup>();
  constexpr int kStatic = (PL + 127) / 128 > 0 ? (PL + 127) / 128 : 1;
  const uint32_t total = PL + tl;
  const uint32_t nb = (total + 17 + 127) >> 7;  // <= kMaxB (callers check)
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t gb = lane & (uint32_t)(kGroup - 1);  // the block this lane schedules
  uint64_t* kw = sha_wave_lds() + (lane / (uint32_t)kGroup) * kMaxB * 80;
  if (gb < nb) {
    uint64_t W[16];
#pragma unroll
    for (int w = 0; w < 16; w++) {
      uint64_t r = 0;
#pragma unroll
      for (int sb = 0; sb < kStatic; sb++)
        if (gb == (uint32_t)sb) r = sha_static_word<PL>(sb, w, prefix, tail, tl, total, nb);
      if (gb >= (uint32_t)kStatic) {
        const uint32_t p0 = gb * 128 + (uint32_t)w * 8;
        r = sha_pad_word(sha_tail_word(tail, p0 - PL, tl), p0, total);
        const uint32_t widx = gb * 16 + (uint32_t)w;
        if (widx == nb * 16 - 1) r = (uint64_t)total << 3;
        else if (widx == nb * 16 - 2) r = 0;
      }
      W[w] = r;
    }
    uint64_t* k = kw + gb * 80;
#pragma unroll
    for (int i = 0; i < 16; i++) k[i] = W[i] + kSha512K[i];
#pragma unroll 1
    for (int r0 = 16; r0 < 80; r0 += 16) {
#pragma unroll
      for (int i = 0; i < 16; i++) {
        const uint64_t w15 = W[(i + 1) & 15], w2 = W[(i + 14) & 15];
        const uint64_t s0 = xor3_64(rotr64(w15, 1), rotr64(w15, 8), shr64(w15, 7));
        const uint64_t s1 = xor3_64(rotr64(w2, 19), rotr64(w2, 61), shr64(w2, 6));
        W[i] += s0 + W[(i + 9) & 15] + s1;
        k[r0 + i] = W[i] + kSha512K[r0 + i];
      }
    }
  }
  // LDS writes of this wave before its reads (one wave: a fence suffices)
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  uint64_t H[8];
  sha512_init(H);
#pragma unroll 1
  for (uint32_t b = 0; b < nb; b++) {
    const uint64_t* k = kw + b * 80;
    uint64_t a = H[0], bb = H[1], c = H[2], d = H[3], e = H[4], f = H[5], g = H[6], h = H[7];
#pragma unroll 1
    for (int t0 = 0; t0 < 80; t0 += 16) {
#pragma unroll
      for (int i = 0; i < 16; i++) sha512_round(a, bb, c, d, e, f, g, h, 0, k[t0 + i]);
    }
    H[0] += a; H[1] += bb; H[2] += c; H[3] += d; H[4] += e; H[5] += f; H[6] += g; H[7] += h;
  }
#pragma unroll
  for (int i = 0; i < 8; i++) out[i] = H[i];
}
#endif

// big-endian digest word i -> little-endian packed byte words
OURO_FI void sha512_digest_words(uint32_t out[16], const uint64_t H[8]) {
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint64_t v = H[i];
    const uint32_t hi = (uint32_t)(v >> 32), lo = (uint32_t)v;
    out[2 * i] = __builtin_bswap32(hi);
    out[2 * i + 1] = __builtin_bswap32(lo);
  }
}

}  // namespace ouro
