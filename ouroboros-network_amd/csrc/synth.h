// synth.h -- signing-side lane routines used ONLY to synthesise benchmark and
// test inputs on the device (Ed25519 keygen/sign, draft-03 VRF prove, Sum6KES
// leaf keys).  Not part of the verifier ABI; the forging side is out of scope
// for the hot path.  Deterministic, so tests pin these
// against the oracle's signer byte for byte.
#pragma once
#include "verify.h"

namespace ouro {

// a*b + c mod L (all 8-word little-endian)
OURO_FI void sc_muladd(uint32_t out[8], const uint32_t a[8], const uint32_t b[8],
                       const uint32_t c[8]) {
  uint32_t p[16];
#pragma unroll
  for (int i = 0; i < 16; i++) p[i] = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint64_t carry = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) {
      uint64_t t = (uint64_t)a[i] * b[j] + p[i + j] + carry;
      p[i + j] = (uint32_t)t;
      carry = t >> 32;
    }
    p[i + 8] = (uint32_t)carry;
  }
  uint64_t carry = 0;
#pragma unroll
  for (int i = 0; i < 16; i++) {
    uint64_t t = (uint64_t)p[i] + (i < 8 ? c[i] : 0u) + carry;
    p[i] = (uint32_t)t;
    carry = t >> 32;
  }
  sc_reduce512(out, p);
}

// [k]B for k < L, through the shared multiplication routine (B table only)
OURO_FI ge_p2 base_mul(const uint32_t k[8], Slot lane, const int32_t* btab) {
  st_words8(lane + kSlotB, k);
  st_carry(lane, 2, sc_recode_b(k));
  dsm(lane, btab, dsm_cfg(0, 0, true));
  return dsm_result(lane);
}

// [k]P for k < L
OURO_FI ge_p2 var_mul(const uint32_t k[8], const ge_p3& P, Slot lane, const int32_t* btab) {
  build_table(lane + kSlotTab1, P);
  st_words8(lane + kSlotA1, k);
  st_carry(lane, 0, sc_recode_carries<4, 64>(k));
  dsm(lane, btab, dsm_cfg(64, 0, false));
  return dsm_result(lane);
}

OURO_FI void encode_p2(uint32_t out[8], const ge_p2& p) { ge_p2_encode(out, p); }

// SHA-512 of a 32-byte register message
OURO_FI void sha512_32(uint32_t out[16], const uint32_t m[8]) {
  uint64_t H[8];
  sha512_prefixed<32>(H, m, ShaNoTail{}, 0);
  sha512_digest_words(out, H);
}

// az = SHA-512(seed) with the Ed25519 clamp; a = az[0:32] mod L
struct ExpandedKey {
  uint32_t a[8];       // clamped scalar reduced mod L
  uint32_t a_raw[8];   // clamped scalar as used for s = k + c x (reduced by muladd)
  uint32_t prefix[8];  // az[32:64]
  uint32_t pk[8];
};

OURO_FI void expand_seed(ExpandedKey& k, const uint32_t seed[8], Slot lane,
                         const int32_t* btab) {
  uint32_t az[16];
  sha512_32(az, seed);
  az[0] &= 0xfffffff8u;
  az[7] &= 0x7fffffffu;
  az[7] |= 0x40000000u;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    k.a_raw[i] = az[i];
    k.prefix[i] = az[8 + i];
  }
  sc_reduce256(k.a, k.a_raw);
  encode_p2(k.pk, base_mul(k.a, lane, btab));
}

// Ed25519 signature of a message (register prefix-free tail source)
template <class Tail>
OURO_FI void ed25519_sign_lane(uint32_t sig[16], const ExpandedKey& k, const Tail& msg,
                               uint32_t mlen, Slot lane, const int32_t* btab) {
  uint64_t H[8];
  uint32_t hw[16], r[8], h[8];
  sha512_prefixed<32>(H, k.prefix, msg, mlen);
  sha512_digest_words(hw, H);
  sc_reduce512(r, hw);
  uint32_t R[8];
  encode_p2(R, base_mul(r, lane, btab));
  uint32_t pre[16];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    pre[i] = R[i];
    pre[8 + i] = k.pk[i];
  }
  sha512_prefixed<64>(H, pre, msg, mlen);
  sha512_digest_words(hw, H);
  sc_reduce512(h, hw);
  uint32_t S[8];
  sc_muladd(S, h, k.a, r);
#pragma unroll
  for (int i = 0; i < 8; i++) {
    sig[i] = R[i];
    sig[8 + i] = S[i];
  }
}

// draft-03 prove (SURVEY.md App. B.3'), 32-byte alpha in registers
OURO_FI void vrf03_prove_lane(uint32_t pi[20], const ExpandedKey& k, const uint32_t alpha[8],
                              Slot lane, const int32_t* btab) {
  uint32_t pre[9];
  pre[0] = 0x04u | (0x01u << 8) | (k.pk[0] << 16);
#pragma unroll
  for (int i = 1; i < 8; i++) pre[i] = (k.pk[i - 1] >> 16) | (k.pk[i] << 16);
  pre[8] = k.pk[7] >> 16;
  struct RegTail32 {
    uint32_t w[8];
    OURO_FI uint32_t tail(uint32_t q) const { return byte_of(w, (int)q); }
  } at;
#pragma unroll
  for (int i = 0; i < 8; i++) at.w[i] = alpha[i];
  uint64_t Hs[8];
  sha512_prefixed<34>(Hs, pre, at, 32);
  uint32_t rw[16];
  sha512_digest_words(rw, Hs);
  rw[7] &= 0x7fffffffu;
  ge_p3 Hp = elligator2_h(rw);
  uint32_t Henc[8];
  ge_encode_with_inv(Henc, Hp.X, Hp.Y, fe_invert(Hp.Z));
  // Gamma = [x]H
  uint32_t G[8];
  encode_p2(G, var_mul(k.a, Hp, lane, btab));
  // nonce k = SHA-512(prefix || H) mod L
  uint32_t nm[16], nw[16], kk[8];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    nm[i] = k.prefix[i];
    nm[8 + i] = Henc[i];
  }
  uint64_t Hn[8];
  sha512_prefixed<64>(Hn, nm, ShaNoTail{}, 0);
  sha512_digest_words(nw, Hn);
  sc_reduce512(kk, nw);
  uint32_t KB[8], KH[8];
  encode_p2(KB, base_mul(kk, lane, btab));
  encode_p2(KH, var_mul(kk, Hp, lane, btab));
  // c = SHA-512(4 || 2 || H || Gamma || kB || kH)[0:16]
  uint32_t hp[33];
  const uint32_t* pts[4] = {Henc, G, KB, KH};
  hp[0] = 0x04u | (0x02u << 8) | (Henc[0] << 16);
#pragma unroll
  for (int q = 0; q < 4; q++) {
#pragma unroll
    for (int i = 1; i < 8; i++) hp[8 * q + i] = (pts[q][i - 1] >> 16) | (pts[q][i] << 16);
    if (q < 3) hp[8 * q + 8] = (pts[q][7] >> 16) | (pts[q + 1][0] << 16);
  }
  hp[32] = KH[7] >> 16;
  uint64_t Hc[8];
  sha512_prefixed<130>(Hc, hp, ShaNoTail{}, 0);
  uint32_t cw[16], c[8], s[8];
  sha512_digest_words(cw, Hc);
#pragma unroll
  for (int i = 0; i < 8; i++) c[i] = i < 4 ? cw[i] : 0u;
  sc_muladd(s, c, k.a, kk);
#pragma unroll
  for (int i = 0; i < 8; i++) {
    pi[i] = G[i];
    pi[12 + i] = s[i];
  }
#pragma unroll
  for (int i = 0; i < 4; i++) pi[8 + i] = c[i];
}

}  // namespace ouro
