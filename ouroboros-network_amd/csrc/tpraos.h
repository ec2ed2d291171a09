// tpraos.h -- the TPraos header combiner as phases.
//
// The crypto subset of SL.updateChainDepState reached from
// ouroboros-consensus-shelley/src/Ouroboros/Consensus/Shelley/Protocol.hs:433-442:
//   OCERT   : Ed25519 by the cold key over hotVk || BE64(n) || BE64(c0),
//             Sum6KES by hotVk over the raw header body
//   OVERLAY : draft-03 VRF verify + output for the eta and leader seeds
// Each check is a *core*: the two Ed25519 checks end in their verdict (the
// half-size equation of lattice.h compares with the identity projectively);
// the VRF cores end in projective points, and one shared *finish* inverts all
// eight Z coordinates with a single field inversion (Montgomery's trick) and
// then does every encoding, comparison and hash.  The cores are independent, so the same code runs
//   * throughput mode: one lane runs all six cores of a header, the VRF key is
//     decoded once and its [1..8](-Y) table serves both U computations;
//   * latency mode (64-header ChainSync windows): eight lanes per header run
//     the cores concurrently -- each V split into [s]H and -[c]Gamma halves so
//     the longest lane is one 252-bit chain -- and a second launch adds the
//     halves (hdr_combine_split) and finishes.
// Verdicts and outputs are identical in both modes (tests pin both against
// the oracle).
#pragma once
#include "verify.h"
#include "../../include/ouro_verify.h"

namespace ouro {

// ---- per-header result record (int32 words) --------------------------------
enum HdrPoint { kPtHe = 0, kPtUe, kPtVe, kPtG8e, kPtHl, kPtUl, kPtVl, kPtG8l, kHdrPoints };
constexpr int kPtWords = 36;                          // X, Y, Z at a 12-word stride
constexpr int kResFlags = kHdrPoints * kPtWords;      // 6 flag words, one per core
constexpr int kResWords = kResFlags + 8;              // 296 words (16-B multiple)
// latency mode: the record plus the two -[c]Gamma partial points, and for the
// fused wave-wide mode (kernels_lat.hip) per VRF the encodings of H, U, V
// (8 words each), its beta (16 words), and the header's arrival counter
constexpr int kLatPart = kResWords;
constexpr int kLatEnc = kLatPart + 2 * kPtWords;      // enc(which, k) at kLatEnc + 8 (3 which + k)
constexpr int kLatBeta = kLatEnc + 48;                // beta(which) at kLatBeta + 16 which
constexpr int kLatCtr = kLatBeta + 32;
// fused mode, each Ed25519 check (OCERT, KES leaf) split over two waves
// (wide_cores.h): its scalars, decoded points and arrival counter
constexpr int kLatEd = kLatCtr + 4;                   // Ed record e at kLatEd + kEdWords e
// (two-wave form: words 0..125; the three-wave split form, wide_cores.h
// ed_split_*: h 0, S 8, ok 16, counters 17..19, then five wave-wide points of
// 64 words from word 32)
constexpr int kEdWords = 352;
// fused mode: the eta nonce's two candidates, Blake2b-256 of the output it
// hashes if the eta VRF verifies (the claimed one when given) and of 64 zero
// bytes (a failed proof), hashed by the eta Gamma core off the critical path
constexpr int kLatNonce = kLatEd + 2 * kEdWords;
// fused split form: per VRF the wave-wide points H, [s_lo]H, [s_hi]H and
// -[c]Gamma (64 words each), combined by the last of three cores
constexpr int kPwWords = 64;
constexpr int kLatVsplit = kLatNonce + 16;            // VRF which at kLatVsplit + 4 kPwWords which
// the four-wave V (wide_cores.h vrf_sh_split; A/B): the V3 item's part per VRF
#ifndef OURO_LAT_V3
#define OURO_LAT_V3 0
#endif
// parties of a VRF's combination in the fused split form: V, V2, Gamma (and V3)
constexpr uint32_t kVParts = OURO_LAT_V3 ? 4u : 3u;
constexpr int kLatV3 = kLatVsplit + 8 * kPwWords;     // VRF which at kLatV3 + kPwWords which
constexpr int kLatResWords = kLatV3 + 2 * kPwWords;   // 1,812 words (16-B multiple)
enum HdrCore { kCoreOcert = 0, kCoreKes, kCoreUe, kCoreUl, kCoreVe, kCoreVl, kHdrCores,
               // latency mode splits each V = [s]H - [c]Gamma over two lanes: the V
               // cores do [s]H (252-bit chain), these do -[c]Gamma (128-bit chain)
               kCoreGe = kHdrCores, kCoreGl, kLatCores };
// flag bits
constexpr int32_t kFlagOk = 1;        // the core's acceptance checks passed
constexpr int32_t kFlagGammaX0 = 2;   // Gamma decoded with x = 0 (re-encodes with sign 0)

// ---- optional members of a batch (include/ouro_verify.h) -------------------
// As bits: taken from the pointers (throughput kernel, host paths) or read
// from device memory next to n (latency kernels replayed from a captured
// graph, whose device struct always points somewhere).
constexpr uint32_t kOptEtaClaim = 1u;     // eta_output given
constexpr uint32_t kOptLeaderClaim = 2u;  // leader_output given
constexpr uint32_t kOptSeeds = 4u;        // slot given: alphas = mkSeed on device
constexpr uint32_t kOptEpochNonce = 8u;   // epoch_nonce given (else NeutralNonce)
constexpr uint32_t kOptEtaNonce = 16u;    // eta_nonce output wanted
OURO_HD inline uint32_t batch_opts(const ouro_tpraos_batch& b) {
  return (b.eta_output ? kOptEtaClaim : 0u) | (b.leader_output ? kOptLeaderClaim : 0u) |
         (b.slot ? kOptSeeds : 0u) | (b.slot && b.epoch_nonce ? kOptEpochNonce : 0u) |
         (b.eta_nonce ? kOptEtaNonce : 0u);
}

OURO_FI void st_point_at(Slot p, const fe& X, const fe& Y, const fe& Z) {
  st_fe(p, X);
  st_fe(p + 12, Y);
  st_fe(p + 24, Z);
}
OURO_FI void st_point(Slot res, int which, const fe& X, const fe& Y, const fe& Z) {
  st_point_at(res + which * kPtWords, X, Y, Z);
}
OURO_FI ge_p2 ld_point_at(Slot p) {
  return ge_p2{ld_fe(p), ld_fe(p + 12), ld_fe(p + 24)};
}
OURO_FI void st_point_from_dsm(Slot res, int which, Slot lane) {
  const ge_p2 r = dsm_result(lane);
  st_point(res, which, r.X, r.Y, r.Z);
}

// ---- cores ---------------------------------------------------------------
// Message bytes held in registers (W words); a select chain keeps a dynamic
// byte index out of scratch -- in every SHA-512 call here the index is a
// compile-time constant after unrolling, so the chain folds away.
template <int W>
struct RegMsg {
  uint32_t w[W];
  OURO_FI uint32_t tail(uint32_t q) const {
    uint32_t r = w[0];
#pragma unroll
    for (int i = 1; i < W; i++) r = ((q >> 2) == (uint32_t)i) ? w[i] : r;
    return (r >> (8 * (q & 3))) & 0xffu;
  }
};
// OCERT signature: message hotVk || BE64(counter) || BE64(c0)
using OcertMsg = RegMsg<12>;
// a 32-byte VRF input (the Seed)
using SeedMsg = RegMsg<8>;

OURO_FI uint32_t bswap32_hd(uint32_t x) {
  return (x >> 24) | ((x >> 8) & 0xff00u) | ((x << 8) & 0xff0000u) | (x << 24);
}

OURO_HD inline void ocert_msg(OcertMsg& m, const uint32_t hot_vk[8], uint64_t ctr, uint64_t c0) {
#pragma unroll
  for (int i = 0; i < 8; i++) m.w[i] = hot_vk[i];
  m.w[8] = bswap32_hd((uint32_t)(ctr >> 32));
  m.w[9] = bswap32_hd((uint32_t)ctr);
  m.w[10] = bswap32_hd((uint32_t)(c0 >> 32));
  m.w[11] = bswap32_hd((uint32_t)c0);
}

// U = [s]B - [c]Y.  With build_y the key is validated/decoded and its [1..8](-Y)
// table written to table slot `yslot`; otherwise a previous call's table is
// reused (throughput mode: both VRFs of a header share the key).
OURO_HD inline bool vrf_u_core(const uint32_t pk[8], const uint32_t pi[20], bool build_y,
                               int yslot, Slot lane, const int32_t* btab,
                               bool quad = false, int phase = kPhaseAll) {
  bool ok = true;
  if (build_y) {
    ge_p3 Y;
    ok = !ge_has_small_order(pk) && ge_is_canonical(pk);
    ok = ge_decode(&Y, pk, false) && ok;
    build_table(lane + yslot * kTabWords, ge_p3_neg(Y), quad);
  }
  uint32_t c[8], s_raw[8], s[8];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    s_raw[i] = pi[12 + i];
    c[i] = i < 4 ? pi[8 + i] : 0u;
  }
  sc_reduce256(s, s_raw);
  st_words8(lane + kSlotA1, c);
  st_words8(lane + kSlotB, s);
  st_carry(lane, 0, sc_recode_carries<4, 33>(c));
  st_carry(lane, 2, sc_recode_b(s));
  dsm_or_defer(lane, btab, dsm_cfg(33, 0, true, yslot, 1), quad, phase);
  return ok;
}

// Gamma checks, H = hash_to_curve(Y, alpha), V = [s]H - [c]Gamma, [8]Gamma.
// Writes H, V, [8]Gamma into res; returns the flag word.  part = 0: all of it
// (throughput mode); part = 1: H and [s]H only, written as V; part = 2: the
// Gamma checks, [8]Gamma and -[c]Gamma, written to `partial` (latency mode:
// the two halves run on two lanes and hdr_combine_split adds them).
template <class Tail>
OURO_HD inline int32_t vrf_v_core(const uint32_t pk[8], const uint32_t pi[20], const Tail& alpha,
                                  uint32_t alen, Slot lane, const int32_t* btab,
                                  Slot res, int ptH, int ptV, int ptG8, int part,
                                  Slot partial, bool quad = false, int phase = kPhaseAll) {
  uint32_t G[8], c[8], s_raw[8], s[8];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    G[i] = pi[i];
    s_raw[i] = pi[12 + i];
    c[i] = i < 4 ? pi[8 + i] : 0u;
  }
  ge_p3 Gamma;
  bool ok = true;
  // throughput mode: Gamma's decode and Elligator2 share one paired
  // exponentiation (fe_pow22523_x2); the latency split cores do one each
  const bool pair = OURO_DECODE_PAIR && part == 0;
  DecodePre gpre;
  fe gbase;
  if (part != 1) {
    ok = ge_is_canonical(G);
    if (pair) gbase = ge_decode_pre(gpre, G);
    else ok = ge_decode(&Gamma, G, false) && ok;
  }
  if (part == 2) {
    build_table(lane + kSlotTab1, ge_p3_neg(Gamma), quad);
    st_words8(lane + kSlotA1, c);
    st_carry(lane, 0, sc_recode_carries<4, 33>(c));
    dsm(lane, btab, dsm_cfg(33, 0, false, 0, 1), quad);
    const ge_p2 r = dsm_result(lane);
    st_point_at(partial, r.X, r.Y, r.Z);
  } else {
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
    if (pair) {
      Ell2Pre epre;
      const fe ebase = elligator2_pre(epre, rw);
      const fe_pair pw = fe_pow22523_x2(gbase, ebase);
      ok = ge_decode_post(&Gamma, gpre, pw.a, G, false) && ok;
      Hp = elligator2_post(epre, pw.b);
    } else {
      Hp = elligator2_h(rw);
    }
    st_point(res, ptH, Hp.X, Hp.Y, Hp.Z);
    build_table(lane + kSlotTab1, Hp, quad);
    st_words8(lane + kSlotA1, s);
    st_carry(lane, 0, sc_recode_carries<4, 64>(s));
    if (part == 0) {
      build_table(lane + kSlotTab2, ge_p3_neg(Gamma), quad);
      st_words8(lane + kSlotA2, c);
      st_carry(lane, 1, sc_recode_carries<4, 33>(c));
      dsm_or_defer(lane, btab, dsm_cfg(64, 33, false, 0, 1), quad, phase);
    } else {
      dsm(lane, btab, dsm_cfg(64, 0, false, 0, 1), quad);
    }
    if (phase != kPhasePre) st_point_from_dsm(res, ptV, lane);
    if (part == 1) return kFlagOk;
  }
  ge_p3 G8 = ge_mul8(Gamma);
  st_point(res, ptG8, G8.X, G8.Y, G8.Z);
  return (ok ? kFlagOk : 0) | (fe_iszero(Gamma.X) ? kFlagGammaX0 : 0);
}

// ---- finish ----------------------------------------------------------------
OURO_FI void pack_shifted(uint32_t* dst, int word0, const uint32_t p[8]) {
  // append 32 bytes at byte offset 4*word0 - 2 (the 2-byte suite/tag prefix
  // shifts every point by 2 bytes); caller seeds dst[word0 - 1] high half
  dst[word0 - 1] |= p[0] << 16;
#pragma unroll
  for (int i = 1; i < 8; i++) dst[word0 - 1 + i] = (p[i - 1] >> 16) | (p[i] << 16);
  dst[word0 + 7] = p[7] >> 16;
}

// beta = SHA-512(suite || 0x03 || encode([8]Gamma))
OURO_HD inline void vrf_beta(uint32_t beta[16], const uint32_t G8enc[8]) {
  uint32_t bp[9];
  bp[0] = 0x04u | (0x03u << 8);
  pack_shifted(bp, 1, G8enc);
  uint64_t Hb[8];
  sha512_prefixed<34>(Hb, bp, ShaNoTail{}, 0);
  sha512_digest_words(beta, Hb);
}

// c' = SHA-512(suite || 0x02 || H || Gamma || U || V)[0..16) == c
OURO_HD inline bool vrf_challenge_ok(const uint32_t Henc[8], const uint32_t Genc[8],
                                     const uint32_t Uenc[8], const uint32_t Venc[8],
                                     const uint32_t c[4]) {
  uint32_t hp[33];
  hp[0] = 0x04u | (0x02u << 8);
  pack_shifted(hp, 1, Henc);
  pack_shifted(hp, 9, Genc);
  pack_shifted(hp, 17, Uenc);
  pack_shifted(hp, 25, Venc);
  uint64_t Hc[8];
  sha512_prefixed<130>(Hc, hp, ShaNoTail{}, 0);
  uint32_t cw[16];
  sha512_digest_words(cw, Hc);
  bool ceq = true;
#pragma unroll
  for (int i = 0; i < 4; i++) ceq = ceq && cw[i] == c[i];
  return ceq;
}

// c' check and beta for one VRF; H/U/V/G8 encodings given
OURO_HD inline bool vrf_finish(uint32_t beta[16], const uint32_t Henc[8], const uint32_t Genc[8],
                               const uint32_t Uenc[8], const uint32_t Venc[8],
                               const uint32_t G8enc[8], const uint32_t c[4]) {
  uint32_t hp[33];
  hp[0] = 0x04u | (0x02u << 8);
  pack_shifted(hp, 1, Henc);
  pack_shifted(hp, 9, Genc);
  pack_shifted(hp, 17, Uenc);
  pack_shifted(hp, 25, Venc);
  uint64_t Hc[8];
  sha512_prefixed<130>(Hc, hp, ShaNoTail{}, 0);
  uint32_t cw[16];
  sha512_digest_words(cw, Hc);
  bool ceq = true;
#pragma unroll
  for (int i = 0; i < 4; i++) ceq = ceq && cw[i] == c[i];
  uint32_t bp[9];
  bp[0] = 0x04u | (0x03u << 8);
  pack_shifted(bp, 1, G8enc);
  uint64_t Hb[8];
  sha512_prefixed<34>(Hb, bp, ShaNoTail{}, 0);
  sha512_digest_words(beta, Hb);
  return ceq;
}

// Latency mode: V = [s]H + (-[c]Gamma) from the two half cores, and the V
// flag word from both (acceptance of both halves; Gamma's x = 0 bit from the
// Gamma half).  Complete projective addition, so no case is special.
OURO_HD inline void hdr_combine_split(Slot res) {
#pragma unroll 1
  for (int which = 0; which < 2; which++) {
    const int ptV = which ? kPtVl : kPtVe;
    const ge_p2 V = ge_p2_add(ld_point_at(res + ptV * kPtWords),
                              ld_point_at(res + kLatPart + which * kPtWords));
    st_point(res, ptV, V.X, V.Y, V.Z);
    int32_t* fv = res.word(kResFlags + (which ? kCoreVl : kCoreVe));
    const int32_t fg = ldg1(res.word(kResFlags + (which ? kCoreGl : kCoreGe)));
    stg1(fv, (ldg1(fv) & fg & kFlagOk) | (fg & kFlagGammaX0));
  }
}

// One inversion for all eight Z; tmp = 8 x 12 scratch words.  Then every
// comparison and hash.  Returns the OURO_HDR_* verdict bits.
OURO_HD inline uint32_t hdr_finish(Slot res, Slot tmp, const uint32_t pie[20],
                                   const uint32_t pil[20], uint32_t beta_e[16],
                                   uint32_t beta_l[16]) {
  // prefix products P_k = Z_0 ... Z_k
  fe acc = ld_fe(res + 24);
  st_fe(tmp, acc);
#pragma unroll 1
  for (int k = 1; k < kHdrPoints; k++) {
    acc = fe_mul(acc, ld_fe(res + k * kPtWords + 24));
    st_fe(tmp + 12 * k, acc);
  }
  fe inv = fe_invert_vartime(acc);
  // walk back: Z_k^-1 = inv * P_{k-1}, inv <- inv * Z_k
#pragma unroll 1
  for (int k = kHdrPoints - 1; k > 0; k--) {
    const fe zk = ld_fe(res + k * kPtWords + 24);
    st_fe(tmp + 12 * k, fe_mul(inv, ld_fe(tmp + 12 * (k - 1))));
    inv = fe_mul(inv, zk);
  }
  st_fe(tmp, inv);
  uint32_t enc[kHdrPoints][8];
#pragma unroll
  for (int k = 0; k < kHdrPoints; k++)
    ge_encode_with_inv(enc[k], ld_fe(res + k * kPtWords), ld_fe(res + k * kPtWords + 12),
                       ld_fe(tmp + 12 * k));
  auto fl = [&](int core) { return ldg1(res.word(kResFlags + core)); };
  uint32_t v = 0;
  if (fl(kCoreOcert) & kFlagOk) v |= 0x01u;
  if (fl(kCoreKes) & kFlagOk) v |= 0x02u;
#pragma unroll 1
  for (int which = 0; which < 2; which++) {
    const uint32_t* pi = which ? pil : pie;
    const int base = which ? kPtHl : kPtHe;
    const int32_t fu = fl(which ? kCoreUl : kCoreUe), fv = fl(which ? kCoreVl : kCoreVe);
    uint32_t Genc[8], c[4], b[16];
#pragma unroll
    for (int i = 0; i < 8; i++) Genc[i] = pi[i];
    if (fv & kFlagGammaX0) Genc[7] &= 0x7fffffffu;
#pragma unroll
    for (int i = 0; i < 4; i++) c[i] = pi[8 + i];
    const bool ceq = vrf_finish(b, enc[base], Genc, enc[base + 1], enc[base + 2], enc[base + 3], c);
    const bool ok = (fu & kFlagOk) && (fv & kFlagOk) && ceq;
    uint32_t* dst = which ? beta_l : beta_e;
#pragma unroll
    for (int i = 0; i < 16; i++) dst[i] = ok ? b[i] : 0u;
    if (ok) v |= which ? 0x08u : 0x04u;
  }
  return v;
}

// Latency-mode finish of ONE VRF (which = 0: eta, 1: leader) straight from
// the split cores' record: V = [s]H + (-[c]Gamma), one inversion for this
// VRF's four Z (H, U, V, [8]Gamma), the c' check and beta.  Returns the VRF's
// verdict bit (OURO_HDR 0x04 / 0x08); beta is zeroed unless it is set.  The
// two VRFs of a header run on two lane pairs of a quad (k_tpraos_finish), so
// a header's finish takes one VRF's time.  Reads res only.
OURO_HD inline uint32_t vrf_finish_split(Slot res, int which, const uint32_t pi[20],
                                         uint32_t beta[16]) {
  const int base = which ? kPtHl : kPtHe;
  const ge_p2 V = ge_p2_add(ld_point_at(res + (base + 2) * kPtWords),
                            ld_point_at(res + kLatPart + which * kPtWords));
  auto fl = [&](int core) { return ldg1(res.word(kResFlags + core)); };
  const int32_t fu = fl(which ? kCoreUl : kCoreUe);
  const int32_t fg = fl(which ? kCoreGl : kCoreGe);
  const int32_t fv = (fl(which ? kCoreVl : kCoreVe) & fg & kFlagOk) | (fg & kFlagGammaX0);
  // Z^-1 of H, U, V, [8]Gamma by one inversion (prefix products)
  const fe z0 = ld_fe(res + base * kPtWords + 24), z1 = ld_fe(res + (base + 1) * kPtWords + 24);
  const fe z3 = ld_fe(res + (base + 3) * kPtWords + 24);
  const fe p1 = fe_mul(z0, z1), p2 = fe_mul(p1, V.Z);
  fe inv = fe_invert_vartime(fe_mul(p2, z3));
  const fe i3 = fe_mul(inv, p2);
  inv = fe_mul(inv, z3);
  const fe i2 = fe_mul(inv, p1);
  inv = fe_mul(inv, V.Z);
  const fe i1 = fe_mul(inv, z0), i0 = fe_mul(inv, z1);
  uint32_t Henc[8], Uenc[8], Venc[8], G8enc[8];
  ge_encode_with_inv(Henc, ld_fe(res + base * kPtWords), ld_fe(res + base * kPtWords + 12), i0);
  ge_encode_with_inv(Uenc, ld_fe(res + (base + 1) * kPtWords),
                     ld_fe(res + (base + 1) * kPtWords + 12), i1);
  ge_encode_with_inv(Venc, V.X, V.Y, i2);
  ge_encode_with_inv(G8enc, ld_fe(res + (base + 3) * kPtWords),
                     ld_fe(res + (base + 3) * kPtWords + 12), i3);
  uint32_t Genc[8], c[4], b[16];
#pragma unroll
  for (int i = 0; i < 8; i++) Genc[i] = pi[i];
  if (fv & kFlagGammaX0) Genc[7] &= 0x7fffffffu;
#pragma unroll
  for (int i = 0; i < 4; i++) c[i] = pi[8 + i];
  const bool ceq = vrf_finish(b, Henc, Genc, Uenc, Venc, G8enc, c);
  const bool ok = (fu & kFlagOk) && (fv & kFlagOk) && ceq;
#pragma unroll
  for (int i = 0; i < 16; i++) beta[i] = ok ? b[i] : 0u;
  return ok ? (which ? 0x08u : 0x04u) : 0u;
}

// The App. B.3 flag bits of a header (include/ouro_verify.h
// OURO_HDR_*_S_UNREDUCED): s = pi[48..80) not below L, from the bytes alone
OURO_FI uint32_t hdr_s_bits(const uint32_t pie[20], const uint32_t pil[20]) {
  return (sc_is_canonical(pie + 12) ? 0u : OURO_HDR_ETA_S_UNREDUCED) |
         (sc_is_canonical(pil + 12) ? 0u : OURO_HDR_LEADER_S_UNREDUCED);
}

// ---- per-header drivers (the kernels' bodies; host-testable) -------------
OURO_FI void ld_words(uint32_t* w, const uint8_t* p, int n16) {
#pragma unroll
  for (int i = 0; i < n16; i++) {
    const int4 v = ldg4(p + 16 * i);
    w[4 * i] = v.x; w[4 * i + 1] = v.y; w[4 * i + 2] = v.z; w[4 * i + 3] = v.w;
  }
}
OURO_FI void st_words(uint8_t* p, const uint32_t* w, int n16) {
#pragma unroll
  for (int i = 0; i < n16; i++)
    stg4(p + 16 * i, make_int4((int)w[4 * i], (int)w[4 * i + 1], (int)w[4 * i + 2], (int)w[4 * i + 3]));
}

// The VRF input of header i: mkSeed seedEta / seedL slot eta0 on the device
// (Shelley/Protocol.hs:409-410; blake2b.h mkseed_hash) when the batch carries
// slots, else the caller's 32 bytes.
// (out of line: the Blake2b state stays out of the cores' register budget)
OURO_NI void hdr_mkseed(uint32_t a[8], const ouro_tpraos_batch& b, size_t i, bool leader,
                        uint32_t opts) {
  uint32_t e0[8];
  if (opts & kOptEpochNonce) ld_words(e0, b.epoch_nonce, 2);
  mkseed_hash(a, b.slot[i], (opts & kOptEpochNonce) ? e0 : nullptr);
#pragma unroll
  for (int k = 0; k < 8; k++) a[k] ^= leader ? kSeedL[k] : kSeedEta[k];
}
OURO_HD inline void hdr_seed(SeedMsg& a, const ouro_tpraos_batch& b, size_t i, bool leader,
                             uint32_t opts) {
  if (opts & kOptSeeds) {
    hdr_mkseed(a.w, b, i, leader, opts);
  } else {
    ld_words(a.w, (leader ? b.leader_alpha : b.eta_alpha) + 32 * i, 2);
  }
}

// One core of header i (tpraos.h); throughput mode reuses the VRF key table
// built by the eta U core (table slot 2) for the leader U core.
// opts: the batch's optional members (batch_opts / the latency launches' word).
// phase (the split header kernel, throughput mode only): kPhasePre runs
// every step before the core's dsm, leaving its inputs in `lane` (the core's
// own task slot) and its flag in res; kPhasePost, after the dsm launch, stores
// the dsm's point or clears the Ed25519 core's flag unless its result is the
// identity.  The leader U core's pre copies the shared key table from the eta
// U core's task slot `ukey` instead of decoding the key again.
OURO_HD inline void hdr_core(const ouro_tpraos_batch& b, size_t i, uint32_t opts, int core,
                             Slot lane, Slot res, const int32_t* btab,
                             bool share_key = true, bool split = false, bool quad = false,
                             int phase = kPhaseAll, Slot ukey = Slot{nullptr}) {
  if (phase == kPhasePost) {
    if (core == kCoreOcert || core == kCoreKes) {
      if (!dsm_result_is_identity(lane)) stg1(res.word(kResFlags + core), 0);
    } else {
      st_point_from_dsm(res, core == kCoreUe ? kPtUe : core == kCoreUl ? kPtUl
                                             : core == kCoreVe ? kPtVe : kPtVl, lane);
    }
    return;
  }
  int32_t flag = 0;
  switch (core) {
    case kCoreOcert: {
      uint32_t s[16], p[8], hv[8];
      ld_words(s, b.ocert_sigma + 64 * i, 4);
      ld_words(p, b.issuer_vk + 32 * i, 2);
      ld_words(hv, b.hot_vk + 32 * i, 2);
      OcertMsg m;
      ocert_msg(m, hv, b.ocert_counter[i], b.ocert_kes_period[i]);
      flag = ed25519_verify_lane(s, p, m, 48, lane, btab, false, quad, phase) ? kFlagOk : 0;
      break;
    }
    case kCoreKes: {
      uint32_t hv[8];
      ld_words(hv, b.hot_vk + 32 * i, 2);
      const uint32_t* sw = reinterpret_cast<const uint32_t*>(b.kes_sig + 448 * i);
      flag = sum6kes_verify_lane(hv, b.kes_t[i], sw, ShaGlobalTail{b.body + b.body_off[i]},
                                 b.body_len[i], lane, btab, quad, phase) ? kFlagOk : 0;
      break;
    }
    case kCoreUe:
    case kCoreUl: {
      const bool leader = core == kCoreUl;
      uint32_t p[8], pi[20];
      ld_words(p, b.vrf_vk + 32 * i, 2);
      ld_words(pi, (leader ? b.leader_proof : b.eta_proof) + 80 * i, 5);
      const bool build = !(share_key && leader);
      if (!build && phase == kPhasePre) {
        // the eta core's [1..8](-Y) into this core's own task slot
#pragma unroll 1
        for (int k = 0; k < kTabWords / 4; k++)
          stg4((lane + kSlotTab3).chunk(k), ldg4((ukey + kSlotTab3).chunk(k)));
      }
      const bool ok = vrf_u_core(p, pi, build, 2, lane, btab, quad, phase);
      flag = build ? (ok ? kFlagOk : 0) : (ldg1(res.word(kResFlags + kCoreUe)) & kFlagOk);
      if (phase != kPhasePre) st_point_from_dsm(res, leader ? kPtUl : kPtUe, lane);
      break;
    }
    default: {  // kCoreVe / kCoreVl, and in latency mode kCoreGe / kCoreGl
      const bool gamma = core == kCoreGe || core == kCoreGl;
      const bool leader = core == kCoreVl || core == kCoreGl;
      uint32_t p[8], pi[20];
      ld_words(p, b.vrf_vk + 32 * i, 2);
      ld_words(pi, (leader ? b.leader_proof : b.eta_proof) + 80 * i, 5);
      // the 32-byte VRF input (the caller's alpha, or mkSeed's output) staged
      // in the lane slot's (still free) result area
      if (!gamma) {
        uint32_t w[8];
        if (opts & kOptSeeds) hdr_mkseed(w, b, i, leader, opts);
        else ld_words(w, (leader ? b.leader_alpha : b.eta_alpha) + 32 * i, 2);
        st_words8(lane + kSlotOut, w);
      }
      flag = vrf_v_core(p, pi, SlotTail{lane + kSlotOut}, 32, lane, btab, res,
                        leader ? kPtHl : kPtHe, leader ? kPtVl : kPtVe,
                        leader ? kPtG8l : kPtG8e, gamma ? 2 : (split ? 1 : 0),
                        res + kLatPart + (leader ? kPtWords : 0), quad, phase);
      break;
    }
  }
  stg1(res.word(kResFlags + core), flag);
}

// The claimed-output bit of one VRF (OURO_HDR_ETA_CLAIM_OK / _LEADER_CLAIM_OK):
// the header's certifiedOutput equals the output computed from a valid proof.
OURO_HD inline uint32_t hdr_claim_bit(const ouro_tpraos_batch& b, size_t i, uint32_t opts,
                                      int which, bool proof_ok, const uint32_t beta[16]) {
  if (!proof_ok || !(opts & (which ? kOptLeaderClaim : kOptEtaClaim))) return 0u;
  uint32_t cl[16];
  ld_words(cl, (which ? b.leader_output : b.eta_output) + 64 * i, 4);
  uint32_t diff = 0;
#pragma unroll
  for (int k = 0; k < 16; k++) diff |= cl[k] ^ beta[k];
  return diff ? 0u : (which ? 0x20u : 0x10u);
}

// eta_nonce[i] = mkNonceFromOutputVRF of the eta output the nonce update
// consumes: Blake2b-256 of the CLAIMED output when the batch carries it (the
// reference's PRTCL rule hashes VRF.certifiedOutput of bheaderEta), else of
// the computed beta_eta (zeros for a failed proof: the header is invalid).
OURO_NI void hdr_eta_nonce(const ouro_tpraos_batch& b, size_t i, uint32_t opts,
                           const uint32_t beta_e[16]) {
  if (!(opts & kOptEtaNonce)) return;
  uint32_t in[16], h[8];
  if (opts & kOptEtaClaim) {
    ld_words(in, b.eta_output + 64 * i, 4);
  } else {
#pragma unroll
    for (int k = 0; k < 16; k++) in[k] = beta_e[k];
  }
  blake2b256_64(h, in);
  st_words(b.eta_nonce + 32 * i, h, 2);
}

// The claimed-output bits and the eta nonce of header i, re-reading the
// outputs the finish has just stored: out of line, so neither the comparison
// nor the Blake2b state lengthens the finish's live ranges (scratch frame).
constexpr uint32_t kOptPost = kOptEtaClaim | kOptLeaderClaim | kOptEtaNonce;
OURO_NI void hdr_post(const ouro_tpraos_batch& b, size_t i, uint32_t opts, uint8_t* verdict,
                      const uint8_t* beta_eta, const uint8_t* beta_leader) {
  uint32_t v = verdict[i], be[16], bl[16];
  ld_words(be, beta_eta + 64 * i, 4);
  ld_words(bl, beta_leader + 64 * i, 4);
  v |= hdr_claim_bit(b, i, opts, 0, (v & 0x04u) != 0, be);
  v |= hdr_claim_bit(b, i, opts, 1, (v & 0x08u) != 0, bl);
  hdr_eta_nonce(b, i, opts, be);
  verdict[i] = (uint8_t)v;
}

// latency-mode finish of header i, VRF by VRF (the host form of the lane-pair
// finish in k_tpraos_finish)
OURO_HD inline void hdr_finish_item_split(const ouro_tpraos_batch& b, size_t i, uint32_t opts,
                                          Slot res, uint8_t* verdict,
                                          uint8_t* beta_eta, uint8_t* beta_leader) {
  uint32_t v = 0;
  if (ldg1(res.word(kResFlags + kCoreOcert)) & kFlagOk) v |= 0x01u;
  if (ldg1(res.word(kResFlags + kCoreKes)) & kFlagOk) v |= 0x02u;
  for (int which = 0; which < 2; which++) {
    uint32_t pi[20], beta[16];
    ld_words(pi, (which ? b.leader_proof : b.eta_proof) + 80 * i, 5);
    if (!sc_is_canonical(pi + 12)) v |= which ? OURO_HDR_LEADER_S_UNREDUCED : OURO_HDR_ETA_S_UNREDUCED;
    const uint32_t bit = vrf_finish_split(res, which, pi, beta);
    v |= bit | hdr_claim_bit(b, i, opts, which, bit != 0, beta);
    if (!which) hdr_eta_nonce(b, i, opts, beta);
    uint8_t* dst = which ? beta_leader : beta_eta;
    if (dst) st_words(dst + 64 * i, beta, 4);
  }
  verdict[i] = (uint8_t)v;
}

OURO_HD inline void hdr_finish_item(const ouro_tpraos_batch& b, size_t i, uint32_t opts,
                                     Slot res, Slot tmp, uint8_t* verdict,
                                     uint8_t* beta_eta, uint8_t* beta_leader) {
  uint32_t pie[20], pil[20], be[16], bl[16];
  ld_words(pie, b.eta_proof + 80 * i, 5);
  ld_words(pil, b.leader_proof + 80 * i, 5);
  const uint32_t v = hdr_finish(res, tmp, pie, pil, be, bl) | hdr_s_bits(pie, pil);
  if (beta_eta) st_words(beta_eta + 64 * i, be, 4);
  if (beta_leader) st_words(beta_leader + 64 * i, bl, 4);
  verdict[i] = (uint8_t)v;
  // claimed outputs / eta nonce: from the results just stored (both outputs
  // are required then; the kernels always pass them)
  if (opts & kOptPost) hdr_post(b, i, opts, verdict, beta_eta, beta_leader);
}


}  // namespace ouro
