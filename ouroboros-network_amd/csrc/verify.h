// verify.h -- lane-level verification routines (one item per lane).
//
// Every routine here is the per-item body of a gfx950 kernel in kernels.hip:
//   ed25519_verify_lane  <- libsodium 1.0.18 crypto_sign_ed25519_verify_detached
//                           
//   vrf03_verify_lane    <- crypto_vrf_ietfdraft03_verify + proof_to_hash
//                           (cardano-crypto-praos; §8(a) a5/a6, App. B.3)
//   sum6kes_verify_lane  <- cardano-crypto-class SumKES/SingleKES verifyKES
//                           (§8(a) a3, App. B.2)
// Control flow is wave-uniform: rejected items still run the arithmetic and
// are masked at the end, so no lane diverges on secret-independent but
// data-dependent checks.
//
// Double-scalar multiplication: signed fixed windows (width 4 for variable
// points, width 8 for the fixed base B), one doubling chain shared by every
// scalar, so the adds happen at the same bit positions in every lane.  Per-lane
// tables of [1..8]P in cached form live in a per-lane global scratch slot;
// the [1..128]B niels table is shared (global, L1/L2 resident).
#pragma once
#include <vector>

#include "blake2b.h"
#include "ge25519.h"
#include "lattice.h"
#include "modinv.h"
#include "sc25519.h"
#include "sha512.h"

namespace ouro {

// ---- per-lane scratch slot layout (int32 words) ----------------------------
constexpr int kCachedWords = 40;                  // 4 fe
constexpr int kTabEntries = 8;                    // [1..8]P
constexpr int kTabWords = kTabEntries * kCachedWords;
constexpr int kSlotTab1 = 0;                      // table slot 0
constexpr int kSlotTab2 = kTabWords;              // table slot 1
constexpr int kSlotTab3 = 2 * kTabWords;          // table slot 2 (header kernel: -Y)
constexpr int kSlotA1 = 3 * kTabWords;            // 8 words
constexpr int kSlotA2 = kSlotA1 + 8;
constexpr int kSlotB = kSlotA2 + 8;
constexpr int kSlotCarry = kSlotB + 8;            // 6 words (3 x u64)
constexpr int kSlotOut = kSlotCarry + 8;          // p2 result: 3 fe at 12-word stride
constexpr int kLaneWords = kSlotOut + 36;         // 1028 words = 4112 B (16-B multiple)

// ---- scratch slots -----------------------------------------------------------
// The slots of kSlotGroup consecutive lanes are interleaved in 16-byte chunks:
// chunk k of slot (g * kSlotGroup + j) sits at words
//   g * kSlotGroup * slot_words + k * kChunkStride + 4 j.
// Every slot offset used is a multiple of 4 words; words inside a chunk are
// contiguous (int2 / uint64 accesses at even words stay inside one chunk).
// kSlotGroup = 1 is the plain lane-major layout (a slot is contiguous), the
// default: the table reads are per-lane GATHERS (each lane's digit picks its
// own entry), so a lane wants its 160-B entry in as few lines as possible.
// Interleaving the 64 slots of a wave (OURO_SLOT_GROUP=64) coalesces the
// uniform accesses (scalars, table stores) but spreads every gathered entry
// over ten 1-KiB-apart lines: measured 2.0x the HBM traffic (411 vs 207
// KB/header), +51 % VMEM instructions and +6.4 % kernel time
// (profiles/r02b).  The host build uses the same layout as the device.
#ifndef OURO_SLOT_GROUP
#define OURO_SLOT_GROUP 1
#endif
constexpr int kSlotGroup = OURO_SLOT_GROUP;
constexpr int kChunkStride = 4 * kSlotGroup;       // words between a slot's chunks
struct Slot {
  int32_t* p;  // chunk 0 of this slot
  // the slot region starting at word w (w a multiple of 4)
  OURO_FI Slot operator+(int w) const {
    OURO_TRK(if (w & 3) ouro_trk_violation();)
    return Slot{p + (w >> 2) * kChunkStride};
  }
  // k chunks further (run-time table entry offsets)
  OURO_FI Slot chunks(int k) const { return Slot{p + k * kChunkStride}; }
  OURO_FI int32_t* word(int w) const { return p + (w >> 2) * kChunkStride + (w & 3); }
  OURO_FI int4* chunk(int k) const { return reinterpret_cast<int4*>(p + k * kChunkStride); }
};
// slot s of a region of slots of slot_words words each (slot_words % 4 == 0;
// the region holds a multiple of kSlotGroup slots)
OURO_FI Slot slot_of(int32_t* base, size_t s, int slot_words) {
  return Slot{base + (s / kSlotGroup) * (size_t)kSlotGroup * slot_words + (s % kSlotGroup) * 4};
}
// words a region of n slots takes (rounded up to whole groups)
constexpr size_t slot_region_words(size_t n, int slot_words) {
  return (n + kSlotGroup - 1) / kSlotGroup * kSlotGroup * (size_t)slot_words;
}

// Fixed base B: the scalar is split at bit 128 (halves with B and 2^128 B, so
// the doubling chain spans 128 bits) and each half is cut into signed digits
// of kBW bits, one every kBW / 4 windows of the chain.  kBW = 16: 8 additions
// per half from tables of 2^15 affine points (2 x 4 MiB, MALL/L2-resident).
#ifndef OURO_BW
#define OURO_BW 16
#endif
constexpr int kBW = OURO_BW;                       // 8, 12 or 16
constexpr int kBStride = kBW / 4;                 // chain windows per B digit
// widths dividing 128 recode b as one number (a carry out of the low half
// continues in the high half); others recode each half alone, with headroom
constexpr bool kBSplitRecode = (128 % kBW) != 0;
constexpr int kBDigitsHalf = kBSplitRecode ? (128 + kBW) / kBW : 128 / kBW;
constexpr int kBTabEntries = 1 << (kBW - 1);      // [1..2^(W-1)]B, then the same of 2^128 B
constexpr int kNielsWords = 32;                   // 30 used, padded to 128 B
constexpr size_t kBTabWords = 2 * (size_t)kBTabEntries * kNielsWords;

// ---- vector load/store helpers ---------------------------------------------
// (the host bound tracker of fe25519.h follows elements through memory)
// one field element at slot word 0: chunks 0, 1 and half of chunk 2
OURO_FI void st_fe(Slot p, const fe& f) {
  stg4(p.chunk(0), make_int4(f.v[0], f.v[1], f.v[2], f.v[3]));
  stg4(p.chunk(1), make_int4(f.v[4], f.v[5], f.v[6], f.v[7]));
  stg2(p.chunk(2), make_int2(f.v[8], f.v[9]));
  OURO_TRK(ouro_trk_store(p.p, f.b));
}
OURO_FI fe ld_fe(Slot p) {
  const int4 a = ldg4(p.chunk(0)), b = ldg4(p.chunk(1));
  const int2 c = ldg2(p.chunk(2));
  fe f = fe_make(a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w, c.x, c.y);
  OURO_TRK(ouro_trk_load(p.p, f.b));
  return f;
}
// one element as five int2 at words w0, w0 + 2, ... (w0 even, run-time) of a
// region whose chunks are `stride` words apart: a slot (kChunkStride) or
// plain memory (4)
OURO_FI fe ld_fe_w2(const int32_t* base, int w0, int stride) {
  int2 q[5];
#pragma unroll
  for (int j = 0; j < 5; j++) {
    const int w = w0 + 2 * j;
    q[j] = ldg2(base + (w >> 2) * stride + (w & 3));
  }
  return fe_make(q[0].x, q[0].y, q[1].x, q[1].y, q[2].x, q[2].y, q[3].x, q[3].y, q[4].x, q[4].y);
}
// cached point: 40 words = 10 chunks, fe k at words [10k, 10k+10)
OURO_FI void st_cached(Slot p, const ge_cached& c) {
  const uint32_t* s[4] = {c.YplusX.v, c.YminusX.v, c.Z2.v, c.T2d.v};
  int32_t w[40];
#pragma unroll
  for (int k = 0; k < 4; k++)
#pragma unroll
    for (int i = 0; i < 10; i++) w[10 * k + i] = s[k][i];
#pragma unroll
  for (int i = 0; i < 10; i++)
    stg4(p.chunk(i), make_int4(w[4 * i], w[4 * i + 1], w[4 * i + 2], w[4 * i + 3]));
  OURO_TRK(ouro_trk_store(p.word(0), c.YplusX.b); ouro_trk_store(p.word(10), c.YminusX.b);
           ouro_trk_store(p.word(20), c.Z2.b); ouro_trk_store(p.word(30), c.T2d.b);)
}
OURO_FI ge_cached ld_cached(Slot p) {
  int32_t w[40];
#pragma unroll
  for (int i = 0; i < 10; i++) {
    int4 v = ldg4(p.chunk(i));
    w[4 * i] = v.x; w[4 * i + 1] = v.y; w[4 * i + 2] = v.z; w[4 * i + 3] = v.w;
  }
  ge_cached c;
#pragma unroll
  for (int i = 0; i < 10; i++) {
    c.YplusX.v[i] = w[i];
    c.YminusX.v[i] = w[10 + i];
    c.Z2.v[i] = w[20 + i];
    c.T2d.v[i] = w[30 + i];
  }
  OURO_TRK(ouro_trk_load(p.word(0), c.YplusX.b); ouro_trk_load(p.word(10), c.YminusX.b);
           ouro_trk_load(p.word(20), c.Z2.b); ouro_trk_load(p.word(30), c.T2d.b);)
  return c;
}
// Packed entries of the per-lane tables (lane mode; lane quads keep the
// 40-word form, which their per-operand loads index).  Each coordinate is
// carried to the limb widths with limb 9 allowed 26 bits and packed into 256
// bits, so an entry is 32 words -- one 128-B line instead of the two a 160-B
// entry touches.  The gathers are the bulk of the kernels' HBM traffic.
#ifndef OURO_TAB_PACK
#define OURO_TAB_PACK 1
#endif
constexpr int kPackedWords = 32;
constexpr int kLaneEntryWords = OURO_TAB_PACK ? kPackedWords : kCachedWords;
// f (limbs < 2^28) as 256 bits: 2^255 wrapped first, then one carry pass that
// leaves limbs 0..8 within their masks and limb 9 below 2^25 + 2^3
OURO_FI void fe_pack256(uint32_t w[8], const fe& f) {
  OURO_TRK(for (int i = 0; i < 10; i++) trk_check(f.b[i] < (1ull << 28));)
  uint32_t h[10];
#pragma unroll
  for (int i = 0; i < 10; i++) h[i] = f.v[i];
  uint32_t c = h[9] >> 25;
  h[9] &= limb_mask(9);
  h[0] += 19 * c;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    c = h[i] >> limb_bits(i);
    h[i] &= limb_mask(i);
    h[i + 1] += c;
  }
  w[0] = h[0] | (h[1] << 26);
  w[1] = (h[1] >> 6) | (h[2] << 19);
  w[2] = (h[2] >> 13) | (h[3] << 13);
  w[3] = (h[3] >> 19) | (h[4] << 6);
  w[4] = h[5] | (h[6] << 25);
  w[5] = (h[6] >> 7) | (h[7] << 19);
  w[6] = (h[7] >> 13) | (h[8] << 12);
  w[7] = (h[8] >> 20) | (h[9] << 6);
}
OURO_FI fe fe_unpack256(const uint32_t w[8]) {
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
  h.v[9] = w[7] >> 6;  // 26 bits
  OURO_TRK(for (int i = 0; i < 9; i++) h.b[i] = limb_mask(i); h.b[9] = (1u << 26) - 1;)
  return h;
}
OURO_FI void st_cached_packed(Slot p, const ge_cached& c) {
  const fe* s[4] = {&c.YplusX, &c.YminusX, &c.Z2, &c.T2d};
#pragma unroll
  for (int k = 0; k < 4; k++) {
    uint32_t w[8];
    fe_pack256(w, *s[k]);
    stg4(p.chunk(2 * k), make_int4((int)w[0], (int)w[1], (int)w[2], (int)w[3]));
    stg4(p.chunk(2 * k + 1), make_int4((int)w[4], (int)w[5], (int)w[6], (int)w[7]));
  }
}
OURO_FI ge_cached ld_cached_packed(Slot p) {
  fe f[4];
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const int4 a = ldg4(p.chunk(2 * k)), b = ldg4(p.chunk(2 * k + 1));
    const uint32_t w[8] = {(uint32_t)a.x, (uint32_t)a.y, (uint32_t)a.z, (uint32_t)a.w,
                           (uint32_t)b.x, (uint32_t)b.y, (uint32_t)b.z, (uint32_t)b.w};
    f[k] = fe_unpack256(w);
  }
  return ge_cached{f[0], f[1], f[2], f[3]};
}
// a lane-mode table entry (packed or not) / a lane-quad one (never packed)
OURO_FI void st_entry(Slot p, const ge_cached& c, bool quad) {
  if (OURO_TAB_PACK && !quad)
    st_cached_packed(p, c);
  else
    st_cached(p, c);
}
OURO_FI ge_niels ld_niels(const int32_t* p) {
  int32_t w[32];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    int4 v = ldg4(p + 4 * i);
    w[4 * i] = v.x; w[4 * i + 1] = v.y; w[4 * i + 2] = v.z; w[4 * i + 3] = v.w;
  }
  ge_niels n;
#pragma unroll
  for (int i = 0; i < 10; i++) {
    n.yplusx.v[i] = w[i];
    n.yminusx.v[i] = w[10 + i];
    n.xy2d.v[i] = w[20 + i];
  }
  OURO_TRK(ouro_trk_load(p, n.yplusx.b); ouro_trk_load(p + 10, n.yminusx.b);
           ouro_trk_load(p + 20, n.xy2d.b);)
  return n;
}
OURO_FI void st_words8(Slot p, const uint32_t w[8]) {
  stg4(p.chunk(0), make_int4((int)w[0], (int)w[1], (int)w[2], (int)w[3]));
  stg4(p.chunk(1), make_int4((int)w[4], (int)w[5], (int)w[6], (int)w[7]));
}
OURO_FI void ld_words8(uint32_t w[8], Slot p) {
  const int4 a = ldg4(p.chunk(0)), b = ldg4(p.chunk(1));
  w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w;
  w[4] = b.x; w[5] = b.y; w[6] = b.z; w[7] = b.w;
}
// the recoding carries of scalars a1, a2, b (k = 0, 1, 2)
OURO_FI uint64_t ld_carry(Slot lane, int k) { return ldg8(lane.word(kSlotCarry + 2 * k)); }
OURO_FI void st_carry(Slot lane, int k, uint64_t c) { stg8(lane.word(kSlotCarry + 2 * k), c); }
// a 32-byte message held in a slot (the VRF input staged by the header cores)
struct SlotTail {
  Slot s;
  OURO_FI uint32_t tail(uint32_t q) const {
    return ((uint32_t)ldg1(s.word((int)(q >> 2))) >> (8 * (q & 3))) & 0xffu;
  }
};

// [1..8]P in cached form into a per-lane table
// (quad: the lane-quad formulas of ge25519.h, latency mode)
OURO_HD inline void build_table(Slot tab, const ge_p3& P, bool quad = false) {
  const int ec = (quad ? kCachedWords : kLaneEntryWords) / 4;  // chunks per entry
  ge_cached c1 = ge_p3_to_cached(P);
  st_entry(tab, c1, quad);
  ge_p3 Pk = quad ? ge_p1p1_to_p3_quad(ge_p2_dbl_quad(ge_p3_to_p2(P)))
                  : ge_p1p1_to_p3(ge_p3_dbl(P));
  st_entry(tab.chunks(ec), ge_p3_to_cached(Pk), quad);
#pragma unroll 1
  for (int k = 2; k < kTabEntries; k++) {
    Pk = quad ? ge_p1p1_to_p3_quad(ge_add_cached_quad(Pk, c1, false))
              : ge_p1p1_to_p3(ge_add_cached(Pk, c1, false));
    st_entry(tab.chunks(k * ec), ge_p3_to_cached(Pk), quad);
  }
}

// recoding carries of the B scalar (b < 2^253) for the split multiplication:
// digits 0..D-1 of its low half at mask bits 0..D-1, of its high half at
// D..2D-1 (one number when kBW divides 128, two otherwise)
OURO_FI uint64_t sc_recode_b(const uint32_t s[8]) {
  if constexpr (!kBSplitRecode) {
    return sc_recode_carries<kBW, 2 * kBDigitsHalf>(s);
  } else {
  uint64_t mask = 0;
#pragma unroll
  for (int h = 0; h < 2; h++) {
    uint32_t c = 0;
#pragma unroll
    for (int k = 0; k < kBDigitsHalf; k++) {
      const int rel = kBW * k, bit = 128 * h + rel;
      const int w = bit >> 5, sh = bit & 31;
      const uint64_t two = (uint64_t)s[w] | ((w + 1 < 8 ? (uint64_t)s[w + 1] : 0ull) << 32);
      uint32_t v = (uint32_t)(two >> sh) & ((1u << kBW) - 1);
      if (128 - rel < kBW) v &= (1u << (128 - rel)) - 1;  // this half's bits only
      mask |= (uint64_t)c << (kBDigitsHalf * h + k);
      c = (v + c) > (1u << (kBW - 1)) ? 1u : 0u;
    }
  }
  return mask;
  }
}

// 160-bit stream shifted right by 0 < bits < 32
OURO_FI void ss_shr5(uint32_t w[5], int bits) {
#pragma unroll
  for (int i = 0; i < 4; i++) w[i] = (w[i] >> bits) | (w[i + 1] << (32 - bits));
  w[4] >>= bits;
}

// ---- the double-scalar multiplication ---------------------------------------
// cfg: bits 0..6 = number of active width-4 windows of scalar a1 (table 1),
//      bits 8..14 = same for a2 (table 2, 0 = unused), bit 16 = add [b]B with
//      b split at bit 128: its kBW-bit digits 0..7 go with B and 8..15 with
//      B' = 2^128 B, so the doubling chain only spans 128 bits,
//      bits 20..21 / 22..23 = table slots (0..2) read for a1 / a2.
// Reads a1/a2/b and their recoding carries from the lane slot, writes the
// resulting p2 point to lane[kSlotOut..].  Out of line: the header kernel calls
// it six times per item, and the loop body is the I-cache-critical code.
constexpr uint32_t dsm_cfg(int nw1, int nw2, bool useB, int tab1 = 0, int tab2 = 1) {
  return (uint32_t)nw1 | ((uint32_t)nw2 << 8) | (useB ? (1u << 16) : 0u) |
         ((uint32_t)tab1 << 20) | ((uint32_t)tab2 << 22);
}

#ifndef OURO_DSM_SKIP_ID
#define OURO_DSM_SKIP_ID 1  // A/B switch: 0 = doublings/addition from the identity kept
#endif
// A/B switches: doublings per loop trip in a window.  One lane per item: 1
// (72.7 ms vs 73.2 / 73.8 for 2 / 4, I-cache); lane quads (latency mode, few
// waves): 4 (configs[4] p50 0.647 -> 0.636 ms).  profiles/r01h/ab_unroll*.json
#ifndef OURO_DBL_UNROLL
#define OURO_DBL_UNROLL 1
#endif
#ifndef OURO_DBL_UNROLL_QUAD
#define OURO_DBL_UNROLL_QUAD 4
#endif
#ifndef OURO_ADD_UNROLL_QUAD
// the four addition sources unrolled in lane-quad mode: configs[4] p50
// 0.643 -> 0.638 ms (two runs each); lane mode keeps the rolled loop
#define OURO_ADD_UNROLL_QUAD 4
#endif
// Where a window's table entries are touched: 3 = before its last doubling
// (the default since round 3; that doubling peeled off the loop), 0 = before
// all four (round 2).  The gathers of ~7 us of doublings over the whole grid
// exceed an XCD's 4 MB L2, so lines touched four doublings ahead were often
// evicted before the additions read them: touching one doubling ahead cuts
// the header kernel's HBM traffic 202 -> 158 KB/header (Ed25519 40 -> 31 KB,
// Sum6KES 43 -> 34 KB, VRF 60 -> 48 KB) and its time 69.57 -> 69.18 ms
// (profiles/r03/ab_finish_prefetch.json).  (An in-loop `if (k == at)` form of
// the same change cost +2.8 % in code generation: profiles/r03/ab_prefetch_position.json.)
#ifndef OURO_PF_AT
#define OURO_PF_AT 3
#endif
// A doubling of the lane chain: its products in lockstep (ge25519.h
// ge_dbl_lockstep, 1, the default since round 4) or as written in ge_p2_dbl
// (0, A/B).
// the same for the chain's additions (ge25519.h ge_add_lockstep): 1 = four
// products at a time, 2 = two, 0 = as written (round 4)
#ifndef OURO_ADD_LOCKSTEP
#define OURO_ADD_LOCKSTEP 1
#endif
#ifndef OURO_DBL_LOCKSTEP
#define OURO_DBL_LOCKSTEP 1
#endif
OURO_FI ge_p1p1 dsm_dbl(const ge_p1p1& t) {
  if constexpr (OURO_DBL_LOCKSTEP) return ge_dbl_lockstep(t);
  else return ge_p2_dbl(ge_p1p1_to_p2(t));
}
template <bool kQuad>
OURO_FI void dsm_body(Slot lane, const int32_t* btab, uint32_t cfg) {
  const int nw1 = (int)(cfg & 0x7f), nw2 = (int)((cfg >> 8) & 0x7f);
  const bool useB = (cfg >> 16) & 1;
  const Slot tab1 = lane.chunks((int)((cfg >> 20) & 3) * (kTabWords / 4));
  const Slot tab2 = lane.chunks((int)((cfg >> 22) & 3) * (kTabWords / 4));
  constexpr int kE = kQuad ? kCachedWords : kLaneEntryWords;  // words per table entry
  uint32_t a1[8], a2[8], b[8];
  ld_words8(a1, lane + kSlotA1);
  ld_words8(a2, lane + kSlotA2);
  ld_words8(b, lane + kSlotB);
  const uint64_t c1 = ld_carry(lane, 0), c2 = ld_carry(lane, 1), cb = ld_carry(lane, 2);
  int top = nw1 > nw2 ? nw1 : nw2;
  if (useB && top < kBStride * kBDigitsHalf) top = kBStride * kBDigitsHalf;
  // digit streams: window top-1 of a1/a2 at the top of the array
#pragma unroll 1
  for (int s = top; s < 64; s++) {
    ss_shl<8>(a1, 4);
    ss_shl<8>(a2, 4);
  }
  // b: two streams (its low and high 128-bit halves, the top digit's bits on
  // top of 160), kBW bits per B window
  constexpr int kBPre = 160 - kBW * kBDigitsHalf;
  uint32_t blo[5] = {0, b[0], b[1], b[2], b[3]};
  uint32_t bhi[5] = {0, b[4], b[5], b[6], b[7]};
  if (kBPre < 32) {
    ss_shr5(blo, 32 - kBPre);
    ss_shr5(bhi, 32 - kBPre);
  }
  uint32_t prefetch = 0;
  // t starts as the identity in p1p1 form (X/Z = 0, Y/T = 1)
  ge_p1p1 t{fe_zero(), fe_one(), fe_one(), fe_one()};
  bool fresh = true;  // t is the identity (wave-uniform)
#pragma unroll 1
  for (int j = top - 1; j >= 0; j--) {
    // this window's digits (wave-uniform activity, per-lane values)
    const bool act1 = j < nw1, act2 = j < nw2;
    const bool actB = useB && (j % kBStride) == 0 && j < kBStride * kBDigitsHalf;
    const bool actB2 = actB;
    int32_t d1 = 0, d2 = 0, d3 = 0, d4 = 0;
    if (act1) d1 = sc_digit_from<4>(a1[7] >> 28, c1, j, 64);
    if (act2) d2 = sc_digit_from<4>(a2[7] >> 28, c2, j, 64);
    ss_shl<8>(a1, 4);
    ss_shl<8>(a2, 4);
    if (actB) {
      const int k = j / kBStride;
      d3 = sc_digit_from<kBW>(blo[4] >> (32 - kBW), cb, k,
                              kBSplitRecode ? kBDigitsHalf : 2 * kBDigitsHalf);
      d4 = sc_digit_from<kBW>(bhi[4] >> (32 - kBW), cb, k + kBDigitsHalf, 2 * kBDigitsHalf);
      ss_shl<5>(blo, kBW);
      ss_shl<5>(bhi, kBW);
    }
    // touch this window's per-lane table entries now, so that the loads
    // after the four doublings hit L2 instead of waiting on HBM
    const int i1 = (d1 < 0 ? -d1 : d1) - 1, i2 = (d2 < 0 ? -d2 : d2) - 1;
    const Slot e1 = tab1.chunks((i1 > 0 ? i1 : 0) * (kE / 4));
    const Slot e2 = tab2.chunks((i2 > 0 ? i2 : 0) * (kE / 4));
    uint32_t pf1 = 0, pf2 = 0, pf3 = 0, pf4 = 0, pf5 = 0, pf6 = 0;
    const int i3 = (d3 < 0 ? -d3 : d3) - 1, i4 = (d4 < 0 ? -d4 : d4) - 1;
#define OURO_TOUCH_ENTRIES()                                                                   \
  do {                                                                                         \
    if (act1) { pf1 = (uint32_t)ldg1(e1.word(0)); if (kE > 32) pf2 = (uint32_t)ldg1(e1.word(kE - 1)); } \
    if (act2) { pf3 = (uint32_t)ldg1(e2.word(0)); if (kE > 32) pf4 = (uint32_t)ldg1(e2.word(kE - 1)); } \
    if (actB) { /* the B entries (one 128-B line each) come from the 8 MiB tables */          \
      pf5 = (uint32_t)ldg1(btab + (size_t)(i3 > 0 ? i3 : 0) * kNielsWords);                    \
      pf6 = (uint32_t)ldg1(btab + ((size_t)kBTabEntries + (i4 > 0 ? i4 : 0)) * kNielsWords);   \
    }                                                                                          \
  } while (0)
    const bool skip_dbl = OURO_DSM_SKIP_ID && j == top - 1;
    if (kQuad || OURO_PF_AT == 0 || skip_dbl) OURO_TOUCH_ENTRIES();
    // (the top window starts from the identity: its doublings are skipped)
    if (!skip_dbl) {
      if constexpr (kQuad) {
#pragma unroll OURO_DBL_UNROLL_QUAD
        for (int k = 0; k < 4; k++) t = ge_dbl_from_p1p1_quad(t);
      } else if (OURO_PF_AT == 0) {
#pragma unroll OURO_DBL_UNROLL
        for (int k = 0; k < 4; k++) t = dsm_dbl(t);
      } else {
#pragma unroll 1
        for (int k = 0; k < 3; k++) t = dsm_dbl(t);
        OURO_TOUCH_ENTRIES();
        t = dsm_dbl(t);
      }
    }
#undef OURO_TOUCH_ENTRIES
    prefetch ^= pf1 ^ pf2 ^ pf3 ^ pf4 ^ pf5 ^ pf6;
    // up to four additions, each from a wave-uniform source
    constexpr int kAddUnroll = kQuad ? OURO_ADD_UNROLL_QUAD : 1;
#pragma unroll kAddUnroll
    for (int src = 0; src < 4; src++) {
      const bool active = src == 0 ? act1 : src == 1 ? act2 : src == 2 ? actB : actB2;
      if (!active) continue;
      const int32_t d = src == 0 ? d1 : src == 1 ? d2 : src == 2 ? d3 : d4;
      const bool neg = d < 0;
      const int32_t mag = neg ? -d : d;
      const int idx = mag > 0 ? mag - 1 : 0;
#if defined(__HIP_DEVICE_COMPILE__)
      if (kQuad && !(OURO_DSM_SKIP_ID && fresh)) {
        // each lane of the quad loads only its own operand of the entry
        const uint32_t qp = threadIdx.x & 3u;
        const bool niels = src >= 2;
        const int k = qp < 2 ? (int)(qp ^ (neg ? 1u : 0u)) : (qp == 2 ? (niels ? 2 : 3) : (niels ? 0 : 2));
        // a B entry is plain memory, a per-lane entry an interleaved slot region
        const int32_t* ent =
            niels ? btab + ((src == 3 ? (size_t)kBTabEntries : 0) + idx) * kNielsWords
                  : (src == 0 ? tab1 : tab2).chunks(idx * (kCachedWords / 4)).p;
        fe b = ld_fe_w2(ent, 10 * k, niels ? 4 : kChunkStride);
        // constants: the identity's operands (1, 1, 0, 2); a niels entry's 2Z = 2
        if (mag == 0 || (niels && qp == 3)) {
          b = fe_zero();
          b.v[0] = qp < 2 ? 1u : (qp == 2 ? 0u : 2u);
        }
        t = ge_add_own_quad(t, b, neg);
        continue;
      }
#endif
      ge_cached q;
      if (src < 2) {
        const Slot e = (src == 0 ? tab1 : tab2).chunks(idx * (kE / 4));
        q = kE == kPackedWords ? ld_cached_packed(e) : ld_cached(e);
      } else {
        const size_t base = src == 3 ? kBTabEntries : 0;
        ge_niels nq = ld_niels(btab + (base + idx) * kNielsWords);
        q = ge_cached{nq.yplusx, nq.yminusx, fe_two(), nq.xy2d};
      }
      if (mag == 0) q = ge_cached_identity();
      if (OURO_DSM_SKIP_ID && fresh) {
        // t is still the identity: O +- q = (2x, 2y, 2z, 2z) with no multiply
        const fe qa = fe_select(q.YminusX, q.YplusX, neg);
        const fe qb = fe_select(q.YplusX, q.YminusX, neg);
        t = ge_p1p1{fe_carry(fe_sub4(qa, qb)), fe_carry(fe_add(qa, qb)), q.Z2, q.Z2};
        fresh = false;
        continue;
      }
      if constexpr (kQuad) t = ge_add_cached_quad(ge_p1p1_to_p3_quad(t), q, neg);
      else if constexpr (OURO_ADD_LOCKSTEP) t = ge_add_lockstep<OURO_ADD_LOCKSTEP == 2>(t, q, neg, src >= 2);
      else t = ge_add_cached(ge_p1p1_to_p3(t), q, neg, src >= 2);
    }
  }
  ge_p2 r = kQuad ? ge_p1p1_to_p2_quad(t) : ge_p1p1_to_p2(t);
  st_fe(lane + kSlotOut, r.X);
  st_fe(lane + kSlotOut + 12, r.Y);
  st_fe(lane + kSlotOut + 24, r.Z);
  // keeps the prefetch loads alive.  The XOR can equal the guard (packed
  // table entries make word 0 full-width), and then this store happens on
  // purpose: it lands on Z's padding word kSlotOut+35, which nothing reads
  if (prefetch == 0xffffffffu) stg1(lane.word(kSlotOut + 35), (int32_t)prefetch);
}
OURO_NI void dsm_lane(Slot lane, const int32_t* btab, uint32_t cfg) {
  dsm_body<false>(lane, btab, cfg);
}
#if defined(__HIPCC__)
// The same for the split header kernel's dsm launch (k_hdr_dsm), a function
// of its own: an out-of-line function gets ONE register allocation, the
// tightest any caller allows, and k_hdr_dsm runs at 4 waves / SIMD (128
// VGPRs) while every other caller has 256.
__device__ __noinline__ void dsm_lane_dsm_launch(Slot lane, const int32_t* btab, uint32_t cfg) {
  dsm_body<false>(lane, btab, cfg);
}
#endif
// latency mode: the four lanes of a quad run one chain (same inputs, same
// slot), splitting each group operation's products
OURO_NI void dsm_quad(Slot lane, const int32_t* btab, uint32_t cfg) {
  dsm_body<true>(lane, btab, cfg);
}
OURO_FI void dsm(Slot lane, const int32_t* btab, uint32_t cfg, bool quad = false) {
  if (quad)
    dsm_quad(lane, btab, cfg);
  else
    dsm_lane(lane, btab, cfg);
}

OURO_FI ge_p2 dsm_result(Slot lane) {
  return ge_p2{ld_fe(lane + kSlotOut), ld_fe(lane + kSlotOut + 12), ld_fe(lane + kSlotOut + 24)};
}

// Phases of a core around its double-scalar multiplication (the split header
// kernel, kernels.hip OURO_SPLIT): kPhasePre stops once the dsm's inputs
// -- tables, scalars, recoding carries -- and its cfg word (kSlotCfg, the
// carry region's spare words) are in the slot; the dsm then runs in a launch
// of its own at a higher occupancy (k_hdr_dsm), and kPhasePost finishes the
// core from the result the dsm left at kSlotOut.  kPhaseAll: all of it.
enum Phase { kPhaseAll = 0, kPhasePre = 1, kPhasePost = 2 };
constexpr int kSlotCfg = kSlotCarry + 6;
OURO_FI void dsm_or_defer(Slot lane, const int32_t* btab, uint32_t cfg, bool quad, int phase) {
  if (phase == kPhasePre) {
    stg1(lane.word(kSlotCfg), (int32_t)cfg);
    return;
  }
  dsm(lane, btab, cfg, quad);
}
// an Ed25519 core's verdict from its dsm result: Q == O, projectively
OURO_FI bool dsm_result_is_identity(Slot lane) {
  const ge_p2 Q = dsm_result(lane);
  return fe_iszero(Q.X) && fe_iszero(fe_sub(Q.Y, Q.Z));
}

// ---- Ed25519 ------------------------------------------------------------------
// Largest x over the wave's active lanes (ballots honour EXEC, so lanes that
// left the grid-stride loop do not contribute); identity on the host.
OURO_FI int wave_max_small(int x) {
#if defined(__HIP_DEVICE_COMPILE__)
  int m = 0;
#pragma unroll
  for (int b = 6; b >= 0; b--) {
    const int trial = m | (1 << b);
    if (__ballot(x >= trial) != 0) m = trial;
  }
  return m;
#else
  return x;
#endif
}

// sig = R || S (16 words), pk (8 words), message bytes from global memory.
// Accepts iff libsodium 1.0.18 does (App. B.1) -- or, for ByronDSIGN, the
// donna-derived cardano-crypto rule (App. B.5) -- through the equivalent
// half-size equation of lattice.h:
//   R_bytes canonical, decodable, x = 0 only with sign 0, and
//   [c1 S mod L]B + [c0](-A) + [c1](-R) == O,  c0 = c1 h (mod 8L), c1 odd,
// with h = SHA-512(R || A || M) mod L.  The doubling chain is ~130 bits
// instead of 253, and no inversion is needed: the result is compared to the
// identity projectively.
// The scalar side of the half-size equation: h = SHA-512(R || A || M) mod L,
// its lattice pair (c0, c1) and b = c1 S mod L.
OURO_HD inline void ed25519_scalars_from_digest(HalfScalars& hs, uint32_t b[8], const uint64_t H[8],
                                                const uint32_t S[8]);
template <class Tail>
OURO_HD inline void ed25519_scalars(HalfScalars& hs, uint32_t b[8], const uint32_t R[8],
                                    const uint32_t S[8], const uint32_t pk[8], const Tail& msg,
                                    uint32_t mlen) {
  uint32_t pre[16];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    pre[i] = R[i];
    pre[8 + i] = pk[i];
  }
  uint64_t H[8];
  sha512_prefixed<64>(H, pre, msg, mlen);
  ed25519_scalars_from_digest(hs, b, H, S);
}
// the rest of ed25519_scalars from the digest H of R || A || M (the latency
// mode hashes on the whole wave, wide_cores.h)
OURO_HD inline void ed25519_scalars_from_digest(HalfScalars& hs, uint32_t b[8], const uint64_t H[8],
                                                const uint32_t S[8]) {
  uint32_t hw[16], h[8];
  sha512_digest_words(hw, H);
  sc_reduce512(h, hw);
  ed25519_half_scalars(hs, h);
  // b = c1 S mod L
  uint32_t prod[16];
#pragma unroll
  for (int i = 0; i < 16; i++) prod[i] = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint64_t carry = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) {
      const uint64_t t = (uint64_t)hs.c1[i] * S[j] + prod[i + j] + carry;
      prod[i + j] = (uint32_t)t;
      carry = t >> 32;
    }
    prod[i + 8] = (uint32_t)carry;
  }
  sc_reduce512(b, prod);
}

// the encoding checks on (S, R, A) before decoding (libsodium / Byron rules)
OURO_FI bool ed25519_precheck(const uint32_t R[8], const uint32_t S[8], const uint32_t pk[8],
                              bool byron) {
  if (byron) return (S[7] >> 29) == 0;  // only the top three bits of S
  bool ok = sc_is_canonical(S) && !ge_has_small_order(R);
  return ok && ge_is_canonical(pk) && !ge_has_small_order(pk);
}

// sig = R || S (16 words), pk (8 words), message bytes from global memory.
// Accepts iff libsodium 1.0.18 does (App. B.1) -- or, for ByronDSIGN, the
// donna-derived cardano-crypto rule (App. B.5) -- through the equivalent
// half-size equation of lattice.h:
//   R_bytes canonical, decodable, x = 0 only with sign 0, and
//   [c1 S mod L]B + [c0](-A) + [c1](-R) == O,  c0 = c1 h (mod 8L), c1 odd,
// with h = SHA-512(R || A || M) mod L.  The doubling chain is ~130 bits
// instead of 253, and no inversion is needed: the result is compared to the
// identity projectively.
// phase (kPhasePre / kPhasePost, the split header kernel): Pre returns the
// checks before the dsm, Post whether its result is the identity.
template <class Tail>
OURO_HD inline bool ed25519_verify_lane(const uint32_t sig[16], const uint32_t pk[8],
                                        const Tail& msg, uint32_t mlen, Slot lane,
                                        const int32_t* btab, bool byron = false,
                                        bool quad = false, int phase = kPhaseAll) {
  if (phase == kPhasePost) return dsm_result_is_identity(lane);
  uint32_t R[8], S[8];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    R[i] = sig[i];
    S[i] = sig[8 + i];
  }
  bool ok = ed25519_precheck(R, S, pk, byron);
  ge_p3 negA, negR;
  bool okA, okR;
  if (quad) {
    ge_decode_pair_quad(&negA, &okA, &negR, &okR, pk, R, true);
  } else {
    ge_decode_pair(&negA, &okA, &negR, &okR, pk, R, true);
  }
  ok = okA && ok;
  // encode(R') == R_bytes  <=>  R_bytes is the canonical encoding of R' (a point)
  ok = ge_is_canonical(R) && ok;
  ok = okR && ok;
  ok = ok && !(fe_iszero(negR.X) && (R[7] >> 31) != 0);
  HalfScalars hs;
  uint32_t b[8];
  ed25519_scalars(hs, b, R, S, pk, msg, mlen);
  // [|c0|](+-A) + [c1](-R) + [b]B, one ~130-bit doubling chain
  build_table(lane + kSlotTab1, hs.c0_neg ? ge_p3_neg(negA) : negA, quad);
  build_table(lane + kSlotTab2, negR, quad);
  st_words8(lane + kSlotA1, hs.c0);
  st_words8(lane + kSlotA2, hs.c1);
  st_words8(lane + kSlotB, b);
  st_carry(lane, 0, sc_recode_carries<4, 64>(hs.c0));
  st_carry(lane, 1, sc_recode_carries<4, 64>(hs.c1));
  st_carry(lane, 2, sc_recode_b(b));
  // windows so that every scalar is < 2^(4 nw - 1) (top carry zero), <= 64
  int nw = wave_max_small((hs.bits + 4) >> 2);
  nw = nw < 1 ? 1 : (nw > 64 ? 64 : nw);
  dsm_or_defer(lane, btab, dsm_cfg(nw, nw, true, 0, 1), quad, phase);
  if (phase == kPhasePre) return ok;
  return ok && dsm_result_is_identity(lane);
}

// ---- ECVRF-ED25519-SHA512-Elligator2 (draft-03) -------------------------------
// libsodium 1.0.18 ge25519_from_uniform with x_sign = 0 (the VRF clears bit 255
// of r before calling it): returns [8] of the Elligator2 image.
//
// Same point as the reference, one exponentiation instead of four.  With
// D = 1 + 2r^2 the candidate Montgomery x's are x1 = -A/D and x2 = -x1 - A =
// 2 r^2 x1, and x1^2 + A x1 + 1 = x2^2 + A x2 + 1 = 1 - x1 x2 = W / D^2 with
// W = D^2 - 2 A^2 r^2.  The Edwards x of the Montgomery point (u, v) is
// sqrt(-(A+2)) u / v, whose square is
//   rho(u) = -(A+2) u^2 / g(u) = -(A+2) u / (u^2 + A u + 1),
// so rho1 = rho(x1) = (A+2) A D / W, rho2 = rho(x2) = 2 r^2 rho1, and
// chi(rho1) = chi(g(x1)) (-(A+2) is a square): libsodium's chi test is the
// squareness of rho1.  One sqrt-ratio exponentiation of num/den = rho1 gives
// beta with beta^2 den = lambda num, lambda a 4th root of unity:
//   lambda =  1: x = beta            lambda =  i: x = r beta (1 - i)
//   lambda = -1: x = beta i          lambda = -i: x = r beta (1 + i)
// (2/i = (1 - i)^2, 2/(-i) = (1 + i)^2, so (r beta (1 -+ i))^2 = rho2).  The
// root's sign is then made even, as ge25519_frombytes does for the
// (canonical, sign 0) encoding of y_ed = (x_final - 1)/(x_final + 1) =
// (Xn - D)/(Xn + D) = n/m with Xn = -A (square) or -2 A r^2 (non-square).
// D != 0 (-2 is a non-square mod p), W != 0 (u^2 + A u + 1 has no root:
// A^2 - 4 is a non-square) and m != 0 (neither (A-1)/2 nor 1/(2(A-1)) is a
// square; tools/check_elligator_exceptions.py), so no inverse of zero can
// occur where libsodium would have computed one.
// pow22523: z -> z^(2^252 - 3); the latency mode's wave-wide item passes the
// wide exponentiation (wide.h), everything else fe_pow22523.  kMul8 = false
// returns the Elligator2 point before the cofactor clearing (the wave-wide
// item doubles it three times on the wave).
// Split around its exponentiation like ge_decode (the throughput header core
// pairs it with Gamma's decode, fe_pow22523_x2): elligator2_pre returns the
// base num W^7, elligator2_post takes its (p-5)/8 power.
struct Ell2Pre {
  fe rr, r2, D, num, W, W3;
};
OURO_HD inline fe elligator2_pre(Ell2Pre& e, const uint32_t r[8]) {
  e.rr = fe_from_words(r);
  e.r2 = fe_sq(e.rr);
  e.D = fe_carry(fe_add(fe_add(e.r2, e.r2), fe_one()));  // 1 + 2 r^2 (re-balanced:
                                                         // n = Xn - D below sums 4 terms)
  fe A2r2 = fe_mul(fe_mont_a2(), e.r2);                  // A^2 r^2
  e.W = fe_carry(fe_sub4(fe_sq(e.D), fe_add(A2r2, A2r2)));  // D^2 - 2 A^2 r^2
  e.num = fe_mul(fe_mont_a2a(), e.D);                    // (A + 2) A D
  // beta = num W^3 (num W^7)^((p-5)/8)
  e.W3 = fe_mul(fe_sq(e.W), e.W);
  const fe W7 = fe_mul(fe_sq(e.W3), e.W);
  return fe_mul(e.num, W7);
}
template <bool kMul8 = true>
OURO_HD inline ge_p3 elligator2_post(const Ell2Pre& e, const fe& pw) {
  const fe A = fe_mont_a();
  const fe rr = e.rr, r2 = e.r2, D = e.D, W = e.W, num = e.num;
  fe beta = fe_mul(fe_mul(num, e.W3), pw);
  fe vxx = fe_mul(fe_sq(beta), W);
  const bool lam_p1 = fe_iszero(fe_sub4(vxx, num));
  const bool lam_m1 = fe_iszero(fe_add(vxx, num));
  const bool lam_pi = fe_iszero(fe_sub4(vxx, fe_mul(num, fe_sqrtm1())));
  const bool nonsq = !(lam_p1 || lam_m1);
  const fe F = fe_select(fe_select(fe_one_minus_i(), fe_one_plus_i(), lam_pi),
                         fe_select(fe_one(), fe_sqrtm1(), lam_p1), nonsq);
  fe x = fe_mul(beta, F);
  x = fe_select(fe_mul(x, rr), x, nonsq);
  x = fe_select(fe_neg(x), x, fe_isnegative(x));  // sign bit 0: even x
  fe Ar2 = fe_mul(A, r2);
  fe Xn = fe_carry(fe_select(fe_neg4(fe_add(Ar2, Ar2)), fe_neg(A), nonsq));
  fe n = fe_sub(Xn, D), m = fe_add(Xn, D);
  const fe nc = fe_carry(n);
  ge_p3 P{fe_mul(x, m), nc, m, fe_mul(x, nc)};
  if constexpr (!kMul8) return P;
  return ge_mul8(P);
}
template <class Pow, bool kMul8 = true>
OURO_HD inline ge_p3 elligator2_h_with(const uint32_t r[8], Pow pow22523) {
  Ell2Pre e;
  const fe base = elligator2_pre(e, r);
  return elligator2_post<kMul8>(e, pow22523(base));
}
OURO_HD inline ge_p3 elligator2_h(const uint32_t r[8]) {
  return elligator2_h_with(r, [](const fe& z) { return fe_pow22523(z); });
}

// The straight restatement of ge25519_from_uniform (4 exponentiations), kept
// for the host tests that pin elligator2_h against it.
OURO_HD inline ge_p3 elligator2_h_ref(const uint32_t r[8]) {
  const fe one = fe_one();
  const fe A = fe_mont_a();
  fe rr = fe_from_words(r);
  fe den = fe_add(fe_sq2(rr), one);          // 1 + 2 r^2
  fe x = fe_neg(fe_mul(A, fe_invert(den)));  // -A / (1 + 2 r^2)
  fe x2 = fe_sq(x);
  fe e = fe_carry(fe_add(fe_add(fe_mul(x, x2), x), fe_mul(x2, A)));  // x^3 + A x^2 + x
  // chi(e) = e^((p-1)/2) = (e^(2^252-3))^4 e^2
  fe chi = fe_mul(fe_sq(fe_sq(fe_pow22523(e))), fe_sq(e));
  uint32_t cw[8];
  fe_to_words(cw, chi);
  const bool e_is_minus_1 = (cw[0] >> 8) & 1;  // byte 1, bit 0 (libsodium's test)
  x = fe_carry(fe_select(fe_sub(fe_neg(x), A), x, e_is_minus_1));
  // y_ed = (x - 1) / (x + 1), decoded with sign 0, then cleared of the cofactor
  fe yed = fe_mul(fe_sub(x, one), fe_invert(fe_add(x, one)));
  uint32_t yw[8];
  fe_to_words(yw, yed);
  ge_p3 P;
  ge_decode(&P, yw, false);  // always a square here (libsodium aborts otherwise)
  return ge_mul8(P);
}

// Montgomery batch inversion of 4 elements
OURO_FI void fe_invert4(fe out[4], const fe z[4]) {
  fe a1 = fe_mul(z[0], z[1]);
  fe a2 = fe_mul(a1, z[2]);
  fe a3 = fe_mul(a2, z[3]);
  fe inv = fe_invert_vartime(a3);
  out[3] = fe_mul(inv, a2);
  inv = fe_mul(inv, z[3]);
  out[2] = fe_mul(inv, a1);
  inv = fe_mul(inv, z[2]);
  out[1] = fe_mul(inv, z[0]);
  out[0] = fe_mul(inv, z[1]);
}

// pi = Gamma (8 words) || c (4 words) || s (8 words); alpha from global memory.
// On success writes beta (16 words, the 64-byte output) and returns true; on
// failure beta is zeroed.
template <class Tail>
OURO_HD inline bool vrf03_verify_lane(uint32_t beta[16], const uint32_t pk[8],
                                      const uint32_t pi[20], const Tail& alpha, uint32_t alen,
                                      Slot lane, const int32_t* btab) {
  uint32_t G[8], c[8], s_raw[8], s[8];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    G[i] = pi[i];
    s_raw[i] = pi[12 + i];
    c[i] = i < 4 ? pi[8 + i] : 0u;
  }
  // validate_key + decode_proof
  ge_p3 Y, Gamma;
  bool okY, okG;
  ge_decode_pair(&Y, &okY, &Gamma, &okG, pk, G, false);
  bool ok = !ge_has_small_order(pk) && ge_is_canonical(pk);
  ok = okY && ok;
  ok = ge_is_canonical(G) && ok;
  ok = okG && ok;
  sc_reduce256(s, s_raw);
  // H = hash_to_curve(Y, alpha): r = SHA-512(0x04 || 0x01 || Y || alpha)[0:32]
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
  ge_p3 Hp = elligator2_h(rw);
  // U = [s]B - [c]Y
  build_table(lane + kSlotTab1, ge_p3_neg(Y));
  st_words8(lane + kSlotA1, c);
  st_words8(lane + kSlotB, s);
  st_carry(lane, 0, sc_recode_carries<4, 33>(c));
  st_carry(lane, 2, sc_recode_b(s));
  dsm(lane, btab, dsm_cfg(33, 0, true));
  ge_p2 U = dsm_result(lane);
  // V = [s]H - [c]Gamma
  build_table(lane + kSlotTab1, Hp);
  build_table(lane + kSlotTab2, ge_p3_neg(Gamma));
  st_words8(lane + kSlotA1, s);
  st_words8(lane + kSlotA2, c);
  st_carry(lane, 0, sc_recode_carries<4, 64>(s));
  st_carry(lane, 1, sc_recode_carries<4, 33>(c));
  dsm(lane, btab, dsm_cfg(64, 33, false));
  ge_p2 V = dsm_result(lane);
  ge_p3 G8 = ge_mul8(Gamma);
  // one inversion for the four encodings
  fe z[4] = {Hp.Z, U.Z, V.Z, G8.Z}, zi[4];
  fe_invert4(zi, z);
  uint32_t Henc[8], Uenc[8], Venc[8], G8enc[8], Genc[8];
  ge_encode_with_inv(Henc, Hp.X, Hp.Y, zi[0]);
  ge_encode_with_inv(Uenc, U.X, U.Y, zi[1]);
  ge_encode_with_inv(Venc, V.X, V.Y, zi[2]);
  ge_encode_with_inv(G8enc, G8.X, G8.Y, zi[3]);
  // Gamma re-encoded: the input bytes, except x = 0 encodes with sign 0
#pragma unroll
  for (int i = 0; i < 8; i++) Genc[i] = G[i];
  if (fe_iszero(Gamma.X)) Genc[7] &= 0x7fffffffu;
  // c' = SHA-512(0x04 || 0x02 || H || Gamma || U || V)[0:16]
  uint32_t hp[33];
  hp[0] = 0x04u | (0x02u << 8) | (Henc[0] << 16);
#pragma unroll
  for (int i = 1; i < 8; i++) hp[i] = (Henc[i - 1] >> 16) | (Henc[i] << 16);
  hp[8] = (Henc[7] >> 16) | (Genc[0] << 16);
#pragma unroll
  for (int i = 1; i < 8; i++) hp[8 + i] = (Genc[i - 1] >> 16) | (Genc[i] << 16);
  hp[16] = (Genc[7] >> 16) | (Uenc[0] << 16);
#pragma unroll
  for (int i = 1; i < 8; i++) hp[16 + i] = (Uenc[i - 1] >> 16) | (Uenc[i] << 16);
  hp[24] = (Uenc[7] >> 16) | (Venc[0] << 16);
#pragma unroll
  for (int i = 1; i < 8; i++) hp[24 + i] = (Venc[i - 1] >> 16) | (Venc[i] << 16);
  hp[32] = Venc[7] >> 16;
  uint64_t Hc[8];
  sha512_prefixed<130>(Hc, hp, ShaNoTail{}, 0);
  uint32_t cw[16];
  sha512_digest_words(cw, Hc);
  bool ceq = true;
#pragma unroll
  for (int i = 0; i < 4; i++) ceq = ceq && cw[i] == c[i];
  ok = ok && ceq;
  // beta = SHA-512(0x04 || 0x03 || encode([8]Gamma))
  uint32_t bp[9];
  bp[0] = 0x04u | (0x03u << 8) | (G8enc[0] << 16);
#pragma unroll
  for (int i = 1; i < 8; i++) bp[i] = (G8enc[i - 1] >> 16) | (G8enc[i] << 16);
  bp[8] = G8enc[7] >> 16;
  uint64_t Hb[8];
  sha512_prefixed<34>(Hb, bp, ShaNoTail{}, 0);
  uint32_t bw[16];
  sha512_digest_words(bw, Hb);
#pragma unroll
  for (int i = 0; i < 16; i++) beta[i] = ok ? bw[i] : 0u;
  return ok;
}

// ---- Sum6KES --------------------------------------------------------------------
// sig (448 B) is read from global memory: leaf signature, then (vk0, vk1) for
// levels 1..6 bottom-up; verification walks top-down from the root vk.
// the Merkle walk: checks the six (vk0, vk1) levels against the root vk and
// returns the leaf's verification key in cur and its signature in sig
OURO_HD inline bool sum6kes_walk(uint32_t cur[8], uint32_t sig[16], const uint32_t vk[8],
                                 uint32_t t, const uint32_t* sigw) {
#pragma unroll
  for (int i = 0; i < 8; i++) cur[i] = vk[i];
  bool ok = true;
#pragma unroll 1
  for (int k = 6; k >= 1; k--) {
    const uint32_t* pair = sigw + 16 + 16 * (k - 1);
    uint32_t pw[16], h[8];
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const int4 v = ldg4(pair + 4 * i);
      pw[4 * i] = v.x; pw[4 * i + 1] = v.y; pw[4 * i + 2] = v.z; pw[4 * i + 3] = v.w;
    }
    blake2b256_64(h, pw);
#pragma unroll
    for (int i = 0; i < 8; i++) ok = ok && h[i] == cur[i];
    const uint32_t half = 1u << (k - 1);
    const bool right = t >= half;
    t = right ? t - half : t;
#pragma unroll
    for (int i = 0; i < 8; i++) cur[i] = right ? pw[8 + i] : pw[i];
  }
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const int4 v = ldg4(sigw + 4 * i);
    sig[4 * i] = v.x; sig[4 * i + 1] = v.y; sig[4 * i + 2] = v.z; sig[4 * i + 3] = v.w;
  }
  return ok;
}

template <class Tail>
OURO_HD inline bool sum6kes_verify_lane(const uint32_t vk[8], uint32_t t, const uint32_t* sigw,
                                        const Tail& msg, uint32_t mlen, Slot lane,
                                        const int32_t* btab, bool quad = false,
                                        int phase = kPhaseAll) {
  if (phase == kPhasePost) return dsm_result_is_identity(lane);
  uint32_t cur[8], sig[16];
  const bool ok = sum6kes_walk(cur, sig, vk, t, sigw);
  const bool leaf = ed25519_verify_lane(sig, cur, msg, mlen, lane, btab, false, quad, phase);
  return ok && leaf;
}

// ---- fixed-base tables (host side, computed once per process) ----------------
// [k]G for k = 1..kBTabEntries as (y + x, y - x, 2 d x y), affine, reduced
// limbs, for G = B and G = 2^128 B (the two halves of the split scalar).  The
// affine conversion inverts the Z coordinates in chunks with one inversion each
// (Montgomery's trick); 2 x 32768 entries take a few tens of ms on the host.
inline void build_btab_one(int32_t* out, const ge_p3& G) {
  constexpr int kChunk = 256;
  std::vector<ge_p3> pts(kChunk);
  std::vector<fe> pre(kChunk);
  ge_p3 P = G;
  for (int k0 = 0; k0 < kBTabEntries; k0 += kChunk) {
    const int n = kBTabEntries - k0 < kChunk ? kBTabEntries - k0 : kChunk;
    for (int i = 0; i < n; i++) {
      if (k0 + i > 0) P = ge_p3_add(P, G);
      pts[i] = P;
      pre[i] = i ? fe_mul(pre[i - 1], P.Z) : P.Z;
    }
    fe inv = fe_invert(pre[n - 1]);
    for (int i = n - 1; i >= 0; i--) {
      const fe zi = i ? fe_mul(inv, pre[i - 1]) : inv;
      if (i) inv = fe_mul(inv, pts[i].Z);
      fe x = fe_mul(pts[i].X, zi), y = fe_mul(pts[i].Y, zi);
      fe yp = fe_carry(fe_add(y, x)), ym = fe_carry(fe_sub(y, x));
      fe xy2d = fe_mul(fe_mul(x, y), fe_d2());
      int32_t* e = out + (size_t)(k0 + i) * kNielsWords;
      for (int l = 0; l < 10; l++) {
        e[l] = yp.v[l];
        e[10 + l] = ym.v[l];
        e[20 + l] = xy2d.v[l];
      }
      OURO_TRK(ouro_trk_store(e, yp.b); ouro_trk_store(e + 10, ym.b); ouro_trk_store(e + 20, xy2d.b);)
      e[30] = 0;
      e[31] = 0;
    }
  }
}

inline void build_btab(int32_t* out) {
  // B = (x, 4/5) with x even: encoding 0x5866...66 (little-endian)
  uint32_t by[8];
  for (int i = 0; i < 8; i++) by[i] = 0x66666666u;
  by[0] = 0x66666658u;
  ge_p3 B;
  ge_decode(&B, by, false);
  build_btab_one(out, B);
  ge_p3 B128 = B;
  for (int i = 0; i < 128; i++) B128 = ge_p1p1_to_p3(ge_p3_dbl(B128));
  build_btab_one(out + (size_t)kBTabEntries * kNielsWords, B128);
}

// The fixed-base tables in the latency mode's wave-wide form (wide.h
// bw_operand), stored after the niels ones: per entry the canonical 16-bit
// limbs of y - x, y + x and 2dxy.
constexpr int kBWideU16 = 48;
constexpr size_t kBTabWideWords = (size_t)kBTabEntries * kBWideU16;  // both halves, int32 words
inline void build_btab_wide(uint16_t* out, const int32_t* niels) {
  for (size_t e = 0; e < 2 * (size_t)kBTabEntries; e++) {
    const int32_t* q = niels + e * kNielsWords;
    for (int k = 0; k < 3; k++) {
      const int32_t* c = q + (k == 0 ? 10 : (k == 1 ? 0 : 20));  // y - x, y + x, 2dxy
      const fe f = fe_make(c[0], c[1], c[2], c[3], c[4], c[5], c[6], c[7], c[8], c[9]);
      uint32_t w[8];
      fe_to_words(w, f);
      for (int j = 0; j < 16; j++)
        out[e * kBWideU16 + 16 * k + j] = (uint16_t)((w[j >> 1] >> (16 * (j & 1))) & 0xffffu);
    }
  }
}

}  // namespace ouro
