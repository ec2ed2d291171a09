// cbor_byron.h -- the Byron header slicer (SURVEY.md §8(f) row 4, §8(a) row
// a11): raw Byron header CBOR as ChainSync receives it -> the key, signature
// and signed message of its PBFT block-signature check.  One header per call,
// no allocation, no recursion (csrc/cbor.h's bounded walker).  Acceptance
// mirrors byron.py parse_byron_header check for check, status for status
// (tests/test_pack_byron.py pins the two against each other).
//
// Wire forms (ouroboros-consensus-byron/src/Ouroboros/Consensus/Byron/Node/Serialisation.hs):
//   F1  #6.24(bytes .cbor [kind, header])                 Byron N2N v1 (:87-92),
//                                                        Cardano N2N v1
//   F2  [[kind, size], #6.24(bytes .cbor header)]         Byron N2N v2 (encodeDisk of
//                                                        the nested context, :197-210)
//   F3  [0, F2]                                           Cardano N2N v2+ (HFC era 0)
// kind 1 = a regular header, 0 = an epoch-boundary header (EBB), which PBFT
// accepts without a signature (ouroboros-consensus/src/Ouroboros/Consensus/Protocol/PBFT.hs:327-328).
// Regular header = [protocolMagic, prevHash, bodyProof, consensusData, extraData],
// consensusData = [slotId, leaderKey, difficulty, [2, [dlgCert, sig]]],
// dlgCert = [epoch, issuerXPub, delegateXPub, certSig].
// The block signature verifies under delegateXPub[0:32] (pbftIssuer,
// ouroboros-consensus-byron/src/Ouroboros/Consensus/Byron/Ledger/PBFT.hs:50-66)
// over signTag magic (SignBlock issuerXPub) || recoverSignedBytes:
//   "01" || issuerXPub (64) || 0x09 || CBOR(magic) || 0x85 || prevHash ||
//   bodyProof || slotId || difficulty || extraData           (raw bytes)
// with magic the node's configured ProtocolMagicId (mkByronContextDSIGN,
// Byron/Ledger/PBFT.hs:43-44) -- or, on request, each header's own field.
#pragma once
#include "cbor.h"

namespace ouro {
namespace cbor {

struct ByronOut {
  uint8_t *pk, *sig, *genesis_vk, *delegate_vk, *msg;
  uint64_t *msg_off, *magic;
  uint32_t* msg_len;
};

// the message of header i lies at msg + msg_off[i] (the caller's layout gives
// every header len[i] + kByronMsgExtra bytes; the message needs at most
// len[i] + 74: the signed fields are disjoint pieces of the header)
constexpr uint64_t kByronMsgExtra = 80;
constexpr uint64_t kWord32Max = 0xffffffffull;

// canonical CBOR head of an unsigned integer (serialize' of a Word32)
OURO_HD inline int put_uint(uint8_t* d, uint64_t v) {
  if (v < 24) {
    d[0] = (uint8_t)v;
    return 1;
  }
  const int w = v < 0x100ull ? 1 : v < 0x10000ull ? 2 : v <= kWord32Max ? 4 : 8;
  d[0] = (uint8_t)(w == 1 ? 24 : w == 2 ? 25 : w == 4 ? 26 : 27);
  for (int k = 0; k < w; k++) d[1 + k] = (uint8_t)(v >> (8 * (w - 1 - k)));
  return 1 + w;
}

OURO_HD inline uint64_t put_span(uint8_t* d, const Cur& c, uint64_t s, uint64_t e) {
#if defined(__HIP_DEVICE_COMPILE__)
  for (uint64_t k = s; k < e; k++) d[k - s] = (uint8_t)cb(c, k);
#else
  __builtin_memcpy(d, c.b + s, e - s);
#endif
  return e - s;
}

// a definite array of exactly `want` items at i (0 = the right shape; else a status)
OURO_HD inline uint8_t fixed_array(const Cur& c, uint64_t i, uint64_t* s, uint64_t* e, int want) {
  int cnt;
  if (!array_items(c, i, s, e, want, &cnt)) return OURO_PACK_ECBOR;
  return cnt == want ? 0 : OURO_PACK_ESHAPE;
}

// a uint no larger than `max` (decodeWord8 / decodeWord32 / a ProtocolMagicId)
OURO_HD inline bool uint_le(const Cur& c, uint64_t i, uint64_t max, uint64_t* v) {
  return uint_at(c, i, v) && *v <= max;
}

// magic_cfg: the configured ProtocolMagicId, or -1 for each header's own
OURO_HD inline uint8_t byron_pack_one(const uint8_t* raw, uint64_t base, uint32_t len,
                                      int64_t magic_cfg, const ByronOut& o, size_t i) {
  const Cur outer{raw + base, len};
  int mt;
  uint64_t arg, j, k, pos = 0, kind = 0;
  bool ind;
  uint64_t s2[2], e2[2];
  uint8_t st;
  if (!head(outer, 0, &mt, &arg, &j, &ind)) return OURO_PACK_ECBOR;
  const bool nested = mt == 4 && !ind && arg == 2;
  if (nested) {  // F3 [era, F2] or F2 [[kind, size], tag]
    int mt1;
    uint64_t a1, j1;
    bool i1;
    if (!head(outer, j, &mt1, &a1, &j1, &i1)) return OURO_PACK_ECBOR;
    if (mt1 == 0) {  // F3: the HFC era, then F2
      if (i1) return OURO_PACK_ESHAPE;
      if (a1 != 0) return OURO_PACK_ESHELLEY;
      pos = j1;
      if (!head(outer, pos, &mt, &arg, &j, &ind)) return OURO_PACK_ECBOR;
      if (mt != 4 || ind || arg != 2) return OURO_PACK_ESHAPE;
    }
    // F2 at pos: [kind, size] (decodeWord8, decodeWord32), then the tag
    if ((st = fixed_array(outer, j, s2, e2, 2))) return st;
    uint64_t size;
    if (!uint_le(outer, s2[0], 255, &kind) || !uint_le(outer, s2[1], kWord32Max, &size))
      return OURO_PACK_ESHAPE;
    if (kind > 1) return OURO_PACK_ESHAPE;  // DecoderErrorUnknownTag
    pos = e2[1];                            // the tag follows [kind, size]
  }
  if (!head(outer, pos, &mt, &arg, &j, &ind)) return OURO_PACK_ECBOR;
  if (mt != 6 || ind || arg != 24) return OURO_PACK_ESHAPE;
  if (!head(outer, j, &mt, &arg, &k, &ind)) return OURO_PACK_ECBOR;
  if (mt != 2 || ind) return OURO_PACK_ESHAPE;
  if (outer.n - k < arg) return OURO_PACK_ECBOR;   // payload past the span
  if (k + arg != outer.n) return OURO_PACK_ECBOR;  // bytes after the header
  const Cur c{raw + base, k + arg};                // the payload bounds the parse
  uint64_t h = k;                                  // the header item
  if (!nested) {  // F1: the payload is [kind, header]
    if ((st = fixed_array(c, k, s2, e2, 2))) return st;
    if (!uint_le(c, s2[0], ~0ull, &kind) || kind > 1) return OURO_PACK_ESHAPE;
    h = s2[1];
  }
  uint64_t fs[5], fe[5], cs[4], ce[4], bs[2], be[2], is[2], ie[2], ds[4], de[4];
  if (kind == 0) {  // no signature; its fields are not checked
    uint64_t he;
    if (!skip(c, h, &he)) return OURO_PACK_ECBOR;
    return he == c.n ? OURO_PACK_EBB : OURO_PACK_ECBOR;
  }
  // one walk of the header's five fields; it must end where the payload does
  if ((st = fixed_array(c, h, fs, fe, 5))) return st;
  if (fe[4] != c.n) return OURO_PACK_ECBOR;  // trailing bytes in CBOR-in-CBOR
  uint64_t magic;
  if (!uint_le(c, fs[0], kWord32Max, &magic)) return OURO_PACK_ESHAPE;
  if ((st = fixed_array(c, fs[3], cs, ce, 4))) return st;
  if ((st = fixed_array(c, cs[3], bs, be, 2))) return st;
  uint64_t sigkind;
  if (!uint_at(c, bs[0], &sigkind) || sigkind != 2) return OURO_PACK_ESHAPE;
  if ((st = fixed_array(c, bs[1], is, ie, 2))) return st;
  if ((st = fixed_array(c, is[0], ds, de, 4))) return st;
  const uint8_t *gvk, *dvk, *sg;
  const int r0 = bytes_at(c, ds[1], 64, &gvk), r1 = bytes_at(c, ds[2], 64, &dvk),
            r2 = bytes_at(c, is[1], 64, &sg);
  if (r0 == kBytesShape || r1 == kBytesShape || r2 == kBytesShape) return OURO_PACK_ESHAPE;
  if (r0 | r1 | r2) return OURO_PACK_ESIZE;
  const uint64_t m = magic_cfg < 0 ? magic : (uint64_t)magic_cfg;
  uint8_t* d = o.msg + o.msg_off[i];
  uint64_t n = 0;
  d[n++] = '0';
  d[n++] = '1';
  n += put_span(d + n, c, (uint64_t)(gvk - c.b), (uint64_t)(gvk - c.b) + 64);
  d[n++] = 0x09;
  n += (uint64_t)put_uint(d + n, m);
  d[n++] = 0x85;  // ToSign: encodeListLen 5
  n += put_span(d + n, c, fs[1], fe[1]);  // prevHash
  n += put_span(d + n, c, fs[2], fe[2]);  // bodyProof
  n += put_span(d + n, c, cs[0], ce[0]);  // slotId
  n += put_span(d + n, c, cs[2], ce[2]);  // difficulty
  n += put_span(d + n, c, fs[4], fe[4]);  // extraData
  o.msg_len[i] = (uint32_t)n;
  const uint64_t g0 = (uint64_t)(gvk - c.b), d0 = (uint64_t)(dvk - c.b), s0 = (uint64_t)(sg - c.b);
  put_span(o.pk + 32 * i, c, d0, d0 + 32);
  put_span(o.sig + 64 * i, c, s0, s0 + 64);
  put_span(o.genesis_vk + 64 * i, c, g0, g0 + 64);
  put_span(o.delegate_vk + 64 * i, c, d0, d0 + 64);
  o.magic[i] = magic;
  return OURO_PACK_OK;
}

OURO_HD inline void byron_zero_row(const ByronOut& o, size_t i) {
  for (int q = 0; q < 32; q++) o.pk[32 * i + q] = 0;
  for (int q = 0; q < 64; q++) o.sig[64 * i + q] = o.genesis_vk[64 * i + q] = o.delegate_vk[64 * i + q] = 0;
  o.msg_len[i] = 0;
  o.magic[i] = 0;
}

// the arena: pk, sig, genesis_vk, delegate_vk, msg_off, msg_len, magic (64-byte
// aligned arrays), then the messages
struct ByronLayout {
  size_t off[8];
  size_t total;
};
constexpr size_t kByronRowBytes[7] = {32, 64, 64, 64, 8, 4, 8};
inline ByronLayout byron_layout(size_t n, size_t msg_bytes) {
  ByronLayout l{};
  size_t at = 0;
  for (int k = 0; k < 7; k++) {
    l.off[k] = at;
    at += (kByronRowBytes[k] * n + 63) & ~(size_t)63;
  }
  l.off[7] = at;
  l.total = at + msg_bytes;
  return l;
}
inline ByronOut byron_arena_out(uint8_t* a, const ByronLayout& l) {
  ByronOut o;
  o.pk = a + l.off[0];
  o.sig = a + l.off[1];
  o.genesis_vk = a + l.off[2];
  o.delegate_vk = a + l.off[3];
  o.msg_off = reinterpret_cast<uint64_t*>(a + l.off[4]);
  o.msg_len = reinterpret_cast<uint32_t*>(a + l.off[5]);
  o.magic = reinterpret_cast<uint64_t*>(a + l.off[6]);
  o.msg = a + l.off[7];
  return o;
}

}  // namespace cbor
}  // namespace ouro
