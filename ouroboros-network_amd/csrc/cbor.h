// cbor.h -- the TPraos header slicer's parse, shared
// by the host slicer (csrc/pack.cpp, ouro_tpraos_pack_cbor) and the device one
// (kernels.hip k_tpraos_pack, ouro_tpraos_pack_cbor_device): one header per
// call, no allocation, no recursion (containers are tracked on a bounded
// stack), byte loops instead of libc, so the same code compiles for gfx950.
// Acceptance mirrors header.py parse_header / pack item for item
// (tests/test_pack.py pins the host build; tests/test_gpu_pack.py the device
// build against the host one).
#pragma once
#include <stddef.h>
#include <stdint.h>

#include "../../include/ouro_verify.h"
#if defined(__HIPCC__)
#include "common.h"
#else  // a plain C++ build of the host slicer (the ASan/UBSan test library)
#define OURO_HD
#endif

namespace ouro {
namespace cbor {

// n bytes (a multiple of 16) to a 16-byte aligned destination.  On the device
// from the aligned dwords covering the source, funnel-shifted into place --
// only dwords that start before the source's end are read, so nothing past
// the raw buffer -- and stored as dwordx4: a lane's field copy is n/4 + 1
// dword loads instead of n byte loads.
OURO_HD inline void copy_bytes(uint8_t* d, const uint8_t* s, int n) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uintptr_t a = reinterpret_cast<uintptr_t>(s);
  const uintptr_t w0 = a & ~uintptr_t(3), end = a + (uintptr_t)n;
  const uint32_t sh = (uint32_t)(a & 3) * 8;
  uint32_t prev = (uint32_t)ldg1(reinterpret_cast<const void*>(w0));
  for (int k = 0; k < n; k += 16) {
    uint32_t o[4];
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const uintptr_t nx = w0 + (uintptr_t)(k + 4 * q + 4);
      const uint32_t next = nx < end ? (uint32_t)ldg1(reinterpret_cast<const void*>(nx)) : 0u;
      o[q] = __builtin_amdgcn_alignbit(next, prev, sh);
      prev = next;
    }
    stg4(d + k, make_int4((int)o[0], (int)o[1], (int)o[2], (int)o[3]));
  }
#else
  __builtin_memcpy(d, s, (size_t)n);
#endif
}
OURO_HD inline void zero_bytes(uint8_t* d, int n) {  // n a multiple of 16, d 16-byte aligned
#if defined(__HIP_DEVICE_COMPILE__)
  for (int k = 0; k < n; k += 16) stg4(d + k, make_int4(0, 0, 0, 0));
#else
  __builtin_memset(d, 0, (size_t)n);
#endif
}

constexpr int kMaxDepth = 64;  // nesting guard for skip() on hostile input

struct Cur {
  const uint8_t* b;
  uint64_t n;  // bytes of this header
};
OURO_HD inline uint32_t cb(const Cur& c, uint64_t i) {  // byte i (global memory on the device)
#if defined(__HIP_DEVICE_COMPILE__)
  return ldg_u8(c.b + i);
#else
  return c.b[i];
#endif
}

// (major type, argument, index after the head); false = truncated/reserved.
// *indef marks an indefinite length (additional info 31; arg is then 0).
OURO_HD inline bool head(const Cur& c, uint64_t i, int* mt, uint64_t* arg, uint64_t* next,
                        bool* indef) {
  if (i >= c.n) return false;
  const uint8_t ib = (uint8_t)cb(c, i);
  *mt = ib >> 5;
  const int ai = ib & 31;
  i++;
  *indef = false;
  if (ai < 24) {
    *arg = (uint64_t)ai;
  } else if (ai <= 27) {
    const int len = 1 << (ai - 24);
    if (c.n - i < (uint64_t)len) return false;
    uint64_t v = 0;
    for (int k = 0; k < len; k++) v = (v << 8) | cb(c, i + k);
    *arg = v;
    i += len;
  } else if (ai == 31) {
    *arg = 0;
    *indef = true;
  } else {
    return false;  // 28..30 reserved
  }
  *next = i;
  return true;
}

// index just past the data item at i (header.py skip), iteratively: rem[d]
// = items still to read in the d-th open container (kIndef: until a break)
constexpr uint64_t kIndef = ~0ull;
OURO_HD inline bool skip(const Cur& c, uint64_t i, uint64_t* out) {
  uint64_t rem[kMaxDepth + 1];
  int d = 0;
  rem[0] = 1;
  for (;;) {
    while (d >= 0 && rem[d] == 0) d--;  // finished definite containers
    if (d < 0) {
      *out = i;
      return true;
    }
    if (rem[d] == kIndef) {
      if (i >= c.n) return false;
      if (cb(c, i) == 0xFF) {  // break: closes the indefinite container
        i++;
        d--;
        continue;
      }
    } else {
      rem[d]--;
    }
    int mt;
    uint64_t arg, j;
    bool ind;
    if (!head(c, i, &mt, &arg, &j, &ind)) return false;
    uint64_t push = 0;
    bool open = true;
    switch (mt) {
      case 0: case 1: case 7:
        open = false;
        i = j;
        break;
      case 2: case 3:
        if (ind) {
          push = kIndef;
        } else {
          if (c.n - j < arg) return false;
          open = false;
          j += arg;
        }
        i = j;
        break;
      case 4: case 5:
        // each element takes at least one byte: a count beyond the input is truncated
        if (!ind && arg > c.n) return false;
        push = ind ? kIndef : (mt == 5 ? 2 * arg : arg);
        i = j;
        break;
      default:  // 6: a tag, then its content
        push = 1;
        i = j;
    }
    if (open) {
      if (d == kMaxDepth) return false;  // nesting guard on hostile input
      rem[++d] = push;
    }
  }
}

// spans of the elements of the definite array at i (at most `cap`)
OURO_HD inline bool array_items(const Cur& c, uint64_t i, uint64_t* starts, uint64_t* ends, int cap, int* count) {
  int mt;
  uint64_t arg, j;
  bool ind;
  if (!head(c, i, &mt, &arg, &j, &ind) || mt != 4 || ind) return false;
  if (arg > (uint64_t)cap) {  // header.py reads every element, then rejects the count
    for (uint64_t k = 0; k < arg; k++)
      if (!skip(c, j, &j)) return false;
    *count = -1;
    return true;
  }
  for (uint64_t k = 0; k < arg; k++) {
    starts[k] = j;
    if (!skip(c, j, &j)) return false;
    ends[k] = j;
  }
  *count = (int)arg;
  return true;
}

OURO_HD inline bool uint_at(const Cur& c, uint64_t i, uint64_t* v) {
  int mt;
  uint64_t arg, j;
  bool ind;
  if (!head(c, i, &mt, &arg, &j, &ind) || mt != 0 || ind) return false;
  *v = arg;
  return true;
}

// definite byte string of exactly `want` bytes at i
enum { kBytesOk = 0, kBytesShape = 1, kBytesSize = 2 };
OURO_HD inline int bytes_at(const Cur& c, uint64_t i, uint64_t want, const uint8_t** p) {
  int mt;
  uint64_t arg, j;
  bool ind;
  if (!head(c, i, &mt, &arg, &j, &ind) || mt != 2 || ind) return kBytesShape;
  if (c.n - j < arg) return kBytesShape;  // (cannot happen after skip; kept for safety)
  if (arg != want) return kBytesSize;
  *p = c.b + j;
  return kBytesOk;
}

struct Out {
  uint8_t *issuer_vk, *vrf_vk, *eta_proof, *leader_proof, *hot_vk, *sigma, *kes_sig;
  uint8_t *eta_output, *leader_output;
  uint64_t *counter, *c0, *body_off;
  uint32_t *kes_t, *body_len;
  uint64_t* slot;
  uint8_t* era;
};

// Integrity.hs:38-44: kesPeriod(slot) - c0 clamped at 0, a Word saturated at
// 2^32 - 1 (every t >= 63 walks to Sum6KES leaf 63, kes.py periods_u32)
OURO_HD inline uint32_t kes_t_of(uint64_t slot, uint64_t spkp, uint64_t c0) {
  const uint64_t cur = slot / spkp;
  const uint64_t t = cur >= c0 ? cur - c0 : 0;
  return t > 0xffffffffull ? 0xffffffffu : (uint32_t)t;
}

// CBOR-in-CBOR as the reference decodes it
// (ouroboros-network/src/Ouroboros/Network/Block.hs:509-514, decodeWrapped):
// the tag-24 byte string must be definite and lie inside the header's span,
// the [header_body, kes_sig] item is parsed from its payload ALONE and must
// end exactly where the payload ends ("trailing bytes in CBOR-in-CBOR"), and
// nothing may follow the header inside its span.
OURO_HD inline uint8_t pack_one(const uint8_t* raw, uint64_t base, uint32_t len, uint64_t spkp, const Out& o,
                 size_t i) {
  const Cur outer{raw + base, len};
  int mt;
  uint64_t arg, j, pos = 0, era = 1;
  bool ind;
  if (!head(outer, 0, &mt, &arg, &j, &ind)) return OURO_PACK_ECBOR;
  if (mt == 4 && !ind && arg == 2) {  // [era, wrapped]
    if (!uint_at(outer, j, &era)) return OURO_PACK_ESHAPE;
    if (era == 0) return OURO_PACK_EBYRON;
    if (!skip(outer, j, &pos)) return OURO_PACK_ECBOR;
  }
  if (!head(outer, pos, &mt, &arg, &j, &ind)) return OURO_PACK_ECBOR;
  if (mt != 6 || ind || arg != 24) return OURO_PACK_ESHAPE;
  uint64_t k;
  if (!head(outer, j, &mt, &arg, &k, &ind)) return OURO_PACK_ECBOR;
  if (mt != 2 || ind) return OURO_PACK_ESHAPE;
  if (outer.n - k < arg) return OURO_PACK_ECBOR;       // payload past the span
  if (k + arg != outer.n) return OURO_PACK_ECBOR;      // bytes after the header
  const Cur c{raw + base, k + arg};                    // the payload's end bounds the parse
  // [header_body, kes_sig]: the body's fields are walked once (the last
  // field's end is the body's end), then the signature
  uint64_t ts[2], te[2], fs[15], fe[15];
  int cnt;
  if (!head(c, k, &mt, &arg, &j, &ind)) return OURO_PACK_ECBOR;
  if (mt != 4 || ind) return OURO_PACK_ECBOR;
  if (arg != 2) return OURO_PACK_ESHAPE;
  ts[0] = j;
  if (!array_items(c, ts[0], fs, fe, 15, &cnt)) return OURO_PACK_ECBOR;
  if (cnt != 15) return OURO_PACK_ESHAPE;
  te[0] = ts[1] = fe[14];
  if (!skip(c, ts[1], &te[1])) return OURO_PACK_ECBOR;
  if (te[1] != c.n) return OURO_PACK_ECBOR;            // trailing bytes in CBOR-in-CBOR
  uint64_t es[2], ee[2], ls[2], le[2];
  int ce, cl;
  if (!array_items(c, fs[5], es, ee, 2, &ce) || !array_items(c, fs[6], ls, le, 2, &cl))
    return OURO_PACK_ECBOR;
  if (ce != 2 || cl != 2) return OURO_PACK_ESHAPE;
  uint64_t block_no, slot, counter, c0;
  if (!uint_at(c, fs[0], &block_no) || !uint_at(c, fs[1], &slot)) return OURO_PACK_ESHAPE;
  // header.py checks the field types in this order, then every size
  const uint8_t *ivk, *vvk, *eo, *ep, *lo, *lp, *hvk, *sg, *ks;
  const int r0 = bytes_at(c, fs[3], 32, &ivk), r1 = bytes_at(c, fs[4], 32, &vvk);
  if (r0 == kBytesShape || r1 == kBytesShape) return OURO_PACK_ESHAPE;
  const int r2 = bytes_at(c, es[0], 64, &eo), r3 = bytes_at(c, es[1], 80, &ep);
  if (r2 == kBytesShape || r3 == kBytesShape) return OURO_PACK_ESHAPE;
  const int r4 = bytes_at(c, ls[0], 64, &lo), r5 = bytes_at(c, ls[1], 80, &lp);
  if (r4 == kBytesShape || r5 == kBytesShape) return OURO_PACK_ESHAPE;
  const int r6 = bytes_at(c, fs[9], 32, &hvk);
  if (r6 == kBytesShape) return OURO_PACK_ESHAPE;
  if (!uint_at(c, fs[10], &counter) || !uint_at(c, fs[11], &c0)) return OURO_PACK_ESHAPE;
  const int r7 = bytes_at(c, fs[12], 64, &sg), r8 = bytes_at(c, ts[1], 448, &ks);
  if (r7 == kBytesShape || r8 == kBytesShape) return OURO_PACK_ESHAPE;
  if (r0 | r1 | r2 | r3 | r4 | r5 | r6 | r7 | r8) return OURO_PACK_ESIZE;
  copy_bytes(o.issuer_vk + 32 * i, ivk, 32);
  copy_bytes(o.vrf_vk + 32 * i, vvk, 32);
  copy_bytes(o.eta_output + 64 * i, eo, 64);
  copy_bytes(o.eta_proof + 80 * i, ep, 80);
  copy_bytes(o.leader_output + 64 * i, lo, 64);
  copy_bytes(o.leader_proof + 80 * i, lp, 80);
  copy_bytes(o.hot_vk + 32 * i, hvk, 32);
  copy_bytes(o.sigma + 64 * i, sg, 64);
  copy_bytes(o.kes_sig + 448 * i, ks, 448);
  o.counter[i] = counter;
  o.c0[i] = c0;
  o.kes_t[i] = kes_t_of(slot, spkp, c0);
  o.body_off[i] = base + ts[0];
  o.body_len[i] = (uint32_t)(te[0] - ts[0]);
  if (o.slot) o.slot[i] = slot;
  if (o.era) o.era[i] = (uint8_t)(era > 255 ? 255 : era);
  return OURO_PACK_OK;
}

OURO_HD inline void zero_row(const Out& o, size_t i) {
  zero_bytes(o.issuer_vk + 32 * i, 32);
  zero_bytes(o.vrf_vk + 32 * i, 32);
  zero_bytes(o.eta_output + 64 * i, 64);
  zero_bytes(o.eta_proof + 80 * i, 80);
  zero_bytes(o.leader_output + 64 * i, 64);
  zero_bytes(o.leader_proof + 80 * i, 80);
  zero_bytes(o.hot_vk + 32 * i, 32);
  zero_bytes(o.sigma + 64 * i, 64);
  zero_bytes(o.kes_sig + 448 * i, 448);
  o.counter[i] = o.c0[i] = 0;
  o.kes_t[i] = 0;
  o.body_off[i] = 0;
  o.body_len[i] = 0;
  if (o.slot) o.slot[i] = 0;
  if (o.era) o.era[i] = 0;
}

// the arena ouro_tpraos_pack_cbor[_device] fills: one array per member, each
// 64-byte aligned (member k of the SoA at off[k])
struct Layout {
  size_t off[14];
  size_t total;
};
constexpr size_t kRowBytes[14] = {32, 32, 80, 80, 32, 8, 8, 64, 4, 448, 8, 4, 64, 64};
inline Layout layout(size_t n) {
  Layout l{};
  size_t at = 0;
  for (int k = 0; k < 14; k++) {
    l.off[k] = at;
    at += (kRowBytes[k] * n + 63) & ~(size_t)63;
  }
  l.total = at;
  return l;
}
// the arena's arrays from its (64-byte aligned) base; slot / era: caller's
inline Out arena_out(uint8_t* a, size_t n, uint64_t* slot, uint8_t* era) {
  const Layout l = layout(n);
  Out o;
  o.issuer_vk = a + l.off[0];
  o.vrf_vk = a + l.off[1];
  o.eta_proof = a + l.off[2];
  o.leader_proof = a + l.off[3];
  o.hot_vk = a + l.off[4];
  o.counter = reinterpret_cast<uint64_t*>(a + l.off[5]);
  o.c0 = reinterpret_cast<uint64_t*>(a + l.off[6]);
  o.sigma = a + l.off[7];
  o.kes_t = reinterpret_cast<uint32_t*>(a + l.off[8]);
  o.kes_sig = a + l.off[9];
  o.body_off = reinterpret_cast<uint64_t*>(a + l.off[10]);
  o.body_len = reinterpret_cast<uint32_t*>(a + l.off[11]);
  o.eta_output = a + l.off[12];
  o.leader_output = a + l.off[13];
  o.slot = slot;
  o.era = era;
  return o;
}
// point the batch's members at the arena's arrays (body = the raw buffer)
inline void batch_from(ouro_tpraos_batch* out, const Out& o, const uint8_t* raw, size_t n) {
  out->n = n;
  out->issuer_vk = o.issuer_vk;
  out->vrf_vk = o.vrf_vk;
  out->eta_proof = o.eta_proof;
  out->leader_proof = o.leader_proof;
  out->hot_vk = o.hot_vk;
  out->ocert_counter = o.counter;
  out->ocert_kes_period = o.c0;
  out->ocert_sigma = o.sigma;
  out->kes_t = o.kes_t;
  out->kes_sig = o.kes_sig;
  out->body = raw;
  out->body_off = o.body_off;
  out->body_len = o.body_len;
  out->eta_output = o.eta_output;
  out->leader_output = o.leader_output;
}
inline uint8_t* arena_base(void* arena) {
  uint8_t* a = static_cast<uint8_t*>(arena);
  return a + ((64 - (reinterpret_cast<uintptr_t>(a) & 63)) & 63);
}

}  // namespace cbor
}  // namespace ouro
