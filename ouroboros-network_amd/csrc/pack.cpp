// pack.cpp -- raw TPraos header CBOR -> the SoA of ouro_tpraos_batch
// (include/ouro_verify.h ouro_tpraos_pack_cbor).
//
// Host code (no device): it sits between the ChainSync client, which hands
// over headers as the raw CBOR it received, and the batch verifier.  Wire
// shapes (ouroboros-network/test/messages.cddl:27-34; the header keeps its
// raw bytes through Annotator at
// ouroboros-consensus-shelley/src/Ouroboros/Consensus/Shelley/Ledger/Block.hs:216-217;
// N2N wrapping at .../Shelley/Node/Serialisation.hs:88-90):
//   header      = #6.24(bytes .cbor [header_body, kes_sig])            N2N v1
//   hfc_header  = [era, #6.24(bytes .cbor [header_body, kes_sig])]     Cardano N2N v2+
//   header_body = [blockNo, slot, prevHash, issuerVk, vrfVk, etaCert, leaderCert,
//                  bodySize, bodyHash, hotVk, counter, kesPeriod, sigma,
//                  protMajor, protMinor]
//   cert        = [output (64 B), proof (80 B)]
// The KES message is the raw header_body, so its span inside `raw` is
// recorded (body = raw, no copy).  Acceptance mirrors the Python slicer
// (header.py parse_header / pack) item for item; tests/test_pack.py pins the
// two against each other on the reference's golden headers and on every
// single-byte corruption and truncation of them.
#include <algorithm>
#include <cstring>
#include <thread>
#include <vector>

#include "../../include/ouro_verify.h"

namespace {

constexpr int kMaxDepth = 64;  // nesting guard for skip() on hostile input

struct Cur {
  const uint8_t* b;
  uint64_t n;  // bytes of this header
};

// (major type, argument, index after the head); false = truncated/reserved.
// arg = UINT64_MAX marks an indefinite length.
inline bool head(const Cur& c, uint64_t i, int* mt, uint64_t* arg, uint64_t* next) {
  if (i >= c.n) return false;
  const uint8_t ib = c.b[i];
  *mt = ib >> 5;
  const int ai = ib & 31;
  i++;
  if (ai < 24) {
    *arg = (uint64_t)ai;
  } else if (ai <= 27) {
    const int len = 1 << (ai - 24);
    if (c.n - i < (uint64_t)len) return false;
    uint64_t v = 0;
    for (int k = 0; k < len; k++) v = (v << 8) | c.b[i + k];
    *arg = v;
    i += len;
  } else if (ai == 31) {
    *arg = UINT64_MAX;
  } else {
    return false;  // 28..30 reserved
  }
  *next = i;
  return true;
}

// index just past the data item at i (header.py skip)
bool skip(const Cur& c, uint64_t i, uint64_t* out, int depth = 0) {
  if (depth > kMaxDepth) return false;
  int mt;
  uint64_t arg, j;
  if (!head(c, i, &mt, &arg, &j)) return false;
  switch (mt) {
    case 0: case 1: case 7:
      *out = j;
      return true;
    case 2: case 3:
      if (arg == UINT64_MAX) {
        while (true) {
          if (j >= c.n) return false;
          if (c.b[j] == 0xFF) break;
          if (!skip(c, j, &j, depth + 1)) return false;
        }
        *out = j + 1;
        return true;
      }
      if (c.n - j < arg) return false;
      *out = j + arg;
      return true;
    case 4: case 5: {
      if (arg == UINT64_MAX) {
        while (true) {
          if (j >= c.n) return false;
          if (c.b[j] == 0xFF) break;
          if (!skip(c, j, &j, depth + 1)) return false;
        }
        *out = j + 1;
        return true;
      }
      // each element takes at least one byte: a count beyond the input is truncated
      if (arg > c.n) return false;
      const uint64_t count = mt == 5 ? 2 * arg : arg;
      for (uint64_t k = 0; k < count; k++)
        if (!skip(c, j, &j, depth + 1)) return false;
      *out = j;
      return true;
    }
    default:  // 6: tag, then its content
      return skip(c, j, out, depth + 1);
  }
}

// spans of the elements of the definite array at i (at most `cap`)
bool array_items(const Cur& c, uint64_t i, uint64_t* starts, uint64_t* ends, int cap, int* count) {
  int mt;
  uint64_t arg, j;
  if (!head(c, i, &mt, &arg, &j) || mt != 4 || arg == UINT64_MAX) return false;
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

bool uint_at(const Cur& c, uint64_t i, uint64_t* v) {
  int mt;
  uint64_t arg, j;
  if (!head(c, i, &mt, &arg, &j) || mt != 0 || arg == UINT64_MAX) return false;
  *v = arg;
  return true;
}

// definite byte string of exactly `want` bytes at i
enum { kBytesOk = 0, kBytesShape = 1, kBytesSize = 2 };
int bytes_at(const Cur& c, uint64_t i, uint64_t want, const uint8_t** p) {
  int mt;
  uint64_t arg, j;
  if (!head(c, i, &mt, &arg, &j) || mt != 2 || arg == UINT64_MAX) return kBytesShape;
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
inline uint32_t kes_t_of(uint64_t slot, uint64_t spkp, uint64_t c0) {
  const uint64_t cur = slot / spkp;
  const uint64_t t = cur >= c0 ? cur - c0 : 0;
  return t > 0xffffffffull ? 0xffffffffu : (uint32_t)t;
}

uint8_t pack_one(const uint8_t* raw, uint64_t base, uint32_t len, uint64_t spkp, const Out& o,
                 size_t i) {
  const Cur c{raw + base, len};
  int mt;
  uint64_t arg, j, pos = 0, era = 1;
  if (!head(c, 0, &mt, &arg, &j)) return OURO_PACK_ECBOR;
  if (mt == 4 && arg == 2) {  // [era, wrapped]
    if (!uint_at(c, j, &era)) return OURO_PACK_ESHAPE;
    if (era == 0) return OURO_PACK_EBYRON;
    if (!skip(c, j, &pos)) return OURO_PACK_ECBOR;
  }
  if (!head(c, pos, &mt, &arg, &j)) return OURO_PACK_ECBOR;
  if (mt != 6 || arg != 24) return OURO_PACK_ESHAPE;
  uint64_t k;
  if (!head(c, j, &mt, &arg, &k)) return OURO_PACK_ECBOR;
  if (mt != 2) return OURO_PACK_ESHAPE;
  // [header_body, kes_sig]: the body's fields are walked once (the last
  // field's end is the body's end), then the signature
  uint64_t ts[2], te[2], fs[15], fe[15];
  int cnt;
  if (!head(c, k, &mt, &arg, &j)) return OURO_PACK_ECBOR;
  if (mt != 4 || arg == UINT64_MAX) return OURO_PACK_ECBOR;
  if (arg != 2) return OURO_PACK_ESHAPE;
  ts[0] = j;
  if (!array_items(c, ts[0], fs, fe, 15, &cnt)) return OURO_PACK_ECBOR;
  if (cnt != 15) return OURO_PACK_ESHAPE;
  te[0] = ts[1] = fe[14];
  if (!skip(c, ts[1], &te[1])) return OURO_PACK_ECBOR;
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
  memcpy(o.issuer_vk + 32 * i, ivk, 32);
  memcpy(o.vrf_vk + 32 * i, vvk, 32);
  memcpy(o.eta_output + 64 * i, eo, 64);
  memcpy(o.eta_proof + 80 * i, ep, 80);
  memcpy(o.leader_output + 64 * i, lo, 64);
  memcpy(o.leader_proof + 80 * i, lp, 80);
  memcpy(o.hot_vk + 32 * i, hvk, 32);
  memcpy(o.sigma + 64 * i, sg, 64);
  memcpy(o.kes_sig + 448 * i, ks, 448);
  o.counter[i] = counter;
  o.c0[i] = c0;
  o.kes_t[i] = kes_t_of(slot, spkp, c0);
  o.body_off[i] = base + ts[0];
  o.body_len[i] = (uint32_t)(te[0] - ts[0]);
  if (o.slot) o.slot[i] = slot;
  if (o.era) o.era[i] = (uint8_t)(era > 255 ? 255 : era);
  return OURO_PACK_OK;
}

void zero_row(const Out& o, size_t i) {
  memset(o.issuer_vk + 32 * i, 0, 32);
  memset(o.vrf_vk + 32 * i, 0, 32);
  memset(o.eta_output + 64 * i, 0, 64);
  memset(o.eta_proof + 80 * i, 0, 80);
  memset(o.leader_output + 64 * i, 0, 64);
  memset(o.leader_proof + 80 * i, 0, 80);
  memset(o.hot_vk + 32 * i, 0, 32);
  memset(o.sigma + 64 * i, 0, 64);
  memset(o.kes_sig + 448 * i, 0, 448);
  o.counter[i] = o.c0[i] = 0;
  o.kes_t[i] = 0;
  o.body_off[i] = 0;
  o.body_len[i] = 0;
  if (o.slot) o.slot[i] = 0;
  if (o.era) o.era[i] = 0;
}

// arena layout: one array per member, each 64-byte aligned
struct Layout {
  size_t off[14];
  size_t total;
};
constexpr size_t kRowBytes[14] = {32, 32, 80, 80, 32, 8, 8, 64, 4, 448, 8, 4, 64, 64};
Layout layout(size_t n) {
  Layout l{};
  size_t at = 0;
  for (int k = 0; k < 14; k++) {
    l.off[k] = at;
    at += (kRowBytes[k] * n + 63) & ~(size_t)63;
  }
  l.total = at;
  return l;
}

}  // namespace

extern "C" {

size_t ouro_tpraos_pack_bytes(size_t n) { return layout(n).total + 64; }

int ouro_tpraos_pack_cbor(const uint8_t* raw, size_t raw_bytes, const uint64_t* off,
                          const uint32_t* len, size_t n, uint64_t slots_per_kes_period,
                          void* arena, size_t arena_bytes, ouro_tpraos_batch* out,
                          uint64_t* slot, uint8_t* era, uint8_t* status, int nthreads) {
  if (!out || !status || slots_per_kes_period == 0) return OURO_EINVAL;
  if (n > 0 && (!raw || !off || !len || !arena)) return OURO_EINVAL;
  if (arena_bytes < ouro_tpraos_pack_bytes(n)) return OURO_EINVAL;
  for (size_t i = 0; i < n; i++)  // every span inside raw (checked without wrapping)
    if (off[i] > raw_bytes || raw_bytes - off[i] < len[i]) return OURO_EINVAL;
  uint8_t* a = static_cast<uint8_t*>(arena);
  a += (64 - (reinterpret_cast<uintptr_t>(a) & 63)) & 63;
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
  auto work = [&](size_t lo, size_t hi) {
    for (size_t i = lo; i < hi; i++) {
      const uint8_t st = pack_one(raw, off[i], len[i], slots_per_kes_period, o, i);
      status[i] = st;
      if (st != OURO_PACK_OK) zero_row(o, i);
    }
  };
  // at least 4096 headers per thread: below that a thread costs more than it saves
  size_t threads = nthreads > 0 ? (size_t)nthreads
                                : std::max<unsigned>(1, std::thread::hardware_concurrency());
  threads = std::max<size_t>(1, std::min(threads, (n + 4095) / 4096));
  threads = std::min<size_t>(threads, 64);
  if (threads <= 1) {
    work(0, n);
  } else {
    std::vector<std::thread> pool;
    const size_t per = (n + threads - 1) / threads;
    for (size_t t = 0; t < threads; t++) {
      const size_t lo = t * per, hi = std::min(n, lo + per);
      if (lo < hi) pool.emplace_back(work, lo, hi);
    }
    for (auto& th : pool) th.join();
  }
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
  return OURO_OK;
}

}  // extern "C"
