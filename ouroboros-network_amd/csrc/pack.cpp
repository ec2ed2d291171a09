// pack.cpp -- raw TPraos header CBOR -> the SoA of ouro_tpraos_batch
// (include/ouro_verify.h ouro_tpraos_pack_cbor), and
// raw Byron header CBOR -> ouro_byron_batch (row 4, ouro_byron_pack_cbor;
// the parse is csrc/cbor_byron.h).
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
#include <vector>

#include "../../include/ouro_verify.h"
#include "cbor.h"
#include "cbor_byron.h"
#include "task_pool.h"

namespace {

using namespace ouro::cbor;

// work(lo, hi) over [0, n) on up to `nthreads` threads (<= 0: one per CPU
// this process may run on) of the library's worker pool (task_pool.h), at
// least 4096 headers each: below that a thread costs more than it saves.
// The parse neither allocates nor throws, so the pool cannot fail it.
template <class F>
void parallel_rows(size_t n, int nthreads, F work) {
  size_t threads = nthreads > 0 ? (size_t)nthreads : (size_t)ouro_pool::usable_cpus();
  threads = std::max<size_t>(1, std::min(threads, (n + 4095) / 4096));
  threads = std::min<size_t>(threads, 64);
  if (threads <= 1) {
    work(0, n);
    return;
  }
  const size_t per = (n + threads - 1) / threads;
  ouro_pool::parallel_for(threads, (int)threads, [&](size_t t) {
    const size_t lo = t * per, hi = std::min(n, lo + per);
    if (lo < hi) work(lo, hi);
  });
}

size_t byron_msg_bytes(size_t n, const uint32_t* len) {
  size_t s = 0;
  for (size_t i = 0; i < n; i++) s += (size_t)len[i] + kByronMsgExtra;
  return s;
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
  const Out o = arena_out(arena_base(arena), n, slot, era);
  parallel_rows(n, nthreads, [&](size_t lo, size_t hi) {
    for (size_t i = lo; i < hi; i++) {
      const uint8_t st = pack_one(raw, off[i], len[i], slots_per_kes_period, o, i);
      status[i] = st;
      if (st != OURO_PACK_OK) zero_row(o, i);
    }
  });
  batch_from(out, o, raw, n);
  return OURO_OK;
}

size_t ouro_byron_pack_bytes(size_t n, const uint32_t* len) {
  if (n > 0 && !len) return 0;
  return byron_layout(n, byron_msg_bytes(n, len)).total + 64;
}

int ouro_byron_pack_cbor(const uint8_t* raw, size_t raw_bytes, const uint64_t* off,
                         const uint32_t* len, size_t n, int64_t protocol_magic, void* arena,
                         size_t arena_bytes, ouro_byron_batch* out, uint8_t* status,
                         int nthreads) {
  if (!out || !status) return OURO_EINVAL;
  if (protocol_magic < -1 || protocol_magic > (int64_t)kWord32Max) return OURO_EINVAL;
  if (n > 0 && (!raw || !off || !len || !arena)) return OURO_EINVAL;
  if (arena_bytes < ouro_byron_pack_bytes(n, len)) return OURO_EINVAL;
  for (size_t i = 0; i < n; i++)
    if (off[i] > raw_bytes || raw_bytes - off[i] < len[i]) return OURO_EINVAL;
  const ByronLayout l = byron_layout(n, byron_msg_bytes(n, len));
  const ByronOut o = byron_arena_out(arena_base(arena), l);
  uint64_t at = 0;  // message slots: len[i] + kByronMsgExtra bytes each, in order
  for (size_t i = 0; i < n; i++) {
    o.msg_off[i] = at;
    at += (uint64_t)len[i] + kByronMsgExtra;
  }
  parallel_rows(n, nthreads, [&](size_t lo, size_t hi) {
    for (size_t i = lo; i < hi; i++) {
      const uint8_t st = byron_pack_one(raw, off[i], len[i], protocol_magic, o, i);
      status[i] = st;
      if (st != OURO_PACK_OK) byron_zero_row(o, i);
    }
  });
  out->n = n;
  out->pk = o.pk;
  out->sig = o.sig;
  out->msg = o.msg;
  out->msg_off = o.msg_off;
  out->msg_len = o.msg_len;
  out->genesis_vk = o.genesis_vk;
  out->delegate_vk = o.delegate_vk;
  out->magic = o.magic;
  return OURO_OK;
}

}  // extern "C"
