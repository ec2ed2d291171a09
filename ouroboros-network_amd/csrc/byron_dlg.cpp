// byron_dlg.cpp -- Byron heavyweight delegation certificates -> verdicts
// (BASELINE.json north star: "Ed25519 DSIGN verify (operational certificates
// and Byron delegation)"; include/ouro_verify.h ouro_byron_dlg_cert_*).
//
// A certificate (cardano-ledger-byron Cardano.Chain.Delegation.Certificate
// [ext]; the reference's PBftDelegationCert,
// ouroboros-consensus-byron/src/Ouroboros/Consensus/Byron/Protocol.hs:30, and
// the mempool's ByronDlg payload, .../Byron/Ledger/Mempool.hs:90) is
// (epoch, issuer XPub, delegate XPub, signature); the ledger checks the
// signature under the issuer's key with the SignCertificate tag.  The signed
// bytes, pinned on the reference's golden Byron header -- its block signature
// carries such a certificate, which verifies under exactly this message
// (tests/test_byron_cert.py) --:
//   0x0a || CBOR(protocol magic) || CBOR bytes("00" || delegate XPub || CBOR(epoch))
// i.e. the tag bytes of SignCertificate followed by the CBOR serialisation of
// the ByteString the certificate signs.  Acceptance is ByronDSIGN's
// (cardano-crypto's donna-derived verify, ouro_byron_ed25519_verify).
//
// Host code: the messages are built here and verified through the ByronDSIGN
// batch (device kernel; host path for single items and after a device error).
#include <algorithm>
#include <cstring>
#include <memory>
#include <new>

#include "../../include/ouro_verify.h"
#include "task_pool.h"

namespace {

// canonical CBOR unsigned integer (major type 0) at o; its length
size_t put_uint(uint8_t* o, uint64_t v, uint8_t major = 0) {
  const uint8_t mt = (uint8_t)(major << 5);
  if (v < 24) {
    o[0] = (uint8_t)(mt | v);
    return 1;
  }
  int w = v < (1ull << 8) ? 1 : v < (1ull << 16) ? 2 : v < (1ull << 32) ? 4 : 8;
  o[0] = (uint8_t)(mt | (w == 1 ? 24 : w == 2 ? 25 : w == 4 ? 26 : 27));
  for (int i = 0; i < w; i++) o[1 + i] = (uint8_t)(v >> (8 * (w - 1 - i)));
  return 1 + (size_t)w;
}

size_t uint_len(uint64_t v) {
  return v < 24 ? 1 : v < (1ull << 8) ? 2 : v < (1ull << 16) ? 3 : v < (1ull << 32) ? 5 : 9;
}

// the signed bytes of one certificate into o (at most OURO_BYRON_DLG_MSG_MAX)
size_t dlg_message(uint8_t* o, uint32_t magic, const uint8_t* delegate_xpub, uint64_t epoch) {
  uint8_t ep[9];
  const size_t eplen = put_uint(ep, epoch);
  size_t at = 0;
  o[at++] = 0x0a;                                         // SignCertificate
  at += put_uint(o + at, magic);                          // serialize' ProtocolMagicId
  at += put_uint(o + at, 2 + 64 + eplen, 2);              // CBOR bytes header
  o[at++] = '0';
  o[at++] = '0';
  memcpy(o + at, delegate_xpub, 64);
  at += 64;
  memcpy(o + at, ep, eplen);
  return at + eplen;
}

}  // namespace

extern "C" {

size_t ouro_byron_dlg_cert_message(uint8_t* out, uint32_t protocol_magic,
                                   const uint8_t* delegate_xpub, uint64_t epoch) {
  if (!out || !delegate_xpub) return 0;
  return dlg_message(out, protocol_magic, delegate_xpub, epoch);
}

int ouro_byron_dlg_cert_verify(uint32_t protocol_magic, const uint8_t* issuer_xpub,
                               const uint8_t* delegate_xpub, uint64_t epoch,
                               const uint8_t* sig) {
  if (!issuer_xpub || !delegate_xpub || !sig) return OURO_EINVAL;
  uint8_t m[OURO_BYRON_DLG_MSG_MAX];
  const size_t len = dlg_message(m, protocol_magic, delegate_xpub, epoch);
  return ouro_byron_ed25519_verify(m, len, issuer_xpub, sig);
}

int ouro_byron_dlg_cert_verify_batch(size_t n, uint32_t protocol_magic,
                                     const uint8_t* issuer_xpub, const uint8_t* delegate_xpub,
                                     const uint64_t* epoch, const uint8_t* sig,
                                     uint8_t* verdict) {
  if (n == 0) return OURO_OK;
  if (!issuer_xpub || !delegate_xpub || !epoch || !sig || !verdict) return OURO_EINVAL;
  if (n > ((size_t)1 << 31)) return OURO_EINVAL;
  std::unique_ptr<uint8_t[]> msg(new (std::nothrow) uint8_t[n * OURO_BYRON_DLG_MSG_MAX]);
  std::unique_ptr<uint8_t[]> pk(new (std::nothrow) uint8_t[n * 32]);
  std::unique_ptr<uint64_t[]> off(new (std::nothrow) uint64_t[n]);
  std::unique_ptr<uint32_t[]> len(new (std::nothrow) uint32_t[n]);
  if (!msg || !pk || !off || !len) return OURO_EDEVICE;  // out of host memory
  // offsets first (a message's length is fixed by the magic and its epoch's
  // CBOR size), then the messages and keys on the library's worker pool:
  // with one thread the first touch of ~100 MB of fresh pages would
  // dominate a 1M-certificate call
  const size_t fixed = 1 + uint_len(protocol_magic) + 2 + 2 + 64;
  uint64_t at = 0;
  for (size_t i = 0; i < n; i++) {
    off[i] = at;
    len[i] = (uint32_t)(fixed + uint_len(epoch[i]));
    at += len[i];
  }
  const size_t rows = 16384;
  const size_t tasks = (n + rows - 1) / rows;
  const int width = std::max(1, std::min(16, ouro_pool::usable_cpus()));
  const int rc = ouro_pool::parallel_for(tasks, width, [&](size_t t) {
    const size_t lo = t * rows, hi = std::min(n, lo + rows);
    for (size_t i = lo; i < hi; i++) {
      dlg_message(msg.get() + off[i], protocol_magic, delegate_xpub + 64 * i, epoch[i]);
      memcpy(pk.get() + 32 * i, issuer_xpub + 64 * i, 32);  // XPub[0:32]
    }
  });
  if (rc) return OURO_EDEVICE;
  return ouro_byron_ed25519_verify_batch(n, pk.get(), sig, msg.get(), off.get(), len.get(),
                                         verdict);
}

}  // extern "C"
