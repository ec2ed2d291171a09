// host_path.hip -- the product's host (CPU) path (host_path.h): the kernels'
// own lane routines compiled for x86 (--offload-host-only), driven item by
// item over host buffers.  Each entry mirrors its kernel in kernels.hip line
// for line (k_ed25519_verify, k_vrf03_verify with its strict-s rule,
// k_sum6kes_verify, k_tpraos_verify, k_leader_check, k_vrf03_proof_to_hash),
// so a host verdict is the device verdict: tests/test_host_path.py pins both
// against the oracle on the same edge-case sets.
// its own host copies of the out-of-line lane routines (common.h)
#define OURO_NI_LINKAGE static

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <new>
#include <vector>

#include "host_fast.h"
#include "host_path.h"
#include "knobs.h"
#include "launch.h"
#include "leader.h"
#include "task_pool.h"
#include "tpraos.h"

using namespace ouro;

namespace {

// one lane's scratch slot (verify.h Slot, lane-major) plus a header record,
// 16-B aligned like a device slot
struct HostLane {
  std::vector<int32_t> buf;
  Slot s;
  HostLane() : buf((size_t)kHdrLaneWords + 4, 0) {
    s = Slot{reinterpret_cast<int32_t*>((reinterpret_cast<uintptr_t>(buf.data()) + 15) &
                                        ~uintptr_t(15))};
  }
};

// one per thread (the caller's, and each pool worker's), allocated on first use
HostLane& thread_lane() {
  thread_local HostLane lane;
  return lane;
}

// items [0, n) over threads_for(n) threads of the library's worker pool
// (task_pool.h: started once, never per batch), fn(i, lane); four tasks per
// thread so uneven items (KES bodies, rejected rows) balance.  A lane that
// cannot be allocated fails the batch with OURO_EDEVICE -- never an
// exception across the C ABI, never a verdict left unwritten as "valid".
template <class Fn>
int parallel_items(size_t n, Fn fn) {
  const int T = ouro_host::threads_for(n);
  const size_t ntasks = T <= 1 ? 1 : std::min<size_t>(n, (size_t)T * 4);
  const int r = ouro_pool::parallel_for(ntasks, T, [&](size_t k) {
    HostLane& l = thread_lane();
    const size_t lo = n * k / ntasks, hi = n * (k + 1) / ntasks;
    for (size_t i = lo; i < hi; i++) fn(i, l.s);
  });
  return r ? OURO_EDEVICE : OURO_OK;
}

}  // namespace

namespace ouro_cpu {

// B and 2^128 B from the encoding of B (y = 4/5, x even), their odd multiples
// [1, 3, .., 127] in affine niels form (x = X/Z, y = Y/Z: y + x, y - x, 2 d x y)
const BaseTables& base_tables() {
  static std::once_flag once;
  static BaseTables* t = nullptr;  // lives until exit
  std::call_once(once, [] {
    BaseTables* bt = new BaseTables;
    uint32_t enc[8];
    for (int i = 0; i < 8; i++) enc[i] = 0x66666666u;
    enc[0] = 0x66666658u;
    P3 B;
    decode(&B, enc, false);
    P3 B128 = B;
    for (int i = 0; i < 128; i++) B128 = to_p3(dbl3(B128));
    for (int which = 0; which < 2; which++) {
      const P3 base = which ? B128 : B;
      Niels* out = which ? bt->b128 : bt->b;
      const P3 twice = to_p3(dbl3(base));
      P3 acc = base;
      for (int k = 0; k < 64; k++) {
        if (k) acc = p3_add(acc, twice);
        const f51 zi = f_invert(acc.Z);
        const f51 x = f_mul(acc.X, zi), y = f_mul(acc.Y, zi);
        out[k] = Niels{f_carry(f_add(y, x)), f_sub(y, x), f_mul(f_mul(x, y), f_d2())};
      }
    }
    t = bt;
  });
  return *t;
}

}  // namespace ouro_cpu

namespace {
// OURO_HOST_IMPL=lanes: the kernels' lane routines compiled for the host (the
// round-4 host path) instead of ouro_cpu -- an A/B switch (bench.py single_item)
bool host_lanes() { return ouro_knobs::get().host_lanes.load(std::memory_order_relaxed) != 0; }
}  // namespace

namespace ouro_host {

const int32_t* btab() {
  static std::once_flag once;
  static std::vector<int32_t>* tab = nullptr;  // lives until exit (no teardown order issues)
  std::call_once(once, [] {
    tab = new std::vector<int32_t>(kBTabWords);
    build_btab(tab->data());
  });
  return tab->data();
}

int threads_for(size_t n) {
  const int cpus = ouro_pool::usable_cpus();
  int cap = 64;
  if (const int t = ouro_knobs::get().host_threads.load(std::memory_order_relaxed)) cap = std::max(1, t);
  const size_t by_items = (n + 15) / 16;
  return (int)std::max<size_t>(1, std::min<size_t>({(size_t)cpus, (size_t)cap, by_items}));
}

int ed_batch(size_t n, const uint8_t* pk, const uint8_t* sig, const uint8_t* msg,
             const uint64_t* off, const uint32_t* len, uint8_t* verdict, uint32_t byron) {
  const int32_t* bt = btab();
  const bool lanes = host_lanes();
  return parallel_items(n, [&](size_t i, Slot lane) {
    uint32_t s[16], p[8];
    ld_words(s, sig + 64 * i, 4);
    ld_words(p, pk + 32 * i, 2);
    const ShaGlobalTail m{msg + off[i]};
    const bool ok = lanes ? ed25519_verify_lane(s, p, m, len[i], lane, bt, byron != 0)
                          : ouro_cpu::ed25519_verify(s, p, m, len[i], byron != 0);
    verdict[i] = ok ? 1 : 0;
  });
}

int vrf_batch(size_t n, const uint8_t* pk, const uint8_t* proof, const uint8_t* alpha,
              const uint64_t* off, const uint32_t* len, uint8_t* beta, uint8_t* verdict,
              uint32_t flags) {
  const int32_t* bt = btab();
  const bool lanes = host_lanes();
  return parallel_items(n, [&](size_t i, Slot lane) {
    uint32_t p[8], pi[20], b[16];
    ld_words(p, pk + 32 * i, 2);
    ld_words(pi, proof + 80 * i, 5);
    const ShaGlobalTail a{alpha + off[i]};
    bool ok;
    if (lanes) {
      ok = vrf03_verify_lane(b, p, pi, a, len[i], lane, bt);
    } else {
      ouro_cpu::VrfKey key;
      ouro_cpu::vrf_key(key, p);
      ok = ouro_cpu::vrf03_verify(b, key, p, pi, a, len[i]);
    }
    if ((flags & OURO_VRF_STRICT_S) && !sc_is_canonical(pi + 12)) ok = false;  // App. B.3
    for (int k = 0; k < 16; k++) b[k] = ok ? b[k] : 0u;
    if (beta) st_words(beta + 64 * i, b, 4);
    verdict[i] = ok ? 1 : 0;
  });
}

int kes_batch(size_t n, const uint8_t* vk, const uint32_t* t, const uint8_t* msg,
              const uint64_t* off, const uint32_t* len, const uint8_t* sig, uint8_t* verdict) {
  const int32_t* bt = btab();
  const bool lanes = host_lanes();
  return parallel_items(n, [&](size_t i, Slot lane) {
    uint32_t v[8];
    ld_words(v, vk + 32 * i, 2);
    const uint32_t* sw = reinterpret_cast<const uint32_t*>(sig + 448 * i);
    const ShaGlobalTail m{msg + off[i]};
    const bool ok = lanes ? sum6kes_verify_lane(v, t[i], sw, m, len[i], lane, bt)
                          : ouro_cpu::sum6kes_verify(v, t[i], sw, m, len[i]);
    verdict[i] = ok ? 1 : 0;
  });
}

int hdr_batch(const ouro_tpraos_batch* b, uint8_t* verdict, uint8_t* beta_eta,
              uint8_t* beta_leader) {
  const int32_t* bt = btab();
  const size_t n = b->n;
  const uint32_t opts = batch_opts(*b);
  // the finish re-reads both outputs for the claimed-output bits / eta nonce
  std::unique_ptr<uint8_t[]> te, tl;
  if (!beta_eta) {
    te.reset(new (std::nothrow) uint8_t[64 * n]);
    if (!te) return OURO_EDEVICE;
    beta_eta = te.get();
  }
  if (!beta_leader) {
    tl.reset(new (std::nothrow) uint8_t[64 * n]);
    if (!tl) return OURO_EDEVICE;
    beta_leader = tl.get();
  }
  if (host_lanes())
    return parallel_items(n, [&](size_t i, Slot lane) {
      const Slot res = lane + kLaneWords;  // k_tpraos_verify's record
      for (int c = kCoreOcert; c <= kCoreVl; c++) hdr_core(*b, i, opts, c, lane, res, bt);
      hdr_finish_item(*b, i, opts, res, lane, verdict, beta_eta, beta_leader);
    });
  // the same verdict bits as hdr_finish_item: OCERT, KES, both VRFs (one key
  // decode), the s-range bits, then the claimed-output bits and the eta nonce
  return parallel_items(n, [&](size_t i, Slot) {
    uint32_t v = 0;
    {
      uint32_t s[16], p[8], hv[8];
      ld_words(s, b->ocert_sigma + 64 * i, 4);
      ld_words(p, b->issuer_vk + 32 * i, 2);
      ld_words(hv, b->hot_vk + 32 * i, 2);
      OcertMsg m;
      ocert_msg(m, hv, b->ocert_counter[i], b->ocert_kes_period[i]);
      if (ouro_cpu::ed25519_verify(s, p, m, 48, false)) v |= OURO_HDR_OCERT_OK;
      const uint32_t* sw = reinterpret_cast<const uint32_t*>(b->kes_sig + 448 * i);
      if (ouro_cpu::sum6kes_verify(hv, b->kes_t[i], sw, ShaGlobalTail{b->body + b->body_off[i]},
                                   b->body_len[i]))
        v |= OURO_HDR_KES_OK;
    }
    uint32_t pk[8], pie[20], pil[20], be[16], bl[16];
    ld_words(pk, b->vrf_vk + 32 * i, 2);
    ld_words(pie, b->eta_proof + 80 * i, 5);
    ld_words(pil, b->leader_proof + 80 * i, 5);
    ouro_cpu::VrfKey key;
    ouro_cpu::vrf_key(key, pk);
    for (int which = 0; which < 2; which++) {
      SeedMsg a;
      hdr_seed(a, *b, i, which != 0, opts);
      if (ouro_cpu::vrf03_verify(which ? bl : be, key, pk, which ? pil : pie, a, 32))
        v |= which ? OURO_HDR_VRF_LEADER_OK : OURO_HDR_VRF_ETA_OK;
    }
    v |= hdr_s_bits(pie, pil);
    st_words(beta_eta + 64 * i, be, 4);
    st_words(beta_leader + 64 * i, bl, 4);
    verdict[i] = (uint8_t)v;
    if (opts & kOptPost) hdr_post(*b, i, opts, verdict, beta_eta, beta_leader);
  });
}

int leader_batch(size_t n, const uint8_t* beta, const uint64_t* num, const uint64_t* den,
                 int64_t act_log_hi, uint64_t act_log_lo, int f_is_one, uint8_t* verdict) {
  return parallel_items(n, [&](size_t i, Slot) {
    const int32_t r = f_is_one ? kLeaderYes
                               : leader_check_lane(beta + 64 * i, num[i], den[i], act_log_lo,
                                                   act_log_hi);
    verdict[i] = r < 0 ? (uint8_t)0xff : (uint8_t)r;
  });
}

int proof_to_hash(uint8_t* out, const uint8_t* proof) {
  if (!host_lanes()) {
    uint32_t pi[20], beta[16];
    ld_words(pi, proof, 5);
    if (!ouro_cpu::vrf03_proof_to_hash(beta, pi)) return OURO_INVALID;
    st_words(out, beta, 4);
    return OURO_OK;
  }
  uint32_t G[8];
  ld_words(G, proof, 2);
  ge_p3 Gamma;
  bool ok = ge_is_canonical(G);
  ok = ge_decode(&Gamma, G, false) && ok;
  if (!ok) return OURO_INVALID;
  const ge_p3 G8 = ge_mul8(Gamma);
  uint32_t enc[8], beta[16];
  ge_encode_with_inv(enc, G8.X, G8.Y, fe_invert(G8.Z));
  vrf_beta(beta, enc);
  st_words(out, beta, 4);
  return OURO_OK;
}

}  // namespace ouro_host
