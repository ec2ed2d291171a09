// host_path.hip -- the product's host (CPU) path (host_path.h): the kernels'
// own lane routines compiled for x86 (--offload-host-only), driven item by
// item over host buffers.  Each entry mirrors its kernel in kernels.hip line
// for line (k_ed25519_verify, k_vrf03_verify with its strict-s rule,
// k_sum6kes_verify, k_tpraos_verify, k_leader_check, k_vrf03_proof_to_hash),
// so a host verdict is the device verdict: tests/test_host_path.py pins both
// against the oracle on the same edge-case sets.
#include <sched.h>

// its own host copies of the out-of-line lane routines (common.h)
#define OURO_NI_LINKAGE static

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "host_path.h"
#include "launch.h"
#include "leader.h"
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

HostLane& thread_lane() {
  thread_local HostLane lane;
  return lane;
}

// items [0, n) over threads_for(n) threads, fn(i, lane)
template <class Fn>
void parallel_items(size_t n, Fn fn) {
  const int T = ouro_host::threads_for(n);
  if (T <= 1) {
    HostLane& l = thread_lane();
    for (size_t i = 0; i < n; i++) fn(i, l.s);
    return;
  }
  std::vector<std::thread> th;
  th.reserve(T);
  for (int k = 0; k < T; k++) {
    th.emplace_back([&, k] {
      HostLane l;
      const size_t lo = n * k / T, hi = n * (k + 1) / T;
      for (size_t i = lo; i < hi; i++) fn(i, l.s);
    });
  }
  for (auto& t : th) t.join();
}

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
  int cpus = 1;
  cpu_set_t set;
  if (sched_getaffinity(0, sizeof(set), &set) == 0) cpus = std::max(1, CPU_COUNT(&set));
  int cap = 64;
  if (const char* e = getenv("OURO_HOST_THREADS")) cap = std::max(1, atoi(e));
  const size_t by_items = (n + 15) / 16;
  return (int)std::max<size_t>(1, std::min<size_t>({(size_t)cpus, (size_t)cap, by_items}));
}

int ed_batch(size_t n, const uint8_t* pk, const uint8_t* sig, const uint8_t* msg,
             const uint64_t* off, const uint32_t* len, uint8_t* verdict, uint32_t byron) {
  const int32_t* bt = btab();
  parallel_items(n, [&](size_t i, Slot lane) {
    uint32_t s[16], p[8];
    ld_words(s, sig + 64 * i, 4);
    ld_words(p, pk + 32 * i, 2);
    const bool ok = ed25519_verify_lane(s, p, ShaGlobalTail{msg + off[i]}, len[i], lane, bt,
                                        byron != 0);
    verdict[i] = ok ? 1 : 0;
  });
  return OURO_OK;
}

int vrf_batch(size_t n, const uint8_t* pk, const uint8_t* proof, const uint8_t* alpha,
              const uint64_t* off, const uint32_t* len, uint8_t* beta, uint8_t* verdict,
              uint32_t flags) {
  const int32_t* bt = btab();
  parallel_items(n, [&](size_t i, Slot lane) {
    uint32_t p[8], pi[20], b[16];
    ld_words(p, pk + 32 * i, 2);
    ld_words(pi, proof + 80 * i, 5);
    bool ok = vrf03_verify_lane(b, p, pi, ShaGlobalTail{alpha + off[i]}, len[i], lane, bt);
    if ((flags & OURO_VRF_STRICT_S) && !sc_is_canonical(pi + 12)) ok = false;  // App. B.3
    for (int k = 0; k < 16; k++) b[k] = ok ? b[k] : 0u;
    if (beta) st_words(beta + 64 * i, b, 4);
    verdict[i] = ok ? 1 : 0;
  });
  return OURO_OK;
}

int kes_batch(size_t n, const uint8_t* vk, const uint32_t* t, const uint8_t* msg,
              const uint64_t* off, const uint32_t* len, const uint8_t* sig, uint8_t* verdict) {
  const int32_t* bt = btab();
  parallel_items(n, [&](size_t i, Slot lane) {
    uint32_t v[8];
    ld_words(v, vk + 32 * i, 2);
    const uint32_t* sw = reinterpret_cast<const uint32_t*>(sig + 448 * i);
    const bool ok = sum6kes_verify_lane(v, t[i], sw, ShaGlobalTail{msg + off[i]}, len[i], lane, bt);
    verdict[i] = ok ? 1 : 0;
  });
  return OURO_OK;
}

int hdr_batch(const ouro_tpraos_batch* b, uint8_t* verdict, uint8_t* beta_eta,
              uint8_t* beta_leader) {
  const int32_t* bt = btab();
  const size_t n = b->n;
  const uint32_t opts = batch_opts(*b);
  // the finish re-reads both outputs for the claimed-output bits / eta nonce
  std::vector<uint8_t> te, tl;
  if (!beta_eta) {
    te.resize(64 * n);
    beta_eta = te.data();
  }
  if (!beta_leader) {
    tl.resize(64 * n);
    beta_leader = tl.data();
  }
  parallel_items(n, [&](size_t i, Slot lane) {
    const Slot res = lane + kLaneWords;  // k_tpraos_verify's record
    for (int c = kCoreOcert; c <= kCoreVl; c++) hdr_core(*b, i, opts, c, lane, res, bt);
    hdr_finish_item(*b, i, opts, res, lane, verdict, beta_eta, beta_leader);
  });
  return OURO_OK;
}

int leader_batch(size_t n, const uint8_t* beta, const uint64_t* num, const uint64_t* den,
                 int64_t act_log_hi, uint64_t act_log_lo, int f_is_one, uint8_t* verdict) {
  parallel_items(n, [&](size_t i, Slot) {
    const int32_t r = f_is_one ? kLeaderYes
                               : leader_check_lane(beta + 64 * i, num[i], den[i], act_log_lo,
                                                   act_log_hi);
    verdict[i] = r < 0 ? (uint8_t)0xff : (uint8_t)r;
  });
  return OURO_OK;
}

int proof_to_hash(uint8_t* out, const uint8_t* proof) {
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
