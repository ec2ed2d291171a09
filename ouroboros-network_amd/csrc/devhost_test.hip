// devhost_test.hip -- TEST-ONLY host build of the kernels' lane routines.
//
// hipcc compiles the __host__ __device__ bodies in verify.h for x86 too; this
// library exports them so tests/test_devcode_host.py can check the exact
// arithmetic the gfx950 kernels run against the oracle and libsodium in a
// container with no GPU.  It is never linked into, or loaded by, the product
// library (lib/libouro_verify.so) and launches nothing.
#include <cstdlib>
#include <algorithm>
#include <cstring>
#include <vector>

#include "leader.h"
#include "tpraos.h"

using namespace ouro;

#if defined(OURO_COUNT_OPS)
thread_local unsigned long long g_ouro_nmul = 0, g_ouro_nsq = 0, g_ouro_bound_violations = 0;

// bound tracker hooks (fe25519.h): shadow bounds of elements stored in memory
#include <array>
#include <unordered_map>
namespace {
thread_local std::unordered_map<const void*, std::array<uint64_t, 10>> g_shadow;
thread_local unsigned long long g_untracked_loads = 0;
}
void ouro_trk_violation() {
  ++g_ouro_bound_violations;
  static const bool do_abort = getenv("OURO_TRK_ABORT") != nullptr;
  if (do_abort) abort();
}
void ouro_trk_store(const void* p, const uint64_t b[10]) {
  std::array<uint64_t, 10> a;
  for (int i = 0; i < 10; i++) a[i] = b[i];
  g_shadow[p] = a;
}
void ouro_trk_load(const void* p, uint64_t b[10]) {
  auto it = g_shadow.find(p);
  if (it == g_shadow.end()) {
    // never stored through st_fe/st_cached: only possible for memory the
    // tracker did not see being written -- assume the worst 32-bit value
    ++g_untracked_loads;
    for (int i = 0; i < 10; i++) b[i] = 0xffffffffu;
    return;
  }
  for (int i = 0; i < 10; i++) b[i] = it->second[i];
}
#endif

namespace {
const int32_t* host_btab() {
  static std::vector<int32_t> tab = [] {
    std::vector<int32_t> t(kBTabWords);
    build_btab(t.data());
    return t;
  }();
  return tab.data();
}
// one slot (column 0) of a kSlotGroup-slot region, laid out as on the device
struct SlotRegion {
  std::vector<int32_t> buf;
  Slot s;
  explicit SlotRegion(int slot_words) : buf(slot_region_words(1, slot_words) + 4, 0) {
    s = Slot{reinterpret_cast<int32_t*>((reinterpret_cast<uintptr_t>(buf.data()) + 15) & ~uintptr_t(15))};
  }
};
struct Lane : SlotRegion {
  Lane() : SlotRegion(kLaneWords) {}
};
fe fe_from_bytes(const uint8_t* b) {
  uint32_t w[8];
  bytes_to_words8(w, b);
  return fe_from_words(w);
}
void fe_to_bytes(uint8_t* out, const fe& f) {
  uint32_t w[8];
  fe_to_words(w, f);
  memcpy(out, w, 32);
}
}  // namespace

extern "C" {

// field-operation counters (valid when built with -DOURO_COUNT_OPS)
void dh_count_reset(void) {
#if defined(OURO_COUNT_OPS)
  g_ouro_nmul = g_ouro_nsq = 0;
#endif
}
unsigned long long dh_bound_violations(void) {
#if defined(OURO_COUNT_OPS)
  return g_ouro_bound_violations;
#else
  return ~0ull;
#endif
}
void dh_count_get(unsigned long long* nmul, unsigned long long* nsq) {
#if defined(OURO_COUNT_OPS)
  *nmul = g_ouro_nmul;
  *nsq = g_ouro_nsq;
#else
  *nmul = *nsq = 0;
#endif
}

// field ops on canonical 32-byte encodings
void dh_fe_mul(uint8_t* out, const uint8_t* a, const uint8_t* b) {
  fe_to_bytes(out, fe_mul(fe_from_bytes(a), fe_from_bytes(b)));
}
void dh_fe_sq(uint8_t* out, const uint8_t* a) { fe_to_bytes(out, fe_sq(fe_from_bytes(a))); }
void dh_fe_sub(uint8_t* out, const uint8_t* a, const uint8_t* b) {
  fe_to_bytes(out, fe_sub(fe_from_bytes(a), fe_from_bytes(b)));
}
void dh_fe_invert(uint8_t* out, const uint8_t* a) {
  fe_to_bytes(out, fe_invert(fe_from_bytes(a)));
}
void dh_fe_invert_vartime(uint8_t* out, const uint8_t* a) {
  fe_to_bytes(out, fe_invert_vartime(fe_from_bytes(a)));
}
// the same with at most 10 bits cancelled per divstep step (the latency
// mode's wave inversion, wide_inv.h OURO_INV_CAP)
void dh_fe_invert_vartime_cap10(uint8_t* out, const uint8_t* a) {
  fe_to_bytes(out, fe_invert_vartime<10>(fe_from_bytes(a)));
}
void dh_fe_invert_vartime_sel(uint8_t* out, const uint8_t* a) {
  fe_to_bytes(out, fe_invert_vartime<10, true>(fe_from_bytes(a)));
}
void dh_fe_invert_vartime_spec(uint8_t* out, const uint8_t* a) {
  fe_to_bytes(out, fe_invert_vartime<30, true, true>(fe_from_bytes(a)));
}
// the same from raw limbs (< 2^31 each: unreduced representations)
void dh_fe_invert_vartime_limbs(uint8_t* out, const uint32_t* limbs) {
  fe f = fe_make(limbs[0], limbs[1], limbs[2], limbs[3], limbs[4], limbs[5], limbs[6], limbs[7],
                 limbs[8], limbs[9]);
  fe_to_bytes(out, fe_invert_vartime(f));
}
// raw-limb round trip: limbs given as 10 uint32 (< 2^31), canonical encoding out
void dh_fe_limbs_tobytes(uint8_t* out, const uint32_t* limbs) {
  fe f = fe_make(limbs[0], limbs[1], limbs[2], limbs[3], limbs[4], limbs[5], limbs[6], limbs[7],
                 limbs[8], limbs[9]);
  fe_to_bytes(out, f);
}
// a per-lane table coordinate's 256-bit packing (verify.h fe_pack256, limbs
// < 2^28 in) and the limbs its unpacking yields
void dh_fe_pack256(uint32_t* words8, uint32_t* limbs_out, const uint32_t* limbs) {
  fe f = fe_make(limbs[0], limbs[1], limbs[2], limbs[3], limbs[4], limbs[5], limbs[6], limbs[7],
                 limbs[8], limbs[9]);
  fe_pack256(words8, f);
  const fe g = fe_unpack256(words8);
  for (int i = 0; i < 10; i++) limbs_out[i] = g.v[i];
}
unsigned long long dh_untracked_loads(void) {
#if defined(OURO_COUNT_OPS)
  return g_untracked_loads;
#else
  return 0;
#endif
}
void dh_sc_reduce64(uint8_t* out, const uint8_t* in64) {
  uint32_t w[16], r[8];
  for (int i = 0; i < 16; i++) w[i] = ld_le32(in64 + 4 * i);
  sc_reduce512(r, w);
  memcpy(out, r, 32);
}
void dh_sha512_prefixed64(uint8_t* out, const uint8_t* prefix64, const uint8_t* msg,
                          uint32_t mlen) {
  uint32_t pre[16];
  for (int i = 0; i < 16; i++) pre[i] = ld_le32(prefix64 + 4 * i);
  uint64_t H[8];
  sha512_prefixed<64>(H, pre, ShaGlobalTail{msg}, mlen);
  uint32_t w[16];
  sha512_digest_words(w, H);
  memcpy(out, w, 64);
}
void dh_blake2b256_64(uint8_t* out, const uint8_t* in64) {
  uint32_t w[16], h[8];
  for (int i = 0; i < 16; i++) w[i] = ld_le32(in64 + 4 * i);
  blake2b256_64(h, w);
  memcpy(out, h, 32);
}
void dh_elligator2(uint8_t* out, const uint8_t* r32) {
  uint32_t r[8];
  bytes_to_words8(r, r32);
  r[7] &= 0x7fffffffu;
  ge_p3 H = elligator2_h(r);
  uint32_t enc[8];
  ge_encode_with_inv(enc, H.X, H.Y, fe_invert(H.Z));
  memcpy(out, enc, 32);
}
void dh_elligator2_ref(uint8_t* out, const uint8_t* r32) {
  uint32_t r[8];
  bytes_to_words8(r, r32);
  r[7] &= 0x7fffffffu;
  ge_p3 H = elligator2_h_ref(r);
  uint32_t enc[8];
  ge_encode_with_inv(enc, H.X, H.Y, fe_invert(H.Z));
  memcpy(out, enc, 32);
}
// leader.h: 1 leader, 0 not, -1 outside the supported domain
int dh_leader_check(const uint8_t* beta64, uint64_t num, uint64_t den, uint64_t act_log_lo,
                    int64_t act_log_hi) {
  return leader_check_lane(beta64, num, den, act_log_lo, act_log_hi);
}
// lattice.h: (|c0|, c1, sign of c0) for h (32 bytes, < 2^253); returns the bit size
int dh_half_scalars(const uint8_t* h32, uint8_t* c0, uint8_t* c1, int* c0_neg) {
  uint32_t h[8];
  bytes_to_words8(h, h32);
  HalfScalars hs;
  ed25519_half_scalars(hs, h);
  memcpy(c0, hs.c0, 32);
  memcpy(c1, hs.c1, 32);
  *c0_neg = hs.c0_neg ? 1 : 0;
  return hs.bits;
}
// the round-1 reduction (lattice.h ed25519_half_scalars_v1), for the
// equivalence test of the round-6 step
int dh_half_scalars_v1(const uint8_t* h32, uint8_t* c0, uint8_t* c1, int* c0_neg) {
  uint32_t h[8];
  bytes_to_words8(h, h32);
  HalfScalars hs;
  ed25519_half_scalars_v1(hs, h);
  memcpy(c0, hs.c0, 32);
  memcpy(c1, hs.c1, 32);
  *c0_neg = hs.c0_neg ? 1 : 0;
  return hs.bits;
}
int dh_ed25519_verify(const uint8_t* sig, const uint8_t* m, uint32_t mlen, const uint8_t* pk) {
  uint32_t s[16], p[8];
  for (int i = 0; i < 16; i++) s[i] = ld_le32(sig + 4 * i);
  bytes_to_words8(p, pk);
  Lane lane;
  return ed25519_verify_lane(s, p, ShaGlobalTail{m}, mlen, lane.s, host_btab()) ? 0 : -1;
}
int dh_vrf03_verify(uint8_t* beta, const uint8_t* pk, const uint8_t* proof, const uint8_t* alpha,
                    uint32_t alen) {
  uint32_t p[8], pi[20], b[16];
  bytes_to_words8(p, pk);
  for (int i = 0; i < 20; i++) pi[i] = ld_le32(proof + 4 * i);
  Lane lane;
  bool ok = vrf03_verify_lane(b, p, pi, ShaGlobalTail{alpha}, alen, lane.s, host_btab());
  memcpy(beta, b, 64);
  return ok ? 0 : -1;
}
int dh_sum6kes_verify(const uint8_t* vk, uint32_t t, const uint8_t* m, uint32_t mlen,
                      const uint8_t* sig) {
  uint32_t v[8];
  bytes_to_words8(v, vk);
  alignas(16) uint32_t sw[112];
  memcpy(sw, sig, 448);
  Lane lane;
  return sum6kes_verify_lane(v, t, sw, ShaGlobalTail{m}, mlen, lane.s, host_btab()) ? 0 : -1;
}
// mkSeed through the header kernels' own path (tpraos.h hdr_seed: blake2b.h
// mkseed_hash and the seedEta / seedL constants); eta0 = NULL: NeutralNonce.
void dh_mk_seed(uint8_t* out, int leader, uint64_t slot, const uint8_t* eta0) {
  alignas(16) uint8_t e0[32];
  if (eta0) memcpy(e0, eta0, 32);
  ouro_tpraos_batch b{};
  b.n = 1;
  b.slot = &slot;
  b.epoch_nonce = eta0 ? e0 : nullptr;
  SeedMsg a;
  hdr_seed(a, b, 0, leader != 0, batch_opts(b));
  memcpy(out, a.w, 32);
}
// The header drivers of tpraos.h for every header of a host SoA batch.
// mode 0 = throughput (one lane, key table shared), 1 = latency (a fresh lane
// per core, no sharing), 2 = latency on lane quads (the four products of each
// group operation emulated in sequence, with the merged operand bounds; the
// finish VRF by VRF as the lane pairs run it).  Pointers must be 16-B aligned like device buffers.
int dh_tpraos_verify(const ouro_tpraos_batch* b, int mode, uint8_t* verdict, uint8_t* beta_eta,
                     uint8_t* beta_leader) {
  std::vector<Lane> lanes(kLatCores);
  SlotRegion rr(kLatResWords);
  const Slot r = rr.s;
  const uint32_t opts = batch_opts(*b);
  for (size_t i = 0; i < b->n; i++) {
    std::fill(rr.buf.begin(), rr.buf.end(), 0);
    if (mode == 3) {
      // the split header kernel's phases (k_hdr_pre / k_hdr_dsm / k_hdr_post):
      // each core in its own task slot, the dsm from the cfg word the pre
      // phase left there
      for (int core = 0; core < kHdrCores; core++)
        hdr_core(*b, i, opts, core, lanes[core].s, r, host_btab(), true, false, false, kPhasePre,
                 lanes[kCoreUe].s);
      for (int core = 0; core < kHdrCores; core++)
        dsm_lane(lanes[core].s, host_btab(), (uint32_t)*lanes[core].s.word(kSlotCfg));
      for (int core = 0; core < kHdrCores; core++)
        hdr_core(*b, i, opts, core, lanes[core].s, r, nullptr, true, false, false, kPhasePost);
      hdr_finish_item(*b, i, opts, r, lanes[0].s, verdict, beta_eta, beta_leader);
      continue;
    }
    const int cores = mode ? kLatCores : kHdrCores;
    for (int core = 0; core < cores; core++)
      hdr_core(*b, i, opts, core, lanes[mode ? core : 0].s, r, host_btab(), mode == 0, mode != 0,
               mode == 2);
    if (mode == 2) {
      hdr_finish_item_split(*b, i, opts, r, verdict, beta_eta, beta_leader);
      continue;
    }
    if (mode) hdr_combine_split(r);
    hdr_finish_item(*b, i, opts, r, lanes[0].s, verdict, beta_eta, beta_leader);
  }
  return 0;
}
}
