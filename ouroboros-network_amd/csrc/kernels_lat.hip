// kernels_lat.hip -- the latency-mode kernels (configs[4] ChainSync windows):
// eight cores per header, each on one wave (wide_cores.h) or on a DPP lane
// quad, then the lane-pair finish.
//
// A translation unit of its own so that its lane routines use the row-order
// field products (OURO_FE_SCAN=0): a lane quad issues one product per lane,
// and the column-scan form's dependent multiply-add chains, which the
// throughput kernel's two resident waves hide, would stall the few waves of a
// small window (A/B in one process: p50 0.5875 -> 0.5712 ms,
// profiles/r02d/ablat_rows_scan.json).  Its copies of the lane routines live in
// namespace ouro_lat, so no symbol is shared with kernels.hip's.
#ifndef OURO_FE_SCAN
#define OURO_FE_SCAN 0
#endif
#define ouro ouro_lat
#include <hip/hip_runtime.h>

#include "../../include/ouro_verify.h"
#include "launch.h"

#include "wide_cores.h"
#include "wide_blake2b.h"

// A/B switch: 1 = the V core computes the whole V = [s]H - [c]Gamma (Gamma
// decoded on its other rows); 0 = -[c]Gamma on the Gamma core and the second
// of the two to arrive combines (the default: the V core is the critical item)
#ifndef OURO_V_WHOLE
#define OURO_V_WHOLE 0
#endif
// A/B switch: 1 = the fused launch's split form (hdr_item_fused: three waves
// per Ed25519 check, V over V / V2 / Gamma), 0 = the two-wave form
#ifndef OURO_LAT_SPLIT
#define OURO_LAT_SPLIT 1
#endif
// waves per SIMD the cores kernel is compiled for: a window's 640 waves never
// put two on one SIMD, so 1 gives each wave the whole register file (AGPRs
// instead of scratch for the wide items' spills); 2 = the round-2 form
#ifndef OURO_LAT_WAVES
#define OURO_LAT_WAVES 2
#endif

using namespace ouro;

// mkSeed's Blake2b on the lane quads (wide_blake2b.h, 1) or on one lane
// (tpraos.h hdr_seed, 0) in the V / V2 items (node configuration)
#ifndef OURO_SEED_QUAD
#define OURO_SEED_QUAD 1
#endif
__device__ __forceinline__ void lat_seed(SeedMsg& a, const ouro_tpraos_batch& b, size_t i,
                                         bool leader, uint32_t opts) {
  if (OURO_SEED_QUAD) hdr_seed_wave(a, b, i, leader, opts);
  else hdr_seed(a, b, i, leader, opts);
}


// One core of header i on one wave (wide_cores.h): the same checks and the
// same record fields (lane 0 stores) as hdr_core with split V on a lane or
// quad.  bw: the wide B tables (after the niels ones in btab).
// fused: U, V and Gamma cores store encodings and beta instead of points
// (the whole V on the V core; hdr_tail_wide finishes), for the fused launch.
__device__ __noinline__ void hdr_core_wide(const ouro_tpraos_batch& b, size_t i, uint32_t opts,
                                           int core, Slot res, const uint16_t* bw, bool fused) {
#if defined(__HIP_DEVICE_COMPILE__)  // wave-collective code (wide.h) is device-only
  using namespace wide;
  const bool lead = (threadIdx.x & 63u) == 0;
  const bool leader = core == kCoreUl || core == kCoreVl || core == kCoreGl;
  int32_t flag = 0;
  switch (core) {
    case kCoreOcert: {
      uint32_t s[16], p[8], hv[8];
      ld_words(s, b.ocert_sigma + 64 * i, 4);
      ld_words(p, b.issuer_vk + 32 * i, 2);
      ld_words(hv, b.hot_vk + 32 * i, 2);
      OcertMsg m;
      ocert_msg(m, hv, b.ocert_counter[i], b.ocert_kes_period[i]);
      flag = ed25519_verify_wide(s, p, m, 48, bw) ? kFlagOk : 0;
      break;
    }
    case kCoreKes: {
      uint32_t hv[8];
      ld_words(hv, b.hot_vk + 32 * i, 2);
      const uint32_t* sw = reinterpret_cast<const uint32_t*>(b.kes_sig + 448 * i);
      flag = sum6kes_verify_wide(hv, b.kes_t[i], sw, ShaGlobalTail{b.body + b.body_off[i]},
                                 b.body_len[i], bw) ? kFlagOk : 0;
      break;
    }
    case kCoreUe:
    case kCoreUl: {
      uint32_t p[8], pi[20];
      ld_words(p, b.vrf_vk + 32 * i, 2);
      ld_words(pi, (leader ? b.leader_proof : b.eta_proof) + 80 * i, 5);
      if (fused && OURO_LAT_SPLIT) {  // the encoding on the wave (wide_cores.h encode1_wide)
        pw Uw;
        flag = vrf_u_wide_pw(Uw, p, pi, bw) ? kFlagOk : 0;
        uint32_t enc[8];
        encode1_wide(enc, Uw);
        if (lead) st_words8(res + kLatEnc + 8 * (3 * (int)leader + 1), enc);
        break;
      }
      ge_p2 U;
      flag = vrf_u_wide(U, p, pi, bw) ? kFlagOk : 0;
      if (fused) {
        uint32_t enc[8];
        encode_p2(enc, U);
        if (lead) st_words8(res + kLatEnc + 8 * (3 * (int)leader + 1), enc);
      } else if (lead) {
        st_point(res, leader ? kPtUl : kPtUe, U.X, U.Y, U.Z);
      }
      break;
    }
    case kCoreVe:
    case kCoreVl: {
      uint32_t p[8], pi[20];
      ld_words(p, b.vrf_vk + 32 * i, 2);
      ld_words(pi, (leader ? b.leader_proof : b.eta_proof) + 80 * i, 5);
      SeedMsg alpha;
      lat_seed(alpha, b, i, leader, opts);
      if (fused && OURO_V_WHOLE) {
        uint32_t Henc[8], Venc[8];
        vrf_v_full_wide(Henc, Venc, p, pi, alpha);
        if (lead) {
          st_words8(res + kLatEnc + 8 * (3 * (int)leader + 0), Henc);
          st_words8(res + kLatEnc + 8 * (3 * (int)leader + 2), Venc);
        }
        flag = kFlagOk;
        break;
      }
      if (fused && OURO_LAT_SPLIT) {  // [s windows 0..31]H; V2 and Gamma do the rest
        vrf_sh_split(res + kLatVsplit + 4 * kPwWords * (int)leader, res, p, pi, alpha, 0);
        flag = kFlagOk;
        break;
      }
      // (fused, split V: H and [s]H to the record; vrf_combine_encode adds
      // the Gamma core's -[c]Gamma)
      ge_p3 H;
      ge_p2 V;
      vrf_sh(H, V, p, pi, alpha);
      if (lead) {
        st_point(res, leader ? kPtHl : kPtHe, H.X, H.Y, H.Z);
        st_point(res, leader ? kPtVl : kPtVe, V.X, V.Y, V.Z);
      }
      flag = kFlagOk;
      break;
    }
    default: {  // kCoreGe / kCoreGl
      uint32_t pi[20];
      ld_words(pi, (leader ? b.leader_proof : b.eta_proof) + 80 * i, 5);
      if (fused) {
        uint32_t beta[16];
        ge_p2 part;
        const Slot vs = res + kLatVsplit + 4 * kPwWords * (int)leader + 3 * kPwWords;
        flag = vrf_gamma_beta_wide(beta, part, pi, OURO_LAT_SPLIT ? &vs : nullptr);
        if (lead) {
          st_words8(res + kLatBeta + 16 * (int)leader, beta);
          st_words8(res + kLatBeta + 16 * (int)leader + 8, beta + 8);
          if (!OURO_V_WHOLE && !OURO_LAT_SPLIT)
            st_point_at(res + kLatPart + (leader ? kPtWords : 0), part.X, part.Y, part.Z);
        }
        if (!leader && (opts & kOptEtaNonce)) eta_nonce_candidates(b, i, opts, res, beta);
        break;
      }
      ge_p2 part;
      ge_p3 G8;
      flag = vrf_gamma_wide(part, G8, pi);
      if (lead) {
        st_point_at(res + kLatPart + (leader ? kPtWords : 0), part.X, part.Y, part.Z);
        st_point(res, leader ? kPtG8l : kPtG8e, G8.X, G8.Y, G8.Z);
      }
      break;
    }
  }
  if (lead) stg1(res.word(kResFlags + core), flag);
#endif
}

// Fused mode, two-wave form (OURO_LAT_SPLIT=0): ten items per header -- the
// eight cores, with the OCERT and KES Ed25519 checks each split into a points
// item (0 / 1) and a scalars item (8 / 9) whose second to arrive runs the
// chain (wide_cores.h ed_*).  Every finished core arrives at the header's
// counter; the eighth runs the finish (hdr_tail_wide).
// Split form (OURO_LAT_SPLIT=1, the default): fourteen items -- each Ed25519
// check over three waves with no lattice pair (points 0 / 1, scalars 8 / 9,
// doubling 10 / 11: wide_cores.h eds_*), each V over the V core (4 / 5, low
// windows of s), a V2 item (12 / 13: H again, 2^128 H, high windows) and the
// Gamma core (6 / 7); the last of a check's chains or of a VRF's three parts
// finishes that check, and eight arrivals (two Ed25519 checks, two U, two VRF
// combinations, two Gamma betas) complete a header.  skip: the timing probe's mask (cores
// 0..7; the doubling and V2 items follow their cores).
static_assert(!(OURO_V_WHOLE && OURO_LAT_SPLIT), "OURO_V_WHOLE needs the two-wave form");
constexpr int kFusedItems = OURO_LAT_SPLIT ? kLatCores + 6 + (OURO_LAT_V3 ? 2 : 0) : kLatCores + 2;
[[maybe_unused]] constexpr uint32_t kHdrParties = OURO_LAT_SPLIT ? 8u : (uint32_t)kLatCores;
// stamps (a timing probe, tools/lat_stamps.py: a build with
// -DOURO_LAT_STAMPS=1, run with OURO_LAT_STAMPS set): header 0's items print
// their start / end times (s_memrealtime, 100 MHz) and the tail's end.  The
// product build has no printf.
#ifndef OURO_LAT_STAMPS
#define OURO_LAT_STAMPS 0
#endif
// true when this wave ran the header's tail (its outputs are written)
__device__ __noinline__ bool hdr_item_fused(const ouro_tpraos_batch& b, size_t i, uint32_t opts,
                                            int item, Slot res, const uint16_t* bw, uint32_t skip,
                                            uint32_t gen,
                                            uint8_t* verdict, uint8_t* beta_eta,
                                            uint8_t* beta_leader, bool stamps) {
#if defined(__HIP_DEVICE_COMPILE__)
  using namespace wide;
  const bool lead = (threadIdx.x & 63u) == 0;
  (void)stamps;
  lstamp(0);
  // probe tags (wide_cores.h lstamp): 1 own part done, 2 / 3 chain X / Y done,
  // 4..7 a VRF combination (start, adds, inverted, encoded), 8 the item's end,
  // 9 / 10 / 11 the tail (start, challenges, end); V / V2 phases 12..18
  auto stamp = [&](const char* what) {
    const char c = what[0], c1 = what[1], c2 = what[2];
    lstamp(c == 'w' ? 1 : c == 'c' && c1 == 'h' && c2 == 'x' ? 2 : c == 'c' && c1 == 'h' ? 3
           : c == 't' ? 11 : c == 'c' && c1 == 'o' && c2 == 'm' ? 7 : 8);
  };
  const bool ed_item = item == kCoreOcert || item == kCoreKes ||
                       (item >= kLatCores && item < kLatCores + (OURO_LAT_SPLIT ? 4 : 2));
  if (ed_item && OURO_LAT_SPLIT) {
    // e: 0 OCERT, 1 KES; role: 0 points, 1 scalars, 2 doubling
    const int e = item < kLatCores ? item : (item - kLatCores) & 1;
    const int role = item < kLatCores ? 0 : (item < kLatCores + 2 ? 1 : 2);
    const Slot ed = res + kLatEd + kEdWords * e;
    const bool skipped = (skip >> e) & 1u;
    bool run_x = false, run_y = false;
    if (!skipped) {
      uint32_t sig[16], pk[8];
      bool walk_ok = true;
      if (e == 0) {
        ld_words(sig, b.ocert_sigma + 64 * i, 4);
        ld_words(pk, b.issuer_vk + 32 * i, 2);
      } else {
        uint32_t hv[8];
        ld_words(hv, b.hot_vk + 32 * i, 2);
        const uint32_t* sw = reinterpret_cast<const uint32_t*>(b.kes_sig + 448 * i);
        walk_ok = sum6kes_walk_wide(pk, sig, hv, b.kes_t[i], sw);
      }
      if (role == 0) {
        eds_points(ed, sig, pk, walk_ok);
      } else if (role == 2) {
        eds_double(ed, pk);
      } else if (e == 0) {
        uint32_t hv[8];
        ld_words(hv, b.hot_vk + 32 * i, 2);
        OcertMsg m;
        ocert_msg(m, hv, b.ocert_counter[i], b.ocert_kes_period[i]);
        eds_scalars(ed, sig, pk, m, 48);
      } else {
        eds_scalars(ed, sig, pk, ShaGlobalTail{b.body + b.body_off[i]}, b.body_len[i]);
      }
    }
    stamp("work");
    // the scalars item is a party of both chains: it arrives at both before
    // running either (X first: its other party, the points item, is earlier)
    if (role != 0) run_y = arrive_last(ed.word(kEsCy), gen, 2);
    if (role != 2) run_x = arrive_last(ed.word(kEsCx), gen, 2);
    bool done = false;
    if (run_x) {
      if (!skipped) eds_chain(ed, bw, false);
      stamp("chx");
      done = arrive_last(ed.word(kEsCd), gen, 2) || done;
    }
    if (run_y) {
      if (!skipped) eds_chain(ed, bw, true);
      stamp("chy");
      done = arrive_last(ed.word(kEsCd), gen, 2) || done;
    }
    if (!done) {
      stamp("half");
      return false;
    }
    const int32_t flag = (!skipped && eds_combine(ed)) ? kFlagOk : 0;
    if (lead) stg1(res.word(kResFlags + e), flag);
  } else if (ed_item) {
    const int e = item >= kLatCores ? item - kLatCores : item;  // 0 OCERT, 1 KES
    const bool scal = item >= kLatCores;
    const Slot ed = res + kLatEd + kEdWords * e;
    const bool skipped = (skip >> e) & 1u;
    if (!skipped && e == 0) {
      uint32_t s[16], p[8], hv[8];
      ld_words(s, b.ocert_sigma + 64 * i, 4);
      ld_words(p, b.issuer_vk + 32 * i, 2);
      ld_words(hv, b.hot_vk + 32 * i, 2);
      if (scal) {
        OcertMsg m;
        ocert_msg(m, hv, b.ocert_counter[i], b.ocert_kes_period[i]);
        ed_scalars_item(ed, s, p, m, 48);
      } else {
        ed_points_item(ed, s, p, true);
      }
    } else if (!skipped) {
      kstamp(0);
      uint32_t hv[8], cur[8], sig[16];
      ld_words(hv, b.hot_vk + 32 * i, 2);
      const uint32_t* sw = reinterpret_cast<const uint32_t*>(b.kes_sig + 448 * i);
      const bool walk_ok = sum6kes_walk_wide(cur, sig, hv, b.kes_t[i], sw);
      kstamp(1);
      if (scal)
        ed_scalars_item(ed, sig, cur, ShaGlobalTail{b.body + b.body_off[i]}, b.body_len[i]);
      else
        ed_points_item(ed, sig, cur, walk_ok);
      kstamp(2);
    }
    if (!arrive_last(ed.word(125), gen, 2)) {
      stamp("half");
      return false;
    }
    kstamp(3);
    const int32_t flag = (!skipped && ed_chain(ed, bw)) ? kFlagOk : 0;
    kstamp(4);
    if (lead) stg1(res.word(kResFlags + e), flag);
  } else if (OURO_LAT_SPLIT && item >= kLatCores + 4) {
    // V2 (items 12 / 13): [s windows K..](2^(4K) H); V3 (14 / 15, OURO_LAT_V3):
    // the top windows; then the VRF's combination arrival
    const int which = (item - (kLatCores + 4)) & 1;
    const int part = item >= kLatCores + 6 ? 2 : 1;
    const bool skipped = (skip >> (kCoreVe + which)) & 1u;
    const bool none = ((skip >> (kCoreVe + which)) | (skip >> (kCoreGe + which))) & 1u;
    int32_t* vctr = res.word(kLatCtr + 1 + which);
    pw mine{0, 0, 0, 0};
    if (!skipped) {
      uint32_t p[8], pi[20];
      ld_words(p, b.vrf_vk + 32 * i, 2);
      ld_words(pi, (which ? b.leader_proof : b.eta_proof) + 80 * i, 5);
      SeedMsg alpha;
      lat_seed(alpha, b, i, which != 0, opts);
      mine = vrf_sh_split(res + kLatVsplit + 4 * kPwWords * which, res + kLatV3 + kPwWords * which,
                          p, pi, alpha, part, /*store=*/false);
    }
    // the usual last party: V and Gamma already arrived -> combine with the
    // part still in registers (OURO_LAST_PEEK); else publish it and arrive
    const bool v2_last = part == 1 && !OURO_LAT_V3 && others_arrived(vctr, gen, kVParts);
    if (!v2_last) {
      if (!skipped)
        st_pw(part == 2 ? res + kLatV3 + kPwWords * which
                        : res + kLatVsplit + 4 * kPwWords * which + 2 * kPwWords,
              mine);
      if (!arrive_last(vctr, gen, kVParts)) {
        stamp("half");
        return false;
      }
    }
    if (!none) vrf_split_combine_encode(res, which, v2_last ? &mine : nullptr);
    stamp("comb");
    // the header's last party likewise runs the tail without arriving
    if (others_arrived(res.word(kLatCtr), gen, kHdrParties)) {
      // lane 0's encodings (vrf_split_combine_encode) to the wave's other lanes
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
      hdr_tail_wide(b, i, opts, res, verdict, beta_eta, beta_leader);
      stamp("tail");
      return true;
    }
  } else if (OURO_LAT_SPLIT && (item == kCoreGe || item == kCoreGl)) {
    // Gamma: -[c]Gamma first (the VRF's three-party combination waits for
    // it), then [8]Gamma, beta and the nonce candidates (only the tail reads
    // them: this item arrives at the header counter itself)
    const int which = item == kCoreGl ? 1 : 0;
    const bool skipped = (skip >> item) & 1u;
    uint32_t pi[20];
    pw Gw{0, 0, 0, 0};
    int32_t flag = 0;
    if (!skipped) {
      ld_words(pi, (which ? b.leader_proof : b.eta_proof) + 80 * i, 5);
      flag = vrf_gamma_part_wide(res + kLatVsplit + 4 * kPwWords * which + 3 * kPwWords, Gw, pi);
    }
    stamp("work");
    if (arrive_last(res.word(kLatCtr + 1 + which), gen, kVParts)) {
      if (!(((skip >> (kCoreVe + which)) | skipped) & 1u)) vrf_split_combine_encode(res, which);
      stamp("comb");
      // the combination's own arrival (this item arrives again for beta below)
      if (arrive_last(res.word(kLatCtr), gen, kHdrParties))
        hdr_tail_wide(b, i, opts, res, verdict, beta_eta, beta_leader);
    }
    if (!skipped) {
      uint32_t beta[16];
      vrf_gamma_beta_part_wide(beta, Gw);
      if (lead) {
        st_words8(res + kLatBeta + 16 * which, beta);
        st_words8(res + kLatBeta + 16 * which + 8, beta + 8);
      }
      if (!which && (opts & kOptEtaNonce)) eta_nonce_candidates(b, i, opts, res, beta);
    }
    if (lead) stg1(res.word(kResFlags + item), flag);
  } else {
    if (!((skip >> item) & 1u)) hdr_core_wide(b, i, opts, item, res, bw, true);
    // split V: the last of a VRF's V and Gamma cores (and V2) combines and encodes
    const bool vg = item == kCoreVe || item == kCoreVl || item == kCoreGe || item == kCoreGl;
    if (!OURO_V_WHOLE && vg) {
      const int which = (item == kCoreVl || item == kCoreGl) ? 1 : 0;
      const bool last = arrive_last(res.word(kLatCtr + 1 + which), gen, OURO_LAT_SPLIT ? kVParts : 2u);
      const bool skipped = ((skip >> (kCoreVe + which)) | (skip >> (kCoreGe + which))) & 1u;
      if (OURO_LAT_SPLIT) {
        if (!last) {
          stamp("half");
          return false;
        }
        stamp("work");
        if (!skipped) vrf_split_combine_encode(res, which);
        stamp("comb");
      } else if (last && !skipped) {
        vrf_combine_encode(res, which);
      }
    }
  }
  stamp("core");
  if (arrive_last(res.word(kLatCtr), gen, kHdrParties)) {
    hdr_tail_wide(b, i, opts, res, verdict, beta_eta, beta_leader);
    stamp("tail");
    return true;
  }
  return false;
#else
  return false;
#endif
}

// items per header of the fused launch (the host sizes the grid with it)
int lat_fused_items_host() { return kFusedItems; }

// the probe's stamps of the last launch (a -DOURO_LAT_STAMPS=1 build; else -1)
int lat_stamps_read(unsigned long long* out) {
#if OURO_LAT_STAMPS
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_lat_stamps),
                             sizeof(unsigned long long) * kStampItems * kStampTags) ==
                 hipSuccess ? kStampItems * kStampTags : -1;
#else
  (void)out;
  return -1;
#endif
}

// the k-th set bit of m (k < popcount(m))
__device__ __forceinline__ int nth_set_bit(uint32_t m, int k) {
  for (int c = 0; c < 8; c++) {
    if ((m >> c) & 1u) {
      if (k == 0) return c;
      k--;
    }
  }
  return 7;
}
// the k-th clear bit of m among bits 0..7
__device__ __forceinline__ int nth_clear_bit(uint32_t m, int k) { return nth_set_bit(~m & 0xffu, k); }

// Latency mode, launch 1: eight cores per header, results to a per-header
// record.  `mode` bit 0: the cores not run wide go on DPP lane quads (four
// lanes share a scratch slot and split every group operation's products,
// ge25519.h) or one lane each; bits 8..15: cores to skip (a timing probe,
// OURO_LAT_SKIP; the verdicts are then wrong); bits 16..23: the cores run on
// one wave each (wide_cores.h, OURO_LAT_WIDE); bit 24 (all eight wide): the
// fused form -- ten items per header (hdr_item_fused), each core encodes its
// points, the header's last core to arrive runs the finish (hdr_tail_wide),
// and there is no second launch.  The first wide_waves waves of
// the grid run the wide items (wave w: core number w % nwide of header
// w / nwide; fused: item w % 10 of header w / 10), the lanes after them the other cores (work item c * n + i:
// core number c of header i, so each wave runs one core type).  n (d_n[0])
// and the batch's optional members (d_n[1], tpraos.h kOpt*) are read from
// device memory so a captured graph serves any batch of n <= capacity.
__global__ void __launch_bounds__(kBlock, OURO_LAT_WAVES) k_tpraos_cores(ouro_tpraos_batch b,
                                                            const uint32_t* __restrict__ d_n,
                                                            int32_t* res_buf, int32_t* scratch,
                                                            const int32_t* __restrict__ btab,
                                                            int mode, int wide_waves,
                                                            uint8_t* __restrict__ verdict,
                                                            uint8_t* __restrict__ beta_eta,
                                                            uint8_t* __restrict__ beta_leader,
                                                            uint32_t* win_ctr, uint32_t* done) {
  const size_t n = d_n[0];
  const uint32_t opts = d_n[1];
  const uint32_t gen = d_n[2];  // the launch's generation (arrive_last), never 0
  const int quad = mode & 1;
  const uint32_t skip = ((uint32_t)mode >> 8) & 0xffu;
  const uint32_t wmask = ((uint32_t)mode >> 16) & 0xffu;
  const int nwide = __builtin_popcount(wmask);
  const bool fused = ((uint32_t)mode >> 24) & 1u;
  // bit 26: a plan's timing probe (OURO_PLAN_TIMING): s_memrealtime at the
  // start (first workgroup) and at the window's end into the done block
  const bool stamps = (((uint32_t)mode >> 26) & 1u) && done;
  const size_t gtid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (stamps && gtid == 0)
    __hip_atomic_store(reinterpret_cast<uint64_t*>(done) + 2,
                       (uint64_t)__builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  const size_t wide_lanes = (size_t)wide_waves * 64;
  if (gtid < wide_lanes && fused) {  // wave-uniform
    const size_t wv = gtid >> 6, i = wv / kFusedItems;
    if (i < n &&
        hdr_item_fused(b, i, opts, (int)(wv % kFusedItems), slot_of(res_buf, i, kLatResWords),
                       reinterpret_cast<const uint16_t*>(btab + kBTabWords), skip, gen, verdict,
                       beta_eta, beta_leader, ((uint32_t)mode >> 25) & 1u) &&
        done) {
      // the window's done word (a plan's pinned output block, OURO_PLAN_FLAG):
      // each header's tail releases its outputs to the host and counts itself
      // in win_ctr (zeroed by the window's input copy); the last one writes the
      // launch's generation, which the plan's wait spins on instead of the
      // stream's completion.  Every lane of the wave first releases its own
      // stores at system scope (the tail's lanes write the verdict and both
      // outputs -- lane 32 beta_leader -- not only lane 0), so the done word
      // can never become visible before any of them.
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      if ((threadIdx.x & 63u) == 0) {
        const uint32_t prev =
            __hip_atomic_fetch_add(win_ctr, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_SYSTEM);
        if (prev + 1u == (uint32_t)n) {
          if (stamps)
            __hip_atomic_store(reinterpret_cast<uint64_t*>(done) + 3,
                               (uint64_t)__builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
          __hip_atomic_store(done, gen, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
      }
    }
    return;
  }
  if (gtid < wide_lanes) {  // wave-uniform
    const size_t wv = gtid >> 6, i = wv / nwide;
    const int core = nth_set_bit(wmask, (int)(wv % nwide));
    if (i < n && !((skip >> core) & 1u))
      hdr_core_wide(b, i, opts, core, slot_of(res_buf, i, kLatResWords),
                    reinterpret_cast<const uint16_t*>(btab + kBTabWords), false);
    return;
  }
  const int sh = quad ? 2 : 0;
  const size_t tid = (gtid - wide_lanes) >> sh;
  const size_t nth = ((size_t)gridDim.x * blockDim.x - wide_lanes) >> sh;
  const Slot lane = slot_of(scratch, tid, kSlotWords);
  const int ncores = kLatCores - nwide;
  for (size_t w = tid; w < (size_t)ncores * n; w += nth) {
    const int c = (int)(w / n);
    const size_t i = w - (size_t)c * n;
    const int core = nth_clear_bit(wmask, c);
    if ((skip >> core) & 1u) continue;
    hdr_core(b, i, opts, core, lane, slot_of(res_buf, i, kLatResWords), btab, /*share_key=*/false,
             /*split=*/true, quad != 0);
  }
}

// Latency mode, launch 2: the finish.  quad = 1: a lane quad per header, its
// lane pairs finishing one VRF each (vrf_finish_split: one inversion of four
// Z per VRF), quad position 0 assembling the verdict; quad = 0: one lane per
// header with one inversion of all eight Z.
__global__ void __launch_bounds__(kBlock, OURO_WAVES) k_tpraos_finish(ouro_tpraos_batch b,
                                                             const uint32_t* __restrict__ d_n,
                                                             int32_t* res_buf,
                                                             uint8_t* __restrict__ verdict,
                                                             uint8_t* __restrict__ beta_eta,
                                                             uint8_t* __restrict__ beta_leader,
                                                             int32_t* scratch, int quad) {
  const size_t n = d_n[0];
  const uint32_t opts = d_n[1];
  const int sh = quad ? 2 : 0;
  const size_t tid = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> sh;
  const size_t nth = ((size_t)gridDim.x * blockDim.x) >> sh;
  const Slot lane = slot_of(scratch, tid, kSlotWords);
  const uint32_t q = threadIdx.x & 3u;
  for (size_t i = tid; i < n; i += nth) {
    const Slot res = slot_of(res_buf, i, kLatResWords);
    if (!quad) {
      hdr_combine_split(res);
      hdr_finish_item(b, i, opts, res, lane, verdict, beta_eta, beta_leader);
      continue;
    }
    const int which = (int)(q >> 1);
    uint32_t pi[20], beta[16];
    load_words(pi, (which ? b.leader_proof : b.eta_proof) + 80 * i, 5);
    uint32_t bit = vrf_finish_split(res, which, pi, beta);
    bit |= hdr_claim_bit(b, i, opts, which, bit != 0, beta);
    if (!sc_is_canonical(pi + 12)) bit |= which ? OURO_HDR_LEADER_S_UNREDUCED : OURO_HDR_ETA_S_UNREDUCED;
    if (q == 0) hdr_eta_nonce(b, i, opts, beta);
    // quad position 0 takes position 2's (the leader VRF's) bits
    const uint32_t other = (uint32_t)__builtin_amdgcn_mov_dpp((int)bit, 0x0a, 0xf, 0xf, true);
    uint8_t* dst = which ? beta_leader : beta_eta;
    if ((q & 1u) == 0 && dst) store_words(dst + 64 * i, beta, 4);
    if (q == 0) {
      uint32_t v = bit | other;
      if (ldg1(res.word(kResFlags + kCoreOcert)) & kFlagOk) v |= 0x01u;
      if (ldg1(res.word(kResFlags + kCoreKes)) & kFlagOk) v |= 0x02u;
      verdict[i] = (uint8_t)v;
    }
  }
}

// Small batches on whole waves (one item per wave, wide_cores.h): the
// latency of a single-item call or a few items is one wave's chain instead of
// one lane's (launch_ed / launch_vrf route n <= OURO_WIDE_SMALL_MAX here).
// Same verdicts and outputs as k_ed25519_verify / k_vrf03_verify.
__global__ void __launch_bounds__(64) k_ed25519_wide(size_t n, const uint8_t* __restrict__ pk,
                                                     const uint8_t* __restrict__ sig,
                                                     const uint8_t* __restrict__ msg,
                                                     const uint64_t* __restrict__ msg_off,
                                                     const uint32_t* __restrict__ msg_len,
                                                     uint8_t* __restrict__ verdict,
                                                     const int32_t* __restrict__ btab,
                                                     uint32_t byron) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint16_t* bw = reinterpret_cast<const uint16_t*>(btab + kBTabWords);
  for (size_t i = blockIdx.x; i < n; i += gridDim.x) {
    uint32_t s[16], p[8];
    load_words(s, sig + 64 * i, 4);
    load_words(p, pk + 32 * i, 2);
    const bool ok = wide::ed25519_verify_wide(s, p, ShaGlobalTail{msg + msg_off[i]}, msg_len[i],
                                              bw, byron != 0);
    if (threadIdx.x == 0) verdict[i] = ok ? 1 : 0;
  }
#endif
}

__global__ void __launch_bounds__(64) k_vrf03_wide(size_t n, const uint8_t* __restrict__ pk,
                                                   const uint8_t* __restrict__ proof,
                                                   const uint8_t* __restrict__ alpha,
                                                   const uint64_t* __restrict__ alpha_off,
                                                   const uint32_t* __restrict__ alpha_len,
                                                   uint8_t* __restrict__ beta,
                                                   uint8_t* __restrict__ verdict,
                                                   const int32_t* __restrict__ btab,
                                                   uint32_t flags) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint16_t* bw = reinterpret_cast<const uint16_t*>(btab + kBTabWords);
  for (size_t i = blockIdx.x; i < n; i += gridDim.x) {
    uint32_t p[8], pi[20], b[16];
    load_words(p, pk + 32 * i, 2);
    load_words(pi, proof + 80 * i, 5);
    bool ok = wide::vrf03_verify_wide(b, p, pi, ShaGlobalTail{alpha + alpha_off[i]},
                                      alpha_len[i], bw);
    if ((flags & OURO_VRF_STRICT_S) && !sc_is_canonical(pi + 12)) ok = false;  // App. B.3
#pragma unroll
    for (int k = 0; k < 16; k++) b[k] = ok ? b[k] : 0u;
    if (threadIdx.x == 0) {
      store_words(beta + 64 * i, b, 4);
      verdict[i] = ok ? 1 : 0;
    }
  }
#endif
}
