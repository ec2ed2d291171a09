// kernels.hip -- gfx950 kernels and the C-ABI runtime (include/ouro_verify.h).
//
// One item per lane, 256-thread workgroups, grid-stride over the batch with a
// grid capped at the resident capacity the occupancy API reports, so the
// per-lane scratch slots (verify.h) are bounded by the grid, not the batch.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <new>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/ouro_verify.h"
#include "cbor.h"
#include "cbor_byron.h"
#include "host_path.h"
#include "knobs.h"
#include "launch.h"
#include "leader.h"
#include "task_pool.h"
#include "tpraos.h"

using namespace ouro;

// numa.cpp: NUMA placement of a device's host side
namespace ouro_numa {
int node_of_pci(const char* busid);
int bind_thread(int node);
}  // namespace ouro_numa


// ---------------------------------------------------------------- kernels ----

__global__ void __launch_bounds__(kBlock, OURO_WAVES) k_ed25519_verify(
    size_t n, const uint8_t* __restrict__ pk, const uint8_t* __restrict__ sig,
    const uint8_t* __restrict__ msg, const uint64_t* __restrict__ msg_off,
    const uint32_t* __restrict__ msg_len, uint8_t* __restrict__ verdict, int32_t* scratch,
    const int32_t* __restrict__ btab, uint32_t byron) {
  const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t nth = (size_t)gridDim.x * blockDim.x;
  const Slot lane = slot_of(scratch, tid, kSlotWords);
  for (size_t i = tid; i < n; i += nth) {
    uint32_t s[16], p[8];
    load_words(s, sig + 64 * i, 4);
    load_words(p, pk + 32 * i, 2);
    const bool ok = ed25519_verify_lane(s, p, ShaGlobalTail{msg + msg_off[i]}, msg_len[i], lane,
                                        btab, byron != 0);
    verdict[i] = ok ? 1 : 0;
  }
}

__global__ void __launch_bounds__(kBlock, OURO_WAVES) k_vrf03_verify(
    size_t n, const uint8_t* __restrict__ pk, const uint8_t* __restrict__ proof,
    const uint8_t* __restrict__ alpha, const uint64_t* __restrict__ alpha_off,
    const uint32_t* __restrict__ alpha_len, uint8_t* __restrict__ beta,
    uint8_t* __restrict__ verdict, int32_t* scratch, const int32_t* __restrict__ btab,
    uint32_t flags) {
  const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t nth = (size_t)gridDim.x * blockDim.x;
  const Slot lane = slot_of(scratch, tid, kSlotWords);
  for (size_t i = tid; i < n; i += nth) {
    uint32_t p[8], pi[20], b[16];
    load_words(p, pk + 32 * i, 2);
    load_words(pi, proof + 80 * i, 5);
    bool ok = vrf03_verify_lane(b, p, pi, ShaGlobalTail{alpha + alpha_off[i]}, alpha_len[i], lane, btab);
    if ((flags & OURO_VRF_STRICT_S) && !sc_is_canonical(pi + 12)) ok = false;  // App. B.3
#pragma unroll
    for (int k = 0; k < 16; k++) b[k] = ok ? b[k] : 0u;
    store_words(beta + 64 * i, b, 4);
    verdict[i] = ok ? 1 : 0;
  }
}

// OURO_KES_STAGE=1: the leaf message's tail (the header body) staged by the
// wave into LDS with coalesced loads (sha512.h ShaStagedTail); the loop then
// runs whole waves (a lane past the batch end repeats the last item, its
// verdict not stored) because staging needs every lane.
#ifndef OURO_KES_STAGE
#define OURO_KES_STAGE 0
#endif
__global__ void __launch_bounds__(kBlock, OURO_WAVES) k_sum6kes_verify(
    size_t n, const uint8_t* __restrict__ vk, const uint32_t* __restrict__ t,
    const uint8_t* __restrict__ msg, const uint64_t* __restrict__ msg_off,
    const uint32_t* __restrict__ msg_len, const uint8_t* __restrict__ sig,
    uint8_t* __restrict__ verdict, int32_t* scratch, const int32_t* __restrict__ btab) {
  const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t nth = (size_t)gridDim.x * blockDim.x;
  const Slot lane = slot_of(scratch, tid, kSlotWords);
#if OURO_KES_STAGE
  __shared__ uint32_t s_stage[kBlock / 64 * kStageWaveDw];
  uint32_t* rows = s_stage + (threadIdx.x >> 6) * kStageWaveDw;
  const size_t lid = threadIdx.x & 63u;
  for (size_t base = tid - lid; base < n; base += nth) {  // wave-uniform
    const size_t i0 = base + lid;
    const size_t i = i0 < n ? i0 : n - 1;
    uint32_t v[8];
    load_words(v, vk + 32 * i, 2);
    const uint32_t* sw = reinterpret_cast<const uint32_t*>(sig + 448 * i);
    const bool ok = sum6kes_verify_lane(v, t[i], sw, ShaStagedTail{msg + msg_off[i], rows},
                                        msg_len[i], lane, btab);
    if (i0 < n) verdict[i0] = ok ? 1 : 0;
  }
  return;
#endif
  for (size_t i = tid; i < n; i += nth) {
    uint32_t v[8];
    load_words(v, vk + 32 * i, 2);
    const uint32_t* sw = reinterpret_cast<const uint32_t*>(sig + 448 * i);
    const bool ok = sum6kes_verify_lane(v, t[i], sw, ShaGlobalTail{msg + msg_off[i]}, msg_len[i], lane, btab);
    verdict[i] = ok ? 1 : 0;
  }
}

// The six cores from one run-time-dispatched copy of the dispatch (1, the
// default since round 3) or six inlined calls (0): the same time (r01h 73.76
// vs 73.62 ms; r03e 70.92 vs 70.90 ms) with the kernel's VGPR spills
// 107 -> 48 and its scratch 3,904 -> 3,760 B/lane.
#ifndef OURO_HDR_LOOP
#define OURO_HDR_LOOP 1
#endif
// The finish (inversion, encodings, hashes) out of line with its own
// register allocation (1, the default since round 3): kernel VGPR spills
// 48 -> 9, scratch 3,760 -> 3,152 B/lane, time 69.57 -> 69.43 ms
// (profiles/r03/ab_finish_prefetch.json).
#ifndef OURO_HDR_FINISH_NI
#define OURO_HDR_FINISH_NI 1
#endif
#if OURO_HDR_FINISH_NI
// A/B: the finish (inversion, encodings, hashes) with its own register allocation
__device__ __noinline__ void hdr_finish_item_ni(const ouro_tpraos_batch& b, size_t i,
                                                uint32_t opts, Slot res, Slot tmp,
                                                uint8_t* verdict, uint8_t* beta_eta,
                                                uint8_t* beta_leader) {
  hdr_finish_item(b, i, opts, res, tmp, verdict, beta_eta, beta_leader);
}
#endif

// CLOCK PROBE (a separate diagnostic build, lib/libouro_verify_clock.so,
// -DOURO_CLOCK_STAMPS=1; in the product build no stamp executes): thread 0 of
// each workgroup stamps s_memtime (shader clock) and s_memrealtime (100 MHz)
// at entry and exit of k_tpraos_verify, so bench.py reads the clock the
// header kernel itself ran at (MI355X_MICROARCH.md "DVFS give-back" item 6)
// for roofline.frac_clock.  Every workgroup of the capped grid lives for the
// whole launch.
#ifndef OURO_CLOCK_STAMPS
#define OURO_CLOCK_STAMPS 0
#endif
[[maybe_unused]] constexpr int kClockSlots = 8192;
#if OURO_CLOCK_STAMPS
__device__ unsigned long long g_clock_stamps[kClockSlots][4];
#endif

// Throughput mode: one lane per header runs every core of tpraos.h, sharing
// the VRF key decode and its table, then the single-inversion finish.
__global__ void __launch_bounds__(kBlock, OURO_WAVES) k_tpraos_verify(ouro_tpraos_batch b,
                                                             uint8_t* __restrict__ verdict,
                                                             uint8_t* __restrict__ beta_eta,
                                                             uint8_t* __restrict__ beta_leader,
                                                             int32_t* scratch,
                                                             const int32_t* __restrict__ btab) {
  const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t nth = (size_t)gridDim.x * blockDim.x;
  const Slot lane = slot_of(scratch, tid, kHdrLaneWords);
  const Slot res = lane + kLaneWords;
  const uint32_t opts = batch_opts(b);
#if OURO_CLOCK_STAMPS
  unsigned long long c0 = 0, r0 = 0;
  if (threadIdx.x == 0) {
    r0 = __builtin_amdgcn_s_memrealtime();
    c0 = __builtin_amdgcn_s_memtime();
  }
#endif
  for (size_t i = tid; i < b.n; i += nth) {
#if OURO_HDR_LOOP
    // one copy of the core dispatch, the core chosen at run time
#pragma unroll 1
    for (int c = kCoreOcert; c <= kCoreVl; c++) hdr_core(b, i, opts, c, lane, res, btab);
#else
    hdr_core(b, i, opts, kCoreOcert, lane, res, btab);
    hdr_core(b, i, opts, kCoreKes, lane, res, btab);
    hdr_core(b, i, opts, kCoreUe, lane, res, btab);
    hdr_core(b, i, opts, kCoreUl, lane, res, btab);
    hdr_core(b, i, opts, kCoreVe, lane, res, btab);
    hdr_core(b, i, opts, kCoreVl, lane, res, btab);
#endif
#if OURO_HDR_FINISH_NI
    hdr_finish_item_ni(b, i, opts, res, lane, verdict, beta_eta, beta_leader);
#else
    hdr_finish_item(b, i, opts, res, lane, verdict, beta_eta, beta_leader);
#endif
  }
#if OURO_CLOCK_STAMPS
  __syncthreads();  // the whole workgroup's work inside the stamps
  if (threadIdx.x == 0 && blockIdx.x < kClockSlots) {
    const unsigned long long c1 = __builtin_amdgcn_s_memtime();
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    g_clock_stamps[blockIdx.x][0] = c0;
    g_clock_stamps[blockIdx.x][1] = c1;
    g_clock_stamps[blockIdx.x][2] = r0;
    g_clock_stamps[blockIdx.x][3] = r1;
  }
#endif
}

// ---- the split header kernel (OURO_SPLIT, round 4) ---------------------------
// The same cores as k_tpraos_verify in three launches per chunk of headers, so
// the double-scalar multiplications -- ~70 % of a header's time, and code
// whose chains fit in 128 VGPRs -- run at OURO_DSM_WAVES waves per SIMD while
// the decodes, hashes, table builds and the finish keep the 2-wave budget they
// need (3 waves spill there: +2.7 %, profiles/r04b/ab_waves_w2_vs_w3.json):
//   k_hdr_pre   header li of the chunk: every core's kPhasePre into its own
//               task slot (core * chunk + li), flags into the header's record;
//   k_hdr_dsm   task t: dsm_lane with the cfg the pre phase left in the slot
//               (t = core * chunk + li: a wave's 64 tasks are one core of 64
//               consecutive headers, the same grouping the pre phase's
//               wave_max_small saw, so the window count is wave-uniform);
//   k_hdr_post  header li: every core's kPhasePost, then the finish.
#ifndef OURO_DSM_WAVES
#define OURO_DSM_WAVES 4
#endif
#ifndef OURO_PRE_WAVES
#define OURO_PRE_WAVES OURO_WAVES  // the pre / post kernels' own budgets (A/B)
#endif
#ifndef OURO_POST_WAVES
#define OURO_POST_WAVES OURO_WAVES
#endif
constexpr int kHdrResWords = round_slot(kResWords);
__global__ void __launch_bounds__(kBlock, OURO_PRE_WAVES) k_hdr_pre(ouro_tpraos_batch b, size_t base,
                                                               size_t count, size_t chunk,
                                                               int32_t* tasks, int32_t* res_buf,
                                                               const int32_t* __restrict__ btab) {
  const size_t nth = (size_t)gridDim.x * blockDim.x;
  const uint32_t opts = batch_opts(b);
  for (size_t li = (size_t)blockIdx.x * blockDim.x + threadIdx.x; li < count; li += nth) {
    const size_t i = base + li;
    const Slot res = slot_of(res_buf, li, kHdrResWords);
    const Slot ukey = slot_of(tasks, (size_t)kCoreUe * chunk + li, kSlotWords);
#pragma unroll 1
    for (int c = kCoreOcert; c <= kCoreVl; c++)
      hdr_core(b, i, opts, c, slot_of(tasks, (size_t)c * chunk + li, kSlotWords), res, btab, true,
               false, false, kPhasePre, ukey);
  }
}
__global__ void __launch_bounds__(kBlock, OURO_DSM_WAVES) k_hdr_dsm(size_t count, size_t chunk,
                                                                   int ncores, int32_t* tasks,
                                                                   const int32_t* __restrict__ btab) {
  const size_t nth = (size_t)gridDim.x * blockDim.x;
  const size_t ntasks = (size_t)ncores * chunk;
  for (size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x; t < ntasks; t += nth) {
    if (t % chunk >= count) continue;  // the last chunk's unused headers
    const Slot s = slot_of(tasks, t, kSlotWords);
    dsm_lane_dsm_launch(s, btab, (uint32_t)ldg1(s.word(kSlotCfg)));
  }
}
__global__ void __launch_bounds__(kBlock, OURO_POST_WAVES) k_hdr_post(ouro_tpraos_batch b, size_t base,
                                                                size_t count, size_t chunk,
                                                                int32_t* tasks, int32_t* res_buf,
                                                                uint8_t* __restrict__ verdict,
                                                                uint8_t* __restrict__ beta_eta,
                                                                uint8_t* __restrict__ beta_leader) {
  const size_t nth = (size_t)gridDim.x * blockDim.x;
  const uint32_t opts = batch_opts(b);
  for (size_t li = (size_t)blockIdx.x * blockDim.x + threadIdx.x; li < count; li += nth) {
    const size_t i = base + li;
    const Slot res = slot_of(res_buf, li, kHdrResWords);
#pragma unroll 1
    for (int c = kCoreOcert; c <= kCoreVl; c++)
      hdr_core(b, i, opts, c, slot_of(tasks, (size_t)c * chunk + li, kSlotWords), res, nullptr,
               true, false, false, kPhasePost);
    // the finish's 8 x 12 scratch words: the header's (spent) OCERT task slot
#if OURO_HDR_FINISH_NI
    hdr_finish_item_ni(b, i, opts, res, slot_of(tasks, li, kSlotWords), verdict, beta_eta,
                       beta_leader);
#else
    hdr_finish_item(b, i, opts, res, slot_of(tasks, li, kSlotWords), verdict, beta_eta,
                    beta_leader);
#endif
  }
}

// The standalone Ed25519 / Sum6KES kernels split the same way (one task per
// item; the checks before the dsm in the slot's spare word kSlotCfg + 1).
constexpr int kSlotPreOk = kSlotCfg + 1;
__global__ void __launch_bounds__(kBlock, OURO_PRE_WAVES) k_ed25519_pre(
    size_t base, size_t count, const uint8_t* __restrict__ pk, const uint8_t* __restrict__ sig,
    const uint8_t* __restrict__ msg, const uint64_t* __restrict__ msg_off,
    const uint32_t* __restrict__ msg_len, int32_t* tasks, const int32_t* __restrict__ btab,
    uint32_t byron) {
  const size_t nth = (size_t)gridDim.x * blockDim.x;
  for (size_t li = (size_t)blockIdx.x * blockDim.x + threadIdx.x; li < count; li += nth) {
    const size_t i = base + li;
    const Slot s = slot_of(tasks, li, kSlotWords);
    uint32_t sg[16], p[8];
    load_words(sg, sig + 64 * i, 4);
    load_words(p, pk + 32 * i, 2);
    const bool ok = ed25519_verify_lane(sg, p, ShaGlobalTail{msg + msg_off[i]}, msg_len[i], s, btab,
                                        byron != 0, false, kPhasePre);
    stg1(s.word(kSlotPreOk), ok ? 1 : 0);
  }
}
__global__ void __launch_bounds__(kBlock, OURO_PRE_WAVES) k_sum6kes_pre(
    size_t base, size_t count, const uint8_t* __restrict__ vk, const uint32_t* __restrict__ t,
    const uint8_t* __restrict__ msg, const uint64_t* __restrict__ msg_off,
    const uint32_t* __restrict__ msg_len, const uint8_t* __restrict__ sig, int32_t* tasks,
    const int32_t* __restrict__ btab) {
  const size_t nth = (size_t)gridDim.x * blockDim.x;
  for (size_t li = (size_t)blockIdx.x * blockDim.x + threadIdx.x; li < count; li += nth) {
    const size_t i = base + li;
    const Slot s = slot_of(tasks, li, kSlotWords);
    uint32_t v[8];
    load_words(v, vk + 32 * i, 2);
    const uint32_t* sw = reinterpret_cast<const uint32_t*>(sig + 448 * i);
    const bool ok = sum6kes_verify_lane(v, t[i], sw, ShaGlobalTail{msg + msg_off[i]}, msg_len[i], s,
                                        btab, false, kPhasePre);
    stg1(s.word(kSlotPreOk), ok ? 1 : 0);
  }
}
// verdict = the pre checks and [the dsm's result] == O
__global__ void __launch_bounds__(kBlock) k_ed_post(size_t base, size_t count, int32_t* tasks,
                                                    uint8_t* __restrict__ verdict) {
  const size_t nth = (size_t)gridDim.x * blockDim.x;
  for (size_t li = (size_t)blockIdx.x * blockDim.x + threadIdx.x; li < count; li += nth) {
    const Slot s = slot_of(tasks, li, kSlotWords);
    verdict[base + li] = (ldg1(s.word(kSlotPreOk)) && dsm_result_is_identity(s)) ? 1 : 0;
  }
}

// Latency mode (k_tpraos_cores, k_tpraos_finish): kernels_lat.hip, its own
// translation unit built with the row-order field products (lane quads issue
// one product per lane, whose dependent column-scan chains would stall: A/B
// p50 0.5875 -> 0.5712 ms, profiles/r02d/ablat_rows_scan.json).
__global__ void k_tpraos_cores(ouro_tpraos_batch b, const uint32_t* __restrict__ d_n,
                               int32_t* res_buf, int32_t* scratch,
                               const int32_t* __restrict__ btab, int mode, int wide_waves,
                               uint8_t* __restrict__ verdict, uint8_t* __restrict__ beta_eta,
                               uint8_t* __restrict__ beta_leader, uint32_t* win_ctr,
                               uint32_t* done);
int lat_fused_items_host();  // kernels_lat.hip: waves per header of the fused launch
int lat_stamps_read(unsigned long long* out);  // kernels_lat.hip: the latency probe's stamps
__global__ void k_ed25519_wide(size_t n, const uint8_t* __restrict__ pk,
                               const uint8_t* __restrict__ sig, const uint8_t* __restrict__ msg,
                               const uint64_t* __restrict__ msg_off,
                               const uint32_t* __restrict__ msg_len, uint8_t* __restrict__ verdict,
                               const int32_t* __restrict__ btab, uint32_t byron);
__global__ void k_vrf03_wide(size_t n, const uint8_t* __restrict__ pk,
                             const uint8_t* __restrict__ proof, const uint8_t* __restrict__ alpha,
                             const uint64_t* __restrict__ alpha_off,
                             const uint32_t* __restrict__ alpha_len, uint8_t* __restrict__ beta,
                             uint8_t* __restrict__ verdict, const int32_t* __restrict__ btab,
                             uint32_t flags);
__global__ void k_tpraos_finish(ouro_tpraos_batch b, const uint32_t* __restrict__ d_n,
                                int32_t* res_buf, uint8_t* __restrict__ verdict,
                                uint8_t* __restrict__ beta_eta, uint8_t* __restrict__ beta_leader,
                                int32_t* scratch, int quad);

// Raw wire headers -> the SoA on the device, one lane
// per header: the host slicer's parse (cbor.h, pinned to header.py by
// tests/test_pack.py), spans checked against raw_bytes here (status
// OURO_PACK_ESPAN) since a device call cannot return OURO_EINVAL per header.
__global__ void __launch_bounds__(kBlock) k_tpraos_pack(const uint8_t* __restrict__ raw,
                                                        size_t raw_bytes,
                                                        const uint64_t* __restrict__ off,
                                                        const uint32_t* __restrict__ len, size_t n,
                                                        uint64_t spkp, cbor::Out o,
                                                        uint8_t* __restrict__ status) {
  const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t nth = (size_t)gridDim.x * blockDim.x;
  for (size_t i = tid; i < n; i += nth) {
    const uint64_t o0 = off[i];
    const uint32_t l0 = len[i];
    uint8_t st = (o0 > raw_bytes || raw_bytes - o0 < l0)
                     ? (uint8_t)OURO_PACK_ESPAN
                     : cbor::pack_one(raw, o0, l0, spkp, o, i);
    if (st != OURO_PACK_OK) cbor::zero_row(o, i);
    status[i] = st;
  }
}

// The Byron slicer (cbor_byron.h byron_pack_one, the host slicer's parse) on
// the device, one lane per header, over a chunk staged densely by raw_stage:
// header i's bytes at off[i] = the lengths' prefix sum, so its message slot
// (len + kByronMsgExtra bytes, ouro_byron_pack_cbor's layout) starts at
// off[i] + kByronMsgExtra * i.  A rejected row is zeroed (msg_len 0).
__global__ void __launch_bounds__(kBlock) k_byron_pack(const uint8_t* __restrict__ raw,
                                                       size_t raw_bytes,
                                                       const uint64_t* __restrict__ off,
                                                       const uint32_t* __restrict__ len, size_t n,
                                                       int64_t magic, cbor::ByronOut o,
                                                       uint8_t* __restrict__ status) {
  const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t nth = (size_t)gridDim.x * blockDim.x;
  for (size_t i = tid; i < n; i += nth) {
    const uint64_t o0 = off[i];
    const uint32_t l0 = len[i];
    o.msg_off[i] = o0 + cbor::kByronMsgExtra * i;
    uint8_t st = (o0 > raw_bytes || raw_bytes - o0 < l0)
                     ? (uint8_t)OURO_PACK_ESPAN
                     : cbor::byron_pack_one(raw, o0, l0, magic, o, i);
    if (st != OURO_PACK_OK) cbor::byron_zero_row(o, i);
    status[i] = st;
  }
}

// leader threshold (leader.h), one item per lane; verdict 1 / 0 / 0xff
__global__ void __launch_bounds__(kBlock) k_leader_check(size_t n, const uint8_t* __restrict__ beta,
                                                         const uint64_t* __restrict__ num,
                                                         const uint64_t* __restrict__ den,
                                                         uint64_t act_log_lo, int64_t act_log_hi,
                                                         uint32_t f_is_one,
                                                         uint8_t* __restrict__ verdict) {
  const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t nth = (size_t)gridDim.x * blockDim.x;
  for (size_t i = tid; i < n; i += nth) {
    const int32_t r = f_is_one ? kLeaderYes
                               : leader_check_lane(beta + 64 * i, num[i], den[i], act_log_lo,
                                                   act_log_hi);
    verdict[i] = r < 0 ? (uint8_t)0xff : (uint8_t)r;
  }
}

// proof_to_hash only (no verification): beta = H(0x04 || 0x03 || [8]Gamma)
__global__ void __launch_bounds__(kBlock, OURO_WAVES) k_vrf03_proof_to_hash(size_t n,
                                                                const uint8_t* __restrict__ proof,
                                                                uint8_t* __restrict__ beta,
                                                                uint8_t* __restrict__ verdict) {
  const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t nth = (size_t)gridDim.x * blockDim.x;
  for (size_t i = tid; i < n; i += nth) {
    uint32_t G[8];
    load_words(G, proof + 80 * i, 2);
    ge_p3 Gamma;
    bool ok = ge_is_canonical(G);
    ok = ge_decode(&Gamma, G, false) && ok;
    ge_p3 G8 = ge_mul8(Gamma);
    uint32_t enc[8];
    ge_encode_with_inv(enc, G8.X, G8.Y, fe_invert(G8.Z));
    uint32_t bp[9];
    bp[0] = 0x04u | (0x03u << 8) | (enc[0] << 16);
#pragma unroll
    for (int k = 1; k < 8; k++) bp[k] = (enc[k - 1] >> 16) | (enc[k] << 16);
    bp[8] = enc[7] >> 16;
    uint64_t H[8];
    sha512_prefixed<34>(H, bp, ShaNoTail{}, 0);
    uint32_t w[16];
    sha512_digest_words(w, H);
#pragma unroll
    for (int k = 0; k < 16; k++) w[k] = ok ? w[k] : 0u;
    store_words(beta + 64 * i, w, 4);
    verdict[i] = ok ? 1 : 0;
  }
}

// ---------------------------------------------------------------- runtime ----

namespace {

thread_local std::string t_last_error;
thread_local int t_device = -1;

int fail(int code, const std::string& what) {
  t_last_error = what;
  return code;
}

#define OURO_HIP(call)                                                               \
  do {                                                                               \
    hipError_t e_ = (call);                                                          \
    if (e_ != hipSuccess)                                                            \
      return fail(OURO_EDEVICE, std::string(#call) + ": " + hipGetErrorString(e_)); \
  } while (0)

struct DeviceState {
  bool ready = false;
  int err = OURO_OK;
  std::string err_msg;
  int32_t* btab = nullptr;
  int cus = 0;
  int max_blocks[16] = {0};  // per KernelId (kNumKernels <= 16)
};

std::mutex g_dev_mu;
std::map<int, DeviceState> g_dev;

enum KernelId { kEd = 0, kVrf = 1, kKes = 2, kHdr = 3, kP2H = 4, kCores = 5, kFinish = 6,
                kLeader = 7, kHdrPre = 8, kHdrDsm = 9, kHdrPost = 10, kEdPre = 11, kKesPre = 12,
                kNumKernels = 13 };

const void* kernel_ptr(int id) {
  switch (id) {
    case kEd: return reinterpret_cast<const void*>(&k_ed25519_verify);
    case kVrf: return reinterpret_cast<const void*>(&k_vrf03_verify);
    case kKes: return reinterpret_cast<const void*>(&k_sum6kes_verify);
    case kHdr: return reinterpret_cast<const void*>(&k_tpraos_verify);
    case kCores: return reinterpret_cast<const void*>(&k_tpraos_cores);
    case kFinish: return reinterpret_cast<const void*>(&k_tpraos_finish);
    case kLeader: return reinterpret_cast<const void*>(&k_leader_check);
    case kHdrPre: return reinterpret_cast<const void*>(&k_hdr_pre);
    case kHdrDsm: return reinterpret_cast<const void*>(&k_hdr_dsm);
    case kHdrPost: return reinterpret_cast<const void*>(&k_hdr_post);
    case kEdPre: return reinterpret_cast<const void*>(&k_ed25519_pre);
    case kKesPre: return reinterpret_cast<const void*>(&k_sum6kes_pre);
    default: return reinterpret_cast<const void*>(&k_vrf03_proof_to_hash);
  }
}

// ---- NUMA placement (numa.cpp) ----
// the NUMA node of device `dev` (sysfs numa_node of its PCI function), -1 if unknown
int device_numa_node(int dev) {
  char busid[64] = {0};
  if (hipDeviceGetPCIBusId(busid, (int)sizeof(busid), dev) != hipSuccess) return -1;
  return ouro_numa::node_of_pci(busid);
}

int current_device(int* dev) {
  // no usable device at all is OURO_ENODEV (not a device error: nothing is
  // recomputed on the host path behind the caller's back)
  auto nodev = [](hipError_t e) {
    return e == hipErrorNoDevice || e == hipErrorInvalidDevice || e == hipErrorInsufficientDriver;
  };
  if (t_device < 0) {
    int d = 0;
    const hipError_t e = hipGetDevice(&d);
    if (nodev(e)) return fail(OURO_ENODEV, std::string("hipGetDevice: ") + hipGetErrorString(e));
    OURO_HIP(e);
    t_device = d;
  }
  const hipError_t e = hipSetDevice(t_device);
  if (nodev(e)) return fail(OURO_ENODEV, std::string("hipSetDevice: ") + hipGetErrorString(e));
  OURO_HIP(e);
  *dev = t_device;
  return OURO_OK;
}

int device_state(DeviceState** out) {
  int dev;
  int rc = current_device(&dev);
  if (rc) return rc;
  std::lock_guard<std::mutex> g(g_dev_mu);
  DeviceState& s = g_dev[dev];
  if (!s.ready) {
    hipDeviceProp_t prop;
    OURO_HIP(hipGetDeviceProperties(&prop, dev));
    if (std::string(prop.gcnArchName).rfind("gfx950", 0) != 0)
      return fail(OURO_ENODEV, std::string("device is ") + prop.gcnArchName + ", need gfx950");
    s.cus = prop.multiProcessorCount;
    // niels B tables, then their wave-wide form (latency mode, wide.h)
    std::vector<int32_t> tab(kBTabWords + kBTabWideWords);
    memcpy(tab.data(), ouro_host::btab(), sizeof(int32_t) * kBTabWords);  // built once per process
    build_btab_wide(reinterpret_cast<uint16_t*>(tab.data() + kBTabWords), tab.data());
    OURO_HIP(hipMalloc(&s.btab, sizeof(int32_t) * tab.size()));
    OURO_HIP(hipMemcpy(s.btab, tab.data(), sizeof(int32_t) * tab.size(), hipMemcpyHostToDevice));
    for (int id = 0; id < kNumKernels; id++) {
      int per_cu = 0;
      OURO_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel_ptr(id), kBlock, 0));
      s.max_blocks[id] = std::max(1, per_cu) * s.cus;
    }
    s.ready = true;
  }
  *out = &s;
  return OURO_OK;
}

// Per-thread, per-DEVICE stream and growable device buffers: a buffer
// allocated on one GPU is never handed to a launch on another, whatever the
// order of ouro_set_device calls or of a multi-GPU call's device list.
struct Buf {
  void* p = nullptr;
  size_t cap = 0;
};

// The bytes a batch addresses by (offset, length) pairs: the window
// [lo, hi) over the items with length > 0, and the offsets rebased to lo, so
// only that window is uploaded (a slice or shard of a larger batch with
// absolute offsets does not drag the bytes before it along).
struct Window {
  uint64_t lo = 0, hi = 0;
  std::vector<uint64_t> off;  // rebased; alive until the upload has completed
  size_t span() const { return (size_t)(hi - lo); }
};

// rows [lo, lo + m) of a host batch on the device: `d` points at the copies
// (optional members only when given), ver/be/bl/nonce at the result buffers
struct StagedHdr {
  ouro_tpraos_batch d{};
  uint8_t *ver = nullptr, *be = nullptr, *bl = nullptr, *nonce = nullptr;
  Window body;
};

// ---- pipelined host-buffer header batches (state) ----
// A large batch from pageable host memory is cut into chunks of one full grid
// of lanes.  Two slots (stream, device buffers, pinned result staging) take
// turns: while chunk c's kernel runs on one stream, the host uploads chunk
// c + 1 on the other and copies chunk c - 1's results out, so PCIe and the
// host copies hide behind the kernel instead of adding to it.
constexpr size_t kOutRow = 1 + 64 + 64 + 32;  // verdict | beta_eta | beta_leader | eta_nonce
struct PipeSlot {
  hipStream_t st = nullptr;
  hipEvent_t done = nullptr;
  Buf in[28];
  uint8_t* h_out = nullptr;  // pinned: verdict (m) | beta_eta (64 m) | beta_leader (64 m) | eta_nonce (32 m)
  size_t h_cap = 0;
  StagedHdr staged;  // its rebased body offsets stay alive for the async upload
  size_t lo = 0, m = 0;
  bool busy = false;
};
struct Pipe {
  bool ready = false;
  PipeSlot s[2];
};

// ---- raw header CBOR from host memory (state; the engine is raw_run) ----
// A slot of the raw-CBOR pipeline: its stream, pinned NUMA-local staging for
// one chunk's gathered header bytes and for its results, and the chunk's
// device buffers (raw bytes, the slicer's arena, results).
constexpr int kRawMaxSlots = 8;
struct RawSlot {
  hipStream_t st = nullptr;
  hipEvent_t done = nullptr;
  uint8_t* h_in = nullptr;   // rebased offsets | lengths | eta0 | alphas | raw bytes
  size_t h_in_cap = 0;
  uint8_t* h_out = nullptr;  // status | verdict | beta_eta | beta_leader | eta_nonce
  size_t h_out_cap = 0;
  Buf d_in, d_arena, d_out;
  size_t lo = 0, m = 0;
  bool busy = false;
};
struct RawPipe {
  bool ready = false;
  RawSlot s[kRawMaxSlots];
};

// Everything a calling thread needs on one device: its stream, the scratch
// slots of each stream it launches on, staging buffers and the two-slot
// pipeline.  Contexts are POOLED per device ("a per-thread
// or pooled stream"): a thread borrows one on its first call for a device and
// its thread-exit guard (Lease) hands it back, so the node's churning FFI
// worker threads reuse a few contexts instead of leaking one each.  A
// returned context has nothing in flight: host-buffer calls synchronise
// before returning, and device-API launches on a caller stream only use the
// scratch keyed by that stream (work later enqueued on the same stream is
// ordered after them).  Only the pool itself outlives the process (never
// freed: the HIP runtime may be gone at teardown).
struct ThreadCtx {
  hipStream_t stream = nullptr;
  std::map<hipStream_t, Buf> scratch;  // per stream: concurrent launches never share slots
  Buf in[32];  // staging slots; a header batch uses up to 24
  Pipe pipe;
  RawPipe raw;  // ouro_tpraos_verify_cbor / ouro_integrity_verify_cbor
};
struct CtxPool {
  std::mutex mu;
  std::map<int, std::vector<ThreadCtx*>> free;  // per device
  std::map<int, size_t> created;
};
CtxPool& ctx_pool() {
  static CtxPool* p = new CtxPool;  // leaked on purpose (see above)
  return *p;
}
struct Lease {
  std::map<int, ThreadCtx*> held;  // device -> the context this thread borrowed
  ~Lease() {
    if (held.empty()) return;
    CtxPool& P = ctx_pool();
    std::lock_guard<std::mutex> g(P.mu);
    for (auto& kv : held) P.free[kv.first].push_back(kv.second);
  }
};
thread_local Lease t_lease;

// the calling thread's context on device `dev`
ThreadCtx& ctx_of(int dev) {
  auto it = t_lease.held.find(dev);
  if (it != t_lease.held.end()) return *it->second;
  ThreadCtx* c = nullptr;
  {
    CtxPool& P = ctx_pool();
    std::lock_guard<std::mutex> g(P.mu);
    std::vector<ThreadCtx*>& v = P.free[dev];
    if (!v.empty()) {
      c = v.back();
      v.pop_back();
    } else {
      c = new ThreadCtx;
      P.created[dev]++;
    }
  }
  t_lease.held[dev] = c;
  return *c;
}
// ... on its current device (valid after current_device())
ThreadCtx& ctx() { return ctx_of(t_device); }

int ensure(Buf& b, size_t bytes) {
  if (b.cap >= bytes) return OURO_OK;
  if (b.p) OURO_HIP(hipFree(b.p));
  b.p = nullptr;
  b.cap = 0;
  size_t want = std::max<size_t>(bytes, 4096);
  OURO_HIP(hipMalloc(&b.p, want));
  b.cap = want;
  return OURO_OK;
}

int thread_stream(hipStream_t* s) {
  int dev;
  int rc = current_device(&dev);
  if (rc) return rc;
  ThreadCtx& c = ctx_of(dev);
  if (c.stream == nullptr) OURO_HIP(hipStreamCreateWithFlags(&c.stream, hipStreamNonBlocking));
  *s = c.stream;
  return OURO_OK;
}

// grid for n items of kernel `id`; returns the scratch slot count
int plan(DeviceState* ds, int id, size_t n, hipStream_t stream, int* grid, int32_t** scratch,
         int lane_words = kSlotWords) {
  size_t blocks = (n + kBlock - 1) / kBlock;
  blocks = std::max<size_t>(1, std::min<size_t>(blocks, (size_t)ds->max_blocks[id]));
  *grid = (int)blocks;
  if (scratch) {
    Buf& b = ctx().scratch[stream];
    int rc = ensure(b, blocks * kBlock * sizeof(int32_t) * lane_words);
    if (rc) return rc;
    *scratch = static_cast<int32_t*>(b.p);
  }
  return OURO_OK;
}

// TEST HOOKS, compiled only into the test build (lib/libouro_verify_test.so,
// -DOURO_TEST_HOOKS=1; tests/test_gpu_hooks.py runs the hook tests in a child
// process on it): with OURO_TEST_DEVICE_ERROR set in the environment every
// launch reports a device error, so the tests reach the host recompute path
// on a healthy GPU; OURO_TEST_PLAN_POISON (plan_poison below).  The product
// library reads neither variable.
#ifndef OURO_TEST_HOOKS
#define OURO_TEST_HOOKS 0
#endif
#if OURO_TEST_HOOKS
bool injected_device_error() { return ouro_knobs::get().test_device_error.load(std::memory_order_relaxed); }
#else
constexpr bool injected_device_error() { return false; }
#endif

int launch_check() {
  OURO_HIP(hipGetLastError());
  if (injected_device_error()) return fail(OURO_EDEVICE, "injected device error (OURO_TEST_DEVICE_ERROR)");
  return OURO_OK;
}

// ---- the host path (host_path.h) -------------------------------------------
// A host-buffer batch whose device run fails with OURO_EDEVICE is recomputed
// on the host path (SURVEY.md §5, §8(b) "Errors": never a silent accept, and
// the caller still gets verdicts); OURO_ON_DEVICE_ERROR=fail returns the error
// instead.  Device-pointer calls (*_batch_device) cannot: their buffers are
// device memory, so they return the error.
std::atomic<unsigned long long> g_host_single{0}, g_host_recompute{0};
bool recompute_on_error() {
  return !ouro_knobs::get().on_device_error_fail.load(std::memory_order_relaxed);
}
template <class F>
int or_host(int rc, F&& recompute) {
  if (rc != OURO_EDEVICE || !recompute_on_error()) return rc;
  g_host_recompute++;
  const std::string why = t_last_error;
  const int r = recompute();
  t_last_error = r == OURO_OK ? "recomputed on the host path after: " + why
                              : "host path failed (" + t_last_error + ") after: " + why;
  return r;
}
// Single items run on the host path (one GPU round trip is ~220-420 us, the
// host path ~1.5x libsodium); OURO_SINGLE_ITEM=gpu sends them to the device
// (A/B, bench.py single_item).
bool single_on_gpu() { return ouro_knobs::get().single_on_gpu.load(std::memory_order_relaxed); }

// Small batches (n <= OURO_WIDE_SMALL_MAX, default 2048; 0 = never) run one
// item per wave (kernels_lat.hip k_ed25519_wide / k_vrf03_wide): a single
// item's latency is then one wave's chain, not one lane's.
size_t wide_small_max() { return ouro_knobs::get().wide_small_max.load(std::memory_order_relaxed); }
int wide_grid(size_t n) { return (int)std::min<size_t>(n, 8192); }

// ---- device-pointer launches (shared by the host-buffer and device APIs) ----
// The split kernels (pre / dsm at OURO_DSM_WAVES / post) instead of the
// one-pass k_tpraos_verify, k_ed25519_verify and k_sum6kes_verify (measured
// and rejected): fixed at compile time in the product
// (OURO_SPLIT_DEFAULT); only the test-hook build lets OURO_SPLIT=1 select them
// (tests/test_gpu_variants.py keeps them bit-exact).
#ifndef OURO_SPLIT_DEFAULT
#define OURO_SPLIT_DEFAULT 0
#endif
bool split_launch() {
#if OURO_TEST_HOOKS
  if (ouro_knobs::get().split.load(std::memory_order_relaxed)) return true;
#endif
  return OURO_SPLIT_DEFAULT != 0;
}
// One Ed25519-shaped item per task: chunks of 4 resident grids of the pre
// kernel, so the 4-wave dsm launch has 2 grids of tasks to spread.
template <class LaunchPre>
int launch_split_items(DeviceState* ds, hipStream_t st, size_t n, int pre_id, uint8_t* verdict,
                       LaunchPre&& launch_pre) {
  const size_t cap = (size_t)ds->max_blocks[pre_id] * kBlock;
  const size_t chunk = std::min<size_t>((n + kBlock - 1) / kBlock * kBlock, 4 * cap);
  Buf& sb = ctx().scratch[st];
  int rc = ensure(sb, slot_region_words(chunk, kSlotWords) * sizeof(int32_t));
  if (rc) return rc;
  int32_t* tasks = static_cast<int32_t*>(sb.p);
  const int gp = (int)std::min<size_t>(chunk / kBlock, (size_t)ds->max_blocks[pre_id]);
  const int gd = (int)std::min<size_t>(chunk / kBlock, (size_t)ds->max_blocks[kHdrDsm]);
  for (size_t base = 0; base < n; base += chunk) {
    const size_t count = std::min(chunk, n - base);
    launch_pre(gp, base, count, tasks);
    hipLaunchKernelGGL(k_hdr_dsm, dim3(gd), dim3(kBlock), 0, st, count, chunk, 1, tasks, ds->btab);
    hipLaunchKernelGGL(k_ed_post, dim3(gp), dim3(kBlock), 0, st, base, count, tasks, verdict);
    if ((rc = launch_check())) return rc;
  }
  return OURO_OK;
}
// byron = 1: ByronDSIGN acceptance (cardano-crypto)
int launch_ed(hipStream_t st, size_t n, const uint8_t* pk, const uint8_t* sig, const uint8_t* msg,
              const uint64_t* off, const uint32_t* len, uint8_t* verdict, uint32_t byron = 0) {
  DeviceState* ds;
  int rc = device_state(&ds);
  if (rc) return rc;
  if (n <= wide_small_max()) {
    hipLaunchKernelGGL(k_ed25519_wide, dim3(wide_grid(n)), dim3(64), 0, st, n, pk, sig, msg, off,
                       len, verdict, ds->btab, byron);
    return launch_check();
  }
  if (split_launch())
    return launch_split_items(ds, st, n, kEdPre, verdict, [&](int g, size_t base, size_t count,
                                                               int32_t* tasks) {
      hipLaunchKernelGGL(k_ed25519_pre, dim3(g), dim3(kBlock), 0, st, base, count, pk, sig, msg,
                         off, len, tasks, ds->btab, byron);
    });
  int grid;
  int32_t* scr;
  if ((rc = plan(ds, kEd, n, st, &grid, &scr))) return rc;
  hipLaunchKernelGGL(k_ed25519_verify, dim3(grid), dim3(kBlock), 0, st, n, pk, sig, msg, off, len,
                     verdict, scr, ds->btab, byron);
  return launch_check();
}

int launch_vrf(hipStream_t st, size_t n, const uint8_t* pk, const uint8_t* proof,
               const uint8_t* alpha, const uint64_t* off, const uint32_t* len, uint8_t* beta,
               uint8_t* verdict, uint32_t flags = 0) {
  DeviceState* ds;
  int rc = device_state(&ds);
  if (rc) return rc;
  if (n <= wide_small_max()) {
    hipLaunchKernelGGL(k_vrf03_wide, dim3(wide_grid(n)), dim3(64), 0, st, n, pk, proof, alpha,
                       off, len, beta, verdict, ds->btab, flags);
    return launch_check();
  }
  int grid;
  int32_t* scr;
  if ((rc = plan(ds, kVrf, n, st, &grid, &scr))) return rc;
  hipLaunchKernelGGL(k_vrf03_verify, dim3(grid), dim3(kBlock), 0, st, n, pk, proof, alpha, off,
                     len, beta, verdict, scr, ds->btab, flags);
  return launch_check();
}

int launch_kes(hipStream_t st, size_t n, const uint8_t* vk, const uint32_t* t, const uint8_t* msg,
               const uint64_t* off, const uint32_t* len, const uint8_t* sig, uint8_t* verdict) {
  DeviceState* ds;
  int rc = device_state(&ds);
  if (rc) return rc;
  if (split_launch())
    return launch_split_items(ds, st, n, kKesPre, verdict, [&](int g, size_t base, size_t count,
                                                                int32_t* tasks) {
      hipLaunchKernelGGL(k_sum6kes_pre, dim3(g), dim3(kBlock), 0, st, base, count, vk, t, msg, off,
                         len, sig, tasks, ds->btab);
    });
  int grid;
  int32_t* scr;
  if ((rc = plan(ds, kKes, n, st, &grid, &scr))) return rc;
  hipLaunchKernelGGL(k_sum6kes_verify, dim3(grid), dim3(kBlock), 0, st, n, vk, t, msg, off, len,
                     sig, verdict, scr, ds->btab);
  return launch_check();
}


int launch_hdr(hipStream_t st, const ouro_tpraos_batch& b, uint8_t* verdict, uint8_t* be,
               uint8_t* bl) {
  DeviceState* ds;
  int rc = device_state(&ds);
  if (rc) return rc;
  int grid;
  int32_t* scr;
  if (split_launch()) {
    // chunks of one resident grid of the pre / post kernels; per chunk the
    // six task slots of each header and its result record
    const size_t chunk = std::min<size_t>((b.n + kBlock - 1) / kBlock * kBlock,
                                          (size_t)ds->max_blocks[kHdrPre] * kBlock);
    const size_t words = (size_t)kHdrCores * slot_region_words(chunk, kSlotWords) +
                         slot_region_words(chunk, kHdrResWords);
    Buf& sb = ctx().scratch[st];
    if ((rc = ensure(sb, words * sizeof(int32_t)))) return rc;
    int32_t* tasks = static_cast<int32_t*>(sb.p);
    int32_t* res = tasks + (size_t)kHdrCores * slot_region_words(chunk, kSlotWords);
    const int gpp = (int)std::min<size_t>(chunk / kBlock, (size_t)ds->max_blocks[kHdrPre]);
    const int gpo = (int)std::min<size_t>(chunk / kBlock, (size_t)ds->max_blocks[kHdrPost]);
    const int gd = (int)std::min<size_t>((size_t)kHdrCores * chunk / kBlock,
                                         (size_t)ds->max_blocks[kHdrDsm]);
    for (size_t base = 0; base < b.n; base += chunk) {
      const size_t count = std::min(chunk, b.n - base);
      hipLaunchKernelGGL(k_hdr_pre, dim3(gpp), dim3(kBlock), 0, st, b, base, count, chunk, tasks,
                         res, ds->btab);
      hipLaunchKernelGGL(k_hdr_dsm, dim3(gd), dim3(kBlock), 0, st, count, chunk, (int)kHdrCores,
                         tasks, ds->btab);
      hipLaunchKernelGGL(k_hdr_post, dim3(gpo), dim3(kBlock), 0, st, b, base, count, chunk, tasks,
                         res, verdict, be, bl);
      if ((rc = launch_check())) return rc;
    }
    return OURO_OK;
  }
  if ((rc = plan(ds, kHdr, b.n, st, &grid, &scr, kHdrLaneWords))) return rc;
  hipLaunchKernelGGL(k_tpraos_verify, dim3(grid), dim3(kBlock), 0, st, b, verdict, be, bl, scr,
                     ds->btab);
  return launch_check();
}

int launch_leader(hipStream_t st, size_t n, const uint8_t* beta, const uint64_t* num,
                  const uint64_t* den, int64_t lhi, uint64_t llo, int f_is_one,
                  uint8_t* verdict) {
  DeviceState* ds;
  int rc = device_state(&ds);
  if (rc) return rc;
  int grid;
  if ((rc = plan(ds, kLeader, n, st, &grid, nullptr))) return rc;
  hipLaunchKernelGGL(k_leader_check, dim3(grid), dim3(kBlock), 0, st, n, beta, num, den, llo, lhi,
                     f_is_one ? 1u : 0u, verdict);
  return launch_check();
}

// Workgroup size of the latency-mode launches (OURO_LAT_BLOCK = 64/128/256).
// A small window fills only a few waves; one-wave workgroups spread them over
// as many CUs (own L1, TA and instruction fetch per wave) instead of packing
// four onto each CU.
int lat_block() {
  const int v = ouro_knobs::get().lat_block.load(std::memory_order_relaxed);
  return v == 64 || v == 128 || v == 256 ? v : kLatBlock;
}

// Latency-mode cores on lane quads (1, default) or one lane per core
// (OURO_LAT_QUAD=0, for A/B).
int lat_quad() { return ouro_knobs::get().lat_quad.load(std::memory_order_relaxed) != 0; }

// Latency-mode cores run on one wave each (wide_cores.h): a mask over
// tpraos.h HdrCore + kCoreGe/kCoreGl, default all eight (OURO_LAT_WIDE; 0 =
// every core on lane quads, for A/B).
int lat_wide_mask() { return ouro_knobs::get().lat_wide.load(std::memory_order_relaxed) & 0xff; }

int lat_fuse() { return ouro_knobs::get().lat_fuse.load(std::memory_order_relaxed) != 0; }

// latency mode: eight cores per header (x4 lanes in quad mode), then the
// finish; n and the option bits read from d_n[0..1].
// Lanes used <= the kBlock-rounded count lowlat_scratch_words provides for.
// The launch shape (grids, option bits: the OURO_LAT_* switches) is fixed per
// capacity; a plan computes it once at build (lat_shape) and issues it per
// window (lat_issue) when it launches without a graph.
struct LatShape {
  int g1 = 0, g2 = 0, blk = 0, quad = 0, wide_lanes = 0;
  bool fused = false;
  uint32_t flags = 0;
  const int32_t* btab = nullptr;
};

int lat_shape(size_t n_cap, LatShape* s) {
  DeviceState* ds;
  int rc = device_state(&ds);
  if (rc) return rc;
  const int blk = lat_block();
  const size_t per = kBlock / blk;
  auto grid = [&](size_t items, int id) {
    size_t g = (items + blk - 1) / blk;
    return (int)std::max<size_t>(1, std::min<size_t>(g, (size_t)ds->max_blocks[id] * per));
  };
  const int quad = lat_quad();
  // the wide cores on one wave each (nwide n_cap waves, rounded to whole
  // workgroups) ahead of the other cores' lanes
  const int wmask = lat_wide_mask();
  const int nwide = __builtin_popcount((unsigned)wmask);
  // fused (all eight cores wide): the last core of a header finishes it, no
  // second launch (OURO_LAT_FUSE=0 keeps the finish launch, for A/B); its
  // items per header: kernels_lat.hip kFusedItems
  const bool fused = wmask == 0xff && lat_fuse();
  const size_t wide_waves = (size_t)(fused ? lat_fused_items_host() : nwide) * n_cap;
  const size_t wide_blocks = (wide_waves * 64 + blk - 1) / blk;
  const size_t quad_items = (size_t)(kLatCores - nwide) * n_cap;
  // timing probe: OURO_LAT_SKIP = mask of cores left out (verdicts then
  // wrong), honoured by the test-hook build only
#if OURO_TEST_HOOKS
  const int skip = ouro_knobs::get().lat_skip.load(std::memory_order_relaxed) & 0xff;
#else
  const int skip = 0;
#endif
  s->g1 = (int)wide_blocks + grid(quad_items << (quad ? 2 : 0), kCores);
  s->g2 = grid(n_cap << (quad ? 2 : 0), kFinish);
  s->blk = blk;
  s->quad = quad;
  s->wide_lanes = (int)(wide_blocks * blk / 64);
  s->fused = fused;
  s->flags = (uint32_t)(quad | (skip << 8) | (wmask << 16) | (fused ? 1 << 24 : 0) |
                        (ouro_knobs::get().lat_stamps.load(std::memory_order_relaxed) ? 1 << 25 : 0));
  s->btab = ds->btab;
  return OURO_OK;
}

// (win_ctr / done: a plan's window counter and done word, or null)
void lat_issue(hipStream_t st, const LatShape& s, const ouro_tpraos_batch& b, const uint32_t* d_n,
               int32_t* res_buf, int32_t* scratch, uint8_t* verdict, uint8_t* be, uint8_t* bl,
               uint32_t* win_ctr = nullptr, uint32_t* done = nullptr) {
  hipLaunchKernelGGL(k_tpraos_cores, dim3(s.g1), dim3(s.blk), 0, st, b, d_n, res_buf, scratch,
                     s.btab, (int)s.flags, s.wide_lanes, verdict, be, bl, win_ctr, done);
  if (s.fused) return;
  hipLaunchKernelGGL(k_tpraos_finish, dim3(s.g2), dim3(s.blk), 0, st, b, d_n, res_buf, verdict, be,
                     bl, scratch, s.quad);
}

int launch_lowlat(hipStream_t st, const ouro_tpraos_batch& b, const uint32_t* d_n, size_t n_cap,
                  int32_t* res_buf, int32_t* scratch, uint8_t* verdict, uint8_t* be,
                  uint8_t* bl) {
  LatShape s;
  int rc = lat_shape(n_cap, &s);
  if (rc) return rc;
  lat_issue(st, s, b, d_n, res_buf, scratch, verdict, be, bl);
  return launch_check();
}

size_t lowlat_scratch_words(DeviceState* ds, size_t n_cap) {
  size_t b1 = std::min<size_t>(((size_t)kLatCores * n_cap + kBlock - 1) / kBlock,
                               (size_t)ds->max_blocks[kCores]);
  size_t b2 = std::min<size_t>((n_cap + kBlock - 1) / kBlock, (size_t)ds->max_blocks[kFinish]);
  return std::max<size_t>(1, std::max(b1, b2)) * kBlock * kSlotWords;
}

// ---- host-buffer staging ----
struct Stager {
  hipStream_t st;
  int slot = 0;
  int rc = OURO_OK;
  Buf* bufs = ctx().in;  // device buffers, one per up()/out() call
  int nbufs = 32;
  Buf* next() {
    if (slot >= nbufs) {
      rc = fail(OURO_EDEVICE, "staging slots exhausted");
      return nullptr;
    }
    return &bufs[slot++];
  }
  template <class T>
  T* up(const T* host, size_t count) {
    if (rc) return nullptr;
    const size_t bytes = std::max<size_t>(count * sizeof(T), 16);
    Buf* b = next();
    if (!b || (rc = ensure(*b, bytes))) return nullptr;
    if (count) {
      hipError_t e = hipMemcpyAsync(b->p, host, count * sizeof(T), hipMemcpyHostToDevice, st);
      if (e != hipSuccess) rc = fail(OURO_EDEVICE, std::string("H2D: ") + hipGetErrorString(e));
    }
    return static_cast<T*>(b->p);
  }
  template <class T>
  T* out(size_t count) {
    if (rc) return nullptr;
    Buf* b = next();
    if (!b || (rc = ensure(*b, std::max<size_t>(count * sizeof(T), 16)))) return nullptr;
    return static_cast<T*>(b->p);
  }
};

// Window of a batch (see struct Window); EINVAL when an offset + length
// overflows.
int window_of(size_t n, const uint64_t* off, const uint32_t* len, Window* w) {
  uint64_t lo = ~0ull, hi = 0;
  for (size_t i = 0; i < n; i++) {
    if (!len[i]) continue;
    const uint64_t e = off[i] + len[i];
    if (e < off[i]) return fail(OURO_EINVAL, "offset + length overflows");
    lo = std::min(lo, off[i]);
    hi = std::max(hi, e);
  }
  if (hi == 0) lo = 0;
  w->lo = lo;
  w->hi = hi;
  w->off.resize(n);
  for (size_t i = 0; i < n; i++) w->off[i] = len[i] ? off[i] - lo : 0;
  return OURO_OK;
}

int finish(hipStream_t st) {
  OURO_HIP(hipStreamSynchronize(st));
  return OURO_OK;
}

int download(hipStream_t st, void* host, const void* dev, size_t bytes) {
  if (!host || !bytes) return OURO_OK;
  OURO_HIP(hipMemcpyAsync(host, dev, bytes, hipMemcpyDeviceToHost, st));
  return OURO_OK;
}

// ---- header batches ----
// The required members present?  (The alphas only when the batch has no slots.)
int check_hdr_batch(const ouro_tpraos_batch* b) {
  if (!b->issuer_vk || !b->vrf_vk || !b->eta_proof || !b->leader_proof || !b->hot_vk ||
      !b->ocert_counter || !b->ocert_kes_period || !b->ocert_sigma || !b->kes_t || !b->kes_sig ||
      !b->body_off || !b->body_len)
    return fail(OURO_EINVAL, "null argument");
  if (!b->slot && (!b->eta_alpha || !b->leader_alpha))
    return fail(OURO_EINVAL, "null alpha (and no slots to derive it from)");
  return OURO_OK;
}

int stage_hdr(Stager& sg, const ouro_tpraos_batch* b, size_t lo, size_t m, StagedHdr* s) {
  int rc = window_of(m, b->body_off + lo, b->body_len + lo, &s->body);
  if (rc) return rc;
  const size_t span = s->body.span();
  if (span && !b->body) return fail(OURO_EINVAL, "null body buffer");
  ouro_tpraos_batch& d = s->d;
  d = ouro_tpraos_batch{};
  d.n = m;
  d.issuer_vk = sg.up(b->issuer_vk + 32 * lo, 32 * m);
  d.vrf_vk = sg.up(b->vrf_vk + 32 * lo, 32 * m);
  d.eta_proof = sg.up(b->eta_proof + 80 * lo, 80 * m);
  d.leader_proof = sg.up(b->leader_proof + 80 * lo, 80 * m);
  if (b->slot) {
    d.slot = sg.up(b->slot + lo, m);
    if (b->epoch_nonce) d.epoch_nonce = sg.up(b->epoch_nonce, 32);
  } else {
    d.eta_alpha = sg.up(b->eta_alpha + 32 * lo, 32 * m);
    d.leader_alpha = sg.up(b->leader_alpha + 32 * lo, 32 * m);
  }
  d.hot_vk = sg.up(b->hot_vk + 32 * lo, 32 * m);
  d.ocert_counter = sg.up(b->ocert_counter + lo, m);
  d.ocert_kes_period = sg.up(b->ocert_kes_period + lo, m);
  d.ocert_sigma = sg.up(b->ocert_sigma + 64 * lo, 64 * m);
  d.kes_t = sg.up(b->kes_t + lo, m);
  d.kes_sig = sg.up(b->kes_sig + 448 * lo, 448 * m);
  d.body = sg.up(span ? b->body + s->body.lo : b->body, span);
  d.body_off = sg.up(s->body.off.data(), m);
  d.body_len = sg.up(b->body_len + lo, m);
  if (b->eta_output) d.eta_output = sg.up(b->eta_output + 64 * lo, 64 * m);
  if (b->leader_output) d.leader_output = sg.up(b->leader_output + 64 * lo, 64 * m);
  s->ver = sg.out<uint8_t>(m);
  s->be = sg.out<uint8_t>(64 * m);
  s->bl = sg.out<uint8_t>(64 * m);
  if (b->eta_nonce) d.eta_nonce = s->nonce = sg.out<uint8_t>(32 * m);
  return sg.rc;
}

}  // namespace

// ---------------------------------------------------------------- C ABI ------
extern "C" {

int ouro_set_device(int device) {
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || device < 0 || device >= count)
    return fail(OURO_ENODEV, "no such device");
  t_device = device;
  return OURO_OK;
}

const char* ouro_last_error(void) { return t_last_error.c_str(); }

}  // extern "C"

namespace {
int ed_batch_host(size_t n, const uint8_t* pk, const uint8_t* sig, const uint8_t* msg,
                  const uint64_t* msg_off, const uint32_t* msg_len, uint8_t* verdict,
                  uint32_t byron) {
  if (n == 0) return OURO_OK;
  if (!pk || !sig || !msg_off || !msg_len || !verdict) return fail(OURO_EINVAL, "null argument");
  hipStream_t st;
  int rc = thread_stream(&st);
  if (rc) return rc;
  Window w;
  if ((rc = window_of(n, msg_off, msg_len, &w))) return rc;
  if (w.span() && !msg) return fail(OURO_EINVAL, "null message buffer");
  Stager sg{st};
  auto dpk = sg.up(pk, 32 * n);
  auto dsig = sg.up(sig, 64 * n);
  auto dmsg = sg.up(w.span() ? msg + w.lo : msg, w.span());
  auto doff = sg.up(w.off.data(), n);
  auto dlen = sg.up(msg_len, n);
  auto dver = sg.out<uint8_t>(n);
  if (sg.rc) return sg.rc;
  if ((rc = launch_ed(st, n, dpk, dsig, dmsg, doff, dlen, dver, byron))) return rc;
  std::vector<uint8_t> tmp(n);
  if ((rc = download(st, tmp.data(), dver, n))) return rc;
  if ((rc = finish(st))) return rc;
  memcpy(verdict, tmp.data(), n);
  return OURO_OK;
}
}  // namespace

extern "C" {

int ouro_ed25519_verify_batch(size_t n, const uint8_t* pk, const uint8_t* sig, const uint8_t* msg,
                              const uint64_t* msg_off, const uint32_t* msg_len, uint8_t* verdict) {
  return or_host(ed_batch_host(n, pk, sig, msg, msg_off, msg_len, verdict, 0), [&] {
    return ouro_host::ed_batch(n, pk, sig, msg, msg_off, msg_len, verdict, 0);
  });
}

int ouro_byron_ed25519_verify_batch(size_t n, const uint8_t* pk, const uint8_t* sig,
                                    const uint8_t* msg, const uint64_t* msg_off,
                                    const uint32_t* msg_len, uint8_t* verdict) {
  return or_host(ed_batch_host(n, pk, sig, msg, msg_off, msg_len, verdict, 1), [&] {
    return ouro_host::ed_batch(n, pk, sig, msg, msg_off, msg_len, verdict, 1);
  });
}


int ouro_vrf03_verify_batch(size_t n, const uint8_t* pk, const uint8_t* proof, const uint8_t* alpha,
                            const uint64_t* alpha_off, const uint32_t* alpha_len, uint8_t* beta,
                            uint8_t* verdict) {
  return ouro_vrf03_verify_batch_flags(n, pk, proof, alpha, alpha_off, alpha_len, beta, verdict, 0);
}

}  // extern "C"

namespace {
int vrf_batch_dev(size_t n, const uint8_t* pk, const uint8_t* proof, const uint8_t* alpha,
                  const uint64_t* alpha_off, const uint32_t* alpha_len, uint8_t* beta,
                  uint8_t* verdict, uint32_t flags) {
  if (n == 0) return OURO_OK;
  if (flags & ~OURO_VRF_STRICT_S) return fail(OURO_EINVAL, "unknown VRF flags");
  if (!pk || !proof || !alpha_off || !alpha_len || !verdict) return fail(OURO_EINVAL, "null argument");
  hipStream_t st;
  int rc = thread_stream(&st);
  if (rc) return rc;
  Window w;
  if ((rc = window_of(n, alpha_off, alpha_len, &w))) return rc;
  if (w.span() && !alpha) return fail(OURO_EINVAL, "null alpha buffer");
  Stager sg{st};
  auto dpk = sg.up(pk, 32 * n);
  auto dpi = sg.up(proof, 80 * n);
  auto dal = sg.up(w.span() ? alpha + w.lo : alpha, w.span());
  auto doff = sg.up(w.off.data(), n);
  auto dlen = sg.up(alpha_len, n);
  auto dbeta = sg.out<uint8_t>(64 * n);
  auto dver = sg.out<uint8_t>(n);
  if (sg.rc) return sg.rc;
  if ((rc = launch_vrf(st, n, dpk, dpi, dal, doff, dlen, dbeta, dver, flags))) return rc;
  std::vector<uint8_t> tv(n), tb(beta ? 64 * n : 0);
  if ((rc = download(st, tv.data(), dver, n))) return rc;
  if (beta && (rc = download(st, tb.data(), dbeta, 64 * n))) return rc;
  if ((rc = finish(st))) return rc;
  memcpy(verdict, tv.data(), n);
  if (beta) memcpy(beta, tb.data(), 64 * n);
  return OURO_OK;
}

int kes_batch_dev(size_t n, const uint8_t* vk, const uint32_t* t, const uint8_t* msg,
                  const uint64_t* msg_off, const uint32_t* msg_len, const uint8_t* sig,
                  uint8_t* verdict) {
  if (n == 0) return OURO_OK;
  if (!vk || !t || !msg_off || !msg_len || !sig || !verdict) return fail(OURO_EINVAL, "null argument");
  hipStream_t st;
  int rc = thread_stream(&st);
  if (rc) return rc;
  Window w;
  if ((rc = window_of(n, msg_off, msg_len, &w))) return rc;
  if (w.span() && !msg) return fail(OURO_EINVAL, "null message buffer");
  Stager sg{st};
  auto dvk = sg.up(vk, 32 * n);
  auto dt = sg.up(t, n);
  auto dmsg = sg.up(w.span() ? msg + w.lo : msg, w.span());
  auto doff = sg.up(w.off.data(), n);
  auto dlen = sg.up(msg_len, n);
  auto dsig = sg.up(sig, 448 * n);
  auto dver = sg.out<uint8_t>(n);
  if (sg.rc) return sg.rc;
  if ((rc = launch_kes(st, n, dvk, dt, dmsg, doff, dlen, dsig, dver))) return rc;
  std::vector<uint8_t> tv(n);
  if ((rc = download(st, tv.data(), dver, n))) return rc;
  if ((rc = finish(st))) return rc;
  memcpy(verdict, tv.data(), n);
  return OURO_OK;
}
}  // namespace

extern "C" {

int ouro_vrf03_verify_batch_flags(size_t n, const uint8_t* pk, const uint8_t* proof,
                                  const uint8_t* alpha, const uint64_t* alpha_off,
                                  const uint32_t* alpha_len, uint8_t* beta, uint8_t* verdict,
                                  uint32_t flags) {
  return or_host(vrf_batch_dev(n, pk, proof, alpha, alpha_off, alpha_len, beta, verdict, flags),
                 [&] {
                   return ouro_host::vrf_batch(n, pk, proof, alpha, alpha_off, alpha_len, beta,
                                               verdict, flags);
                 });
}

int ouro_sum6kes_verify_batch(size_t n, const uint8_t* vk, const uint32_t* t, const uint8_t* msg,
                              const uint64_t* msg_off, const uint32_t* msg_len, const uint8_t* sig,
                              uint8_t* verdict) {
  return or_host(kes_batch_dev(n, vk, t, msg, msg_off, msg_len, sig, verdict), [&] {
    return ouro_host::kes_batch(n, vk, t, msg, msg_off, msg_len, sig, verdict);
  });
}

}  // extern "C"

namespace {
// ---- pipelined host-buffer header batches (PipeSlot / Pipe above) ----
int pipe_of(int dev, Pipe** out) {
  Pipe& p = ctx_of(dev).pipe;
  if (!p.ready) {
    for (PipeSlot& q : p.s) {
      if (!q.st) OURO_HIP(hipStreamCreateWithFlags(&q.st, hipStreamNonBlocking));
      if (!q.done) OURO_HIP(hipEventCreateWithFlags(&q.done, hipEventDisableTiming));
    }
    p.ready = true;
  }
  *out = &p;
  return OURO_OK;
}

struct HdrOut {
  uint8_t *verdict, *beta_eta, *beta_leader, *eta_nonce;
};

int pipe_drain(PipeSlot& p, const HdrOut& o) {
  if (!p.busy) return OURO_OK;
  p.busy = false;
  OURO_HIP(hipEventSynchronize(p.done));
  const size_t m = p.m;
  memcpy(o.verdict + p.lo, p.h_out, m);
  if (o.beta_eta) memcpy(o.beta_eta + 64 * p.lo, p.h_out + m, 64 * m);
  if (o.beta_leader) memcpy(o.beta_leader + 64 * p.lo, p.h_out + 65 * m, 64 * m);
  if (o.eta_nonce) memcpy(o.eta_nonce + 32 * p.lo, p.h_out + 129 * m, 32 * m);
  return OURO_OK;
}

int pipe_chunk(PipeSlot& p, const ouro_tpraos_batch* b, size_t lo, size_t m, const HdrOut& o) {
  Stager sg{p.st};
  sg.bufs = p.in;
  sg.nbufs = (int)(sizeof(p.in) / sizeof(p.in[0]));
  int rc = stage_hdr(sg, b, lo, m, &p.staged);
  if (rc) return rc;
  const StagedHdr& s = p.staged;
  if ((rc = launch_hdr(p.st, s.d, s.ver, s.be, s.bl))) return rc;
  if (p.h_cap < kOutRow * m) {
    if (p.h_out) OURO_HIP(hipHostFree(p.h_out));
    p.h_out = nullptr;
    p.h_cap = 0;
    // (hipHostMallocNumaUser: on the calling thread's NUMA policy -- a
    // multi-device worker is bound to its GPU's node, numa.cpp)
    OURO_HIP(hipHostMalloc(reinterpret_cast<void**>(&p.h_out), kOutRow * m, hipHostMallocNumaUser));
    p.h_cap = kOutRow * m;
  }
  OURO_HIP(hipMemcpyAsync(p.h_out, s.ver, m, hipMemcpyDeviceToHost, p.st));
  if (o.beta_eta) OURO_HIP(hipMemcpyAsync(p.h_out + m, s.be, 64 * m, hipMemcpyDeviceToHost, p.st));
  if (o.beta_leader)
    OURO_HIP(hipMemcpyAsync(p.h_out + 65 * m, s.bl, 64 * m, hipMemcpyDeviceToHost, p.st));
  if (o.eta_nonce)
    OURO_HIP(hipMemcpyAsync(p.h_out + 129 * m, s.nonce, 32 * m, hipMemcpyDeviceToHost, p.st));
  OURO_HIP(hipEventRecord(p.done, p.st));
  p.lo = lo;
  p.m = m;
  p.busy = true;
  return OURO_OK;
}

// headers per chunk: one full grid of the header kernel (OURO_HOST_CHUNK
// overrides; 0 = the whole batch in one piece)
size_t host_chunk(DeviceState* ds) {
  const long long v = ouro_knobs::get().host_chunk.load(std::memory_order_relaxed);
  return v >= 0 ? (size_t)v : (size_t)ds->max_blocks[kHdr] * kBlock;
}

int hdr_batch_pipelined(const ouro_tpraos_batch* b, size_t chunk, const HdrOut& o) {
  int dev, rc = current_device(&dev);
  if (rc) return rc;
  Pipe* pp;
  if ((rc = pipe_of(dev, &pp))) return rc;
  size_t c = 0;
  for (size_t lo = 0; lo < b->n && !rc; lo += chunk, c++) {
    PipeSlot& p = pp->s[c & 1];
    rc = pipe_drain(p, o);
    if (!rc) rc = pipe_chunk(p, b, lo, std::min(chunk, b->n - lo), o);
  }
  // older chunk first; on an error, still wait for everything in flight
  for (int k = 0; k < 2; k++) {
    PipeSlot& p = pp->s[(c + k) & 1];
    if (rc) {
      (void)hipStreamSynchronize(p.st);
      p.busy = false;
    } else {
      rc = pipe_drain(p, o);
    }
  }
  return rc;
}

// one synchronous launch of the whole batch (throughput kernel, or the
// latency-mode kernels with lowlat), results copied out after the sync
int hdr_batch_once(const ouro_tpraos_batch* b, const HdrOut& o, bool lowlat) {
  const size_t n = b->n;
  hipStream_t st;
  int rc = thread_stream(&st);
  if (rc) return rc;
  DeviceState* ds;
  if ((rc = device_state(&ds))) return rc;
  Stager sg{st};
  StagedHdr s;
  if ((rc = stage_hdr(sg, b, 0, n, &s))) return rc;
  if (lowlat) {
    // {n, option bits, generation (arrive_last; res is zeroed below), 0}
    const uint32_t nw[4] = {(uint32_t)n, batch_opts(s.d), 1u, 0u};
    const uint32_t* d_n = sg.up(nw, 4);
    int32_t* res = sg.out<int32_t>(slot_region_words(n, kLatResWords));
    int32_t* scr = sg.out<int32_t>(lowlat_scratch_words(ds, n));
    if (sg.rc) return sg.rc;
    // the arrival records are generation-tagged (generation 1 here) and never
    // reset by the kernel: this one-shot buffer starts from zero
    OURO_HIP(hipMemsetAsync(res, 0, sizeof(int32_t) * slot_region_words(n, kLatResWords), st));
    // (nw is read by the H2D above; this frame outlives the sync below)
    if ((rc = launch_lowlat(st, s.d, d_n, n, res, scr, s.ver, s.be, s.bl))) return rc;
  } else if ((rc = launch_hdr(st, s.d, s.ver, s.be, s.bl))) {
    return rc;
  }
  std::vector<uint8_t> tv(n), te(o.beta_eta ? 64 * n : 0), tl(o.beta_leader ? 64 * n : 0),
      tn(o.eta_nonce ? 32 * n : 0);
  if ((rc = download(st, tv.data(), s.ver, n))) return rc;
  if (o.beta_eta && (rc = download(st, te.data(), s.be, 64 * n))) return rc;
  if (o.beta_leader && (rc = download(st, tl.data(), s.bl, 64 * n))) return rc;
  if (o.eta_nonce && (rc = download(st, tn.data(), s.nonce, 32 * n))) return rc;
  if ((rc = finish(st))) return rc;
  memcpy(o.verdict, tv.data(), n);
  if (o.beta_eta) memcpy(o.beta_eta, te.data(), 64 * n);
  if (o.beta_leader) memcpy(o.beta_leader, tl.data(), 64 * n);
  if (o.eta_nonce) memcpy(o.eta_nonce, tn.data(), 32 * n);
  return OURO_OK;
}
}  // namespace

extern "C" {

int ouro_tpraos_verify_batch(const ouro_tpraos_batch* b, uint8_t* verdict, uint8_t* beta_eta,
                             uint8_t* beta_leader) {
  if (!b) return fail(OURO_EINVAL, "null batch");
  if (b->n == 0) return OURO_OK;
  if (!verdict) return fail(OURO_EINVAL, "null verdict");
  int rc = check_hdr_batch(b);
  if (rc) return rc;
  DeviceState* ds;
  if ((rc = device_state(&ds))) return rc;
  const HdrOut o{verdict, beta_eta, beta_leader, b->eta_nonce};
  const size_t chunk = host_chunk(ds);
  rc = chunk && b->n > chunk ? hdr_batch_pipelined(b, chunk, o) : hdr_batch_once(b, o, false);
  return or_host(rc, [&] { return ouro_host::hdr_batch(b, verdict, beta_eta, beta_leader); });
}

// ---- latency mode (ChainSync windows) ----
int ouro_tpraos_verify_batch_lowlat(const ouro_tpraos_batch* b, uint8_t* verdict,
                                    uint8_t* beta_eta, uint8_t* beta_leader) {
  if (!b) return fail(OURO_EINVAL, "null batch");
  if (b->n == 0) return OURO_OK;
  if (b->n > 0xffffffffu) return fail(OURO_EINVAL, "batch too large");
  if (!verdict) return fail(OURO_EINVAL, "null verdict");
  int rc = check_hdr_batch(b);
  if (rc) return rc;
  return or_host(hdr_batch_once(b, HdrOut{verdict, beta_eta, beta_leader, b->eta_nonce}, true),
                 [&] { return ouro_host::hdr_batch(b, verdict, beta_eta, beta_leader); });
}

int ouro_nonce_fold(size_t n, const uint8_t* eta_nonce, const uint64_t* slot,
                    uint64_t first_slot_next_epoch, uint64_t stability_window, uint8_t* eta_v,
                    uint8_t* eta_c, int* is_neutral) {
  if (n == 0) return OURO_OK;
  if (!eta_nonce || !slot || !eta_v || !eta_c) return fail(OURO_EINVAL, "null argument");
  bool v_neutral = is_neutral && is_neutral[0], c_neutral = is_neutral && is_neutral[1];
  uint32_t v[8], c[8];
  memcpy(v, eta_v, 32);
  memcpy(c, eta_c, 32);
  for (size_t i = 0; i < n; i++) {
    // eta_v <- eta_v (*) eta, with NeutralNonce (*) x = x
    uint32_t in[16];
    memcpy(in + 8, eta_nonce + 32 * i, 32);
    if (v_neutral) {
      memcpy(v, in + 8, 32);
    } else {
      memcpy(in, v, 32);
      blake2b256_64(v, in);
    }
    v_neutral = false;
    // UPDN: s +* Duration sp < firstSlotNextEpoch (Word64 arithmetic, as SlotNo)
    if (slot[i] + stability_window < first_slot_next_epoch) {
      memcpy(c, v, 32);
      c_neutral = false;
    }
  }
  memcpy(eta_v, v, 32);
  memcpy(eta_c, c, 32);
  if (is_neutral) {
    is_neutral[0] = v_neutral;
    is_neutral[1] = c_neutral;
  }
  return OURO_OK;
}

int ouro_leader_check_batch(size_t n, const uint8_t* beta, const uint64_t* sigma_num,
                            const uint64_t* sigma_den, int64_t act_log_hi, uint64_t act_log_lo,
                            int f_is_one, uint8_t* verdict) {
  if (n == 0) return OURO_OK;
  if (!beta || !sigma_num || !sigma_den || !verdict) return fail(OURO_EINVAL, "null argument");
  auto dev = [&]() -> int {
    hipStream_t st;
    int rc = thread_stream(&st);
    if (rc) return rc;
    Stager sg{st};
    auto dbeta = sg.up(beta, 64 * n);
    auto dnum = sg.up(sigma_num, n);
    auto dden = sg.up(sigma_den, n);
    auto dver = sg.out<uint8_t>(n);
    if (sg.rc) return sg.rc;
    if ((rc = launch_leader(st, n, dbeta, dnum, dden, act_log_hi, act_log_lo, f_is_one, dver)))
      return rc;
    std::vector<uint8_t> tv(n);
    if ((rc = download(st, tv.data(), dver, n))) return rc;
    if ((rc = finish(st))) return rc;
    memcpy(verdict, tv.data(), n);
    return OURO_OK;
  };
  return or_host(dev(), [&] {
    return ouro_host::leader_batch(n, beta, sigma_num, sigma_den, act_log_hi, act_log_lo, f_is_one,
                                   verdict);
  });
}

// ---- single item: a batch of one (ABI-identical to the symbols replaced) ----
int ouro_ed25519_verify(const unsigned char* sig, const unsigned char* m, unsigned long long mlen,
                        const unsigned char* pk) {
  if (!sig || !pk || (mlen && !m)) return OURO_INVALID;
  const uint64_t off = 0;
  const uint32_t len = (uint32_t)mlen;
  if ((unsigned long long)len != mlen) return fail(OURO_EINVAL, "message too long");
  uint8_t v = 0;
  static const uint8_t empty[1] = {0};
  int rc;
  if (single_on_gpu()) {
    rc = ouro_ed25519_verify_batch(1, pk, sig, mlen ? m : empty, &off, &len, &v);
  } else {
    g_host_single++;
    rc = ouro_host::ed_batch(1, pk, sig, mlen ? m : empty, &off, &len, &v, 0);
  }
  if (rc) return rc;
  return v ? OURO_OK : OURO_INVALID;
}

int ouro_byron_ed25519_verify(const unsigned char* m, size_t mlen, const unsigned char* pk,
                              const unsigned char* sig) {
  if (!sig || !pk || (mlen && !m)) return OURO_INVALID;
  const uint64_t off = 0;
  const uint32_t len = (uint32_t)mlen;
  if ((size_t)len != mlen) return fail(OURO_EINVAL, "message too long");
  uint8_t v = 0;
  static const uint8_t empty[1] = {0};
  int rc;
  if (single_on_gpu()) {
    rc = ouro_byron_ed25519_verify_batch(1, pk, sig, mlen ? m : empty, &off, &len, &v);
  } else {
    g_host_single++;
    rc = ouro_host::ed_batch(1, pk, sig, mlen ? m : empty, &off, &len, &v, 1);
  }
  if (rc) return rc;
  return v ? OURO_OK : OURO_INVALID;
}

int ouro_vrf03_verify(unsigned char* output, const unsigned char* pk, const unsigned char* proof,
                      const unsigned char* msg, unsigned long long msglen) {
  if (!pk || !proof || (msglen && !msg)) return OURO_INVALID;
  const uint64_t off = 0;
  const uint32_t len = (uint32_t)msglen;
  if ((unsigned long long)len != msglen) return fail(OURO_EINVAL, "message too long");
  uint8_t v = 0, beta[64];
  static const uint8_t empty[1] = {0};
  int rc;
  if (single_on_gpu()) {
    rc = ouro_vrf03_verify_batch(1, pk, proof, msglen ? msg : empty, &off, &len, beta, &v);
  } else {
    g_host_single++;
    rc = ouro_host::vrf_batch(1, pk, proof, msglen ? msg : empty, &off, &len, beta, &v, 0);
  }
  if (rc) return rc;
  if (!v) return OURO_INVALID;
  if (output) memcpy(output, beta, 64);  // written only on success, like the original
  return OURO_OK;
}

int ouro_vrf03_proof_to_hash(unsigned char* output, const unsigned char* proof) {
  if (!output || !proof) return OURO_INVALID;
  if (!single_on_gpu()) {
    g_host_single++;
    return ouro_host::proof_to_hash(output, proof);
  }
  hipStream_t st;
  int rc = thread_stream(&st);
  if (rc) return rc;
  DeviceState* ds;
  if ((rc = device_state(&ds))) return rc;
  Stager sg{st};
  auto dpi = sg.up(proof, 80);
  auto dbeta = sg.out<uint8_t>(64);
  auto dver = sg.out<uint8_t>(1);
  if (sg.rc) return sg.rc;
  hipLaunchKernelGGL(k_vrf03_proof_to_hash, dim3(1), dim3(kBlock), 0, st, (size_t)1, dpi, dbeta, dver);
  if ((rc = launch_check())) return rc;
  uint8_t beta[64], v = 0;
  if ((rc = download(st, beta, dbeta, 64))) return rc;
  if ((rc = download(st, &v, dver, 1))) return rc;
  if ((rc = finish(st))) return rc;
  if (!v) return OURO_INVALID;
  memcpy(output, beta, 64);
  return OURO_OK;
}

// (The cardano-crypto-praos names are NOT exported here: the opt-in
// lib/libouro_vrf_shim.so, csrc/vrf_shim.cpp, provides them.)

int ouro_sum6kes_verify(const unsigned char* vk, unsigned int t, const unsigned char* m,
                        unsigned long long mlen, const unsigned char* sig) {
  if (!vk || !sig || (mlen && !m)) return OURO_INVALID;
  const uint64_t off = 0;
  const uint32_t len = (uint32_t)mlen;
  if ((unsigned long long)len != mlen) return fail(OURO_EINVAL, "message too long");
  uint8_t v = 0;
  const uint32_t tt = t;
  static const uint8_t empty[1] = {0};
  int rc;
  if (single_on_gpu()) {
    rc = ouro_sum6kes_verify_batch(1, vk, &tt, mlen ? m : empty, &off, &len, sig, &v);
  } else {
    g_host_single++;
    rc = ouro_host::kes_batch(1, vk, &tt, mlen ? m : empty, &off, &len, sig, &v);
  }
  if (rc) return rc;
  return v ? OURO_OK : OURO_INVALID;
}

// ---- device-resident batches ----
int ouro_ed25519_verify_batch_device(void* stream, size_t n, const uint8_t* pk, const uint8_t* sig,
                                     const uint8_t* msg, const uint64_t* msg_off,
                                     const uint32_t* msg_len, uint8_t* verdict) {
  if (n == 0) return OURO_OK;
  hipStream_t st = static_cast<hipStream_t>(stream);  // NULL = HIP's default stream
  return launch_ed(st, n, pk, sig, msg, msg_off, msg_len, verdict);
}

int ouro_byron_ed25519_verify_batch_device(void* stream, size_t n, const uint8_t* pk,
                                           const uint8_t* sig, const uint8_t* msg,
                                           const uint64_t* msg_off, const uint32_t* msg_len,
                                           uint8_t* verdict) {
  if (n == 0) return OURO_OK;
  hipStream_t st = static_cast<hipStream_t>(stream);  // NULL = HIP's default stream
  return launch_ed(st, n, pk, sig, msg, msg_off, msg_len, verdict, 1);
}

int ouro_vrf03_verify_batch_device(void* stream, size_t n, const uint8_t* pk, const uint8_t* proof,
                                   const uint8_t* alpha, const uint64_t* alpha_off,
                                   const uint32_t* alpha_len, uint8_t* beta, uint8_t* verdict) {
  if (n == 0) return OURO_OK;
  hipStream_t st = static_cast<hipStream_t>(stream);  // NULL = HIP's default stream
  return launch_vrf(st, n, pk, proof, alpha, alpha_off, alpha_len, beta, verdict);
}

int ouro_vrf03_verify_batch_device_flags(void* stream, size_t n, const uint8_t* pk,
                                         const uint8_t* proof, const uint8_t* alpha,
                                         const uint64_t* alpha_off, const uint32_t* alpha_len,
                                         uint8_t* beta, uint8_t* verdict, uint32_t flags) {
  if (n == 0) return OURO_OK;
  if (flags & ~OURO_VRF_STRICT_S) return fail(OURO_EINVAL, "unknown VRF flags");
  hipStream_t st = static_cast<hipStream_t>(stream);  // NULL = HIP's default stream
  return launch_vrf(st, n, pk, proof, alpha, alpha_off, alpha_len, beta, verdict, flags);
}

int ouro_sum6kes_verify_batch_device(void* stream, size_t n, const uint8_t* vk, const uint32_t* t,
                                     const uint8_t* msg, const uint64_t* msg_off,
                                     const uint32_t* msg_len, const uint8_t* sig,
                                     uint8_t* verdict) {
  if (n == 0) return OURO_OK;
  hipStream_t st = static_cast<hipStream_t>(stream);  // NULL = HIP's default stream
  return launch_kes(st, n, vk, t, msg, msg_off, msg_len, sig, verdict);
}

int ouro_tpraos_verify_batch_device(void* stream, const ouro_tpraos_batch* b, uint8_t* verdict,
                                    uint8_t* beta_eta, uint8_t* beta_leader) {
  if (!b) return fail(OURO_EINVAL, "null batch");
  if (b->n == 0) return OURO_OK;
  if (!beta_eta || !beta_leader) return fail(OURO_EINVAL, "device API needs both beta buffers");
  if (!verdict) return fail(OURO_EINVAL, "null verdict");
  int rc = check_hdr_batch(b);
  if (rc) return rc;
  hipStream_t st = static_cast<hipStream_t>(stream);  // NULL = HIP's default stream
  return launch_hdr(st, *b, verdict, beta_eta, beta_leader);
}

int ouro_tpraos_pack_cbor_device(void* stream, const uint8_t* raw, size_t raw_bytes,
                                 const uint64_t* off, const uint32_t* len, size_t n,
                                 uint64_t slots_per_kes_period, void* arena, size_t arena_bytes,
                                 ouro_tpraos_batch* out, uint64_t* slot, uint8_t* era,
                                 uint8_t* status) {
  if (!out || slots_per_kes_period == 0) return fail(OURO_EINVAL, "null batch / zero period");
  if (n > 0 && (!raw || !off || !len || !arena || !status)) return fail(OURO_EINVAL, "null buffer");
  if (arena_bytes < ouro_tpraos_pack_bytes(n)) return fail(OURO_EINVAL, "arena too small");
  const cbor::Out o = cbor::arena_out(cbor::arena_base(arena), n, slot, era);
  cbor::batch_from(out, o, raw, n);
  if (n == 0) return OURO_OK;
  DeviceState* ds;
  int rc = device_state(&ds);
  if (rc) return rc;
  hipStream_t st = static_cast<hipStream_t>(stream);  // NULL = HIP's default stream
  const size_t blocks = std::min<size_t>((n + kBlock - 1) / kBlock, 4096);
  hipLaunchKernelGGL(k_tpraos_pack, dim3((unsigned)blocks), dim3(kBlock), 0, st, raw, raw_bytes,
                     off, len, n, slots_per_kes_period, o, status);
  return launch_check();
}

}  // extern "C"

// ---- raw header CBOR in host memory -> verdicts in one call -----------------
// The reference's bulk callers hold raw header bytes in host memory: ChainDB's
// re-validation of a chain suffix (ouroboros-consensus/src/Ouroboros/Consensus/
// Storage/ChainDB/Impl/LgrDB.hs:350-368), ChainSync windows
// (.../MiniProtocol/ChainSync/Client.hs:792), and storage integrity on every
// block (.../Storage/VolatileDB/Impl/Parser.hs:66-85,
// .../Storage/ImmutableDB/Impl/Validation.hs:358-365).  raw_run takes such a
// batch straight through the device:
//   * the batch is cut into chunks of whole headers (OURO_CBOR_CHUNK headers,
//     default 65,536, and at most kRawChunkBytes of raw bytes each);
//   * chunk c runs on slot c % S (S = OURO_CBOR_SLOTS streams, default 6 for
//     headers, 4 for integrity):
//     the library's worker pool gathers its header spans from the caller's
//     pageable buffer into the slot's pinned, NUMA-local staging (runs of
//     adjacent spans as one memcpy; offsets rebased by a prefix sum), the
//     slot's stream uploads that block -- the raw bytes, ~1 KB per header,
//     not the 1.4 KB SoA --, runs the device slicer (k_tpraos_pack) into the
//     slot's arena, then the header kernel with mkSeed from (slot, eta0) on
//     the device (or the Sum6KES kernel, for integrity), and copies status,
//     verdicts and outputs back into pinned memory;
//   * before reusing a slot the host harvests its previous chunk into the
//     caller's buffers, so up to S chunks are in flight: the host's gathers,
//     the uploads and the other slots' kernels overlap, and the kernels of
//     neighbouring chunks share the CUs as each one's waves retire.
// A device error stops the pipeline (everything in flight is waited for) and
// the whole batch is recomputed on the host path (raw_host).
namespace {
constexpr size_t a16(size_t x) { return (x + 15) & ~(size_t)15; }
constexpr size_t kRawChunkBytes = (size_t)96 << 20;

enum RawKind { kRawHdr = 0, kRawKes = 1, kRawByron = 2 };
struct RawCall {
  RawKind kind;
  const uint8_t* raw;
  size_t raw_bytes;
  const uint64_t* off;
  const uint32_t* len;
  size_t n;
  uint64_t spkp;
  const uint8_t* eta0;           // epoch nonce (32 B), or null = NeutralNonce
  const uint8_t *ea, *la;        // explicit VRF inputs (n x 32 each), or null: mkSeed
  uint8_t* status;
  uint8_t* verdict;
  uint8_t *be, *bl, *nonce;      // optional outputs (header kind)
  int64_t magic = -1;            // Byron: the configured ProtocolMagicId (-1: each header's)
};
struct RawChunk {
  size_t lo, m, bytes;
};

// the pinned / device input block of a chunk of m headers and `bytes` raw bytes
struct RawIn {
  size_t off, len, eta0, alpha, raw, total;
};
RawIn raw_in(size_t m, size_t bytes, bool alphas) {
  RawIn l;
  l.off = 0;
  l.len = a16(8 * m);
  l.eta0 = l.len + a16(4 * m);
  l.alpha = l.eta0 + 32;
  l.raw = a16(l.alpha + (alphas ? 64 * m : 0));
  l.total = l.raw + a16(std::max<size_t>(bytes, 16));
  return l;
}
// its result block: status | verdict | beta_eta | beta_leader | eta_nonce | slot
struct RawOut {
  size_t status, verdict, be, bl, nonce, slot, total;
};
RawOut raw_out(size_t m) {
  RawOut o;
  o.status = 0;
  o.verdict = a16(m);
  o.be = o.verdict + a16(m);
  o.bl = o.be + 64 * m;
  o.nonce = o.bl + 64 * m;
  o.slot = o.nonce + 32 * m;  // device only: the slicer's slots for mkSeed
  o.total = o.slot + 8 * m;
  return o;
}
// bytes of the result block copied back
size_t raw_out_bytes(const RawCall& c, const RawOut& o, size_t m) {
  if (c.kind != kRawHdr) return o.verdict + m;
  if (c.nonce) return o.slot;
  if (c.bl) return o.nonce;
  if (c.be) return o.bl;
  return o.verdict + m;
}

// Every span inside raw (as ouro_tpraos_pack_cbor demands), and the chunks.
// a raw-CBOR knob (knobs.h; 0 = unset) if inside [lo, hi], else the default
size_t knob_size(const std::atomic<size_t>& k, size_t dflt, size_t lo, size_t hi) {
  const size_t v = k.load(std::memory_order_relaxed);
  return v && v >= lo && v <= hi ? v : dflt;
}

// Headers in chunk j when `left` headers (this chunk's included) remain.
// ramp (OURO_CBOR_RAMP=1, A/B): the first chunks a quarter and a half of
// `per`, so the first kernel starts after a short gather and upload, and the
// last ones halving down to a quarter, so the chip is not left running one
// full chunk's kernel alone at the end.  It lost: 77.5 -> 85.3 ms per 1M
// headers (profiles/r05o/cbor_ramp_ab.jsonl) -- a small chunk's kernel runs
// at a fraction of the chip with nothing beside it; off by default.
size_t raw_chunk_target(size_t j, size_t left, size_t per, bool ramp) {
  if (!ramp) return per;
  size_t t = j == 0 ? per / 4 : (j == 1 ? per / 2 : per);
  if (left <= per + per / 2) t = std::min(t, std::max(per / 4, left / 2));
  return std::max<size_t>(t, 256);
}

int raw_chunks(const RawCall& c, size_t per, std::vector<RawChunk>* out) {
  out->clear();
  const bool ramp = ouro_knobs::get().cbor_ramp.load(std::memory_order_relaxed) == 1;
  RawChunk k{0, 0, 0};
  size_t target = raw_chunk_target(0, c.n, per, ramp);
  for (size_t i = 0; i < c.n; i++) {
    if (c.off[i] > c.raw_bytes || c.raw_bytes - c.off[i] < c.len[i])
      return fail(OURO_EINVAL, "header " + std::to_string(i) + ": span outside raw_bytes");
    if (k.m && (k.m >= target || k.bytes + c.len[i] > kRawChunkBytes)) {
      out->push_back(k);
      k = RawChunk{i, 0, 0};
      target = raw_chunk_target(out->size(), c.n - i, per, ramp);
    }
    k.m++;
    k.bytes += c.len[i];
  }
  if (k.m) out->push_back(k);
  return OURO_OK;
}


// last call's phases on this thread (ouro_debug_cbor_stats)
thread_local double t_raw_stats[6] = {-1, -1, -1, -1, -1, -1};

int pinned_at_least(uint8_t** p, size_t* cap, size_t bytes) {
  if (*cap >= bytes) return OURO_OK;
  if (*p) OURO_HIP(hipHostFree(*p));
  *p = nullptr;
  *cap = 0;
  // (hipHostMallocNumaUser: the calling thread's NUMA policy -- a bench rank
  // or multi-device worker is bound to its GPU's node, numa.cpp)
  OURO_HIP(hipHostMalloc(reinterpret_cast<void**>(p), bytes, hipHostMallocNumaUser));
  *cap = bytes;
  return OURO_OK;
}

// the chunk's header spans from the caller's buffer into the slot's pinned block
int raw_stage(RawSlot& s, const RawCall& c, const RawChunk& k, int width) {
  const bool alphas = c.ea != nullptr;
  const RawIn L = raw_in(k.m, k.bytes, alphas);
  int rc = pinned_at_least(&s.h_in, &s.h_in_cap, L.total + L.total / 8);
  if (rc) return rc;
  uint64_t* noff = reinterpret_cast<uint64_t*>(s.h_in + L.off);
  uint64_t at = 0;
  for (size_t i = 0; i < k.m; i++) {
    noff[i] = at;
    at += c.len[k.lo + i];
  }
  memcpy(s.h_in + L.len, c.len + k.lo, 4 * k.m);
  if (c.eta0) memcpy(s.h_in + L.eta0, c.eta0, 32);
  if (alphas) {
    memcpy(s.h_in + L.alpha, c.ea + 32 * k.lo, 32 * k.m);
    memcpy(s.h_in + L.alpha + 32 * k.m, c.la + 32 * k.lo, 32 * k.m);
  }
  uint8_t* dst = s.h_in + L.raw;
  // tasks of ~1 MB: enough to balance, few enough to keep each memcpy long
  const size_t ntasks = std::max<size_t>(1, std::min<size_t>(k.m, k.bytes >> 20));
  const int r = ouro_pool::parallel_for(ntasks, width, [&](size_t t) {
    const size_t a = k.m * t / ntasks, b = k.m * (t + 1) / ntasks;
    for (size_t i = a; i < b;) {
      // a run of headers adjacent in the caller's buffer: one memcpy
      const uint64_t src = c.off[k.lo + i];
      uint64_t bytes = c.len[k.lo + i];
      size_t j = i + 1;
      while (j < b && c.off[k.lo + j] == src + bytes) bytes += c.len[k.lo + j++];
      memcpy(dst + noff[i], c.raw + src, bytes);
      i = j;
    }
  });
  return r ? fail(OURO_EDEVICE, "raw CBOR gather failed") : OURO_OK;
}

// the slot's stream: upload, device slicer, kernel, results back
int raw_launch(RawSlot& s, const RawCall& c, const RawChunk& k) {
  const bool alphas = c.ea != nullptr;
  const RawIn L = raw_in(k.m, k.bytes, alphas);
  const RawOut O = raw_out(k.m);
  const size_t back = raw_out_bytes(c, O, k.m);
  int rc;
  if ((rc = ensure(s.d_in, L.total)) || (rc = ensure(s.d_arena, ouro_tpraos_pack_bytes(k.m))) ||
      (rc = ensure(s.d_out, O.total)) || (rc = pinned_at_least(&s.h_out, &s.h_out_cap, back)))
    return rc;
  uint8_t* din = static_cast<uint8_t*>(s.d_in.p);
  uint8_t* dout = static_cast<uint8_t*>(s.d_out.p);
  OURO_HIP(hipMemcpyAsync(din, s.h_in, L.total, hipMemcpyHostToDevice, s.st));
  const size_t blocks = std::min<size_t>((k.m + kBlock - 1) / kBlock, 4096);
  if (c.kind == kRawByron) {
    // the device Byron slicer into the slot's arena, then the Ed25519 kernel
    // with ByronDSIGN acceptance (cardano-crypto: SURVEY.md App. B.5)
    const cbor::ByronLayout bl = cbor::byron_layout(k.m, k.bytes + cbor::kByronMsgExtra * k.m);
    if ((rc = ensure(s.d_arena, bl.total + 64))) return rc;
    const cbor::ByronOut o = cbor::byron_arena_out(cbor::arena_base(s.d_arena.p), bl);
    hipLaunchKernelGGL(k_byron_pack, dim3((unsigned)blocks), dim3(kBlock), 0, s.st, din + L.raw,
                       k.bytes, reinterpret_cast<const uint64_t*>(din + L.off),
                       reinterpret_cast<const uint32_t*>(din + L.len), k.m, c.magic, o,
                       dout + O.status);
    if ((rc = launch_check())) return rc;
    if ((rc = launch_ed(s.st, k.m, o.pk, o.sig, o.msg, o.msg_off, o.msg_len, dout + O.verdict, 1)))
      return rc;
    OURO_HIP(hipMemcpyAsync(s.h_out, dout, back, hipMemcpyDeviceToHost, s.st));
    OURO_HIP(hipEventRecord(s.done, s.st));
    s.lo = k.lo;
    s.m = k.m;
    s.busy = true;
    return OURO_OK;
  }
  uint64_t* dslot = reinterpret_cast<uint64_t*>(dout + O.slot);
  const bool seeds = c.kind == kRawHdr && !alphas;
  const cbor::Out o = cbor::arena_out(cbor::arena_base(s.d_arena.p), k.m, seeds ? dslot : nullptr,
                                      nullptr);
  const uint8_t* draw = din + L.raw;
  hipLaunchKernelGGL(k_tpraos_pack, dim3((unsigned)blocks), dim3(kBlock), 0, s.st, draw, k.bytes,
                     reinterpret_cast<const uint64_t*>(din + L.off),
                     reinterpret_cast<const uint32_t*>(din + L.len), k.m, c.spkp, o,
                     dout + O.status);
  if ((rc = launch_check())) return rc;
  ouro_tpraos_batch b{};
  cbor::batch_from(&b, o, draw, k.m);
  if (c.kind == kRawKes) {
    rc = launch_kes(s.st, k.m, b.hot_vk, b.kes_t, b.body, b.body_off, b.body_len, b.kes_sig,
                    dout + O.verdict);
  } else {
    if (alphas) {
      b.eta_alpha = din + L.alpha;
      b.leader_alpha = din + L.alpha + 32 * k.m;
    } else {
      b.slot = dslot;
      b.epoch_nonce = c.eta0 ? din + L.eta0 : nullptr;
    }
    if (c.nonce) b.eta_nonce = dout + O.nonce;
    rc = launch_hdr(s.st, b, dout + O.verdict, dout + O.be, dout + O.bl);
  }
  if (rc) return rc;
  OURO_HIP(hipMemcpyAsync(s.h_out, dout, back, hipMemcpyDeviceToHost, s.st));
  OURO_HIP(hipEventRecord(s.done, s.st));
  s.lo = k.lo;
  s.m = k.m;
  s.busy = true;
  return OURO_OK;
}

// the slot's finished chunk into the caller's buffers
int raw_drain(RawSlot& s, const RawCall& c) {
  if (!s.busy) return OURO_OK;
  s.busy = false;
  OURO_HIP(hipEventSynchronize(s.done));
  const RawOut O = raw_out(s.m);
  const uint8_t* st = s.h_out + O.status;
  const uint8_t* v = s.h_out + O.verdict;
  memcpy(c.status + s.lo, st, s.m);
  if (c.kind == kRawByron) {
    // PBFT accepts an epoch-boundary header without a signature
    // (ouroboros-consensus/src/Ouroboros/Consensus/Protocol/PBFT.hs:327-328)
    for (size_t i = 0; i < s.m; i++)
      c.verdict[s.lo + i] = st[i] == OURO_PACK_EBB ? 1 : (st[i] == OURO_PACK_OK && v[i] ? 1 : 0);
    return OURO_OK;
  }
  // a header the slicer rejected is invalid (its zeroed row cannot verify;
  // masked so that no bit at all is set for it)
  for (size_t i = 0; i < s.m; i++) c.verdict[s.lo + i] = st[i] == OURO_PACK_OK ? v[i] : 0;
  if (c.kind == kRawHdr) {
    if (c.be) memcpy(c.be + 64 * s.lo, s.h_out + O.be, 64 * s.m);
    if (c.bl) memcpy(c.bl + 64 * s.lo, s.h_out + O.bl, 64 * s.m);
    if (c.nonce) memcpy(c.nonce + 32 * s.lo, s.h_out + O.nonce, 32 * s.m);
  }
  return OURO_OK;
}

int raw_run(const RawCall& c, const std::vector<RawChunk>& chunks) {
  using clk = std::chrono::steady_clock;
  const auto t0 = clk::now();
  double gather_ms = 0, wait_ms = 0;
  DeviceState* ds;
  int dev, rc = device_state(&ds);
  if (rc || (rc = current_device(&dev))) return rc;
  RawPipe& p = ctx_of(dev).raw;
  // chunks in flight: the header kernel wants ~3 grids of work queued (6 x
  // 64 K headers); the Sum6KES kernel is PCIe-bound, 4 suffice
  // (profiles/r05a/cbor_sweep.jsonl); Byron's Ed25519 runs best with 5
  // (66.7--67.1 M headers/s against ~61 with 4 and 60--68 with 6, interleaved
  // on one box: profiles/r06k/byron_ab.jsonl)
  const int S = (int)knob_size(ouro_knobs::get().cbor_slots, c.kind == kRawHdr ? 6 : (c.kind == kRawByron ? 5 : 4), 1,
                                kRawMaxSlots);
  for (int k = 0; k < S; k++) {
    RawSlot& s = p.s[k];
    if (!s.st) OURO_HIP(hipStreamCreateWithFlags(&s.st, hipStreamNonBlocking));
    if (!s.done) OURO_HIP(hipEventCreateWithFlags(&s.done, hipEventDisableTiming));
  }
  const int width = (int)knob_size(ouro_knobs::get().cbor_copy_threads, 8, 1, 64);
  size_t ci = 0;
  for (; ci < chunks.size() && !rc; ci++) {
    RawSlot& s = p.s[ci % S];
    const auto a = clk::now();
    rc = raw_drain(s, c);
    const auto b = clk::now();
    if (!rc) rc = raw_stage(s, c, chunks[ci], width);
    const auto d = clk::now();
    if (!rc) rc = raw_launch(s, c, chunks[ci]);
    wait_ms += std::chrono::duration<double, std::milli>(b - a).count();
    gather_ms += std::chrono::duration<double, std::milli>(d - b).count();
  }
  // the rest in chunk order; after an error, wait for everything in flight
  for (int k = 0; k < S; k++) {
    RawSlot& s = p.s[(ci + k) % S];
    if (rc) {
      (void)hipStreamSynchronize(s.st);
      s.busy = false;
    } else {
      const auto a = clk::now();
      rc = raw_drain(s, c);
      wait_ms += std::chrono::duration<double, std::milli>(clk::now() - a).count();
    }
  }
  const double total = std::chrono::duration<double, std::milli>(clk::now() - t0).count();
  const double st[6] = {total, gather_ms, wait_ms, (double)chunks.size(), (double)S, (double)width};
  memcpy(t_raw_stats, st, sizeof st);
  return rc;
}

// the host path over the same batch: host slicer + host verification, in
// chunks (no batch-sized arena), results straight into the caller's buffers
int raw_host_byron(const RawCall& c) {
  const size_t C = 1 << 16;
  for (size_t lo = 0; lo < c.n; lo += C) {
    const size_t m = std::min(C, c.n - lo);
    const size_t nb = ouro_byron_pack_bytes(m, c.len + lo);
    std::unique_ptr<uint8_t[]> arena(new (std::nothrow) uint8_t[nb]);  // every row written
    if (!arena) return fail(OURO_EDEVICE, "raw Byron host path: out of host memory");
    ouro_byron_batch b;
    int rc = ouro_byron_pack_cbor(c.raw, c.raw_bytes, c.off + lo, c.len + lo, m, c.magic,
                                  arena.get(), nb, &b, c.status + lo, 0);
    if (rc) return fail(rc, "ouro_byron_pack_cbor: bad arguments");
    if ((rc = ouro_host::ed_batch(m, b.pk, b.sig, b.msg, b.msg_off, b.msg_len, c.verdict + lo, 1)))
      return fail(rc, "raw Byron host path failed");
    for (size_t i = lo; i < lo + m; i++)
      c.verdict[i] = c.status[i] == OURO_PACK_EBB ? 1
                                                  : (c.status[i] == OURO_PACK_OK && c.verdict[i]);
  }
  return OURO_OK;
}

int raw_host(const RawCall& c) {
  if (c.kind == kRawByron) return raw_host_byron(c);
  const size_t C = 1 << 16;
  const size_t cap = std::min(C, c.n);
  const size_t nb = ouro_tpraos_pack_bytes(cap);
  std::unique_ptr<uint8_t[]> arena(new (std::nothrow) uint8_t[nb]);
  std::unique_ptr<uint64_t[]> slots(new (std::nothrow) uint64_t[cap]);
  if (!arena || !slots) return fail(OURO_EDEVICE, "raw CBOR host path: out of host memory");
  for (size_t lo = 0; lo < c.n; lo += C) {
    const size_t m = std::min(C, c.n - lo);
    ouro_tpraos_batch b{};  // (the slicer sets the required members only)
    int rc = ouro_tpraos_pack_cbor(c.raw, c.raw_bytes, c.off + lo, c.len + lo, m, c.spkp,
                                   arena.get(), nb, &b, slots.get(), nullptr, c.status + lo, 0);
    if (rc) return fail(rc, "ouro_tpraos_pack_cbor: bad arguments");
    if (c.kind == kRawKes) {
      rc = ouro_host::kes_batch(m, b.hot_vk, b.kes_t, b.body, b.body_off, b.body_len, b.kes_sig,
                                c.verdict + lo);
    } else {
      if (c.ea) {
        b.eta_alpha = c.ea + 32 * lo;
        b.leader_alpha = c.la + 32 * lo;
      } else {
        b.slot = slots.get();
        b.epoch_nonce = c.eta0;
      }
      if (c.nonce) b.eta_nonce = c.nonce + 32 * lo;
      rc = ouro_host::hdr_batch(&b, c.verdict + lo, c.be ? c.be + 64 * lo : nullptr,
                                c.bl ? c.bl + 64 * lo : nullptr);
    }
    if (rc) return fail(rc, "raw CBOR host path failed");
    for (size_t i = lo; i < lo + m; i++)
      if (c.status[i] != OURO_PACK_OK) c.verdict[i] = 0;
  }
  return OURO_OK;
}

int raw_verify(const RawCall& c) {
  if (c.n == 0) return OURO_OK;
  if (!c.raw || !c.off || !c.len || !c.status || !c.verdict)
    return fail(OURO_EINVAL, "null argument");
  if (c.kind != kRawByron && c.spkp == 0) return fail(OURO_EINVAL, "zero slots per KES period");
  if (c.kind == kRawByron && (c.magic < -1 || c.magic > (int64_t)0xffffffffll))
    return fail(OURO_EINVAL, "protocol magic outside Word32 (or -1)");
  if ((c.ea == nullptr) != (c.la == nullptr))
    return fail(OURO_EINVAL, "give both VRF input arrays or neither");
  std::vector<RawChunk> chunks;
  const size_t per = knob_size(ouro_knobs::get().cbor_chunk, 65536, 256, (size_t)1 << 24);
  int rc = raw_chunks(c, per, &chunks);
  if (rc) return rc;
  return or_host(raw_run(c, chunks), [&] { return raw_host(c); });
}
}  // namespace

extern "C" {

// ---- storage integrity (KES only) over raw headers ----
// verifyHeaderIntegrity (ouroboros-consensus-shelley/src/Ouroboros/Consensus/
// Shelley/Ledger/Integrity.hs:20-44): Sum6KES of the raw header body under the
// opcert's hot key at t = kesPeriod(slot) - c0 (0 below c0) -- the check the
// VolatileDB parser runs on every block at open
// (ouroboros-consensus/src/Ouroboros/Consensus/Storage/VolatileDB/Impl/Parser.hs:66-85)
// and ImmutableDB chunk validation on every block of a chunk
// (.../ImmutableDB/Impl/Validation.hs:358-365).  The raw-CBOR pipeline above:
// the device slicer (cbor.h, kes_t_of = Integrity.hs:38-44), then the Sum6KES
// kernel on its rows; a header the slicer rejects is 0.
int ouro_integrity_verify_cbor(const uint8_t* raw, size_t raw_bytes, const uint64_t* off,
                               const uint32_t* len, size_t n, uint64_t slots_per_kes_period,
                               uint8_t* status, uint8_t* verdict) {
  RawCall c{kRawKes, raw, raw_bytes, off, len, n, slots_per_kes_period, nullptr, nullptr,
            nullptr, status, verdict, nullptr, nullptr, nullptr};
  return raw_verify(c);
}

// Raw TPraos headers -> the full header check (ouroboros-consensus-shelley/
// src/Ouroboros/Consensus/Shelley/Protocol.hs:433-442 over each decoded
// header) in one call through the raw-CBOR pipeline above.
int ouro_tpraos_verify_cbor(const uint8_t* raw, size_t raw_bytes, const uint64_t* off,
                            const uint32_t* len, size_t n, uint64_t slots_per_kes_period,
                            const uint8_t* epoch_nonce, const uint8_t* eta_alpha,
                            const uint8_t* leader_alpha, uint8_t* status, uint8_t* verdict,
                            uint8_t* beta_eta, uint8_t* beta_leader, uint8_t* eta_nonce) {
  RawCall c{kRawHdr, raw, raw_bytes, off, len, n, slots_per_kes_period, epoch_nonce, eta_alpha,
            leader_alpha, status, verdict, beta_eta, beta_leader, eta_nonce};
  return raw_verify(c);
}

// Raw Byron headers -> PBFT's block-signature verdicts (ouroboros-consensus/
// src/Ouroboros/Consensus/Protocol/PBFT.hs:332-338; the storage integrity
// check ouroboros-consensus-byron/src/Ouroboros/Consensus/Byron/Ledger/
// Integrity.hs:24-35) through the raw-CBOR pipeline above: chunks gathered
// into pinned NUMA-local staging, the device Byron slicer (k_byron_pack, the
// host slicer's cbor_byron.h parse), then the Ed25519 kernel with ByronDSIGN
// acceptance, five chunks in flight.  An epoch-boundary header is 1 (status
// OURO_PACK_EBB); a rejected one 0.
int ouro_byron_verify_cbor(const uint8_t* raw, size_t raw_bytes, const uint64_t* off,
                           const uint32_t* len, size_t n, int64_t protocol_magic,
                           uint8_t* status, uint8_t* verdict) {
  RawCall c{kRawByron, raw, raw_bytes, off, len, n, 0, nullptr, nullptr, nullptr, status,
            verdict, nullptr, nullptr, nullptr, protocol_magic};
  return raw_verify(c);
}

// DIAGNOSTIC: 1 in the test-hook build (lib/libouro_verify_test.so), 0 in the product
int ouro_debug_test_hooks(void) { return OURO_TEST_HOOKS; }

void ouro_debug_reload_knobs(void) { ouro_knobs::reload(); }

// DIAGNOSTIC: the calling thread's last raw-CBOR call (ms and counts)
int ouro_debug_cbor_stats(double* out6) {
  if (!out6) return fail(OURO_EINVAL, "null buffer");
  memcpy(out6, t_raw_stats, sizeof t_raw_stats);
  return OURO_OK;
}

// The same on raw headers already in device memory (raw, off, len, arena,
// status, verdict: device pointers; arena >= ouro_tpraos_pack_bytes(n)):
// the device slicer and the Sum6KES kernel enqueued on `stream`, not
// synchronised.  A rejected header's zeroed row (OURO_PACK_*) cannot verify.
int ouro_integrity_verify_cbor_device(void* stream, const uint8_t* raw, size_t raw_bytes,
                                      const uint64_t* off, const uint32_t* len, size_t n,
                                      uint64_t slots_per_kes_period, void* arena,
                                      size_t arena_bytes, uint8_t* status, uint8_t* verdict) {
  if (n == 0) return OURO_OK;
  if (!verdict) return fail(OURO_EINVAL, "null verdict");
  ouro_tpraos_batch b{};
  int rc = ouro_tpraos_pack_cbor_device(stream, raw, raw_bytes, off, len, n,
                                        slots_per_kes_period, arena, arena_bytes, &b, nullptr,
                                        nullptr, status);
  if (rc) return rc;
  hipStream_t st = static_cast<hipStream_t>(stream);
  return launch_kes(st, n, b.hot_vk, b.kes_t, b.body, b.body_off, b.body_len, b.kes_sig, verdict);
}

int ouro_leader_check_batch_device(void* stream, size_t n, const uint8_t* beta,
                                   const uint64_t* sigma_num, const uint64_t* sigma_den,
                                   int64_t act_log_hi, uint64_t act_log_lo, int f_is_one,
                                   uint8_t* verdict) {
  if (n == 0) return OURO_OK;
  hipStream_t st = static_cast<hipStream_t>(stream);  // NULL = HIP's default stream
  return launch_leader(st, n, beta, sigma_num, sigma_den, act_log_hi, act_log_lo, f_is_one,
                       verdict);
}

}  // extern "C"

// A plan's window read straight from its pinned input block by a copy kernel
// (OURO_PLAN_STAGE >= 1; A/B against the DMA copy node): one 16-B load per
// thread, every load of the window in flight at once.
// stamp (a plan's timing probe, OURO_PLAN_TIMING; else null): the copy's start
// in s_memrealtime ticks (100 MHz), written to the plan's pinned done block.
__device__ __forceinline__ void plan_stamp(uint64_t* stamp) {
  if (stamp && blockIdx.x == 0 && threadIdx.x == 0)
    __hip_atomic_store(stamp, (uint64_t)__builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
}
__global__ void __launch_bounds__(256) k_plan_stage(const uint4* __restrict__ src,
                                                    uint4* __restrict__ dst, size_t n16,
                                                    uint64_t* stamp) {
  plan_stamp(stamp);
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n16) dst[i] = src[i];
}
// The same over the byte ranges a window actually uses (the block header, and
// per member given its n rows or the body span -- not the capacity), in 16-B
// units: thread t copies unit t of the concatenated ranges (round 5: the
// copy reads pinned memory over PCIe, so its bytes are its time).
constexpr int kPlanMaxRanges = 24;
struct PlanRanges {
  uint32_t count;
  uint32_t start16[kPlanMaxRanges];
  uint32_t len16[kPlanMaxRanges];
};
__global__ void __launch_bounds__(256) k_plan_stage_ranges(const uint4* __restrict__ src,
                                                           uint4* __restrict__ dst,
                                                           PlanRanges r, uint64_t* stamp) {
  plan_stamp(stamp);
  uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  for (uint32_t k = 0; k < r.count; k++) {
    if (t < r.len16[k]) {
      const uint32_t i = r.start16[k] + t;
      dst[i] = src[i];
      return;
    }
    t -= r.len16[k];
  }
}

// ---- plans: pinned staging, the window's copy kernel + latency kernel -------
// issued straight on the plan's stream per window (default), or replayed from
// one captured hipGraph (OURO_PLAN_GRAPH=1, A/B): the graph's GPU-side
// dispatch of its two kernel nodes cost 8-10 us more per window than two
// stream launches (profiles/r04m/ablat_plan_graph.json, lat_phases_graph.json).
// The packed input block: 16 bytes {n, option bits (tpraos.h kOpt*), the
// launch's generation (wide_cores.h arrive_last), 0}, then
// every member of ouro_tpraos_batch in order, each 16-byte aligned at
// capacity size; the output block: verdict | beta_eta | beta_leader | eta_nonce.
namespace {
constexpr int kPlanFields = 19;
// bytes per header of each member; 0 = the body (capacity-sized), -1 = a
// fixed 32 bytes (epoch_nonce)
constexpr int kFieldBytes[kPlanFields] = {32, 32, 80, 80, 32, 32, 32, 8, 8, 64,
                                          4,  448, 0, 8, 4, 64, 64, 8, -1};
enum PlanField { kFBody = 12, kFBodyOff = 13, kFEtaAlpha = 4, kFLeaderAlpha = 5, kFEpochNonce = 18 };
constexpr size_t align16(size_t x) { return (x + 15) & ~(size_t)15; }
}  // namespace

struct ouro_tpraos_plan {
  int dev = -1;
  size_t cap = 0, body_cap = 0;
  hipStream_t st = nullptr;
  hipGraph_t graph = nullptr;
  hipGraphExec_t exec = nullptr;
  uint8_t *h_in = nullptr, *d_in = nullptr, *h_out = nullptr, *d_out = nullptr;
  size_t in_bytes = 0, out_bytes = 0;
  int32_t *res = nullptr, *scratch = nullptr;
  size_t off[kPlanFields] = {0};  // byte offsets of the members in the packed input block
  ouro_tpraos_batch dev_batch{};
  uint32_t gen = 0;             // generation of the last launch (arrive_last), 1..2^28-1
  size_t pending = 0;           // headers of the batch in flight (submit .. wait)
  uint8_t* nonce_dst = nullptr;  // that batch's eta_nonce (written by wait)
  uint32_t opts = 0;             // that batch's option bits (tpraos.h kOpt*)
  bool inflight = false;
  bool failed = false;           // its launch failed: wait recomputes it on the host path
  // TIMING PROBE (OURO_PLAN_TIMING set at submit; bench.py latency phases):
  // events around the window's launches on the plan's stream
  // (without the done word, the A/B forms: events around the launches; with
  // it, the kernels' own s_memrealtime stamps in the done block -- events
  // recorded every window made the runtime stall one submit in ~250 for
  // ~125 us, profiles/r06b/submit_probe.json)
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  bool timed = false;
  uint64_t* stamps = nullptr;  // device view of the done block's stamps (timing + flag)
  const volatile uint64_t* stamps_host = nullptr;
  bool timing = false;  // OURO_PLAN_TIMING at create
  float last_gpu_ms = -1.0f;
  float copy_us = -1.0f, launch_us = -1.0f;  // host side of its last submit
  int stage = 2;  // OURO_PLAN_STAGE at capture (plan_build)
  int spin = 0;   // OURO_PLAN_SPIN at capture: wait spins on hipStreamQuery
  int use_graph = 0;  // OURO_PLAN_GRAPH at build: 1 = the launches captured into one hipGraph
  void* hin = nullptr;  // device view of h_in (stage >= 1)
  uint8_t *dver = nullptr, *dbe = nullptr, *dbl = nullptr;  // the latency kernel's outputs
  LatShape shape;  // the latency launch at capacity (lat_shape, once)
  // OURO_PLAN_FLAG (default 1; stage 2, fused kernel): the latency kernel's
  // last header tail writes the generation into a done word in the pinned
  // output block, and wait spins on it instead of the stream's completion
  bool flag = false;
  uint32_t* done_dev = nullptr;              // that word as the kernel sees it
  const volatile uint32_t* done_host = nullptr;
  // the window's used byte ranges of the input block (recorded at submit):
  // the copy kernel moves those instead of the whole capacity block
  // (OURO_PLAN_TRIM=0 at create: the whole block, the round-4 form)
  bool trim = true;
  PlanRanges ranges{};
};

namespace {
void plan_free(ouro_tpraos_plan* p) {
  if (!p) return;
  // no DMA into freed staging (and, with the done word, a waited-for launch
  // may still be retiring its last waves)
  if (p->st) (void)hipStreamSynchronize(p->st);
  if (p->ev0) (void)hipEventDestroy(p->ev0);
  if (p->ev1) (void)hipEventDestroy(p->ev1);
  if (p->exec) (void)hipGraphExecDestroy(p->exec);
  if (p->graph) (void)hipGraphDestroy(p->graph);
  if (p->h_in) (void)hipHostFree(p->h_in);
  if (p->h_out) (void)hipHostFree(p->h_out);
  if (p->d_in) (void)hipFree(p->d_in);
  if (p->d_out) (void)hipFree(p->d_out);
  if (p->res) (void)hipFree(p->res);
  if (p->scratch) (void)hipFree(p->scratch);
  if (p->st) (void)hipStreamDestroy(p->st);
  delete p;
}

// the window's launches on the plan's stream: issued per submit (the
// default), or captured once into the graph (OURO_PLAN_GRAPH=1, A/B)
int plan_enqueue(ouro_tpraos_plan* p) {
  if ((p->stage == 1 || p->stage == 2) && p->ranges.count && !p->use_graph) {
    uint32_t units = 0;
    for (uint32_t k = 0; k < p->ranges.count; k++) units += p->ranges.len16[k];
    hipLaunchKernelGGL(k_plan_stage_ranges, dim3((units + 255) / 256), dim3(256), 0, p->st,
                       static_cast<const uint4*>(p->hin), reinterpret_cast<uint4*>(p->d_in),
                       p->ranges, p->stamps);
  } else if (p->stage == 1 || p->stage == 2) {
    const size_t n16 = p->in_bytes / 16;  // in_bytes is a multiple of 16
    hipLaunchKernelGGL(k_plan_stage, dim3((unsigned)((n16 + 255) / 256)), dim3(256), 0, p->st,
                       static_cast<const uint4*>(p->hin), reinterpret_cast<uint4*>(p->d_in), n16,
                       p->stamps);
  } else if (p->stage <= 0) {
    OURO_HIP(hipMemcpyAsync(p->d_in, p->h_in, p->in_bytes, hipMemcpyHostToDevice, p->st));
  }
  const uint8_t* d = p->stage >= 3 ? static_cast<const uint8_t*>(p->hin) : p->d_in;
  // the window counter: word 3 of the input block, zeroed by the copy
  lat_issue(p->st, p->shape, p->dev_batch, reinterpret_cast<const uint32_t*>(d), p->res,
            p->scratch, p->dver, p->dbe, p->dbl,
            p->flag ? reinterpret_cast<uint32_t*>(p->d_in) + 3 : nullptr, p->done_dev);
  OURO_HIP(hipGetLastError());
  if (p->stage < 2)
    OURO_HIP(hipMemcpyAsync(p->h_out, p->d_out, p->out_bytes, hipMemcpyDeviceToHost, p->st));
  return OURO_OK;
}

size_t field_cap_bytes(const ouro_tpraos_plan* p, int f) {
  return kFieldBytes[f] > 0 ? (size_t)kFieldBytes[f] * p->cap
                            : (kFieldBytes[f] == 0 ? p->body_cap : 32);
}

int plan_build(ouro_tpraos_plan* p) {
  DeviceState* ds;
  int rc = device_state(&ds);
  if (rc) return rc;
  if ((rc = current_device(&p->dev))) return rc;
  OURO_HIP(hipStreamCreateWithFlags(&p->st, hipStreamNonBlocking));
  size_t o = 16;  // n and the option bits live in the first 16 bytes
  for (int f = 0; f < kPlanFields; f++) {
    p->off[f] = o;
    o += align16(field_cap_bytes(p, f));
  }
  p->in_bytes = o;
  p->out_bytes = align16(p->cap) + 160 * p->cap + 64;  // + the done word (OURO_PLAN_FLAG)
  OURO_HIP(hipHostMalloc(&p->h_in, p->in_bytes, hipHostMallocNumaUser));
  OURO_HIP(hipHostMalloc(&p->h_out, p->out_bytes, hipHostMallocNumaUser));
  OURO_HIP(hipMalloc(&p->d_in, p->in_bytes));
  OURO_HIP(hipMalloc(&p->d_out, p->out_bytes));
  OURO_HIP(hipMalloc(&p->res, sizeof(int32_t) * slot_region_words(p->cap, kLatResWords)));
  // the arrival records are generation-tagged (each submit bumps the plan's
  // generation) and never reset by the kernel; they start from zero once here
  OURO_HIP(hipMemset(p->res, 0, sizeof(int32_t) * slot_region_words(p->cap, kLatResWords)));
  OURO_HIP(hipMalloc(&p->scratch, sizeof(int32_t) * lowlat_scratch_words(ds, p->cap)));
  memset(p->h_in, 0, p->in_bytes);
  memset(p->h_out, 0, p->out_bytes);  // the done word starts at 0, never a generation
  // OURO_PLAN_STAGE (the window's copies, read here once): 0 = DMA copies in
  // and out; 1 = a copy kernel reads the pinned input block; 2 (default) =
  // that, and the latency kernel writes the results straight into the pinned
  // output block -- one node fewer, 2-3 us of the window (profiles/r04c:
  // ablat_plan_stage.json, lat_phases.json; the copy nodes' own time is
  // ~5 us each, the rest is the graph's node-to-node dispatch); 3 = no input
  // copy either: the latency kernel reads the pinned block over PCIe (A/B).
  // OURO_PLAN_GRAPH=1: capture them into a hipGraph (the form before r04m).
  const ouro_knobs::Knobs& kn = ouro_knobs::get();
  p->stage = kn.plan_stage.load(std::memory_order_relaxed);
  p->spin = kn.plan_spin.load(std::memory_order_relaxed);
  p->use_graph = kn.plan_graph.load(std::memory_order_relaxed) != 0;
  p->trim = kn.plan_trim.load(std::memory_order_relaxed) != 0;
  p->timing = kn.plan_timing.load(std::memory_order_relaxed) != 0;
  if (p->stage >= 1) OURO_HIP(hipHostGetDevicePointer(&p->hin, p->h_in, 0));
  uint8_t* d = p->stage >= 3 ? static_cast<uint8_t*>(p->hin) : p->d_in;
  ouro_tpraos_batch& b = p->dev_batch;
  b.n = p->cap;
  b.issuer_vk = d + p->off[0];
  b.vrf_vk = d + p->off[1];
  b.eta_proof = d + p->off[2];
  b.leader_proof = d + p->off[3];
  b.eta_alpha = d + p->off[4];
  b.leader_alpha = d + p->off[5];
  b.hot_vk = d + p->off[6];
  b.ocert_counter = reinterpret_cast<const uint64_t*>(d + p->off[7]);
  b.ocert_kes_period = reinterpret_cast<const uint64_t*>(d + p->off[8]);
  b.ocert_sigma = d + p->off[9];
  b.kes_t = reinterpret_cast<const uint32_t*>(d + p->off[10]);
  b.kes_sig = d + p->off[11];
  b.body = d + p->off[12];
  b.body_off = reinterpret_cast<const uint64_t*>(d + p->off[13]);
  b.body_len = reinterpret_cast<const uint32_t*>(d + p->off[14]);
  b.eta_output = d + p->off[15];
  b.leader_output = d + p->off[16];
  b.slot = reinterpret_cast<const uint64_t*>(d + p->off[17]);
  b.epoch_nonce = d + p->off[18];
  uint8_t* dver = p->d_out;
  uint8_t* dbe = dver + align16(p->cap);
  uint8_t* dbl = dbe + 64 * p->cap;
  b.eta_nonce = dbl + 64 * p->cap;  // written only when the option bit says so
  if (p->stage >= 2) {
    void* hout = nullptr;
    OURO_HIP(hipHostGetDevicePointer(&hout, p->h_out, 0));
    dver = static_cast<uint8_t*>(hout);
    dbe = dver + align16(p->cap);
    dbl = dbe + 64 * p->cap;
    b.eta_nonce = dbl + 64 * p->cap;
  }
  p->dver = dver;
  p->dbe = dbe;
  p->dbl = dbl;
  if ((rc = lat_shape(p->cap, &p->shape))) return rc;
  {
    p->flag = p->stage == 2 && p->shape.fused && kn.plan_flag.load(std::memory_order_relaxed) != 0;
    if (p->flag) {
      uint8_t* w = p->h_out + p->out_bytes - 64;
      void* wd = nullptr;
      OURO_HIP(hipHostGetDevicePointer(&wd, w, 0));
      p->done_dev = static_cast<uint32_t*>(wd);
      p->done_host = reinterpret_cast<const volatile uint32_t*>(w);
      if (p->timing) {
        // the done block: word 0 the done word; u64 1 the latency kernel's
        // start, u64 2 the last tail's end, u64 3 the copy kernel's start
        p->stamps = reinterpret_cast<uint64_t*>(static_cast<uint8_t*>(wd) + 8);
        p->stamps_host = reinterpret_cast<const volatile uint64_t*>(w + 8);
        p->shape.flags |= 1u << 26;
      }
    }
  }
  if (!p->use_graph) return OURO_OK;
  OURO_HIP(hipStreamBeginCapture(p->st, hipStreamCaptureModeThreadLocal));
  if ((rc = plan_enqueue(p))) {
    hipGraph_t g = nullptr;
    (void)hipStreamEndCapture(p->st, &g);
    if (g) (void)hipGraphDestroy(g);
    return rc;
  }
  OURO_HIP(hipStreamEndCapture(p->st, &p->graph));
  OURO_HIP(hipGraphInstantiate(&p->exec, p->graph, nullptr, nullptr, 0));
  return OURO_OK;
}

// The batch in the plan's pinned input block as a host batch (the layout
// ouro_tpraos_plan_submit wrote), for the host recompute after a failed
// launch; results go straight to the caller's buffers.
ouro_tpraos_batch plan_host_batch(const ouro_tpraos_plan* p) {
  const uint8_t* h = p->h_in;
  ouro_tpraos_batch b{};
  b.n = p->pending;
  b.issuer_vk = h + p->off[0];
  b.vrf_vk = h + p->off[1];
  b.eta_proof = h + p->off[2];
  b.leader_proof = h + p->off[3];
  b.hot_vk = h + p->off[6];
  b.ocert_counter = reinterpret_cast<const uint64_t*>(h + p->off[7]);
  b.ocert_kes_period = reinterpret_cast<const uint64_t*>(h + p->off[8]);
  b.ocert_sigma = h + p->off[9];
  b.kes_t = reinterpret_cast<const uint32_t*>(h + p->off[10]);
  b.kes_sig = h + p->off[11];
  b.body = h + p->off[12];
  b.body_off = reinterpret_cast<const uint64_t*>(h + p->off[13]);
  b.body_len = reinterpret_cast<const uint32_t*>(h + p->off[14]);
  if (p->opts & kOptEtaClaim) b.eta_output = h + p->off[15];
  if (p->opts & kOptLeaderClaim) b.leader_output = h + p->off[16];
  if (p->opts & kOptSeeds) {
    b.slot = reinterpret_cast<const uint64_t*>(h + p->off[17]);
    if (p->opts & kOptEpochNonce) b.epoch_nonce = h + p->off[18];
  } else {
    b.eta_alpha = h + p->off[4];
    b.leader_alpha = h + p->off[5];
  }
  if (p->opts & kOptEtaNonce) b.eta_nonce = p->nonce_dst;
  return b;
}

// TEST HOOK (tests/test_gpu_claims.py::test_plan_counters_from_cut_off_launch;
// the test build only, OURO_TEST_HOOKS): OURO_TEST_PLAN_POISON set at
// ouro_tpraos_plan_submit leaves every arrival counter of the
// plan's records as a launch of its last generation would have left them had
// it been cut off one arrival short of each finish, so the test can show the
// next launch ignores them.
#if OURO_TEST_HOOKS
int plan_poison(ouro_tpraos_plan* p) {
  OURO_HIP(hipSetDevice(p->dev));
  OURO_HIP(hipStreamSynchronize(p->st));  // the last launch retired (done word: maybe not yet)
  const size_t words = slot_region_words(p->cap, kLatResWords);
  std::vector<int32_t> h(words);
  OURO_HIP(hipMemcpy(h.data(), p->res, sizeof(int32_t) * words, hipMemcpyDeviceToHost));
  const int32_t tag = (int32_t)((p->gen & 0x0fffffffu) << 4);
  for (size_t i = 0; i < p->cap; i++) {
    const Slot r = slot_of(h.data(), i, kLatResWords);
    *r.word(kLatCtr) = tag | (kLatCores - 1);     // the header's tail one arrival away
    *r.word(kLatCtr + 1) = tag | 1;                // each V / Gamma pair (or V / V2 /
    *r.word(kLatCtr + 2) = tag | 1;                // Gamma triple), one in
    for (int e = 0; e < 2; e++) {
      *r.word(kLatEd + kEdWords * e + 125) = tag | 1;  // each Ed25519 points / scalars pair
      for (int k = 17; k <= 19; k++)                // split form: the chain and done counters
        *r.word(kLatEd + kEdWords * e + k) = tag | 1;
    }
  }
  OURO_HIP(hipMemcpy(p->res, h.data(), sizeof(int32_t) * words, hipMemcpyHostToDevice));
  return OURO_OK;
}
#endif
}  // namespace

extern "C" {

ouro_tpraos_plan* ouro_tpraos_plan_create(size_t max_headers, size_t max_body_bytes) {
  if (max_headers == 0 || max_headers > 0xffffffffu) {
    fail(OURO_EINVAL, "bad plan size");
    return nullptr;
  }
  auto* p = new ouro_tpraos_plan;
  p->cap = max_headers;
  p->body_cap = std::max<size_t>(max_body_bytes, 16);
  if (plan_build(p) != OURO_OK) {
    plan_free(p);
    return nullptr;
  }
  return p;
}

int ouro_tpraos_plan_submit(ouro_tpraos_plan* p, const ouro_tpraos_batch* b) {
  if (!p || !b) return fail(OURO_EINVAL, "null argument");
  if (p->inflight) return fail(OURO_EINVAL, "the plan already has a batch in flight");
  const size_t n = b->n;
  if (n > p->cap) return fail(OURO_EINVAL, "batch larger than the plan");
  if (n == 0) {
    p->pending = 0;
    p->nonce_dst = nullptr;
    p->inflight = true;
    return OURO_OK;
  }
  int rc = check_hdr_batch(b);
  if (rc) return rc;
  Window w;
  if ((rc = window_of(n, b->body_off, b->body_len, &w))) return rc;
  if (w.span() > p->body_cap) return fail(OURO_EINVAL, "body bytes exceed the plan");
  if (w.span() && !b->body) return fail(OURO_EINVAL, "null body buffer");
  const void* src[kPlanFields] = {
      b->issuer_vk,  b->vrf_vk,           b->eta_proof,   b->leader_proof, b->eta_alpha,
      b->leader_alpha, b->hot_vk,         b->ocert_counter, b->ocert_kes_period,
      b->ocert_sigma, b->kes_t,           b->kes_sig,     w.span() ? b->body + w.lo : nullptr,
      w.off.data(),  b->body_len,         b->eta_output,  b->leader_output, b->slot,
      b->epoch_nonce};
  p->timed = p->timing;
  const auto tc0 = std::chrono::steady_clock::now();
  if (b->slot) src[kFEtaAlpha] = src[kFLeaderAlpha] = nullptr;  // derived on the device
  else src[kFEpochNonce] = nullptr;
  bool trim = p->trim;
  p->ranges.count = 0;
  if (trim) {  // the block header: n, option bits, generation, window counter
    p->ranges.start16[0] = 0;
    p->ranges.len16[0] = 1;
    p->ranges.count = 1;
  }
  for (int f = 0; f < kPlanFields; f++) {
    const size_t bytes = kFieldBytes[f] > 0 ? (size_t)kFieldBytes[f] * n
                                            : (kFieldBytes[f] == 0 ? w.span() : 32);
    if (bytes && src[f]) {
      memcpy(p->h_in + p->off[f], src[f], bytes);
      if (trim) {
        PlanRanges& r = p->ranges;
        const uint32_t s16 = (uint32_t)(p->off[f] / 16), l16 = (uint32_t)((bytes + 15) / 16);
        if (r.start16[r.count - 1] + r.len16[r.count - 1] == s16) r.len16[r.count - 1] += l16;
        else if (r.count < (uint32_t)kPlanMaxRanges) {
          r.start16[r.count] = s16;
          r.len16[r.count++] = l16;
        } else {
          r.count = 0;  // (cannot happen: 19 members) copy the whole block
          trim = false;
        }
      }
    }
  }
  if (p->timed)
    p->copy_us = std::chrono::duration<float, std::micro>(std::chrono::steady_clock::now() - tc0).count();
#if OURO_TEST_HOOKS
  if (p->gen && ouro_knobs::get().test_plan_poison.load() && (rc = plan_poison(p))) return rc;
#endif
  // every launch a new generation, so no counter an earlier launch left
  // behind (one that never completed) is ever counted again
  p->gen = p->gen % 0x0fffffffu + 1u;
  p->opts = batch_opts(*b);
  const uint32_t nw[3] = {(uint32_t)n, p->opts, p->gen};
  memcpy(p->h_in, nw, sizeof nw);
  p->pending = n;
  p->nonce_dst = b->eta_nonce;
  p->failed = false;
#if OURO_TEST_HOOKS
  // TEST HOOK (tests/test_gpu_hooks_plan.py): every result byte of the pinned
  // output block (not the done word) set to a sentinel before the launch, so
  // a wait that returned before the kernel's stores were visible would hand
  // back the sentinel instead of the oracle's verdicts and outputs
  if (ouro_knobs::get().test_plan_sentinel.load()) memset(p->h_out, 0xEE, p->out_bytes - 64);
#endif
  const bool injected = injected_device_error();
  hipError_t e = hipSetDevice(p->dev);
  const bool events = p->timed && !p->stamps;
  if (events && !p->ev0 && e == hipSuccess) {
    e = hipEventCreate(&p->ev0);
    if (e == hipSuccess) e = hipEventCreate(&p->ev1);
  }
  if (events && e == hipSuccess) e = hipEventRecord(p->ev0, p->st);
  const auto tl0 = std::chrono::steady_clock::now();
  if (e == hipSuccess && !injected) {
    if (p->exec) e = hipGraphLaunch(p->exec, p->st);
    else if (plan_enqueue(p) != OURO_OK) e = hipErrorLaunchFailure;
  }
  if (p->timed)
    p->launch_us = std::chrono::duration<float, std::micro>(std::chrono::steady_clock::now() - tl0).count();
  if (events && e == hipSuccess) e = hipEventRecord(p->ev1, p->st);
  if (e != hipSuccess || injected) {
    fail(OURO_EDEVICE, std::string("plan launch: ") +
                           (e != hipSuccess ? hipGetErrorString(e) : "injected device error"));
    if (!recompute_on_error()) return OURO_EDEVICE;
    p->failed = true;  // the inputs stay staged in h_in: wait verifies them on the host
  }
  p->inflight = true;
  return OURO_OK;
}

int ouro_tpraos_plan_wait(ouro_tpraos_plan* p, uint8_t* verdict, uint8_t* beta_eta,
                          uint8_t* beta_leader) {
  if (!p) return fail(OURO_EINVAL, "null plan");
  if (!p->inflight) return fail(OURO_EINVAL, "no batch in flight on this plan");
  const size_t n = p->pending;
  if (n && !verdict) return fail(OURO_EINVAL, "null verdict");
  p->inflight = false;
  if (n == 0) return OURO_OK;
  int rc = OURO_OK;
  if (!p->failed) {
    hipError_t e = hipSetDevice(p->dev);
    if (e == hipSuccess && p->flag) {
      // the kernel's done word; the stream is asked now and then, so a launch
      // that never writes it (a fault) still ends the wait with its error
      for (uint32_t k = 1;; k++) {
        if (*p->done_host == p->gen) break;
        if ((k & 255u) == 0) {
          e = hipStreamQuery(p->st);
          if (e != hipErrorNotReady) break;
          e = hipSuccess;
        }
        __builtin_ia32_pause();
      }
      std::atomic_thread_fence(std::memory_order_acquire);
      if (e == hipSuccess && p->timed && !p->stamps) e = hipEventSynchronize(p->ev1);
    } else if (e == hipSuccess && p->spin) {
      // poll the stream instead of the runtime's wait, which may sleep on the
      // completion interrupt
      while ((e = hipStreamQuery(p->st)) == hipErrorNotReady) __builtin_ia32_pause();
    }
    if (e == hipSuccess && !p->flag) e = hipStreamSynchronize(p->st);
    if (e != hipSuccess) rc = fail(OURO_EDEVICE, std::string("plan wait: ") + hipGetErrorString(e));
  } else {
    rc = OURO_EDEVICE;
  }
  if (rc) {
    const ouro_tpraos_batch hb = plan_host_batch(p);
    p->nonce_dst = nullptr;
    p->failed = false;
    return or_host(rc, [&] { return ouro_host::hdr_batch(&hb, verdict, beta_eta, beta_leader); });
  }
  p->last_gpu_ms = -1.0f;
  if (p->timed && p->stamps) {
    // the copy kernel's start to the last header's end, 100 MHz ticks
    const uint64_t t0 = p->stamps_host[0], t2 = p->stamps_host[2];
    p->last_gpu_ms = t2 > t0 ? (float)((double)(t2 - t0) * 1e-5) : -1.0f;
  } else if (p->timed) {
    (void)hipEventElapsedTime(&p->last_gpu_ms, p->ev0, p->ev1);
  }
  const uint8_t* o = p->h_out + align16(p->cap);
  memcpy(verdict, p->h_out, n);
  if (beta_eta) memcpy(beta_eta, o, 64 * n);
  if (beta_leader) memcpy(beta_leader, o + 64 * p->cap, 64 * n);
  if (p->nonce_dst) memcpy(p->nonce_dst, o + 128 * p->cap, 32 * n);
  p->nonce_dst = nullptr;
  return OURO_OK;
}

int ouro_tpraos_plan_run(ouro_tpraos_plan* p, const ouro_tpraos_batch* b, uint8_t* verdict,
                         uint8_t* beta_eta, uint8_t* beta_leader) {
  if (!p || !b || !verdict) return fail(OURO_EINVAL, "null argument");
  if (b->n == 0) return OURO_OK;
  int rc = ouro_tpraos_plan_submit(p, b);
  if (rc) return rc;
  return ouro_tpraos_plan_wait(p, verdict, beta_eta, beta_leader);
}

void ouro_tpraos_plan_destroy(ouro_tpraos_plan* p) { plan_free(p); }

// TIMING PROBE (tools/lat_stamps.py): header 0's per-item stamps of the last
// fused latency launch, 16 items x 24 tags of s_memrealtime (100 MHz), from a
// library built with -DOURO_LAT_STAMPS=1 and run with OURO_LAT_STAMPS set;
// returns the count, or -1 in the product build.
int ouro_debug_lat_stamps(unsigned long long* out) { return lat_stamps_read(out); }

// CLOCK PROBE (bench.py roofline.frac_clock): the last k_tpraos_verify
// launch's per-workgroup {s_memtime, s_memtime, s_memrealtime, s_memrealtime}
// at entry / exit, min(grid, max_slots) rows, from a -DOURO_CLOCK_STAMPS=1
// build (lib/libouro_verify_clock.so); -1 in the product build.
int ouro_debug_clock_stamps(unsigned long long* out, int max_slots) {
#if OURO_CLOCK_STAMPS
  if (!out || max_slots <= 0) return fail(OURO_EINVAL, "null buffer");
  const int n = std::min(max_slots, kClockSlots);
  if (hipDeviceSynchronize() != hipSuccess) return fail(OURO_EDEVICE, "sync");
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_clock_stamps), sizeof(unsigned long long) * 4 * n) !=
      hipSuccess)
    return fail(OURO_EDEVICE, "hipMemcpyFromSymbol");
  return n;
#else
  (void)out;
  (void)max_slots;
  return -1;
#endif
}

}  // extern "C"

namespace {
// The (offset, length) spans of a host-path batch: the same argument checks
// as the device calls' window_of: an offset + length that wraps,
// or a null buffer with any nonzero length, is OURO_EINVAL -- never a read of
// invalid memory.
int check_spans(size_t n, const uint64_t* off, const uint32_t* len, const void* buf,
                const char* what) {
  for (size_t i = 0; i < n; i++) {
    if (!len[i]) continue;
    if (off[i] + len[i] < off[i]) return fail(OURO_EINVAL, "offset + length overflows");
    if (!buf) return fail(OURO_EINVAL, std::string("null ") + what + " buffer");
  }
  return OURO_OK;
}
}  // namespace

extern "C" {

// ---- the host path, called explicitly (host_path.h) ----
int ouro_ed25519_verify_batch_host(size_t n, const uint8_t* pk, const uint8_t* sig,
                                   const uint8_t* msg, const uint64_t* msg_off,
                                   const uint32_t* msg_len, uint8_t* verdict) {
  if (n == 0) return OURO_OK;
  if (!pk || !sig || !msg_off || !msg_len || !verdict) return fail(OURO_EINVAL, "null argument");
  if (int rc = check_spans(n, msg_off, msg_len, msg, "message")) return rc;
  return ouro_host::ed_batch(n, pk, sig, msg, msg_off, msg_len, verdict, 0);
}
int ouro_byron_ed25519_verify_batch_host(size_t n, const uint8_t* pk, const uint8_t* sig,
                                         const uint8_t* msg, const uint64_t* msg_off,
                                         const uint32_t* msg_len, uint8_t* verdict) {
  if (n == 0) return OURO_OK;
  if (!pk || !sig || !msg_off || !msg_len || !verdict) return fail(OURO_EINVAL, "null argument");
  if (int rc = check_spans(n, msg_off, msg_len, msg, "message")) return rc;
  return ouro_host::ed_batch(n, pk, sig, msg, msg_off, msg_len, verdict, 1);
}
int ouro_vrf03_verify_batch_host(size_t n, const uint8_t* pk, const uint8_t* proof,
                                 const uint8_t* alpha, const uint64_t* alpha_off,
                                 const uint32_t* alpha_len, uint8_t* beta, uint8_t* verdict,
                                 uint32_t flags) {
  if (n == 0) return OURO_OK;
  if (flags & ~OURO_VRF_STRICT_S) return fail(OURO_EINVAL, "unknown VRF flags");
  if (!pk || !proof || !alpha_off || !alpha_len || !verdict) return fail(OURO_EINVAL, "null argument");
  if (int rc = check_spans(n, alpha_off, alpha_len, alpha, "alpha")) return rc;
  return ouro_host::vrf_batch(n, pk, proof, alpha, alpha_off, alpha_len, beta, verdict, flags);
}
int ouro_sum6kes_verify_batch_host(size_t n, const uint8_t* vk, const uint32_t* t,
                                   const uint8_t* msg, const uint64_t* msg_off,
                                   const uint32_t* msg_len, const uint8_t* sig, uint8_t* verdict) {
  if (n == 0) return OURO_OK;
  if (!vk || !t || !msg_off || !msg_len || !sig || !verdict) return fail(OURO_EINVAL, "null argument");
  if (int rc = check_spans(n, msg_off, msg_len, msg, "message")) return rc;
  return ouro_host::kes_batch(n, vk, t, msg, msg_off, msg_len, sig, verdict);
}
int ouro_tpraos_verify_batch_host(const ouro_tpraos_batch* b, uint8_t* verdict,
                                  uint8_t* beta_eta, uint8_t* beta_leader) {
  if (!b) return fail(OURO_EINVAL, "null batch");
  if (b->n == 0) return OURO_OK;
  if (!verdict) return fail(OURO_EINVAL, "null verdict");
  int rc = check_hdr_batch(b);
  if (rc) return rc;
  if ((rc = check_spans(b->n, b->body_off, b->body_len, b->body, "body"))) return rc;
  return ouro_host::hdr_batch(b, verdict, beta_eta, beta_leader);
}
int ouro_leader_check_batch_host(size_t n, const uint8_t* beta, const uint64_t* sigma_num,
                                 const uint64_t* sigma_den, int64_t act_log_hi,
                                 uint64_t act_log_lo, int f_is_one, uint8_t* verdict) {
  if (n == 0) return OURO_OK;
  if (!beta || !sigma_num || !sigma_den || !verdict) return fail(OURO_EINVAL, "null argument");
  return ouro_host::leader_batch(n, beta, sigma_num, sigma_den, act_log_hi, act_log_lo, f_is_one,
                                 verdict);
}

// TIMING PROBE: the GPU time of the plan's last waited-for window (events
// around its launches: input copy, the latency kernel, output), recorded when
// OURO_PLAN_TIMING was set at its submit; -1 otherwise.
int ouro_debug_plan_timing(ouro_tpraos_plan* p, float* gpu_ms, float* copy_us, float* launch_us) {
  if (!p) return fail(OURO_EINVAL, "null plan");
  if (gpu_ms) *gpu_ms = p->last_gpu_ms;
  if (copy_us) *copy_us = p->timed ? p->copy_us : -1.0f;
  if (launch_us) *launch_us = p->timed ? p->launch_us : -1.0f;
  return OURO_OK;
}

// Items the host path has verified: single items routed there, and host-
// buffer batches recomputed there after a device error.
int ouro_debug_host_path(unsigned long long* single_items, unsigned long long* recomputed_batches) {
  if (single_items) *single_items = g_host_single.load();
  if (recomputed_batches) *recomputed_batches = g_host_recompute.load();
  return OURO_OK;
}

// Contexts of the per-thread pool on `device` (kernels.hip ThreadCtx):
// created so far and idle (returned by exited threads).
int ouro_debug_contexts(int device, size_t* created, size_t* idle) {
  CtxPool& P = ctx_pool();
  std::lock_guard<std::mutex> g(P.mu);
  if (created) *created = P.created[device];
  if (idle) *idle = P.free[device].size();
  return OURO_OK;
}

}  // extern "C"

// ---- one process, several GPUs ----------------------------
// Persistent worker threads, pooled per device: a multi-device call borrows
// one worker per shard (a device listed k times gets k workers) and returns
// them when every shard is done, so two callers -- ChainSync windows and
// ChainDB's suffix re-validation, say -- run their calls at once on workers of
// their own instead of queueing behind one process-wide lock (VERDICT r05
// item 2).  A worker's thread-local context -- streams, device buffers,
// pinned staging, the raw-CBOR slots -- belongs to its one device and lives as
// long as the process, so repeated calls allocate nothing; the worker is
// bound to its GPU's NUMA node.  Each worker verifies one contiguous shard
// straight into the caller's buffers; in one process no collective is needed.
namespace {
struct Worker {
  std::mutex mu;
  std::condition_variable cv;
  bool has_job = false, done = false;
  int dev = 0, rc = OURO_OK;
  int numa_node = -1, bound_cpus = 0;
  std::string err;
  std::function<int()> job;

  void loop() {
    // this worker's host side -- its copies, its pinned staging (allocated
    // with hipHostMallocNumaUser), its gathers -- on the GPU's node
    numa_node = device_numa_node(dev);
    if (numa_node >= 0) bound_cpus = ouro_numa::bind_thread(numa_node);
    for (;;) {
      std::unique_lock<std::mutex> lk(mu);
      cv.wait(lk, [&] { return has_job; });
      has_job = false;
      std::function<int()> f = std::move(job);
      lk.unlock();
      int r = ouro_set_device(dev);
      // nothing thrown in a shard (a host allocation, say) may end the
      // process from this detached thread: it fails the shard instead
      if (r == OURO_OK) {
        try {
          r = f();
        } catch (const std::bad_alloc&) {
          r = fail(OURO_EDEVICE, "out of host memory");
        } catch (...) {
          r = fail(OURO_EDEVICE, "shard failed with an exception");
        }
      }
      lk.lock();
      rc = r;
      err = r ? t_last_error : std::string();
      done = true;
      cv.notify_all();
    }
  }
};

struct WorkerPool {
  std::mutex mu;
  std::map<int, std::vector<Worker*>> idle;  // per device
  std::vector<Worker*> all;                   // never freed: threads outlive every call
};
WorkerPool& worker_pool() {
  static WorkerPool* p = new WorkerPool;
  return *p;
}

// an idle worker of `dev`, or a new one; nullptr if no thread could be
// started (no exception ever crosses the C ABI)
Worker* borrow_worker(int dev) {
  WorkerPool& P = worker_pool();
  std::lock_guard<std::mutex> g(P.mu);
  std::vector<Worker*>& v = P.idle[dev];
  if (!v.empty()) {
    Worker* w = v.back();
    v.pop_back();
    return w;
  }
  Worker* w = new (std::nothrow) Worker;
  if (!w) return nullptr;
  w->dev = dev;
  try {
    P.all.reserve(P.all.size() + 1);
    std::thread([w] { w->loop(); }).detach();
  } catch (...) {
    delete w;
    return nullptr;
  }
  P.all.push_back(w);
  return w;
}

void return_worker(Worker* w) {
  WorkerPool& P = worker_pool();
  std::lock_guard<std::mutex> g(P.mu);
  P.idle[w->dev].push_back(w);
}

// the device list of a multi-device call (NULL: every visible device)
int multi_devices(const int* devices, int ndev, std::vector<int>* devs) {
  const int count = ouro_device_count();
  if (devices) {
    if (ndev <= 0 || ndev > 64) return fail(OURO_EINVAL, "bad device count");
    devs->assign(devices, devices + ndev);
    for (int d : *devs)
      if (d < 0 || d >= count) return fail(OURO_ENODEV, "no such device " + std::to_string(d));
  } else {
    for (int d = 0; d < count; d++) devs->push_back(d);
    if (devs->empty()) return fail(OURO_ENODEV, "no device");
  }
  return OURO_OK;
}

// n items in contiguous shards of ceil(n / G) over the listed devices, shard
// k = job(k's first item, its count) on a borrowed worker of devices[k]; the
// first failing shard's code (its message prefixed with the device)
template <class Job>
int run_multi(const std::vector<int>& devs, size_t n, Job&& job) {
  const size_t g = std::min<size_t>(devs.size(), n);
  const size_t per = (n + g - 1) / g;
  // every shard's worker first, so a worker that cannot be started fails the
  // call before any shard runs
  std::vector<Worker*> used;
  for (size_t k = 0; k < g && k * per < n; k++) {
    Worker* w = borrow_worker(devs[k]);
    if (!w) {
      for (Worker* u : used) return_worker(u);
      return fail(OURO_EDEVICE, "cannot start a worker thread for device " +
                                    std::to_string(devs[k]));
    }
    used.push_back(w);
  }
  for (size_t k = 0; k < used.size(); k++) {
    const size_t lo = k * per;
    const size_t m = std::min(per, n - lo);
    Worker* w = used[k];
    {
      std::lock_guard<std::mutex> lk(w->mu);
      w->job = [&job, lo, m] { return job(lo, m); };
      w->done = false;
      w->has_job = true;
    }
    w->cv.notify_all();
  }
  int rc = OURO_OK;
  for (Worker* w : used) {  // wait for every shard, errors included
    {
      std::unique_lock<std::mutex> lk(w->mu);
      w->cv.wait(lk, [&] { return w->done; });
      if (w->rc && rc == OURO_OK) {
        rc = w->rc;
        t_last_error = "device " + std::to_string(w->dev) + ": " + w->err;
      }
    }
    return_worker(w);
  }
  return rc;
}

ouro_tpraos_batch shard_of(const ouro_tpraos_batch& b, size_t lo, size_t m) {
  ouro_tpraos_batch s = b;  // body + absolute offsets shared, epoch_nonce shared
  s.n = m;
  s.issuer_vk = b.issuer_vk + 32 * lo;
  s.vrf_vk = b.vrf_vk + 32 * lo;
  s.eta_proof = b.eta_proof + 80 * lo;
  s.leader_proof = b.leader_proof + 80 * lo;
  if (b.eta_alpha) s.eta_alpha = b.eta_alpha + 32 * lo;
  if (b.leader_alpha) s.leader_alpha = b.leader_alpha + 32 * lo;
  s.hot_vk = b.hot_vk + 32 * lo;
  s.ocert_counter = b.ocert_counter + lo;
  s.ocert_kes_period = b.ocert_kes_period + lo;
  s.ocert_sigma = b.ocert_sigma + 64 * lo;
  s.kes_t = b.kes_t + lo;
  s.kes_sig = b.kes_sig + 448 * lo;
  s.body_off = b.body_off + lo;
  s.body_len = b.body_len + lo;
  if (b.eta_output) s.eta_output = b.eta_output + 64 * lo;
  if (b.leader_output) s.leader_output = b.leader_output + 64 * lo;
  if (b.slot) s.slot = b.slot + lo;
  if (b.eta_nonce) s.eta_nonce = b.eta_nonce + 32 * lo;
  return s;
}

// shard [lo, lo + m) of a raw-CBOR call: the buffer and its offsets are
// shared (the offsets are absolute into raw), every per-header array offset
RawCall raw_shard(const RawCall& c, size_t lo, size_t m) {
  RawCall s = c;
  s.n = m;
  s.off = c.off + lo;
  s.len = c.len + lo;
  if (c.ea) s.ea = c.ea + 32 * lo;
  if (c.la) s.la = c.la + 32 * lo;
  s.status = c.status + lo;
  s.verdict = c.verdict + lo;
  if (c.be) s.be = c.be + 64 * lo;
  if (c.bl) s.bl = c.bl + 64 * lo;
  if (c.nonce) s.nonce = c.nonce + 32 * lo;
  return s;
}

// a raw-CBOR call over several devices: its argument checks once, then each
// shard through the one-device pipeline (raw_verify: chunks over the worker's
// slots, the host-path recompute of that shard after a device error)
int raw_verify_multi(const RawCall& c, const int* devices, int ndev) {
  if (c.n == 0) return OURO_OK;
  if (!c.raw || !c.off || !c.len || !c.status || !c.verdict)
    return fail(OURO_EINVAL, "null argument");
  for (size_t i = 0; i < c.n; i++)  // every span inside raw before any shard starts
    if (c.off[i] > c.raw_bytes || c.raw_bytes - c.off[i] < c.len[i])
      return fail(OURO_EINVAL, "header " + std::to_string(i) + ": span outside raw_bytes");
  std::vector<int> devs;
  int rc = multi_devices(devices, ndev, &devs);
  if (rc) return rc;
  return run_multi(devs, c.n, [&](size_t lo, size_t m) { return raw_verify(raw_shard(c, lo, m)); });
}
}  // namespace

extern "C" {

int ouro_device_count(void) {
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess) return 0;
  return count;
}

int ouro_device_numa_node(int device) {
  const int count = ouro_device_count();
  if (device < 0 || device >= count) return fail(OURO_ENODEV, "no such device");
  return device_numa_node(device);
}

int ouro_bind_thread_to_device(int device) {
  const int node = ouro_device_numa_node(device);
  if (node >= 0) ouro_numa::bind_thread(node);
  return node;
}

int ouro_debug_multi_workers(int* devices, int* nodes, int* cpus, int max) {
  WorkerPool& P = worker_pool();
  std::lock_guard<std::mutex> guard(P.mu);
  int k = 0;
  for (Worker* w : P.all) {
    if (k < max) {
      if (devices) devices[k] = w->dev;
      if (nodes) nodes[k] = w->numa_node;
      if (cpus) cpus[k] = w->bound_cpus;
    }
    k++;
  }
  return k;
}

int ouro_tpraos_verify_batch_multi(const ouro_tpraos_batch* b, const int* devices, int ndev,
                                   uint8_t* verdict, uint8_t* beta_eta, uint8_t* beta_leader) {
  if (!b) return fail(OURO_EINVAL, "null batch");
  if (b->n == 0) return OURO_OK;
  if (!verdict) return fail(OURO_EINVAL, "null verdict");
  int rc = check_hdr_batch(b);
  if (rc) return rc;
  std::vector<int> devs;
  if ((rc = multi_devices(devices, ndev, &devs))) return rc;
  return run_multi(devs, b->n, [&](size_t lo, size_t m) {
    const ouro_tpraos_batch s = shard_of(*b, lo, m);
    return ouro_tpraos_verify_batch(&s, verdict + lo, beta_eta ? beta_eta + 64 * lo : nullptr,
                                    beta_leader ? beta_leader + 64 * lo : nullptr);
  });
}

// The raw-CBOR entries over several devices of one process (SURVEY.md §8(e):
// static contiguous shards, one per listed device, each on that device's
// NUMA-bound worker with its own chunk pipeline and pinned staging; results
// straight into the caller's buffers).
int ouro_tpraos_verify_cbor_multi(const int* devices, int ndev, const uint8_t* raw,
                                  size_t raw_bytes, const uint64_t* off, const uint32_t* len,
                                  size_t n, uint64_t slots_per_kes_period,
                                  const uint8_t* epoch_nonce, const uint8_t* eta_alpha,
                                  const uint8_t* leader_alpha, uint8_t* status, uint8_t* verdict,
                                  uint8_t* beta_eta, uint8_t* beta_leader, uint8_t* eta_nonce) {
  if (n && slots_per_kes_period == 0) return fail(OURO_EINVAL, "zero slots per KES period");
  if ((eta_alpha == nullptr) != (leader_alpha == nullptr))
    return fail(OURO_EINVAL, "give both VRF input arrays or neither");
  RawCall c{kRawHdr, raw, raw_bytes, off, len, n, slots_per_kes_period, epoch_nonce, eta_alpha,
            leader_alpha, status, verdict, beta_eta, beta_leader, eta_nonce};
  return raw_verify_multi(c, devices, ndev);
}

int ouro_integrity_verify_cbor_multi(const int* devices, int ndev, const uint8_t* raw,
                                     size_t raw_bytes, const uint64_t* off, const uint32_t* len,
                                     size_t n, uint64_t slots_per_kes_period, uint8_t* status,
                                     uint8_t* verdict) {
  if (n && slots_per_kes_period == 0) return fail(OURO_EINVAL, "zero slots per KES period");
  RawCall c{kRawKes, raw, raw_bytes, off, len, n, slots_per_kes_period, nullptr, nullptr,
            nullptr, status, verdict, nullptr, nullptr, nullptr};
  return raw_verify_multi(c, devices, ndev);
}

int ouro_byron_verify_cbor_multi(const int* devices, int ndev, const uint8_t* raw,
                                 size_t raw_bytes, const uint64_t* off, const uint32_t* len,
                                 size_t n, int64_t protocol_magic, uint8_t* status,
                                 uint8_t* verdict) {
  if (protocol_magic < -1 || protocol_magic > (int64_t)0xffffffffll)
    return fail(OURO_EINVAL, "protocol magic outside Word32 (or -1)");
  RawCall c{kRawByron, raw, raw_bytes, off, len, n, 0, nullptr, nullptr, nullptr, status,
            verdict, nullptr, nullptr, nullptr, protocol_magic};
  return raw_verify_multi(c, devices, ndev);
}

}  // extern "C"
