// kernels_lat.hip -- the latency-mode kernels (configs[4] ChainSync windows):
// eight cores per header on DPP lane quads, then the lane-pair finish.
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

using namespace ouro;

// Latency mode, launch 1: eight cores per header (work item w = core * n + i,
// so each wave runs one core type), results to a per-header record.
// quad = 1: each work item runs on the four lanes of a DPP quad, which share
// its scratch slot and split every group operation's products (ge25519.h);
// quad = 0: one lane per item.  n (d_n[0]) and the batch's optional members
// (d_n[1], tpraos.h kOpt*) are read from device memory so a captured graph
// serves any batch of n <= capacity.
__global__ void __launch_bounds__(kBlock, OURO_WAVES) k_tpraos_cores(ouro_tpraos_batch b,
                                                            const uint32_t* __restrict__ d_n,
                                                            int32_t* res_buf, int32_t* scratch,
                                                            const int32_t* __restrict__ btab,
                                                            int quad) {
  const size_t n = d_n[0];
  const uint32_t opts = d_n[1];
  const int sh = quad ? 2 : 0;
  const size_t tid = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> sh;
  const size_t nth = ((size_t)gridDim.x * blockDim.x) >> sh;
  const Slot lane = slot_of(scratch, tid, kSlotWords);
  for (size_t w = tid; w < (size_t)kLatCores * n; w += nth) {
    const int core = (int)(w / n);
    const size_t i = w - (size_t)core * n;
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

