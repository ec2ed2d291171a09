// host_path.h -- the product's host (CPU) path: the same lane routines the
// kernels run (verify.h, tpraos.h, leader.h), compiled for x86 in
// host_path.hip and called by the runtime in kernels.hip.
//
// Two uses (VERDICT r03 "next" item 4; SURVEY.md §5 and §8(b) "Errors"):
//   * single items.  The reference calls the crypto one header at a time
//     (ouroboros-consensus-shelley/src/Ouroboros/Consensus/Shelley/Protocol.hs:433-442,
//     .../Shelley/Ledger/Integrity.hs:20-44,
//     ouroboros-consensus-byron/src/Ouroboros/Consensus/Byron/Crypto/DSIGN.hs:110-113);
//     a GPU round trip per call costs ~220-420 us, this path ~1.5x libsodium;
//   * the recompute path after a device or runtime error: a host-buffer batch
//     whose launch fails is verified here instead, never reported valid
//     without having been verified.
// Not the oracle: nothing under oracle/ is compiled into or loaded by the
// product.  Plain host memory, any alignment (common.h host accessors).
#pragma once
#include <stddef.h>
#include <stdint.h>

#include "../../include/ouro_verify.h"

namespace ouro_host {

// The fixed-base niels tables (verify.h build_btab), built once per process
// on first use; the device runtime uploads the same copy.
const int32_t* btab();

// Batches over host buffers, split over host threads; each returns OURO_OK.
// Same arguments and outputs as the ouro_*_batch calls they back.
int ed_batch(size_t n, const uint8_t* pk, const uint8_t* sig, const uint8_t* msg,
             const uint64_t* off, const uint32_t* len, uint8_t* verdict, uint32_t byron);
int vrf_batch(size_t n, const uint8_t* pk, const uint8_t* proof, const uint8_t* alpha,
              const uint64_t* off, const uint32_t* len, uint8_t* beta, uint8_t* verdict,
              uint32_t flags);
int kes_batch(size_t n, const uint8_t* vk, const uint32_t* t, const uint8_t* msg,
              const uint64_t* off, const uint32_t* len, const uint8_t* sig, uint8_t* verdict);
int hdr_batch(const ouro_tpraos_batch* b, uint8_t* verdict, uint8_t* beta_eta,
              uint8_t* beta_leader);
int leader_batch(size_t n, const uint8_t* beta, const uint64_t* num, const uint64_t* den,
                 int64_t act_log_hi, uint64_t act_log_lo, int f_is_one, uint8_t* verdict);
// proof_to_hash without verification: OURO_OK and out written, or OURO_INVALID
int proof_to_hash(uint8_t* out, const uint8_t* proof);

// Threads a batch of n items uses (OURO_HOST_THREADS caps it; default: the
// CPUs this process may run on, at most 64, and at least 16 items each).
int threads_for(size_t n);

}  // namespace ouro_host
