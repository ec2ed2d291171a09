// The production double-scalar multiplication (verify.h dsm_lane: per-lane
// tables in scratch slots, packed entries, the window loop) at 2, 3 or 4
// waves per SIMD (round 4).  tools/microbench/occupancy.hip showed a lone
// doubling runs 13 % faster per op at 4 waves than at 2 when its chain fits
// 128 VGPRs; the header kernel is held at 2 by its other phases (decodes,
// hashes, the finish).  This measures what the real window loop -- table
// gathers included -- gains at each occupancy, to size a split of the header
// kernel into a 2-wave prepare / finish and an N-wave dsm phase.
//
// Build (one binary per occupancy: the callee's VGPR budget follows its
// kernel's launch bounds):
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -DMB_WAVES=4 -o dsm_w4 dsm_occupancy.hip
// Run: ./dsm_w4 [items]  -> one JSON line (ms per launch, ns per dsm chip-wide)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../ouroboros-network_amd/csrc/verify.h"

#ifndef MB_WAVES
#define MB_WAVES 2
#endif

#define CHECK(x)                                                                          \
  do {                                                                                    \
    hipError_t e_ = (x);                                                                  \
    if (e_ != hipSuccess) {                                                               \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));          \
      exit(1);                                                                            \
    }                                                                                     \
  } while (0)

using namespace ouro;

// per item: tables of B and -B's multiples (any valid points do: the work is
// data-independent), a1 a 253-bit and a2 a 128-bit pseudo-random scalar
__global__ void __launch_bounds__(256, 2) k_prep(int32_t* slots, size_t n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const Slot lane = slot_of(slots, i, kLaneWords);
  uint32_t enc[8];
  enc[0] = 0x66666658u;
#pragma unroll
  for (int k = 1; k < 8; k++) enc[k] = 0x66666666u;
  ge_p3 P;
  (void)ge_decode(&P, enc, false);
  build_table(lane + kSlotTab1, P);
  build_table(lane + kSlotTab2, ge_p3_neg(P));
  uint32_t a1[8], a2[8], b[8];
  uint32_t x = (uint32_t)i * 2654435761u + 12345u;
#pragma unroll
  for (int k = 0; k < 8; k++) {
    x ^= x << 13; x ^= x >> 17; x ^= x << 5;
    a1[k] = x;
    x ^= x << 13; x ^= x >> 17; x ^= x << 5;
    a2[k] = k < 4 ? x : 0u;
    b[k] = 0u;
  }
  a1[7] &= 0x0fffffffu;
  st_words8(lane + kSlotA1, a1);
  st_words8(lane + kSlotA2, a2);
  st_words8(lane + kSlotB, b);
  st_carry(lane, 0, sc_recode_carries<4, 64>(a1));
  st_carry(lane, 1, sc_recode_carries<4, 33>(a2));
  st_carry(lane, 2, 0);
}

__global__ void __launch_bounds__(256, MB_WAVES) k_dsm(int32_t* slots, size_t n, uint32_t cfg) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    dsm_lane(slot_of(slots, i, kLaneWords), nullptr, cfg);
}

// fold of the results (so a variant that computes something else shows)
__global__ void k_fold(const int32_t* slots, size_t n, unsigned long long* out) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const Slot lane = slot_of(const_cast<int32_t*>(slots), i, kLaneWords);
  uint32_t x = 0;
  for (int w = 0; w < 36; w++) x = x * 31u + (uint32_t)*lane.word(kSlotOut + w);
  atomicAdd(out, (unsigned long long)x);
}

int main(int argc, char** argv) {
  const size_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : 524288;
  int32_t* slots;
  CHECK(hipMalloc(&slots, slot_region_words(n, kLaneWords) * sizeof(int32_t)));
  unsigned long long* d_fold;
  CHECK(hipMalloc(&d_fold, sizeof(unsigned long long)));
  CHECK(hipMemset(d_fold, 0, sizeof(unsigned long long)));
  const int blocks = (int)((n + 255) / 256);
  hipLaunchKernelGGL(k_prep, dim3(blocks), dim3(256), 0, 0, slots, n);
  CHECK(hipGetLastError());
  int per_cu = 0;
  CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_dsm, 256, 0));
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int grid = std::min<int>(blocks, per_cu * prop.multiProcessorCount);
  const uint32_t cfg = dsm_cfg(64, 33, false, 0, 1);  // a VRF V core: [a1]T1 + [a2]T2
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL(k_dsm, dim3(grid), dim3(256), 0, 0, slots, n, cfg);  // warm-up
  CHECK(hipDeviceSynchronize());
  std::vector<float> ms;
  for (int r = 0; r < 7; r++) {
    CHECK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(k_dsm, dim3(grid), dim3(256), 0, 0, slots, n, cfg);
    CHECK(hipEventRecord(e1, 0));
    CHECK(hipEventSynchronize(e1));
    float t;
    CHECK(hipEventElapsedTime(&t, e0, e1));
    ms.push_back(t);
  }
  hipLaunchKernelGGL(k_fold, dim3(blocks), dim3(256), 0, 0, slots, n, d_fold);
  unsigned long long fold;
  CHECK(hipMemcpy(&fold, d_fold, sizeof fold, hipMemcpyDeviceToHost));
  std::sort(ms.begin(), ms.end());
  printf("{\"waves\": %d, \"blocks_per_cu\": %d, \"items\": %zu, \"median_ms\": %.4f, "
         "\"min_ms\": %.4f, \"ns_per_dsm_chip\": %.4f, \"fold\": \"%016llx\"}\n",
         MB_WAVES, per_cu, n, ms[3], ms[0], ms[3] * 1e6 / (double)n, fold);
  return 0;
}
