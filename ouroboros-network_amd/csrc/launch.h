// launch.h -- launch shape, slot sizes and vector helpers shared by the
// kernel translation units (kernels.hip, kernels_lat.hip).
#pragma once
#include "tpraos.h"

namespace ouro {

constexpr int kBlock = 256;
// resident waves per SIMD the kernels are compiled for (VGPR budget 512 / W)
#ifndef OURO_WAVES
#define OURO_WAVES 2
#endif
// throughput header kernel: scratch slot + the per-header result record
// rounded up to whole 128-B lines (OURO_SLOT_ALIGN): every table entry then
// starts 32-B aligned and a gathered 160-B entry touches exactly two lines
#ifndef OURO_SLOT_ALIGN
#define OURO_SLOT_ALIGN 32
#endif
constexpr int round_slot(int w) { return (w + OURO_SLOT_ALIGN - 1) / OURO_SLOT_ALIGN * OURO_SLOT_ALIGN; }
constexpr int kHdrLaneWords = round_slot(kLaneWords + kResWords);
constexpr int kSlotWords = round_slot(kLaneWords);  // the other kernels' slots
constexpr int kLatBlock = 64;  // default latency-mode workgroup (lat_block(); A/B: tools/ab_latency.py)

__device__ __forceinline__ void load_words(uint32_t* w, const uint8_t* p, int nwords16) {
#pragma unroll
  for (int i = 0; i < nwords16; i++) {
    const int4 v = ldg4(p + 16 * i);
    w[4 * i] = v.x; w[4 * i + 1] = v.y; w[4 * i + 2] = v.z; w[4 * i + 3] = v.w;
  }
}
__device__ __forceinline__ void store_words(uint8_t* p, const uint32_t* w, int nwords16) {
#pragma unroll
  for (int i = 0; i < nwords16; i++)
    stg4(p + 16 * i, make_int4((int)w[4 * i], (int)w[4 * i + 1], (int)w[4 * i + 2], (int)w[4 * i + 3]));
}

__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }


}  // namespace ouro
