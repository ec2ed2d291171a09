// common.h -- shared macros for the gfx950 verifier kernels.
//
// Every lane-level routine is `__host__ __device__` so the exact code the
// kernels run can also be compiled for the host by hipcc and exercised in the
// CPU test suite (tests/test_devcode_host.py) without a GPU.  The product
// library only ever runs these routines inside kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define OURO_HD __host__ __device__
#define OURO_FI __host__ __device__ __forceinline__
#define OURO_NI __host__ __device__ __noinline__

namespace ouro {

OURO_FI uint32_t ld_le32(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

// 8 little-endian words <-> 32 bytes
OURO_FI void bytes_to_words8(uint32_t w[8], const uint8_t* p) {
#pragma unroll
  for (int i = 0; i < 8; i++) w[i] = ld_le32(p + 4 * i);
}

OURO_FI uint32_t byte_of(const uint32_t* w, int i) { return (w[i >> 2] >> (8 * (i & 3))) & 0xffu; }

}  // namespace ouro
