// common.h -- shared macros for the gfx950 verifier kernels.
//
// Every lane-level routine is `__host__ __device__` so the exact code the
// kernels run can also be compiled for the host by hipcc and exercised in the
// CPU test suite (tests/test_devcode_host.py) without a GPU.  The product
// library runs them inside kernels and, since round 4, on the host for single
// items and as the recompute path after a device error (host_path.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define OURO_HD __host__ __device__
#define OURO_FI __host__ __device__ __forceinline__
// Out-of-line routines have external linkage, one definition per library
// (kernels.hip); the host path's translation unit (host_path.hip) defines
// OURO_NI_LINKAGE static to keep its own host copies apart.
#ifndef OURO_NI_LINKAGE
#define OURO_NI_LINKAGE
#endif
#define OURO_NI __host__ __device__ __noinline__ OURO_NI_LINKAGE

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

// ---- global-memory accessors --------------------------------------------------
// Every buffer the lane routines touch (inputs, outputs, scratch slots, the B
// tables) is device global memory, but a pointer that crosses an out-of-line
// call or a struct is generic to LLVM, which then emits FLAT instructions:
// those count on both vmcnt and lgkmcnt, so any s_waitcnt lgkmcnt(0) for a
// scalar load also waits for every table prefetch in flight.  These accessors
// cast to address space 1 (global_load / global_store, vmcnt only).
#if defined(__HIP_DEVICE_COMPILE__)
#define OURO_AS1 __attribute__((address_space(1)))
typedef int ouro_v4i __attribute__((ext_vector_type(4)));
typedef int ouro_v2i __attribute__((ext_vector_type(2)));
OURO_FI int4 ldg4(const void* p) {
  const ouro_v4i v = *(const OURO_AS1 ouro_v4i*)p;
  return make_int4(v.x, v.y, v.z, v.w);
}
OURO_FI int2 ldg2(const void* p) {
  const ouro_v2i v = *(const OURO_AS1 ouro_v2i*)p;
  return make_int2(v.x, v.y);
}
OURO_FI int32_t ldg1(const void* p) { return *(const OURO_AS1 int32_t*)p; }
OURO_FI uint64_t ldg8(const void* p) { return *(const OURO_AS1 uint64_t*)p; }
OURO_FI uint32_t ldg_u8(const void* p) { return *(const OURO_AS1 uint8_t*)p; }
OURO_FI uint32_t ldg_u16(const void* p) { return *(const OURO_AS1 uint16_t*)p; }
OURO_FI void stg4(void* p, int4 v) {
  *(OURO_AS1 ouro_v4i*)p = ouro_v4i{v.x, v.y, v.z, v.w};
}
OURO_FI void stg2(void* p, int2 v) { *(OURO_AS1 ouro_v2i*)p = ouro_v2i{v.x, v.y}; }
OURO_FI void stg1(void* p, int32_t v) { *(OURO_AS1 int32_t*)p = v; }
OURO_FI void stg8(void* p, uint64_t v) { *(OURO_AS1 uint64_t*)p = v; }
#else
// Host: byte-wise copies, so the host path (host_path.hip) reads the caller's
// buffers at any alignment (the kernels' inputs are 16-B aligned device
// buffers; a host caller's ByteStrings need not be).  Same code at -O2.
template <class T>
OURO_FI T ldh(const void* p) {
  T v;
  __builtin_memcpy(&v, p, sizeof(T));
  return v;
}
template <class T>
OURO_FI void sth(void* p, const T& v) {
  __builtin_memcpy(p, &v, sizeof(T));
}
OURO_FI int4 ldg4(const void* p) { return ldh<int4>(p); }
OURO_FI int2 ldg2(const void* p) { return ldh<int2>(p); }
OURO_FI int32_t ldg1(const void* p) { return ldh<int32_t>(p); }
OURO_FI uint64_t ldg8(const void* p) { return ldh<uint64_t>(p); }
OURO_FI uint32_t ldg_u8(const void* p) { return *static_cast<const uint8_t*>(p); }
OURO_FI uint32_t ldg_u16(const void* p) { return ldh<uint16_t>(p); }
OURO_FI void stg4(void* p, int4 v) { sth(p, v); }
OURO_FI void stg2(void* p, int2 v) { sth(p, v); }
OURO_FI void stg1(void* p, int32_t v) { sth(p, v); }
OURO_FI void stg8(void* p, uint64_t v) { sth(p, v); }
#endif

}  // namespace ouro
