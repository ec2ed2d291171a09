// Component microbenchmark: the lane routines of csrc/ (the exact code the
// product kernels run) timed one at a time at the header kernel's occupancy,
// so the header's cost can be split into its parts and each part compared
// with its field-operation count x the measured fe_mul / fe_sq rates
// (fe_mul_variants.hip).  Inputs are valid points/scalars derived from a seed;
// every kernel folds its results into one output word so nothing is dropped.
//
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o components components.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../ouroboros-network_amd/csrc/tpraos.h"

using namespace ouro;

#define CHECK(x)                                                                          \
  do {                                                                                    \
    hipError_t e_ = (x);                                                                  \
    if (e_ != hipSuccess) {                                                               \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));          \
      exit(1);                                                                            \
    }                                                                                     \
  } while (0)

constexpr int kBlock = 256;
#ifndef COMP_WAVES
#define COMP_WAVES 2  // resident waves per SIMD (blocks per CU, launch bounds)
#endif

__device__ void seed_words(uint32_t w[8], uint32_t s) {
  for (int i = 0; i < 8; i++) {
    s ^= s << 13; s ^= s >> 17; s ^= s << 5;
    w[i] = s;
  }
  w[7] &= 0x0fffffffu;  // < 2^252 < L
}

// the base point's encoding
__device__ void base_words(uint32_t w[8]) {
  for (int i = 0; i < 8; i++) w[i] = 0x66666666u;
  w[0] = 0x66666658u;
}

enum Comp { kHalf = 0, kSha1, kPow, kDecode, kTable, kDsmEd, kDsmU, kDsmV, kElligator, kEdFull,
            kVrfFull, kSc512, kDbl, kAddLd, kAddReg, kMulChain, kTo3, kNumComp };
const char* kNames[kNumComp] = {"half_scalars", "sha512_64+32", "fe_pow22523", "ge_decode",
                                "build_table", "dsm_ed(34,34,B split)", "dsm_U(33,-,B split)",
                                "dsm_V(64,33)", "elligator2_h", "ed25519_verify_lane",
                                "vrf03_verify_lane", "sc_reduce512", "x256 p2 doublings",
                                "x64 adds (table loads)", "x64 adds (register q)",
                                "x512 fe_mul chain", "x64 p1p1_to_p3 (4M)"};

template <int C>
__global__ void __launch_bounds__(kBlock, COMP_WAVES) kcomp(int32_t* scratch, const int32_t* btab,
                                                   const uint8_t* msgs, uint32_t* out, int iters) {
  const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  int32_t* lane = scratch + tid * kLaneWords;
  uint32_t w[8];
  seed_words(w, (uint32_t)tid * 2654435761u + 12345u);
  uint32_t acc = 0;
  ge_p3 B;
  uint32_t bw[8];
  base_words(bw);
  ge_decode(&B, bw, false);
  if constexpr (C == kTable || C == kDsmEd || C == kDsmU || C == kDsmV || C == kAddLd ||
                C == kAddReg) {
    build_table(lane + kSlotTab1, B);
    build_table(lane + kSlotTab2, B);
    build_table(lane + kSlotTab3, B);
  }
#pragma unroll 1
  for (int it = 0; it < iters; it++) {
    w[0] ^= acc;
    if constexpr (C == kHalf) {
      HalfScalars hs;
      ed25519_half_scalars(hs, w);
      acc += hs.c0[0] ^ hs.c1[1] ^ (uint32_t)hs.bits;
    } else if constexpr (C == kSha1) {
      uint32_t pre[16];
      for (int i = 0; i < 16; i++) pre[i] = w[i & 7] + i;
      uint64_t H[8];
      sha512_prefixed<64>(H, pre, ShaGlobalTail{msgs + 32 * (tid & 1023)}, 32);
      acc += (uint32_t)H[0] ^ (uint32_t)(H[7] >> 32);
    } else if constexpr (C == kPow) {
      fe x = fe_from_words(w);
      fe y = fe_pow22523(x);
      uint32_t o[8];
      fe_to_words(o, y);
      acc += o[0];
    } else if constexpr (C == kDecode) {
      ge_p3 P;
      uint32_t s[8];
      for (int i = 0; i < 8; i++) s[i] = bw[i];
      s[0] ^= (w[0] & 0xff);  // mostly-valid y values near B's
      const bool ok = ge_decode(&P, s, true);
      uint32_t o[8];
      fe_to_words(o, P.T);
      acc += o[1] + ok;
    } else if constexpr (C == kTable) {
      build_table(lane + kSlotTab1, B);
      acc += (uint32_t)lane[kSlotTab1 + 7 * kCachedWords + (acc & 7)];
      B.X.v[0] ^= acc & 1;
    } else if constexpr (C == kDsmEd || C == kDsmU || C == kDsmV) {
      uint32_t a2[8];
      for (int i = 0; i < 8; i++) a2[i] = w[7 - i] & (i >= 4 ? 0u : 0xffffffffu);
      uint32_t a1[8];
      for (int i = 0; i < 8; i++) a1[i] = (C == kDsmV) ? w[i] : (i >= 4 ? 0u : w[i]);
      st_words8(lane + kSlotA1, a1);
      st_words8(lane + kSlotA2, a2);
      st_words8(lane + kSlotB, w);
      uint64_t* carr = reinterpret_cast<uint64_t*>(lane + kSlotCarry);
      carr[0] = sc_recode_carries<4, 64>(a1);
      carr[1] = sc_recode_carries<4, 64>(a2);
      carr[2] = sc_recode_b(w);
      const uint32_t cfg = C == kDsmEd ? dsm_cfg(34, 34, true, 0, 1)
                         : C == kDsmU  ? dsm_cfg(33, 0, true, 0, 1)
                                       : dsm_cfg(64, 33, false, 0, 1);
      dsm(lane, btab, cfg);
      acc += (uint32_t)lane[kSlotOut + (acc & 7)];
    } else if constexpr (C == kElligator) {
      ge_p3 H = elligator2_h(w);
      uint32_t o[8];
      fe_to_words(o, H.Y);
      acc += o[2];
    } else if constexpr (C == kEdFull) {
      uint32_t sig[16];
      for (int i = 0; i < 8; i++) { sig[i] = bw[i]; sig[8 + i] = w[i]; }
      const bool ok = ed25519_verify_lane(sig, bw, ShaGlobalTail{msgs + 32 * (tid & 1023)}, 32,
                                          lane, btab);
      acc += ok ? 1u : 3u;
    } else if constexpr (C == kVrfFull) {
      uint32_t pi[20], beta[16];
      for (int i = 0; i < 8; i++) { pi[i] = bw[i]; pi[12 + i] = w[i]; }
      for (int i = 0; i < 4; i++) pi[8 + i] = w[i] ^ 0x5a5a5a5au;
      const bool ok = vrf03_verify_lane(beta, bw, pi, ShaGlobalTail{msgs + 32 * (tid & 1023)}, 32,
                                        lane, btab);
      acc += beta[3] + ok;
    } else if constexpr (C == kDbl) {
      ge_p1p1 t{B.X, B.Y, B.Z, B.Z};
      t.X.v[0] ^= acc & 1;
#pragma unroll 1
      for (int k = 0; k < 256; k++) t = ge_p2_dbl(ge_p1p1_to_p2(t));
      uint32_t o[8];
      fe_to_words(o, t.X);
      acc += o[0];
    } else if constexpr (C == kAddLd || C == kAddReg) {
      ge_p1p1 t{B.X, B.Y, B.Z, B.Z};
      t.X.v[0] ^= acc & 1;
      const ge_cached qr = ld_cached(lane + kSlotTab1 + 3 * kCachedWords);
      uint32_t r = w[1] | 1u;
#pragma unroll 1
      for (int k = 0; k < 64; k++) {
        r = r * 1664525u + 1013904223u;
        const int idx = (int)(r >> 29);
        const ge_cached q = C == kAddLd ? ld_cached(lane + kSlotTab1 + idx * kCachedWords) : qr;
        t = ge_add_cached(ge_p1p1_to_p3(t), q, (r >> 28) & 1);
      }
      uint32_t o[8];
      fe_to_words(o, t.X);
      acc += o[0];
    } else if constexpr (C == kMulChain) {
      fe x = B.X, y = B.Y;
      x.v[0] ^= acc & 1;
#pragma unroll 1
      for (int k = 0; k < 512; k++) x = fe_mul(x, y);
      uint32_t o[8];
      fe_to_words(o, x);
      acc += o[0];
    } else if constexpr (C == kTo3) {
      ge_p1p1 t{B.X, B.Y, B.Z, B.T};
      t.X.v[0] ^= acc & 1;
#pragma unroll 1
      for (int k = 0; k < 64; k++) {
        ge_p3 q = ge_p1p1_to_p3(t);
        t = ge_p1p1{q.X, q.Y, q.Z, q.T};
      }
      uint32_t o[8];
      fe_to_words(o, t.X);
      acc += o[0];
    } else if constexpr (C == kSc512) {
      uint32_t x[16], r[8];
      for (int i = 0; i < 16; i++) x[i] = w[i & 7] * (i + 1);
      sc_reduce512(r, x);
      acc += r[0] ^ r[7];
    }
  }
  out[tid] = acc;
}

template <int C>
double time_comp(int32_t* scr, const int32_t* btab, const uint8_t* msgs, uint32_t* out, int blocks,
                 int iters) {
  hipLaunchKernelGGL(kcomp<C>, dim3(blocks), dim3(kBlock), 0, 0, scr, btab, msgs, out, 1);
  CHECK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  CHECK(hipEventRecord(e0, 0));
  hipLaunchKernelGGL(kcomp<C>, dim3(blocks), dim3(kBlock), 0, 0, scr, btab, msgs, out, iters);
  CHECK(hipEventRecord(e1, 0));
  CHECK(hipEventSynchronize(e1));
  float ms;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  // GPU-time per operation (ns): launch time / operations executed by the whole grid
  return (double)ms * 1e6 / ((double)blocks * kBlock * iters);
}

int main(int argc, char** argv) {
  CHECK(hipSetDevice(0));
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int blocks = prop.multiProcessorCount * COMP_WAVES;  // one resident grid
  const size_t lanes = (size_t)blocks * kBlock;
  int32_t *scr, *btab;
  uint32_t* out;
  uint8_t* msgs;
  CHECK(hipMalloc(&scr, lanes * kLaneWords * 4));
  CHECK(hipMalloc(&btab, kBTabWords * 4));
  CHECK(hipMalloc(&out, lanes * 4));
  CHECK(hipMalloc(&msgs, 32 * 1024));
  std::vector<int32_t> tab(kBTabWords);
  build_btab(tab.data());
  CHECK(hipMemcpy(btab, tab.data(), kBTabWords * 4, hipMemcpyHostToDevice));
  std::vector<uint8_t> m(32 * 1024);
  for (size_t i = 0; i < m.size(); i++) m[i] = (uint8_t)(i * 131 + 7);
  CHECK(hipMemcpy(msgs, m.data(), m.size(), hipMemcpyHostToDevice));
  double ns[kNumComp];
  ns[kHalf] = time_comp<kHalf>(scr, btab, msgs, out, blocks, 64);
  ns[kSha1] = time_comp<kSha1>(scr, btab, msgs, out, blocks, 64);
  ns[kPow] = time_comp<kPow>(scr, btab, msgs, out, blocks, 16);
  ns[kDecode] = time_comp<kDecode>(scr, btab, msgs, out, blocks, 16);
  ns[kTable] = time_comp<kTable>(scr, btab, msgs, out, blocks, 16);
  ns[kDsmEd] = time_comp<kDsmEd>(scr, btab, msgs, out, blocks, 4);
  ns[kDsmU] = time_comp<kDsmU>(scr, btab, msgs, out, blocks, 4);
  ns[kDsmV] = time_comp<kDsmV>(scr, btab, msgs, out, blocks, 2);
  ns[kElligator] = time_comp<kElligator>(scr, btab, msgs, out, blocks, 8);
  ns[kEdFull] = time_comp<kEdFull>(scr, btab, msgs, out, blocks, 2);
  ns[kVrfFull] = time_comp<kVrfFull>(scr, btab, msgs, out, blocks, 2);
  ns[kSc512] = time_comp<kSc512>(scr, btab, msgs, out, blocks, 64);
  ns[kDbl] = time_comp<kDbl>(scr, btab, msgs, out, blocks, 2);
  ns[kAddLd] = time_comp<kAddLd>(scr, btab, msgs, out, blocks, 4);
  ns[kAddReg] = time_comp<kAddReg>(scr, btab, msgs, out, blocks, 4);
  ns[kMulChain] = time_comp<kMulChain>(scr, btab, msgs, out, blocks, 2);
  ns[kTo3] = time_comp<kTo3>(scr, btab, msgs, out, blocks, 4);
  printf("{\"lanes\": %zu, \"unit\": \"GPU-ns per operation (whole MI355X)\"", lanes);
  for (int c = 0; c < kNumComp; c++) printf(", \"%s\": %.4f", kNames[c], ns[c]);
  printf("}\n");
  return 0;
}
