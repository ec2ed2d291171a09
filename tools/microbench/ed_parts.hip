// Attribution of the Ed25519 lane verify (verify.h ed25519_verify_lane, the
// code k_ed25519_verify and the header / Sum6KES cores run) to its phases,
// each kernel below runs the real routines up to or
// around one phase on the same synthetic signatures (lib/libouro_synth.so,
// 32-byte messages), one item per lane at the product's launch bounds, so a
// rocprofv3 SQ_INSTS_VALU pass per kernel gives VALU lane-instructions per
// item by subtraction:
//   decode  = K_decode                      (precheck + the A / R decode pair)
//   sha     = K_sha                         (SHA-512 of R || A || M, one block)
//   reduce  = K_sha_reduce - K_sha          (h = digest mod L)
//   lattice = K_scalars - K_sha_reduce      (half-size pair + b = c1 S mod L)
//   tables  = K_tables - K_decode           (the A and R tables, 2 x 8 entries)
//   recode  = K_pre - K_scalars - K_tables  (scalar recoding, slot stores)
//   dsm     = K_full - K_pre                (the 130-bit double-scalar chain)
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o ed_parts ed_parts.hip \
//          -L../../ouroboros-network_amd/lib -louro_synth -Wl,-rpath,...
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../ouroboros-network_amd/csrc/launch.h"

using namespace ouro;

extern "C" int ouro_synth_ed25519(size_t n, uint64_t first, uint8_t* pk, uint8_t* sig,
                                  uint8_t* msg);

#define CHECK(x)                                                                 \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

enum Part { kFull = 0, kPre, kDecode, kSha, kShaReduce, kScalars, kTables, kNumParts };
const char* kNames[kNumParts] = {"full", "pre", "decode", "sha", "sha_reduce", "scalars", "tables"};

template <int P>
__global__ void __launch_bounds__(256, 2) kpart(size_t n, const uint8_t* __restrict__ pk,
                                                const uint8_t* __restrict__ sig,
                                                const uint8_t* __restrict__ msg, int32_t* scratch,
                                                const int32_t* __restrict__ btab, uint32_t* out) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const Slot lane = slot_of(scratch, i, kSlotWords);
  uint32_t s[16], p[8];
  load_words(s, sig + 64 * i, 4);
  load_words(p, pk + 32 * i, 2);
  const ShaGlobalTail tail{msg + 32 * i};
  uint32_t R[8], S[8];
#pragma unroll
  for (int k = 0; k < 8; k++) {
    R[k] = s[k];
    S[k] = s[8 + k];
  }
  uint32_t acc = 0;
  if constexpr (P == kFull) {
    acc = ed25519_verify_lane(s, p, tail, 32, lane, btab) ? 1u : 0u;
  } else if constexpr (P == kPre) {
    acc = ed25519_verify_lane(s, p, tail, 32, lane, btab, false, false, kPhasePre) ? 1u : 0u;
  } else if constexpr (P == kDecode || P == kTables) {
    bool ok = ed25519_precheck(R, S, p, false);
    ge_p3 negA, negR;
    bool okA, okR;
    ge_decode_pair(&negA, &okA, &negR, &okR, p, R, true);
    ok = ok && okA && okR && ge_is_canonical(R);
    if constexpr (P == kTables) {
      build_table(lane + kSlotTab1, negA);
      build_table(lane + kSlotTab2, negR);
      acc = (uint32_t)ldg1(lane.word(kSlotTab2 + 7 * (kLaneEntryWords)));
    } else {
      acc = negA.X.v[0] ^ negR.T.v[3] ^ negA.Y.v[9];
    }
    acc += ok ? 1u : 0u;
  } else if constexpr (P == kSha || P == kShaReduce) {
    uint32_t pre[16];
#pragma unroll
    for (int k = 0; k < 8; k++) {
      pre[k] = R[k];
      pre[8 + k] = p[k];
    }
    uint64_t H[8];
    sha512_prefixed<64>(H, pre, tail, 32);
    if constexpr (P == kShaReduce) {
      uint32_t hw[16], h[8];
      sha512_digest_words(hw, H);
      sc_reduce512(h, hw);
      acc = h[0] ^ h[7];
    } else {
      acc = (uint32_t)H[0] ^ (uint32_t)(H[7] >> 32);
    }
  } else if constexpr (P == kScalars) {
    HalfScalars hs;
    uint32_t b[8];
    ed25519_scalars(hs, b, R, S, p, tail, 32);
    acc = b[0] ^ hs.c0[1] ^ hs.c1[2] ^ (uint32_t)hs.bits;
  }
  out[i] = acc;
}

template <int P>
float run(size_t n, const uint8_t* pk, const uint8_t* sig, const uint8_t* msg, int32_t* scr,
          const int32_t* btab, uint32_t* out) {
  const unsigned blocks = (unsigned)((n + 255) / 256);
  hipLaunchKernelGGL(kpart<P>, dim3(blocks), dim3(256), 0, 0, n, pk, sig, msg, scr, btab, out);
  CHECK(hipGetLastError());
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  CHECK(hipEventRecord(e0, 0));
  hipLaunchKernelGGL(kpart<P>, dim3(blocks), dim3(256), 0, 0, n, pk, sig, msg, scr, btab, out);
  CHECK(hipEventRecord(e1, 0));
  CHECK(hipEventSynchronize(e1));
  float ms;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  return ms;
}

int main(int argc, char** argv) {
  const size_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : 262144;
  CHECK(hipSetDevice(0));
  uint8_t *pk, *sig, *msg;
  int32_t *scr, *btab;
  uint32_t* out;
  CHECK(hipMalloc(&pk, 32 * n));
  CHECK(hipMalloc(&sig, 64 * n));
  CHECK(hipMalloc(&msg, 32 * n));
  CHECK(hipMalloc(&out, 4 * n));
  CHECK(hipMalloc(&scr, (size_t)kSlotWords * 4 * n));
  CHECK(hipMalloc(&btab, kBTabWords * 4));
  std::vector<int32_t> tab(kBTabWords);
  build_btab(tab.data());
  CHECK(hipMemcpy(btab, tab.data(), kBTabWords * 4, hipMemcpyHostToDevice));
  if (ouro_synth_ed25519(n, 0, pk, sig, msg) != 0) {
    fprintf(stderr, "synth failed\n");
    return 1;
  }
  CHECK(hipDeviceSynchronize());
  float ms[kNumParts];
  ms[kFull] = run<kFull>(n, pk, sig, msg, scr, btab, out);
  std::vector<uint32_t> v(n);
  CHECK(hipMemcpy(v.data(), out, 4 * n, hipMemcpyDeviceToHost));
  size_t valid = 0;
  for (uint32_t x : v) valid += x;
  ms[kPre] = run<kPre>(n, pk, sig, msg, scr, btab, out);
  ms[kDecode] = run<kDecode>(n, pk, sig, msg, scr, btab, out);
  ms[kSha] = run<kSha>(n, pk, sig, msg, scr, btab, out);
  ms[kShaReduce] = run<kShaReduce>(n, pk, sig, msg, scr, btab, out);
  ms[kScalars] = run<kScalars>(n, pk, sig, msg, scr, btab, out);
  ms[kTables] = run<kTables>(n, pk, sig, msg, scr, btab, out);
  printf("{\"n\": %zu, \"valid\": %zu, \"unit\": \"ms per launch\"", n, valid);
  for (int k = 0; k < kNumParts; k++) printf(", \"%s\": %.4f", kNames[k], ms[k]);
  printf("}\n");
  return valid == n ? 0 : 2;
}
