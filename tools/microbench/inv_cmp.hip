// Lane-mode inversion: the variable-time Bernstein-Yang inversion
// (modinv.h fe_invert_vartime, what fe_invert4 / the header finish use)
// against z^(p-2) (fe25519.h fe_invert, the exponentiation chain), and the
// whole lane VRF verify for scale -- one item per lane at the product's
// launch bounds, timed, and counted by a rocprofv3 SQ_INSTS_VALU pass.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o inv_cmp inv_cmp.hip \
//          -L../../ouroboros-network_amd/lib -louro_synth -Wl,-rpath,...
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../ouroboros-network_amd/csrc/launch.h"

using namespace ouro;

extern "C" int ouro_synth_vrf(size_t n, uint64_t first, uint8_t* pk, uint8_t* proof,
                              uint8_t* alpha);

#define CHECK(x)                                                                 \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

enum Kind { kVartime = 0, kPow, kVrf, kNum };
const char* kNames[kNum] = {"invert_vartime", "invert_pow", "vrf03_verify_lane"};

template <int K>
__global__ void __launch_bounds__(256, 2) kinv(size_t n, const uint8_t* __restrict__ pk,
                                               const uint8_t* __restrict__ proof,
                                               const uint8_t* __restrict__ alpha,
                                               int32_t* scratch, const int32_t* __restrict__ btab,
                                               uint32_t* out) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t acc = 0;
  if constexpr (K == kVrf) {
    const Slot lane = slot_of(scratch, i, kSlotWords);
    uint32_t p[8], pi[20], b[16];
    load_words(p, pk + 32 * i, 2);
    load_words(pi, proof + 80 * i, 5);
    const bool ok = vrf03_verify_lane(b, p, pi, ShaGlobalTail{alpha + 32 * i}, 32, lane, btab);
    acc = b[0] + (ok ? 1u : 0u);
  } else {
    // a random element per lane (the proof's Gamma bytes, top bit cleared)
    uint32_t w[8];
    load_words(w, proof + 80 * i, 2);
    w[7] &= 0x7fffffffu;
    fe z = fe_from_words(w);
    fe r = K == kVartime ? fe_invert_vartime(z) : fe_invert(z);
    uint32_t o[8];
    fe_to_words(o, fe_mul(r, z));  // = 1
    acc = o[0] ^ o[7] ^ 1u;  // 0 when r z = 1
  }
  out[i] = acc;
}

template <int K>
float run(size_t n, const uint8_t* pk, const uint8_t* proof, const uint8_t* alpha, int32_t* scr,
          const int32_t* btab, uint32_t* out) {
  const unsigned blocks = (unsigned)((n + 255) / 256);
  hipLaunchKernelGGL(kinv<K>, dim3(blocks), dim3(256), 0, 0, n, pk, proof, alpha, scr, btab, out);
  CHECK(hipGetLastError());
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  CHECK(hipEventRecord(e0, 0));
  hipLaunchKernelGGL(kinv<K>, dim3(blocks), dim3(256), 0, 0, n, pk, proof, alpha, scr, btab, out);
  CHECK(hipEventRecord(e1, 0));
  CHECK(hipEventSynchronize(e1));
  float ms;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  return ms;
}

size_t count_ok(const uint32_t* d_out, size_t n, bool zero_is_ok) {
  std::vector<uint32_t> v(n);
  CHECK(hipMemcpy(v.data(), d_out, 4 * n, hipMemcpyDeviceToHost));
  size_t k = 0;
  for (uint32_t x : v) k += zero_is_ok ? (x == 0) : (x & 1u);
  return k;
}

int main(int argc, char** argv) {
  const size_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : 262144;
  CHECK(hipSetDevice(0));
  uint8_t *pk, *proof, *alpha;
  int32_t *scr, *btab;
  uint32_t* out;
  CHECK(hipMalloc(&pk, 32 * n));
  CHECK(hipMalloc(&proof, 80 * n));
  CHECK(hipMalloc(&alpha, 32 * n));
  CHECK(hipMalloc(&out, 4 * n));
  CHECK(hipMalloc(&scr, (size_t)kSlotWords * 4 * n));
  CHECK(hipMalloc(&btab, kBTabWords * 4));
  std::vector<int32_t> tab(kBTabWords);
  build_btab(tab.data());
  CHECK(hipMemcpy(btab, tab.data(), kBTabWords * 4, hipMemcpyHostToDevice));
  if (ouro_synth_vrf(n, 0, pk, proof, alpha) != 0) {
    fprintf(stderr, "synth failed\n");
    return 1;
  }
  CHECK(hipDeviceSynchronize());
  float ms[kNum];
  size_t ok[kNum];
  ms[kVartime] = run<kVartime>(n, pk, proof, alpha, scr, btab, out);
  ok[kVartime] = count_ok(out, n, true);
  ms[kPow] = run<kPow>(n, pk, proof, alpha, scr, btab, out);
  ok[kPow] = count_ok(out, n, true);
  ms[kVrf] = run<kVrf>(n, pk, proof, alpha, scr, btab, out);
  ok[kVrf] = count_ok(out, n, false);
  printf("{\"n\": %zu, \"unit\": \"ms per launch\"", n);
  for (int k = 0; k < kNum; k++) printf(", \"%s\": %.4f, \"%s_ok\": %zu", kNames[k], ms[k], kNames[k], ok[k]);
  printf("}\n");
  return 0;
}
