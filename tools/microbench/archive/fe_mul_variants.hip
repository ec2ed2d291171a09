// Field-multiply microbenchmark: the product's radix-2^25.5 signed 10-limb
// fe_mul/fe_sq (csrc/fe25519.h) against radix-2^32 8-limb prototypes
// (fe8_proto.h).  Every variant runs ITERS dependent multiplies on two
// independent chains per lane at the header kernel's occupancy (256-thread
// blocks, __launch_bounds__(256, 2)), and writes canonical words so the host
// can check all variants agree bit for bit.
//
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o fe_mul_variants fe_mul_variants.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../../ouroboros-network_amd/csrc/fe25519.h"
#include "fe8_proto.h"

#define CHECK(x)                                                                          \
  do {                                                                                    \
    hipError_t e_ = (x);                                                                  \
    if (e_ != hipSuccess) {                                                               \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));          \
      exit(1);                                                                            \
    }                                                                                     \
  } while (0)

constexpr int ITERS = 1024;

template <int V>
__global__ void __launch_bounds__(256, 2) kvar(const uint32_t* in, uint32_t* out, size_t n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t a[8], b[8], c[8];
  for (int k = 0; k < 8; k++) {
    a[k] = in[24 * i + k];
    b[k] = in[24 * i + 8 + k];
    c[k] = in[24 * i + 16 + k];
  }
  uint32_t w1[8], w2[8];
  if constexpr (V == 11 || V == 12) {
    // production fe25519.h, one dependent chain per lane (V 11: sq, V 12: mul)
    ouro::fe x = ouro::fe_from_words(a), y = ouro::fe_from_words(b);
#pragma unroll 1
    for (int it = 0; it < ITERS; it++) {
      if constexpr (V == 11) x = ouro::fe_sq(x);
      else x = ouro::fe_mul(x, y);
    }
    ouro::fe_to_words(w1, x);
    ouro::fe_to_words(w2, y);
  } else if constexpr (V == 0 || V == 3) {
    ouro::fe x = ouro::fe_from_words(a), y = ouro::fe_from_words(b), z = ouro::fe_from_words(c);
    ouro::fe w = y;
#pragma unroll 1
    for (int it = 0; it < ITERS; it++) {
      if constexpr (V == 0) {
        // Fibonacci-style chains: no loop-invariant operand for the compiler to exploit
        ouro::fe t = ouro::fe_mul(x, y), u = ouro::fe_mul(z, w);
        x = y; y = t; z = w; w = u;
      } else {
        x = ouro::fe_sq(x);
        z = ouro::fe_sq(z);
      }
    }
    ouro::fe_to_words(w1, x);
    ouro::fe_to_words(w2, z);
  } else if constexpr (V == 7 || V == 8 || V == 9 || V == 10) {
    fe8p::fe10u x = fe8p::from_words10u(a), y = fe8p::from_words10u(b), z = fe8p::from_words10u(c);
    fe8p::fe10u w = y;
#pragma unroll 1
    for (int it = 0; it < ITERS; it++) {
      if constexpr (V == 7) {
        fe8p::fe10u t = fe8p::mul10u(x, y), u = fe8p::mul10u(z, w);
        x = y; y = t; z = w; w = u;
      } else if constexpr (V == 9) {
        fe8p::fe10u t = fe8p::mul10d(x, y), u = fe8p::mul10d(z, w);
        x = y; y = t; z = w; w = u;
      } else if constexpr (V == 10) {
        x = fe8p::sq10d(x);
        z = fe8p::sq10d(z);
      } else {
        x = fe8p::sq10u(x);
        z = fe8p::sq10u(z);
      }
    }
    fe8p::to_words10u(w1, x);
    fe8p::to_words10u(w2, z);
  } else {
    fe8p::fe8 x = fe8p::from_words(a), y = fe8p::from_words(b), z = fe8p::from_words(c);
    fe8p::fe8 w = y;
#pragma unroll 1
    for (int it = 0; it < ITERS; it++) {
      if constexpr (V == 1) {
        fe8p::fe8 t = fe8p::mul_1chain(x, y), u = fe8p::mul_1chain(z, w);
        x = y; y = t; z = w; w = u;
      } else if constexpr (V == 2) {
        fe8p::fe8 t = fe8p::mul_c(x, y), u = fe8p::mul_c(z, w);
        x = y; y = t; z = w; w = u;
      } else if constexpr (V == 6) {
        fe8p::fe8 t = fe8p::mul_osc(x, y), u = fe8p::mul_osc(z, w);
        x = y; y = t; z = w; w = u;
      } else if constexpr (V == 5) {
        fe8p::fe8 t = fe8p::mul_os(x, y), u = fe8p::mul_os(z, w);
        x = y; y = t; z = w; w = u;
      } else {
        x = fe8p::sq_1chain(x);
        z = fe8p::sq_1chain(z);
      }
    }
    fe8p::to_words(w1, x);
    fe8p::to_words(w2, z);
  }
  for (int k = 0; k < 8; k++) {
    out[16 * i + k] = w1[k];
    out[16 * i + 8 + k] = w2[k];
  }
}

template <int V>
float run(const uint32_t* din, uint32_t* dout, size_t n, int reps) {
  const int blocks = (int)((n + 255) / 256);
  hipLaunchKernelGGL(kvar<V>, dim3(blocks), dim3(256), 0, 0, din, dout, n);
  CHECK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  CHECK(hipEventRecord(e0, 0));
  for (int r = 0; r < reps; r++) hipLaunchKernelGGL(kvar<V>, dim3(blocks), dim3(256), 0, 0, din, dout, n);
  CHECK(hipEventRecord(e1, 0));
  CHECK(hipEventSynchronize(e1));
  float ms;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  return ms / reps;
}

int main(int argc, char** argv) {
  int dev = 0;
  CHECK(hipSetDevice(dev));
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, dev));
  // two resident 256-thread blocks per CU (the header kernel's occupancy), x4 rounds
  const size_t n = (size_t)prop.multiProcessorCount * 2 * 256 * 4;
  std::vector<uint32_t> h(24 * n);
  uint64_t s = 0x9e3779b97f4a7c15ull;
  for (auto& x : h) {
    s ^= s << 13; s ^= s >> 7; s ^= s << 17;
    x = (uint32_t)(s >> 11);
  }
  for (size_t i = 0; i < 3 * n; i++) h[8 * i + 7] &= 0x7fffffff;  // < 2^255
  uint32_t *din, *dout;
  CHECK(hipMalloc(&din, h.size() * 4));
  CHECK(hipMalloc(&dout, 16 * n * 4));
  CHECK(hipMemcpy(din, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  const char* names[13] = {"fe10_mul", "fe8_mul_asm", "fe8_mul_c", "fe10_sq", "fe8_sq_asm",
                           "fe8_mul_opscan", "fe8_mul_opscan_c", "fe10u_mul", "fe10u_sq",
                           "fe10d_mul", "fe10d_sq", "fe_sq_1chain", "fe_mul_1chain"};
  std::vector<std::vector<uint32_t>> res(13, std::vector<uint32_t>(16 * n));
  float ms[13];
  for (int round = 0; round < 2; round++) {
    ms[0] = run<0>(din, dout, n, 3);
    CHECK(hipMemcpy(res[0].data(), dout, 16 * n * 4, hipMemcpyDeviceToHost));
    ms[1] = run<1>(din, dout, n, 3);
    CHECK(hipMemcpy(res[1].data(), dout, 16 * n * 4, hipMemcpyDeviceToHost));
    ms[2] = run<2>(din, dout, n, 3);
    CHECK(hipMemcpy(res[2].data(), dout, 16 * n * 4, hipMemcpyDeviceToHost));
    ms[3] = run<3>(din, dout, n, 3);
    CHECK(hipMemcpy(res[3].data(), dout, 16 * n * 4, hipMemcpyDeviceToHost));
    ms[4] = run<4>(din, dout, n, 3);
    CHECK(hipMemcpy(res[4].data(), dout, 16 * n * 4, hipMemcpyDeviceToHost));
    ms[5] = run<5>(din, dout, n, 3);
    CHECK(hipMemcpy(res[5].data(), dout, 16 * n * 4, hipMemcpyDeviceToHost));
    ms[6] = run<6>(din, dout, n, 3);
    CHECK(hipMemcpy(res[6].data(), dout, 16 * n * 4, hipMemcpyDeviceToHost));
    ms[7] = run<7>(din, dout, n, 3);
    CHECK(hipMemcpy(res[7].data(), dout, 16 * n * 4, hipMemcpyDeviceToHost));
    ms[8] = run<8>(din, dout, n, 3);
    CHECK(hipMemcpy(res[8].data(), dout, 16 * n * 4, hipMemcpyDeviceToHost));
    ms[9] = run<9>(din, dout, n, 3);
    CHECK(hipMemcpy(res[9].data(), dout, 16 * n * 4, hipMemcpyDeviceToHost));
    ms[10] = run<10>(din, dout, n, 3);
    CHECK(hipMemcpy(res[10].data(), dout, 16 * n * 4, hipMemcpyDeviceToHost));
    ms[11] = run<11>(din, dout, n, 3);
    CHECK(hipMemcpy(res[11].data(), dout, 16 * n * 4, hipMemcpyDeviceToHost));
    ms[12] = run<12>(din, dout, n, 3);
    CHECK(hipMemcpy(res[12].data(), dout, 16 * n * 4, hipMemcpyDeviceToHost));
  }
  const bool mul_eq = res[0] == res[1] && res[0] == res[2] && res[0] == res[5] && res[0] == res[6] && res[0] == res[7] &&
                      res[0] == res[9];
  const bool sq_eq = res[3] == res[4] && res[3] == res[8] && res[3] == res[10];
  const double ops = 2.0 * ITERS * n;
  printf("{\"lanes\": %zu, \"iters\": %d, \"mul_equal\": %s, \"sq_equal\": %s", n, ITERS,
         mul_eq ? "true" : "false", sq_eq ? "true" : "false");
  for (int v = 0; v < 13; v++)
    printf(", \"%s\": {\"ms\": %.3f, \"Gops\": %.2f}", names[v], ms[v],
           (v >= 11 ? ops / 2 : ops) / (ms[v] * 1e-3) / 1e9);
  printf("}\n");
  return (mul_eq && sq_eq) ? 0 : 1;
}
