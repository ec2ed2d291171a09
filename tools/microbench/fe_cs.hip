// Column-scan field multiply/square (carry of column k folded into the first
// multiply-add of column k + 1) against the production fe_mul / fe_sq
// (csrc/fe25519.h: row-order accumulation, then a 12-step carry chain).
// Two independent chains per lane at the header kernel's occupancy; outputs
// are compared as canonical words.
//
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o fe_cs fe_cs.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../ouroboros-network_amd/csrc/fe25519.h"

#define CHECK(x)                                                                          \
  do {                                                                                    \
    hipError_t e_ = (x);                                                                  \
    if (e_ != hipSuccess) {                                                               \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));          \
      exit(1);                                                                            \
    }                                                                                     \
  } while (0)

using namespace ouro;

__device__ __forceinline__ fe cs_finish(uint32_t h[10], uint64_t c) {
  const uint64_t t = (uint64_t)h[0] + 19ull * c;
  h[0] = (uint32_t)t & limb_mask(0);
  h[1] += (uint32_t)(t >> 26);
  fe r;
#pragma unroll
  for (int i = 0; i < 10; i++) {
    r.v[i] = h[i];
    asm("" : "+v"(r.v[i]));
  }
  return r;
}

__device__ __forceinline__ fe mul_cs(const fe& f, const fe& g) {
  uint32_t g19[10], f2[10];
#pragma unroll
  for (int i = 0; i < 10; i++) {
    g19[i] = 19u * g.v[i];
    f2[i] = (i & 1) ? 2u * f.v[i] : f.v[i];
  }
  uint32_t h[10];
  uint64_t c = 0;
#pragma unroll
  for (int k = 0; k < 10; k++) {
    uint64_t t = c;
#pragma unroll
    for (int i = 0; i < 10; i++) {
      const int j = (k - i + 10) % 10;
      const uint32_t a = ((i & 1) && (j & 1)) ? f2[i] : f.v[i];
      const uint32_t b = (i + j >= 10) ? g19[j] : g.v[j];
      t += (uint64_t)a * b;
    }
    h[k] = (uint32_t)t & limb_mask(k);
    c = t >> limb_bits(k);
  }
  return cs_finish(h, c);
}

__device__ __forceinline__ fe sq_cs(const fe& f) {
  uint32_t f2[10], f4[10], f19[10];
#pragma unroll
  for (int i = 0; i < 10; i++) {
    f2[i] = 2u * f.v[i];
    f4[i] = 4u * f.v[i];
    f19[i] = 19u * f.v[i];
  }
  uint32_t h[10];
  uint64_t c = 0;
#pragma unroll
  for (int k = 0; k < 10; k++) {
    uint64_t t = c;
#pragma unroll
    for (int i = 0; i < 10; i++) {
#pragma unroll
      for (int j = i; j < 10; j++) {
        if ((i + j) % 10 != k) continue;
        uint32_t a, b;
        if (i == j) {
          a = (i & 1) ? f2[i] : f.v[i];
          b = (2 * i >= 10) ? f19[i] : f.v[i];
        } else {
          a = ((i & 1) && (j & 1)) ? f4[i] : f2[i];
          b = (i + j >= 10) ? f19[j] : f.v[j];
        }
        t += (uint64_t)a * b;
      }
    }
    h[k] = (uint32_t)t & limb_mask(k);
    c = t >> limb_bits(k);
  }
  return cs_finish(h, c);
}


// the same with the multiply-adds as inline asm, so the column carry stays the
// first addend (LLVM otherwise reassociates it into a separate 64-bit add)
#ifndef MAD_OPAQUE
__device__ __forceinline__ uint64_t mad(uint32_t a, uint32_t b, uint64_t c) {
  uint64_t r, sc;
  asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(r), "=s"(sc) : "v"(a), "v"(b), "v"(c));
  return r;
}
#else
// compiler-emitted multiply-add on an opaque accumulator (no reassociation)
__device__ __forceinline__ uint64_t mad(uint32_t a, uint32_t b, uint64_t c) {
  uint64_t r = (uint64_t)a * b + c;
  asm("" : "+v"(r));
  return r;
}
#endif
__device__ __forceinline__ fe mul_cs2(const fe& f, const fe& g) {
  uint32_t g19[10], f2[10];
#pragma unroll
  for (int i = 0; i < 10; i++) {
    g19[i] = 19u * g.v[i];
    f2[i] = (i & 1) ? 2u * f.v[i] : f.v[i];
  }
  uint32_t h[10];
  uint64_t c = 0;
#pragma unroll
  for (int k = 0; k < 10; k++) {
    uint64_t t = c;
#pragma unroll
    for (int i = 0; i < 10; i++) {
      const int j = (k - i + 10) % 10;
      const uint32_t a = ((i & 1) && (j & 1)) ? f2[i] : f.v[i];
      const uint32_t b = (i + j >= 10) ? g19[j] : g.v[j];
      t = mad(a, b, t);
    }
    h[k] = (uint32_t)t & limb_mask(k);
    c = t >> limb_bits(k);
  }
  return cs_finish(h, c);
}
__device__ __forceinline__ fe sq_cs2(const fe& f) {
  uint32_t f2[10], f4[10], f19[10];
#pragma unroll
  for (int i = 0; i < 10; i++) {
    f2[i] = 2u * f.v[i];
    f4[i] = 4u * f.v[i];
    f19[i] = 19u * f.v[i];
  }
  uint32_t h[10];
  uint64_t c = 0;
#pragma unroll
  for (int k = 0; k < 10; k++) {
    uint64_t t = c;
#pragma unroll
    for (int i = 0; i < 10; i++) {
#pragma unroll
      for (int j = i; j < 10; j++) {
        if ((i + j) % 10 != k) continue;
        uint32_t a, b;
        if (i == j) {
          a = (i & 1) ? f2[i] : f.v[i];
          b = (2 * i >= 10) ? f19[i] : f.v[i];
        } else {
          a = ((i & 1) && (j & 1)) ? f4[i] : f2[i];
          b = (i + j >= 10) ? f19[j] : f.v[j];
        }
        t = mad(a, b, t);
      }
    }
    h[k] = (uint32_t)t & limb_mask(k);
    c = t >> limb_bits(k);
  }
  return cs_finish(h, c);
}


// two independent column-scan chains (columns 0..4 and 5..9), then the carry
// out of column 4 into limb 5 and the 2^255 = 19 wrap of column 9's carry
template <bool kSq>
__device__ __forceinline__ fe cs3(const fe& f, const fe& g) {
  uint32_t g19[10], f2[10], f4[10];
#pragma unroll
  for (int i = 0; i < 10; i++) {
    g19[i] = 19u * g.v[i];
    f2[i] = kSq ? 2u * f.v[i] : ((i & 1) ? 2u * f.v[i] : f.v[i]);
    f4[i] = 4u * f.v[i];
  }
  uint32_t h[10];
  uint64_t cA = 0, cB = 0;
#pragma unroll
  for (int s = 0; s < 5; s++) {
    uint64_t tA = cA, tB = cB;
#pragma unroll
    for (int half = 0; half < 2; half++) {
      const int k = half ? s + 5 : s;
      uint64_t t = half ? tB : tA;
#pragma unroll
      for (int i = 0; i < 10; i++) {
#pragma unroll
        for (int j = 0; j < 10; j++) {
          if ((i + j) % 10 != k) continue;
          uint32_t a, b;
          if (kSq) {
            if (j < i) continue;
            if (i == j) {
              a = (i & 1) ? f2[i] : f.v[i];
              b = (2 * i >= 10) ? g19[i] : f.v[i];
            } else {
              a = ((i & 1) && (j & 1)) ? f4[i] : f2[i];
              b = (i + j >= 10) ? g19[j] : f.v[j];
            }
          } else {
            a = ((i & 1) && (j & 1)) ? f2[i] : f.v[i];
            b = (i + j >= 10) ? g19[j] : g.v[j];
          }
          t = mad(a, b, t);
        }
      }
      if (half) tB = t; else tA = t;
    }
    h[s] = (uint32_t)tA & limb_mask(s);
    cA = tA >> limb_bits(s);
    h[s + 5] = (uint32_t)tB & limb_mask(s + 5);
    cB = tB >> limb_bits(s + 5);
  }
  const uint64_t t5 = (uint64_t)h[5] + cA;
  h[5] = (uint32_t)t5 & limb_mask(5);
  h[6] += (uint32_t)(t5 >> 25);
  return cs_finish(h, cB);
}

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
  fe x = fe_from_words(a), y = fe_from_words(b), z = fe_from_words(c), w = y;
#pragma unroll 1
  for (int it = 0; it < ITERS; it++) {
    if constexpr (V == 0) {
      fe t = fe_mul(x, y), u = fe_mul(z, w);
      x = y; y = t; z = w; w = u;
    } else if constexpr (V == 1) {
      fe t = mul_cs(x, y), u = mul_cs(z, w);
      x = y; y = t; z = w; w = u;
    } else if constexpr (V == 2) {
      x = fe_sq(x);
      z = fe_sq(z);
    } else if constexpr (V == 3) {
      x = sq_cs(x);
      z = sq_cs(z);
    } else if constexpr (V == 4) {
      fe t = mul_cs2(x, y), u = mul_cs2(z, w);
      x = y; y = t; z = w; w = u;
    } else if constexpr (V == 5) {
      x = sq_cs2(x);
      z = sq_cs2(z);
    } else if constexpr (V == 6) {
      fe t = cs3<false>(x, y), u = cs3<false>(z, w);
      x = y; y = t; z = w; w = u;
    } else {
      x = cs3<true>(x, x);
      z = cs3<true>(z, z);
    }
  }
  uint32_t w1[8], w2[8];
  fe_to_words(w1, x);
  fe_to_words(w2, z);
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

int main() {
  CHECK(hipSetDevice(0));
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const size_t n = (size_t)prop.multiProcessorCount * 2 * 256 * 4;
  std::vector<uint32_t> h(24 * n);
  uint64_t s = 0x9e3779b97f4a7c15ull;
  for (auto& x : h) {
    s ^= s << 13; s ^= s >> 7; s ^= s << 17;
    x = (uint32_t)(s >> 11);
  }
  for (size_t i = 0; i < 3 * n; i++) h[8 * i + 7] &= 0x7fffffff;
  uint32_t *din, *dout;
  CHECK(hipMalloc(&din, h.size() * 4));
  CHECK(hipMalloc(&dout, 16 * n * 4));
  CHECK(hipMemcpy(din, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  const char* names[8] = {"fe_mul", "mul_cs", "fe_sq", "sq_cs", "mul_cs_asm", "sq_cs_asm", "mul_cs2ch", "sq_cs2ch"};
  std::vector<std::vector<uint32_t>> res(8, std::vector<uint32_t>(16 * n));
  float ms[8];
  for (int round = 0; round < 3; round++) {
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
  }
  const bool mul_eq = res[0] == res[1] && res[0] == res[4] && res[0] == res[6],
             sq_eq = res[2] == res[3] && res[2] == res[5] && res[2] == res[7];
  const double ops = 2.0 * ITERS * n;
  printf("{\"lanes\": %zu, \"iters\": %d, \"mul_equal\": %s, \"sq_equal\": %s", n, ITERS,
         mul_eq ? "true" : "false", sq_eq ? "true" : "false");
  for (int v = 0; v < 8; v++)
    printf(", \"%s\": {\"ms\": %.3f, \"Gops\": %.2f}", names[v], ms[v], ops / (ms[v] * 1e-3) / 1e9);
  printf("}\n");
  return (mul_eq && sq_eq) ? 0 : 1;
}
