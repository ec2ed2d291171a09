// Occupancy A/B for the lane arithmetic (round 4).
//
// tools/microbench/valu_costs.hip showed a wave issues at most one VALU
// instruction per ~4 cycles (v_mad_u64_u32 one per ~7, and a MAD that
// depends on the previous one every ~14), while the SIMD retires a simple
// instruction every ~1.9 cycles and a MAD every ~3.2 once 4 waves share it.
// At the header kernel's 2 waves/SIMD the issue is therefore bound by each
// wave's own cadence.  This runs the production group operations
// (ge25519.h: doublings p2 -> p1p1 -> p2, cached additions) and field
// products out of csrc/ in per-lane register chains at 1..4 waves/SIMD and
// reports ns per operation over the whole chip, with the VGPR budget the
// launch bounds force -- the ceiling a lower-register schedule could reach.
//
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o occupancy occupancy.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "../../ouroboros-network_amd/csrc/ge25519.h"

#define CHECK(x)                                                                          \
  do {                                                                                    \
    hipError_t e_ = (x);                                                                  \
    if (e_ != hipSuccess) {                                                               \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));          \
      exit(1);                                                                            \
    }                                                                                     \
  } while (0)

using namespace ouro;

__device__ __forceinline__ fe load_fe(const uint32_t* in, size_t i, int k) {
  fe f;
#pragma unroll
  for (int l = 0; l < 10; l++) f.v[l] = in[(size_t)(k * 10 + l) * 65536 + (i & 65535)] & 0x1ffffff;
  return f;
}
__device__ __forceinline__ void fold(uint32_t* out, size_t i, const fe& f) {
  uint32_t x = 0;
#pragma unroll
  for (int l = 0; l < 10; l++) x ^= f.v[l];
  out[i] = x;
}

// ---- lockstep prototypes: N independent products, one scan chain each, their
// multiply-adds interleaved (chain n's dependent MADs N instructions apart)
template <int N>
__device__ __forceinline__ void sq_xn(fe* out, const fe* in, const int* scale) {
  uint32_t fs[N][10], f2s[N][10], f4s[N][10], f19[N][10];
#pragma unroll
  for (int e = 0; e < N; e++)
#pragma unroll
    for (int i = 0; i < 10; i++) {
      fs[e][i] = scale[e] * in[e].v[i];
      f2s[e][i] = 2u * scale[e] * in[e].v[i];
      f4s[e][i] = 4u * scale[e] * in[e].v[i];
      f19[e][i] = 19u * in[e].v[i];
    }
  uint32_t h[N][10];
  uint64_t c[N];
#pragma unroll
  for (int e = 0; e < N; e++) c[e] = 0;
#pragma unroll
  for (int k = 0; k < 10; k++) {
    uint64_t t[N];
#pragma unroll
    for (int e = 0; e < N; e++) t[e] = c[e];
#pragma unroll
    for (int i = 0; i < 10; i++)
#pragma unroll
      for (int j = i; j < 10; j++) {
        if ((i + j) % 10 != k) continue;
#pragma unroll
        for (int e = 0; e < N; e++) {
          uint32_t a, b;
          if (i == j) {
            a = (i & 1) ? f2s[e][i] : fs[e][i];
            b = (2 * i >= 10) ? f19[e][i] : in[e].v[i];
          } else {
            a = ((i & 1) && (j & 1)) ? f4s[e][i] : f2s[e][i];
            b = (i + j >= 10) ? f19[e][j] : in[e].v[j];
          }
          t[e] = mad_acc(a, b, t[e]);
        }
      }
#pragma unroll
    for (int e = 0; e < N; e++) {
      h[e][k] = (uint32_t)t[e] & limb_mask(k);
      c[e] = t[e] >> limb_bits(k);
    }
  }
#pragma unroll
  for (int e = 0; e < N; e++) out[e] = scan_finish(h[e], c[e]);
}
template <int N>
__device__ __forceinline__ void mul_xn(fe* out, const fe* f, const fe* g) {
  uint32_t g19[N][10], f2[N][10];
#pragma unroll
  for (int e = 0; e < N; e++)
#pragma unroll
    for (int i = 0; i < 10; i++) {
      g19[e][i] = 19u * g[e].v[i];
      f2[e][i] = (i & 1) ? 2u * f[e].v[i] : f[e].v[i];
    }
  uint32_t h[N][10];
  uint64_t c[N];
#pragma unroll
  for (int e = 0; e < N; e++) c[e] = 0;
#pragma unroll
  for (int k = 0; k < 10; k++) {
    uint64_t t[N];
#pragma unroll
    for (int e = 0; e < N; e++) t[e] = c[e];
#pragma unroll
    for (int i = 0; i < 10; i++) {
      const int j = (k - i + 10) % 10;
#pragma unroll
      for (int e = 0; e < N; e++) {
        const uint32_t a = ((i & 1) && (j & 1)) ? f2[e][i] : f[e].v[i];
        const uint32_t b = (i + j >= 10) ? g19[e][j] : g[e].v[j];
        t[e] = mad_acc(a, b, t[e]);
      }
    }
#pragma unroll
    for (int e = 0; e < N; e++) {
      h[e][k] = (uint32_t)t[e] & limb_mask(k);
      c[e] = t[e] >> limb_bits(k);
    }
  }
#pragma unroll
  for (int e = 0; e < N; e++) out[e] = scan_finish(h[e], c[e]);
}
// doubling with the four squarings in lockstep and the three products in lockstep
__device__ __forceinline__ ge_p1p1 dbl_lockstep(const ge_p1p1& p) {
  // p1p1 -> p2: X = X T, Y = Y Z, Z = Z T
  fe pf[3] = {p.T, p.Z, p.T}, pg[3] = {p.X, p.Y, p.Z}, q[3];
  mul_xn<3>(q, pf, pg);
  fe in[4] = {q[0], q[1], q[2], fe_add(q[0], q[1])}, o[4];
  const int sc[4] = {1, 1, 2, 1};
  sq_xn<4>(o, in, sc);
  const fe A = o[0], B = o[1], C = o[2], S = o[3];
  ge_p1p1 r;
  r.Y = fe_carry(fe_add(B, A));
  r.Z = fe_sub(B, A);
  r.X = fe_sub(S, r.Y);
  r.T = fe_sub(fe_add(C, A), B);
  return r;
}
__device__ __forceinline__ ge_p1p1 dbl_pairs(const ge_p1p1& p) {
  fe pf[2] = {p.T, p.Z}, pg[2] = {p.X, p.Y}, q[2];
  mul_xn<2>(q, pf, pg);
  const fe Z = fe_mul(p.T, p.Z);
  fe in1[2] = {q[0], q[1]}, o1[2];
  const int sc1[2] = {1, 1};
  sq_xn<2>(o1, in1, sc1);
  fe in2[2] = {Z, fe_add(q[0], q[1])}, o2[2];
  const int sc2[2] = {2, 1};
  sq_xn<2>(o2, in2, sc2);
  const fe A = o1[0], B = o1[1], C = o2[0], S = o2[1];
  ge_p1p1 r;
  r.Y = fe_carry(fe_add(B, A));
  r.Z = fe_sub(B, A);
  r.X = fe_sub(S, r.Y);
  r.T = fe_sub(fe_add(C, A), B);
  return r;
}

// cached addition (p1p1 -> p3, then + q) with each layer's four products in lockstep
__device__ __forceinline__ ge_p1p1 add_lockstep(const ge_p1p1& t, const ge_cached& q, bool neg) {
  fe f1[4] = {t.T, t.Z, t.T, t.X}, g1[4] = {t.X, t.Y, t.Z, t.Y}, p3[4];
  mul_xn<4>(p3, f1, g1);  // X, Y, Z, T of the p3 point
  const fe qa = fe_select(q.YminusX, q.YplusX, neg);
  const fe qb = fe_select(q.YplusX, q.YminusX, neg);
  fe f2[4] = {fe_add(p3[1], p3[0]), fe_sub(p3[1], p3[0]), p3[3], p3[2]};
  fe g2[4] = {qa, qb, q.T2d, q.Z2}, r4[4];
  mul_xn<4>(r4, f2, g2);
  const fe A = r4[0], B = r4[1], C = r4[2], D = r4[3];
  const fe Dp = fe_add(D, C), Dm = fe_sub(D, C);
  ge_p1p1 r;
  r.X = fe_sub(A, B);
  r.Y = fe_add(A, B);
  r.Z = fe_select(Dm, Dp, neg);
  r.T = fe_select(Dp, Dm, neg);
  return r;
}

// kind 0: doublings (p2 -> p1p1 -> p2), kind 1: cached additions (p3 + q),
// kind 2: squarings, kind 3: multiplies, kind 4: squarings in pairs (fe_sq_x2),
// kind 5: two-chain squarings (fe_sq_scan2), kind 6: doublings, products in
// lockstep (dbl_lockstep), kind 7: doublings in lockstep pairs (dbl_pairs)
template <int W, int KIND>
__global__ void __launch_bounds__(256, W) kop(const uint32_t* in, uint32_t* out, int iters) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if constexpr (KIND == 0) {
    ge_p1p1 t{load_fe(in, i, 0), load_fe(in, i, 1), load_fe(in, i, 2), load_fe(in, i, 3)};
#pragma unroll 1
    for (int k = 0; k < iters; k++) t = ge_p2_dbl(ge_p1p1_to_p2(t));
    fold(out, i, ge_p1p1_to_p2(t).X);
  } else if constexpr (KIND == 1) {
    ge_p1p1 t{load_fe(in, i, 0), load_fe(in, i, 1), load_fe(in, i, 2), load_fe(in, i, 3)};
    const ge_cached q{load_fe(in, i, 4), load_fe(in, i, 5), load_fe(in, i, 6), load_fe(in, i, 7)};
#pragma unroll 1
    for (int k = 0; k < iters; k++) t = ge_add_cached(ge_p1p1_to_p3(t), q, (k & 1) != 0);
    fold(out, i, ge_p1p1_to_p2(t).X);
  } else if constexpr (KIND == 2) {
    fe a = load_fe(in, i, 0);
#pragma unroll 1
    for (int k = 0; k < iters; k++) a = fe_sq(a);
    fold(out, i, a);
  } else if constexpr (KIND == 3) {
    fe a = load_fe(in, i, 0), b = load_fe(in, i, 1);
#pragma unroll 1
    for (int k = 0; k < iters; k++) a = fe_mul(a, b);
    fold(out, i, a);
  } else if constexpr (KIND == 4) {
    fe a = load_fe(in, i, 0), b = load_fe(in, i, 1);
#pragma unroll 1
    for (int k = 0; k < iters / 2; k++) fe_sq_x2(a, b);
    fold(out, i, fe_add(a, b));
  } else if constexpr (KIND == 5) {
    fe a = load_fe(in, i, 0);
#pragma unroll 1
    for (int k = 0; k < iters; k++) a = fe_sq_scan2<1>(a);
    fold(out, i, a);
  } else if constexpr (KIND == 8) {
    ge_p1p1 t{load_fe(in, i, 0), load_fe(in, i, 1), load_fe(in, i, 2), load_fe(in, i, 3)};
    const ge_cached q{load_fe(in, i, 4), load_fe(in, i, 5), load_fe(in, i, 6), load_fe(in, i, 7)};
#pragma unroll 1
    for (int k = 0; k < iters; k++) t = add_lockstep(t, q, (k & 1) != 0);
    fold(out, i, ge_p1p1_to_p2(t).X);
  } else {
    ge_p1p1 t{load_fe(in, i, 0), load_fe(in, i, 1), load_fe(in, i, 2), load_fe(in, i, 3)};
#pragma unroll 1
    for (int k = 0; k < iters; k++) t = KIND == 6 ? dbl_lockstep(t) : dbl_pairs(t);
    fold(out, i, ge_p1p1_to_p2(t).X);
  }
}

typedef void (*kfn)(const uint32_t*, uint32_t*, int);

int main() {
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  const int cus = p.multiProcessorCount;
  uint32_t *in, *out;
  const size_t in_words = 80 * 65536;
  CHECK(hipMalloc(&in, in_words * 4));
  uint32_t* h = (uint32_t*)malloc(in_words * 4);
  uint32_t s = 12345;
  for (size_t k = 0; k < in_words; k++) h[k] = (s = s * 1664525u + 1013904223u);
  CHECK(hipMemcpy(in, h, in_words * 4, hipMemcpyHostToDevice));
  struct K {
    const char* name;
    int waves, kind;
    kfn f;
  } ks[] = {
      {"dbl", 1, 0, kop<1, 0>}, {"dbl", 2, 0, kop<2, 0>}, {"dbl", 3, 0, kop<3, 0>}, {"dbl", 4, 0, kop<4, 0>},
      {"add", 1, 1, kop<1, 1>}, {"add", 2, 1, kop<2, 1>}, {"add", 3, 1, kop<3, 1>}, {"add", 4, 1, kop<4, 1>},
      {"sq", 1, 2, kop<1, 2>},  {"sq", 2, 2, kop<2, 2>},  {"sq", 3, 2, kop<3, 2>},  {"sq", 4, 2, kop<4, 2>},
      {"mul", 1, 3, kop<1, 3>}, {"mul", 2, 3, kop<2, 3>}, {"mul", 3, 3, kop<3, 3>}, {"mul", 4, 3, kop<4, 3>},
      {"sq_x2", 2, 4, kop<2, 4>}, {"sq_x2", 3, 4, kop<3, 4>}, {"sq_x2", 4, 4, kop<4, 4>},
      {"sq_scan2", 2, 5, kop<2, 5>}, {"sq_scan2", 3, 5, kop<3, 5>}, {"sq_scan2", 4, 5, kop<4, 5>},
      {"dbl_lockstep", 2, 6, kop<2, 6>}, {"dbl_lockstep", 3, 6, kop<3, 6>},
      {"dbl_pairs", 2, 7, kop<2, 7>}, {"dbl_pairs", 3, 7, kop<3, 7>},
      {"add_lockstep", 2, 8, kop<2, 8>}, {"add_lockstep", 3, 8, kop<3, 8>},
  };
  const int iters = 512;
  printf("{\"device\": \"%s\", \"cus\": %d, \"iters\": %d, \"unit\": \"ps of chip time per op "
         "(all lanes), and ns per op per lane\", \"ops\": [\n", p.gcnArchName, cus, iters);
  bool first = true;
  for (auto& k : ks) {
    // exactly `waves` waves per SIMD: 256-thread blocks, waves blocks per CU
    const int blocks = cus * k.waves;
    CHECK(hipMalloc(&out, sizeof(uint32_t) * blocks * 256));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, in, out, 8);
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(e0));
    const int reps = 3;
    for (int r = 0; r < reps; r++) hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, in, out, iters);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    const double ops = (double)blocks * 256 * iters * reps;
    printf("%s  {\"op\": \"%s\", \"waves\": %d, \"ps_per_op_chip\": %.4f, \"ns_per_op_lane\": %.2f}",
           first ? "" : ",\n", k.name, k.waves, ms * 1e9 / ops, ms * 1e6 / (iters * reps));
    first = false;
    fflush(stdout);
    CHECK(hipFree(out));
  }
  printf("\n]}\n");
  return 0;
}
