// Integer-VALU throughput microbenchmark for gfx950 (MI355X).
//
// Measures the issue rate of the instructions a GF(2^255-19) field multiply can
// be built from, so the roofline peak used by bench.py is a measured number and
// not a datasheet guess (SURVEY.md §8(d) "Peak").  Each lane runs NCHAIN
// independent dependency chains of one instruction kind in inline asm so the
// compiler can neither fold nor reorder them.
//
// Build: hipcc --offload-arch=gfx950 -O3 -o int_rates int_rates.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1);} } while (0)

constexpr int ITERS = 4096;

// 8 independent chains of v_mad_u64_u32 (acc = a*b + acc).
__global__ void k_mad_u64_u32(uint64_t* out, uint32_t seed) {
  uint32_t a = seed ^ threadIdx.x, b = a * 2654435761u;
  uint64_t c0 = a, c1 = b, c2 = a + 1, c3 = b + 1, c4 = a + 2, c5 = b + 2, c6 = a + 3, c7 = b + 3;
  uint64_t cc;
  for (int i = 0; i < ITERS; ++i) {
#define MAD(c) asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(c), "=s"(cc) : "v"(a), "v"(b));
    MAD(c0) MAD(c1) MAD(c2) MAD(c3) MAD(c4) MAD(c5) MAD(c6) MAD(c7)
#undef MAD
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = c0 ^ c1 ^ c2 ^ c3 ^ c4 ^ c5 ^ c6 ^ c7;
}

#define SIMPLE_KERNEL(NAME, ASM)                                                     \
  __global__ void NAME(uint64_t* out, uint32_t seed) {                              \
    uint32_t a = seed ^ threadIdx.x, b = a * 2654435761u;                           \
    uint32_t c0 = a, c1 = b, c2 = a + 1, c3 = b + 1, c4 = a + 2, c5 = b + 2,        \
             c6 = a + 3, c7 = b + 3;                                                \
    for (int i = 0; i < ITERS; ++i) {                                               \
      asm volatile(ASM : "+v"(c0) : "v"(a), "v"(b));                                \
      asm volatile(ASM : "+v"(c1) : "v"(a), "v"(b));                                \
      asm volatile(ASM : "+v"(c2) : "v"(a), "v"(b));                                \
      asm volatile(ASM : "+v"(c3) : "v"(a), "v"(b));                                \
      asm volatile(ASM : "+v"(c4) : "v"(a), "v"(b));                                \
      asm volatile(ASM : "+v"(c5) : "v"(a), "v"(b));                                \
      asm volatile(ASM : "+v"(c6) : "v"(a), "v"(b));                                \
      asm volatile(ASM : "+v"(c7) : "v"(a), "v"(b));                                \
    }                                                                               \
    out[blockIdx.x * blockDim.x + threadIdx.x] = c0 ^ c1 ^ c2 ^ c3 ^ c4 ^ c5 ^ c6 ^ c7; \
  }

SIMPLE_KERNEL(k_mul_lo_u32, "v_mul_lo_u32 %0, %1, %0")
SIMPLE_KERNEL(k_mul_hi_u32, "v_mul_hi_u32 %0, %1, %0")
SIMPLE_KERNEL(k_mul_u32_u24, "v_mul_u32_u24 %0, %1, %0")
SIMPLE_KERNEL(k_mul_hi_u32_u24, "v_mul_hi_u32_u24 %0, %1, %0")
SIMPLE_KERNEL(k_mad_u32_u24, "v_mad_u32_u24 %0, %1, %2, %0")
SIMPLE_KERNEL(k_add_u32, "v_add_u32 %0, %1, %0")
SIMPLE_KERNEL(k_add_co_u32, "v_add_co_u32 %0, vcc, %1, %0")
SIMPLE_KERNEL(k_alignbit, "v_alignbit_b32 %0, %1, %0, 7")

__global__ void k_fma_f64(uint64_t* out, uint32_t seed) {
  double a = 1.0 + 1e-9 * (seed ^ threadIdx.x), b = 0.999999;
  double c0 = a, c1 = b, c2 = a + 1, c3 = b + 1, c4 = a + 2, c5 = b + 2, c6 = a + 3, c7 = b + 3;
  for (int i = 0; i < ITERS; ++i) {
#define F(c) asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(c) : "v"(a), "v"(b));
    F(c0) F(c1) F(c2) F(c3) F(c4) F(c5) F(c6) F(c7)
#undef F
  }
  double s = c0 + c1 + c2 + c3 + c4 + c5 + c6 + c7;
  out[blockIdx.x * blockDim.x + threadIdx.x] = *(uint64_t*)&s;
}

typedef void (*kfn)(uint64_t*, uint32_t);

static double run(kfn k, uint64_t* d, int blocks, int threads) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, d, 1u);  // warm-up
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(e0));
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, d, 1u + r);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  return ms / 5.0;
}

int main() {
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  const int cus = p.multiProcessorCount;
  const int threads = 256, blocks = cus * 8;  // 8 waves/SIMD worth of chains
  uint64_t* d;
  CHECK(hipMalloc(&d, sizeof(uint64_t) * blocks * threads));
  struct { const char* name; kfn k; } ks[] = {
      {"v_mad_u64_u32", k_mad_u64_u32}, {"v_mul_lo_u32", k_mul_lo_u32},
      {"v_mul_hi_u32", k_mul_hi_u32},   {"v_mul_u32_u24", k_mul_u32_u24},
      {"v_mul_hi_u32_u24", k_mul_hi_u32_u24}, {"v_mad_u32_u24", k_mad_u32_u24},
      {"v_add_u32", k_add_u32},         {"v_add_co_u32", k_add_co_u32},
      {"v_alignbit_b32", k_alignbit},   {"v_fma_f64", k_fma_f64},
  };
  printf("{\"device\": \"%s\", \"cus\": %d, \"clock_mhz\": %d, \"rates\": {", p.name, cus,
         p.clockRate / 1000);
  bool first = true;
  for (auto& kk : ks) {
    double ms = run(kk.k, d, blocks, threads);
    double ops = double(blocks) * threads * ITERS * 8;
    double tops = ops / (ms * 1e-3) / 1e12;
    // lane-ops per CU per clock at the nominal clock
    double per_cu_clk = ops / (ms * 1e-3) / cus / (p.clockRate * 1e3);
    printf("%s\"%s\": {\"Tops\": %.3f, \"lane_ops_per_cu_clk\": %.2f}", first ? "" : ", ", kk.name,
           tops, per_cu_clk);
    first = false;
  }
  printf("}}\n");
  CHECK(hipFree(d));
  return 0;
}
