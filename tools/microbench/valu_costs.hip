// Issue cost of the integer VALU instructions the field arithmetic is built
// from, on gfx950, in SIMD cycles per wave-instruction.
//
// Round 4: the header kernel is issue-bound, so what matters
// is not a "peak" of one instruction but what each instruction in the mix
// costs.  int_rates.hip timed a few kinds against the nominal clock; this
// one reads the shader clock itself (s_memtime against the 100 MHz
// s_memrealtime, per wave) and reports
//   cyc = SIMD cycles per wave-instruction, at W waves per SIMD,
// for single kinds (8 independent chains per lane, inline asm, no folding)
// and for pairs (one MAD then one other instruction, to see whether their
// costs add or overlap).
//
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o valu_costs valu_costs.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                          \
  do {                                                                                    \
    hipError_t e_ = (x);                                                                  \
    if (e_ != hipSuccess) {                                                               \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));          \
      exit(1);                                                                            \
    }                                                                                     \
  } while (0)

constexpr int ITERS = 2048;

struct Stamp {
  unsigned long long c0, c1, r0, r1;
};

__device__ __forceinline__ void stamp_begin(Stamp* st, unsigned long long& c0,
                                            unsigned long long& r0) {
  (void)st;
  r0 = wall_clock64();
  c0 = clock64();
}
__device__ __forceinline__ void stamp_end(Stamp* st, unsigned long long c0,
                                          unsigned long long r0) {
  const unsigned long long c1 = clock64();
  const unsigned long long r1 = wall_clock64();
  if ((threadIdx.x & 63) == 0) {
    const int w = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    st[w] = Stamp{c0, c1, r0, r1};
  }
}

// 32-bit kinds: 8 chains of "c = op(c, a, b)"
#define K32(NAME, ASM)                                                                    \
  __global__ void __launch_bounds__(256) NAME(uint32_t* out, Stamp* st, uint32_t seed) {  \
    uint32_t a = seed ^ threadIdx.x, b = a * 2654435761u;                                 \
    uint32_t c0 = a, c1 = b, c2 = a + 1, c3 = b + 1, c4 = a + 2, c5 = b + 2, c6 = a + 3,  \
             c7 = b + 3;                                                                  \
    unsigned long long t0, r0;                                                            \
    stamp_begin(st, t0, r0);                                                              \
    for (int i = 0; i < ITERS; ++i) {                                                     \
      asm volatile(ASM : "+v"(c0) : "v"(a), "v"(b));                                      \
      asm volatile(ASM : "+v"(c1) : "v"(a), "v"(b));                                      \
      asm volatile(ASM : "+v"(c2) : "v"(a), "v"(b));                                      \
      asm volatile(ASM : "+v"(c3) : "v"(a), "v"(b));                                      \
      asm volatile(ASM : "+v"(c4) : "v"(a), "v"(b));                                      \
      asm volatile(ASM : "+v"(c5) : "v"(a), "v"(b));                                      \
      asm volatile(ASM : "+v"(c6) : "v"(a), "v"(b));                                      \
      asm volatile(ASM : "+v"(c7) : "v"(a), "v"(b));                                      \
    }                                                                                     \
    stamp_end(st, t0, r0);                                                                \
    out[blockIdx.x * blockDim.x + threadIdx.x] = c0 ^ c1 ^ c2 ^ c3 ^ c4 ^ c5 ^ c6 ^ c7;  \
  }

// 64-bit destination kinds: 8 chains of "c = op(c, a, b)", c 64-bit
#define K64(NAME, ASM)                                                                    \
  __global__ void __launch_bounds__(256) NAME(uint32_t* out, Stamp* st, uint32_t seed) {  \
    uint32_t a = seed ^ threadIdx.x, b = a * 2654435761u;                                 \
    uint64_t c0 = a, c1 = b, c2 = a + 1, c3 = b + 1, c4 = a + 2, c5 = b + 2, c6 = a + 3,  \
             c7 = b + 3;                                                                  \
    uint64_t ab = ((uint64_t)a << 32) | b;                                                \
    unsigned long long t0, r0;                                                            \
    stamp_begin(st, t0, r0);                                                              \
    for (int i = 0; i < ITERS; ++i) {                                                     \
      asm volatile(ASM : "+v"(c0) : "v"(a), "v"(b), "v"(ab));                             \
      asm volatile(ASM : "+v"(c1) : "v"(a), "v"(b), "v"(ab));                             \
      asm volatile(ASM : "+v"(c2) : "v"(a), "v"(b), "v"(ab));                             \
      asm volatile(ASM : "+v"(c3) : "v"(a), "v"(b), "v"(ab));                             \
      asm volatile(ASM : "+v"(c4) : "v"(a), "v"(b), "v"(ab));                             \
      asm volatile(ASM : "+v"(c5) : "v"(a), "v"(b), "v"(ab));                             \
      asm volatile(ASM : "+v"(c6) : "v"(a), "v"(b), "v"(ab));                             \
      asm volatile(ASM : "+v"(c7) : "v"(a), "v"(b), "v"(ab));                             \
    }                                                                                     \
    stamp_end(st, t0, r0);                                                                \
    out[blockIdx.x * blockDim.x + threadIdx.x] =                                          \
        (uint32_t)(c0 ^ c1 ^ c2 ^ c3 ^ c4 ^ c5 ^ c6 ^ c7);                                \
  }

// pairs: 8 chains of [v_mad_u64_u32 on m_i ; OTHER on c_i] (16 instructions per trip)
#define KPAIR(NAME, ASM)                                                                  \
  __global__ void __launch_bounds__(256) NAME(uint32_t* out, Stamp* st, uint32_t seed) {  \
    uint32_t a = seed ^ threadIdx.x, b = a * 2654435761u;                                 \
    uint32_t c0 = a, c1 = b, c2 = a + 1, c3 = b + 1, c4 = a + 2, c5 = b + 2, c6 = a + 3,  \
             c7 = b + 3;                                                                  \
    uint64_t m0 = a, m1 = b, m2 = a + 5, m3 = b + 5, m4 = a + 6, m5 = b + 6, m6 = a + 7,  \
             m7 = b + 7, cc;                                                              \
    unsigned long long t0, r0;                                                            \
    stamp_begin(st, t0, r0);                                                              \
    for (int i = 0; i < ITERS; ++i) {                                                     \
      _Pragma("unroll") for (int q = 0; q < 1; q++) {                                     \
        asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(m0), "=s"(cc) : "v"(a), "v"(b)); \
        asm volatile(ASM : "+v"(c0) : "v"(a), "v"(b));                                    \
        asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(m1), "=s"(cc) : "v"(a), "v"(b)); \
        asm volatile(ASM : "+v"(c1) : "v"(a), "v"(b));                                    \
        asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(m2), "=s"(cc) : "v"(a), "v"(b)); \
        asm volatile(ASM : "+v"(c2) : "v"(a), "v"(b));                                    \
        asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(m3), "=s"(cc) : "v"(a), "v"(b)); \
        asm volatile(ASM : "+v"(c3) : "v"(a), "v"(b));                                    \
        asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(m4), "=s"(cc) : "v"(a), "v"(b)); \
        asm volatile(ASM : "+v"(c4) : "v"(a), "v"(b));                                    \
        asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(m5), "=s"(cc) : "v"(a), "v"(b)); \
        asm volatile(ASM : "+v"(c5) : "v"(a), "v"(b));                                    \
        asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(m6), "=s"(cc) : "v"(a), "v"(b)); \
        asm volatile(ASM : "+v"(c6) : "v"(a), "v"(b));                                    \
        asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(m7), "=s"(cc) : "v"(a), "v"(b)); \
        asm volatile(ASM : "+v"(c7) : "v"(a), "v"(b));                                    \
      }                                                                                   \
    }                                                                                     \
    stamp_end(st, t0, r0);                                                                \
    out[blockIdx.x * blockDim.x + threadIdx.x] = c0 ^ c1 ^ c2 ^ c3 ^ c4 ^ c5 ^ c6 ^ c7 ^  \
        (uint32_t)(m0 ^ m1 ^ m2 ^ m3 ^ m4 ^ m5 ^ m6 ^ m7);                                \
  }

// one dependent chain of v_mad_u64_u32 (each MAD adds into the previous
// result: the column-scan squaring's shape), s_nop between as required
__global__ void __launch_bounds__(256) k_mad_dep1(uint32_t* out, Stamp* st, uint32_t seed) {
  uint32_t a = seed ^ threadIdx.x, b = a * 2654435761u;
  uint64_t m = a, cc;
  unsigned long long t0, r0;
  stamp_begin(st, t0, r0);
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int q = 0; q < 8; q++)
      asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0\n s_nop 0" : "+v"(m), "=s"(cc) : "v"(a), "v"(b));
  }
  stamp_end(st, t0, r0);
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)m;
}
// two interleaved dependent chains, no s_nop (the other chain's MAD between)
__global__ void __launch_bounds__(256) k_mad_dep2(uint32_t* out, Stamp* st, uint32_t seed) {
  uint32_t a = seed ^ threadIdx.x, b = a * 2654435761u;
  uint64_t m = a, n = b, cc;
  unsigned long long t0, r0;
  stamp_begin(st, t0, r0);
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int q = 0; q < 4; q++)
      asm volatile("v_mad_u64_u32 %0, %2, %3, %4, %0\n v_mad_u64_u32 %1, %2, %3, %4, %1"
                   : "+v"(m), "+v"(n), "=s"(cc) : "v"(a), "v"(b));
  }
  stamp_end(st, t0, r0);
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)(m ^ n);
}

K64(k_mad_u64_u32, "v_mad_u64_u32 %0, vcc, %1, %2, %0")
K64(k_mad_i64_i32, "v_mad_i64_i32 %0, vcc, %1, %2, %0")
K64(k_lshrrev_b64, "v_lshrrev_b64 %0, 26, %0")
K64(k_lshlrev_b64, "v_lshlrev_b64 %0, 1, %0")
K64(k_lshl_add_u64, "v_lshl_add_u64 %0, %0, 1, %3")
K64(k_lshl_add_u64_s0, "v_lshl_add_u64 %0, %0, 0, %3")
K64(k_fma_f64, "v_fma_f64 %0, %0, %3, %3")
K64(k_add_f64, "v_add_f64 %0, %0, %3")
K64(k_pk_fma_f32, "v_pk_fma_f32 %0, %0, %3, %3")
K64(k_pk_add_f32, "v_pk_add_f32 %0, %0, %3")
K64(k_pk_mov_b32, "v_pk_mov_b32 %0, %0, %3 op_sel:[1,0]")
K32(k_mul_lo_u32, "v_mul_lo_u32 %0, %1, %0")
K32(k_mul_hi_u32, "v_mul_hi_u32 %0, %1, %0")
K32(k_mul_u32_u24, "v_mul_u32_u24 %0, %1, %0")
K32(k_mad_u32_u24, "v_mad_u32_u24 %0, %1, %2, %0")
K32(k_mul_i32_i24, "v_mul_i32_i24 %0, %1, %0")
K32(k_add_u32, "v_add_u32 %0, %1, %0")
K32(k_sub_u32, "v_sub_u32 %0, %1, %0")
K32(k_add3_u32, "v_add3_u32 %0, %1, %2, %0")
K32(k_xad_u32, "v_xad_u32 %0, %1, %2, %0")
K32(k_and_b32, "v_and_b32 %0, %1, %0")
K32(k_and_lit, "v_and_b32 %0, 0x3ffffff, %0")
K32(k_or_b32, "v_or_b32 %0, %1, %0")
K32(k_xor_b32, "v_xor_b32 %0, %1, %0")
K32(k_or3_b32, "v_or3_b32 %0, %1, %2, %0")
K32(k_and_or_b32, "v_and_or_b32 %0, %1, %2, %0")
K32(k_bitop3_b32, "v_bitop3_b32 %0, %1, %2, %0 bitop3:0x96")
K32(k_lshlrev_b32, "v_lshlrev_b32 %0, 1, %0")
K32(k_lshrrev_b32, "v_lshrrev_b32 %0, 26, %0")
K32(k_lshl_add_u32, "v_lshl_add_u32 %0, %0, 1, %1")
K32(k_add_lshl_u32, "v_add_lshl_u32 %0, %0, %1, 1")
K32(k_lshl_or_b32, "v_lshl_or_b32 %0, %0, 1, %1")
K32(k_bfe_u32, "v_bfe_u32 %0, %0, 26, 6")
K32(k_bfi_b32, "v_bfi_b32 %0, %1, %2, %0")
K32(k_alignbit_b32, "v_alignbit_b32 %0, %1, %0, 7")
K32(k_perm_b32, "v_perm_b32 %0, %1, %0, %2")
K32(k_cndmask_b32, "v_cndmask_b32 %0, %1, %0, vcc")
K32(k_mov_b32, "v_mov_b32 %0, %1")
K32(k_add_co_u32, "v_add_co_u32 %0, vcc, %1, %0")
K32(k_addc_co_u32, "v_addc_co_u32 %0, vcc, %1, %0, vcc")
K32(k_sad_u32, "v_sad_u32 %0, %1, %2, %0")
K32(k_max3_u32, "v_max3_u32 %0, %1, %2, %0")
K32(k_min_u32, "v_min_u32 %0, %1, %0")
K32(k_pk_add_u16, "v_pk_add_u16 %0, %1, %0")
K32(k_pk_mad_u16, "v_pk_mad_u16 %0, %1, %2, %0")
K32(k_mul_u32_u24_dpp, "v_mul_u32_u24_dpp %0, %1, %0 row_ror:1 row_mask:0xf bank_mask:0xf")
K32(k_mov_dpp, "v_mov_b32_dpp %0, %1 row_ror:1 row_mask:0xf bank_mask:0xf")
K32(k_fma_f32, "v_fma_f32 %0, %1, %2, %0")
K32(k_add_f32, "v_add_f32 %0, %1, %0")
K32(k_cvt_f32_u32, "v_cvt_f32_u32 %0, %0")

KPAIR(p_mad_and, "v_and_b32 %0, 0x3ffffff, %0")
KPAIR(p_mad_add, "v_add_u32 %0, %1, %0")
KPAIR(p_mad_lshl, "v_lshlrev_b32 %0, 1, %0")
KPAIR(p_mad_mullo, "v_mul_lo_u32 %0, %1, %0")
KPAIR(p_mad_alignbit, "v_alignbit_b32 %0, %1, %0, 7")
KPAIR(p_mad_cndmask, "v_cndmask_b32 %0, %1, %0, vcc")
KPAIR(p_mad_mov, "v_mov_b32 %0, %1")
KPAIR(p_mad_add3, "v_add3_u32 %0, %1, %2, %0")
KPAIR(p_mad_fma32, "v_fma_f32 %0, %1, %2, %0")
KPAIR(p_mad_mad24, "v_mad_u32_u24 %0, %1, %2, %0")

typedef void (*kfn)(uint32_t*, Stamp*, uint32_t);

struct Res {
  double ms, ghz, cyc;
};

// waves_per_simd W: 256-thread blocks (one wave per SIMD each), 256 * W blocks
static Res run(kfn k, int W, int insts_per_trip, uint32_t* d, Stamp* dst, int cus) {
  const int blocks = cus * W, threads = 256, nw = blocks * 4;
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, d, dst, 1u);
  CHECK(hipDeviceSynchronize());
  const int reps = 3;
  CHECK(hipEventRecord(e0));
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, d, dst, 1u + r);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  std::vector<Stamp> st(nw);
  CHECK(hipMemcpy(st.data(), dst, sizeof(Stamp) * nw, hipMemcpyDeviceToHost));
  // shader clock from the last launch's waves; per-wave loop cycles
  double ghz = 0, cyc_wave = 0;
  for (auto& s : st) {
    ghz += double(s.c1 - s.c0) / double(s.r1 - s.r0) * 0.1;  // s_memrealtime is 100 MHz
    cyc_wave += double(s.c1 - s.c0);
  }
  ghz /= nw;
  cyc_wave /= nw;
  // each wave's loop ran concurrently with W-1 others on its SIMD: SIMD cycles
  // per wave-instruction = loop cycles / (W * instructions of one wave)
  const double insts = double(ITERS) * insts_per_trip;
  Res r{ms / reps, ghz, cyc_wave / (W * insts)};
  CHECK(hipEventDestroy(e0));
  CHECK(hipEventDestroy(e1));
  return r;
}

int main() {
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  const int cus = p.multiProcessorCount;
  uint32_t* d;
  Stamp* dst;
  CHECK(hipMalloc(&d, sizeof(uint32_t) * cus * 8 * 256));
  CHECK(hipMalloc(&dst, sizeof(Stamp) * cus * 8 * 4));
  struct {
    const char* name;
    kfn k;
    int per_trip;
  } ks[] = {
      {"v_mad_u64_u32", k_mad_u64_u32, 8}, {"v_mad_i64_i32", k_mad_i64_i32, 8},
      {"mad_dep1_chain(+s_nop)", k_mad_dep1, 8}, {"mad_dep2_chains", k_mad_dep2, 8},
      {"v_lshrrev_b64", k_lshrrev_b64, 8}, {"v_lshlrev_b64", k_lshlrev_b64, 8},
      {"v_lshl_add_u64", k_lshl_add_u64, 8}, {"v_lshl_add_u64_s0", k_lshl_add_u64_s0, 8},
      {"v_fma_f64", k_fma_f64, 8}, {"v_add_f64", k_add_f64, 8},
      {"v_pk_fma_f32", k_pk_fma_f32, 8}, {"v_pk_add_f32", k_pk_add_f32, 8},
      {"v_pk_mov_b32", k_pk_mov_b32, 8},
      {"v_mul_lo_u32", k_mul_lo_u32, 8}, {"v_mul_hi_u32", k_mul_hi_u32, 8},
      {"v_mul_u32_u24", k_mul_u32_u24, 8}, {"v_mad_u32_u24", k_mad_u32_u24, 8},
      {"v_mul_i32_i24", k_mul_i32_i24, 8}, {"v_add_u32", k_add_u32, 8},
      {"v_sub_u32", k_sub_u32, 8}, {"v_add3_u32", k_add3_u32, 8}, {"v_xad_u32", k_xad_u32, 8},
      {"v_and_b32", k_and_b32, 8}, {"v_and_b32_lit", k_and_lit, 8}, {"v_or_b32", k_or_b32, 8},
      {"v_xor_b32", k_xor_b32, 8}, {"v_or3_b32", k_or3_b32, 8}, {"v_and_or_b32", k_and_or_b32, 8},
      {"v_bitop3_b32", k_bitop3_b32, 8}, {"v_lshlrev_b32", k_lshlrev_b32, 8},
      {"v_lshrrev_b32", k_lshrrev_b32, 8}, {"v_lshl_add_u32", k_lshl_add_u32, 8},
      {"v_add_lshl_u32", k_add_lshl_u32, 8}, {"v_lshl_or_b32", k_lshl_or_b32, 8},
      {"v_bfe_u32", k_bfe_u32, 8}, {"v_bfi_b32", k_bfi_b32, 8},
      {"v_alignbit_b32", k_alignbit_b32, 8}, {"v_perm_b32", k_perm_b32, 8},
      {"v_cndmask_b32", k_cndmask_b32, 8}, {"v_mov_b32", k_mov_b32, 8},
      {"v_add_co_u32", k_add_co_u32, 8}, {"v_addc_co_u32", k_addc_co_u32, 8},
      {"v_sad_u32", k_sad_u32, 8}, {"v_max3_u32", k_max3_u32, 8}, {"v_min_u32", k_min_u32, 8},
      {"v_pk_add_u16", k_pk_add_u16, 8}, {"v_pk_mad_u16", k_pk_mad_u16, 8},
      {"v_mul_u32_u24_dpp", k_mul_u32_u24_dpp, 8}, {"v_mov_b32_dpp", k_mov_dpp, 8},
      {"v_fma_f32", k_fma_f32, 8}, {"v_add_f32", k_add_f32, 8},
      {"v_cvt_f32_u32", k_cvt_f32_u32, 8},
      {"pair mad+and", p_mad_and, 16}, {"pair mad+add", p_mad_add, 16},
      {"pair mad+lshl", p_mad_lshl, 16}, {"pair mad+mul_lo", p_mad_mullo, 16},
      {"pair mad+alignbit", p_mad_alignbit, 16}, {"pair mad+cndmask", p_mad_cndmask, 16},
      {"pair mad+mov", p_mad_mov, 16}, {"pair mad+add3", p_mad_add3, 16},
      {"pair mad+fma_f32", p_mad_fma32, 16}, {"pair mad+mad_u32_u24", p_mad_mad24, 16},
  };
  printf("{\"device\": \"%s\", \"cus\": %d, \"iters\": %d, \"unit\": \"SIMD cycles per wave-instruction (pairs: per instruction of the pair)\",\n \"kinds\": {\n",
         p.gcnArchName, cus, ITERS);
  const int Ws[3] = {1, 2, 4};
  bool first = true;
  for (auto& kk : ks) {
    printf("%s  \"%s\": {", first ? "" : ",\n", kk.name);
    first = false;
    for (int wi = 0; wi < 3; wi++) {
      Res r = run(kk.k, Ws[wi], kk.per_trip, d, dst, cus);
      printf("%s\"w%d\": {\"cyc\": %.3f, \"ghz\": %.3f, \"ms\": %.4f}", wi ? ", " : "", Ws[wi], r.cyc,
             r.ghz, r.ms);
    }
    printf("}");
    fflush(stdout);
  }
  printf("\n }\n}\n");
  CHECK(hipFree(d));
  CHECK(hipFree(dst));
  return 0;
}
