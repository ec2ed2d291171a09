// synth.hip -- on-device synthesis of benchmark/test inputs (BENCH/TEST
// INFRASTRUCTURE, built into lib/libouro_synth.so, never into the verifier).
//
// Seeds (tag zero-padded to 12 bytes so every seed message is
// exactly 32 bytes):
//   seed(tag, i) = SHA-512("ouro-mi355x/" || tag[12] || LE64(i))[0:32]
// Header batches: P pools; header i belongs to pool i mod P, KES period
// t = i mod 64, counter = c0 = 0, alpha_eta = seed("eta", i),
// alpha_leader = seed("lead", i), body = the golden Shelley body template with
// its prevHash payload replaced by seed("body", i).  Sum6KES leaf l of pool j
// has seed SHA-512(seed("kes", j) || LE32(l))[0:32].
// Every routine mirrors oracle/batch.c + oracle/kes.c byte for byte
// (tests/test_synth.py).
#include <hip/hip_runtime.h>

#include <cstring>
#include <vector>

#include "synth.h"

using namespace ouro;

namespace {

constexpr int kBlock = 256;

struct Tag {
  uint32_t w[3];
};

__device__ __forceinline__ void seed_of(uint32_t out[8], Tag tag, uint64_t i) {
  uint32_t m[8];
  m[0] = 0x6f72756fu;  // "ouro"
  m[1] = 0x33696d2du;  // "-mi3"
  m[2] = 0x2f783535u;  // "55x/"
  m[3] = tag.w[0];
  m[4] = tag.w[1];
  m[5] = tag.w[2];
  m[6] = (uint32_t)i;
  m[7] = (uint32_t)(i >> 32);
  uint32_t h[16];
  sha512_32(h, m);
#pragma unroll
  for (int k = 0; k < 8; k++) out[k] = h[k];
}

struct RegTail32 {
  uint32_t w[8];
  __device__ __forceinline__ uint32_t tail(uint32_t q) const { return byte_of(w, (int)q); }
};
struct RegTail4 {
  uint32_t w[1];
  __device__ __forceinline__ uint32_t tail(uint32_t q) const { return (w[0] >> (8 * (q & 3))) & 0xffu; }
};

__device__ __forceinline__ void ld8(uint32_t* w, const uint8_t* p) {
  const uint4* q = reinterpret_cast<const uint4*>(p);
  uint4 a = q[0], b = q[1];
  w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w; w[4] = b.x; w[5] = b.y; w[6] = b.z; w[7] = b.w;
}
__device__ __forceinline__ void st_n(uint8_t* p, const uint32_t* w, int n16) {
  uint4* q = reinterpret_cast<uint4*>(p);
  for (int i = 0; i < n16; i++) q[i] = make_uint4(w[4 * i], w[4 * i + 1], w[4 * i + 2], w[4 * i + 3]);
}

__device__ __forceinline__ void kes_leaf_seed(uint32_t out[8], const uint32_t tree_seed[8], uint32_t l) {
  RegTail4 t;
  t.w[0] = l;
  uint64_t H[8];
  sha512_prefixed<32>(H, tree_seed, t, 4);
  uint32_t h[16];
  sha512_digest_words(h, H);
#pragma unroll
  for (int k = 0; k < 8; k++) out[k] = h[k];
}

}  // namespace

// ---- flat batches ------------------------------------------------------------
__global__ void __launch_bounds__(kBlock) k_synth_ed25519(size_t n, uint64_t first, Tag tseed,
                                                          Tag tmsg, uint8_t* pk, uint8_t* sig,
                                                          uint8_t* msg, int32_t* scratch,
                                                          const int32_t* btab) {
  const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t nth = (size_t)gridDim.x * blockDim.x;
  const Slot lane = slot_of(scratch, tid, kLaneWords);
  for (size_t i = tid; i < n; i += nth) {
    uint32_t seed[8];
    RegTail32 m;
    seed_of(seed, tseed, first + i);
    seed_of(m.w, tmsg, first + i);
    ExpandedKey k;
    expand_seed(k, seed, lane, btab);
    uint32_t s[16];
    ed25519_sign_lane(s, k, m, 32, lane, btab);
    st_n(pk + 32 * i, k.pk, 2);
    st_n(sig + 64 * i, s, 4);
    st_n(msg + 32 * i, m.w, 2);
  }
}

__global__ void __launch_bounds__(kBlock) k_synth_vrf(size_t n, uint64_t first, Tag tseed,
                                                      Tag talpha, uint8_t* pk, uint8_t* proof,
                                                      uint8_t* alpha, int32_t* scratch,
                                                      const int32_t* btab) {
  const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t nth = (size_t)gridDim.x * blockDim.x;
  const Slot lane = slot_of(scratch, tid, kLaneWords);
  for (size_t i = tid; i < n; i += nth) {
    uint32_t seed[8], a[8], pi[20];
    seed_of(seed, tseed, first + i);
    seed_of(a, talpha, first + i);
    ExpandedKey k;
    expand_seed(k, seed, lane, btab);
    vrf03_prove_lane(pi, k, a, lane, btab);
    st_n(pk + 32 * i, k.pk, 2);
    st_n(proof + 80 * i, pi, 5);
    st_n(alpha + 32 * i, a, 2);
  }
}

// ---- header batches ---------------------------------------------------------
// nodes: [pool][127][8 words]: level 0 = 64 leaf vks, then 32, 16, 8, 4, 2, 1
__device__ __forceinline__ int node_index(int level, int idx) {
  return (128 - (128 >> level)) + idx;
}

__global__ void __launch_bounds__(kBlock) k_synth_kes_leaves(int npools, Tag tkes, uint32_t* nodes,
                                                             int32_t* scratch, const int32_t* btab) {
  const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t nth = (size_t)gridDim.x * blockDim.x;
  const Slot lane = slot_of(scratch, tid, kLaneWords);
  for (size_t g = tid; g < (size_t)npools * 64; g += nth) {
    const int j = (int)(g >> 6), l = (int)(g & 63);
    uint32_t ts[8], ls[8];
    seed_of(ts, tkes, (uint64_t)j);
    kes_leaf_seed(ls, ts, (uint32_t)l);
    ExpandedKey k;
    expand_seed(k, ls, lane, btab);
    uint32_t* dst = nodes + ((size_t)j * 127 + node_index(0, l)) * 8;
    for (int w = 0; w < 8; w++) dst[w] = k.pk[w];
  }
}

__global__ void __launch_bounds__(kBlock) k_synth_kes_tree(int npools, uint32_t* nodes) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= npools) return;
  uint32_t* base = nodes + (size_t)j * 127 * 8;
  for (int level = 1; level <= 6; level++) {
    for (int idx = 0; idx < (64 >> level); idx++) {
      uint32_t in[16], h[8];
      const uint32_t* a = base + node_index(level - 1, 2 * idx) * 8;
      for (int w = 0; w < 16; w++) in[w] = a[w];  // the two children are adjacent
      blake2b256_64(h, in);
      uint32_t* d = base + node_index(level, idx) * 8;
      for (int w = 0; w < 8; w++) d[w] = h[w];
    }
  }
}

// per pool: cold key, VRF key (expanded), opcert over the Sum6 root
__global__ void __launch_bounds__(kBlock) k_synth_pools(int npools, Tag tcold, Tag tvrf,
                                                        const uint32_t* nodes, uint32_t* pool,
                                                        int32_t* scratch, const int32_t* btab) {
  // pool record (words): cold_pk 8 | vrf a 8 | vrf prefix 8 | vrf pk 8 | hot_vk 8 | sigma 16
  const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t nth = (size_t)gridDim.x * blockDim.x;
  const Slot lane = slot_of(scratch, tid, kLaneWords);
  for (size_t j = tid; j < (size_t)npools; j += nth) {
    uint32_t cs[8], vs[8];
    seed_of(cs, tcold, j);
    seed_of(vs, tvrf, j);
    ExpandedKey cold, vrf;
    expand_seed(cold, cs, lane, btab);
    expand_seed(vrf, vs, lane, btab);
    const uint32_t* root = nodes + (j * 127 + node_index(6, 0)) * 8;
    struct RegTail48 {
      uint32_t w[12];
      __device__ __forceinline__ uint32_t tail(uint32_t q) const {
        uint32_t r = w[0];
        for (int i = 1; i < 12; i++) r = ((q >> 2) == (uint32_t)i) ? w[i] : r;
        return (r >> (8 * (q & 3))) & 0xffu;
      }
    } m;
    for (int w = 0; w < 8; w++) m.w[w] = root[w];
    for (int w = 8; w < 12; w++) m.w[w] = 0;  // BE64(counter 0) || BE64(c0 0)
    uint32_t sig[16];
    ed25519_sign_lane(sig, cold, m, 48, lane, btab);
    uint32_t* rec = pool + j * 56;
    for (int w = 0; w < 8; w++) {
      rec[w] = cold.pk[w];
      rec[8 + w] = vrf.a[w];
      rec[16 + w] = vrf.prefix[w];
      rec[24 + w] = vrf.pk[w];
      rec[32 + w] = root[w];
    }
    for (int w = 0; w < 16; w++) rec[40 + w] = sig[w];
  }
}

__global__ void __launch_bounds__(kBlock) k_synth_headers(
    size_t n, uint64_t first, int npools, Tag teta, Tag tlead, Tag tbody, Tag tkes, const uint32_t* pool,
    const uint32_t* nodes, const uint8_t* body_tmpl, uint32_t body_len, uint8_t* issuer_vk,
    uint8_t* vrf_vk, uint8_t* eta_proof, uint8_t* leader_proof, uint8_t* eta_alpha,
    uint8_t* leader_alpha, uint8_t* hot_vk, uint64_t* counter, uint64_t* c0, uint8_t* sigma,
    uint32_t* kes_t, uint8_t* kes_sig, uint8_t* body, uint64_t* body_off, uint32_t* body_lens,
    int32_t* scratch, const int32_t* btab) {
  const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t nth = (size_t)gridDim.x * blockDim.x;
  const Slot lane = slot_of(scratch, tid, kLaneWords);
  for (size_t i = tid; i < n; i += nth) {
    const uint64_t g = first + i;  // global header index
    const int j = (int)(g % (uint64_t)npools);
    const uint32_t t = (uint32_t)(g & 63);
    const uint32_t* rec = pool + (size_t)j * 56;
    ExpandedKey vrf;
    for (int w = 0; w < 8; w++) {
      vrf.a[w] = rec[8 + w];
      vrf.prefix[w] = rec[16 + w];
      vrf.pk[w] = rec[24 + w];
    }
    uint32_t ae[8], al[8], pe[20], pl[20];
    seed_of(ae, teta, first + i);
    seed_of(al, tlead, first + i);
    vrf03_prove_lane(pe, vrf, ae, lane, btab);
    vrf03_prove_lane(pl, vrf, al, lane, btab);
    // body: template with the prevHash payload (body bytes 5..36) per header
    uint8_t* bd = body + i * (size_t)body_len;
    uint32_t ph[8];
    seed_of(ph, tbody, first + i);
    for (uint32_t b = 0; b < body_len; b++) {
      const uint32_t k = b - 5;
      bd[b] = (b >= 5 && b < 37) ? (uint8_t)byte_of(ph, (int)k) : body_tmpl[b];
    }
    // KES: leaf key t of pool j signs the body; Merkle pairs bottom-up
    uint32_t ts[8], ls[8];
    seed_of(ts, tkes, (uint64_t)j);
    kes_leaf_seed(ls, ts, t);
    ExpandedKey leaf;
    expand_seed(leaf, ls, lane, btab);
    uint32_t lsig[16];
    ed25519_sign_lane(lsig, leaf, ShaGlobalTail{bd}, body_len, lane, btab);
    uint8_t* ks = kes_sig + i * 448;
    st_n(ks, lsig, 4);
    const uint32_t* nb = nodes + (size_t)j * 127 * 8;
    for (int k = 1; k <= 6; k++) {
      const int idx = (int)(t >> (k - 1)) & ~1;
      st_n(ks + 64 + 64 * (k - 1), nb + node_index(k - 1, idx) * 8, 4);  // vk0 || vk1
    }
    st_n(issuer_vk + 32 * i, rec, 2);
    st_n(vrf_vk + 32 * i, rec + 24, 2);
    st_n(hot_vk + 32 * i, rec + 32, 2);
    st_n(sigma + 64 * i, rec + 40, 4);
    st_n(eta_proof + 80 * i, pe, 5);
    st_n(leader_proof + 80 * i, pl, 5);
    st_n(eta_alpha + 32 * i, ae, 2);
    st_n(leader_alpha + 32 * i, al, 2);
    counter[i] = 0;
    c0[i] = 0;
    kes_t[i] = t;
    body_off[i] = i * (uint64_t)body_len;
    body_lens[i] = body_len;
  }
}

// The node's configuration of a batch made by k_synth_headers (ADVICE r02:
// the bench's "node" latency leg): slot_i = slot0 + i, VRF inputs derived
// as the OVERLAY rule does -- mkSeed seedEta / seedL slot eta0 -- and both
// proofs re-made over them with the pool's VRF key; the claimed outputs are
// the proofs' outputs (proof_to_hash).  eta0 = NULL: NeutralNonce.
__device__ void vrf_output_of(uint8_t* out, const uint32_t pi[20]) {
  uint32_t G[8];
  for (int k = 0; k < 8; k++) G[k] = pi[k];
  ge_p3 Gamma;
  ge_decode(&Gamma, G, false);
  const ge_p3 G8 = ge_mul8(Gamma);
  uint32_t enc[8], bp[9], w[16];
  ge_encode_with_inv(enc, G8.X, G8.Y, fe_invert(G8.Z));
  bp[0] = 0x04u | (0x03u << 8) | (enc[0] << 16);
  for (int k = 1; k < 8; k++) bp[k] = (enc[k - 1] >> 16) | (enc[k] << 16);
  bp[8] = enc[7] >> 16;
  uint64_t H[8];
  sha512_prefixed<34>(H, bp, ShaNoTail{}, 0);
  sha512_digest_words(w, H);
  st_n(out, w, 4);
}

__global__ void __launch_bounds__(kBlock) k_synth_seeded(
    size_t n, uint64_t first, int npools, const uint32_t* pool, uint64_t slot0,
    const uint8_t* eta0, uint64_t* slot, uint8_t* eta_alpha, uint8_t* leader_alpha,
    uint8_t* eta_proof, uint8_t* leader_proof, uint8_t* eta_out, uint8_t* lead_out,
    int32_t* scratch, const int32_t* btab, const uint64_t* slot_in) {
  const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t nth = (size_t)gridDim.x * blockDim.x;
  const Slot lane = slot_of(scratch, tid, kLaneWords);
  uint32_t e0[8];
  if (eta0)
    for (int k = 0; k < 8; k++)
      e0[k] = (uint32_t)eta0[4 * k] | ((uint32_t)eta0[4 * k + 1] << 8) |
              ((uint32_t)eta0[4 * k + 2] << 16) | ((uint32_t)eta0[4 * k + 3] << 24);
  for (size_t i = tid; i < n; i += nth) {
    const int j = (int)((first + i) % (uint64_t)npools);
    const uint32_t* rec = pool + (size_t)j * 56;
    ExpandedKey vrf;
    for (int w = 0; w < 8; w++) {
      vrf.a[w] = rec[8 + w];
      vrf.prefix[w] = rec[16 + w];
      vrf.pk[w] = rec[24 + w];
    }
    const uint64_t s = slot_in ? slot_in[i] : slot0 + i;
    slot[i] = s;
    uint32_t h[8], ae[8], al[8], pe[20], pl[20];
    mkseed_hash(h, s, eta0 ? e0 : nullptr);
    for (int k = 0; k < 8; k++) {
      ae[k] = h[k] ^ kSeedEta[k];
      al[k] = h[k] ^ kSeedL[k];
    }
    vrf03_prove_lane(pe, vrf, ae, lane, btab);
    vrf03_prove_lane(pl, vrf, al, lane, btab);
    st_n(eta_alpha + 32 * i, ae, 2);
    st_n(leader_alpha + 32 * i, al, 2);
    st_n(eta_proof + 80 * i, pe, 5);
    st_n(leader_proof + 80 * i, pl, 5);
    vrf_output_of(eta_out + 64 * i, pe);
    vrf_output_of(lead_out + 64 * i, pl);
  }
}

// Raw wire headers (#6.24(bytes .cbor [header_body, kes_sig])) consistent with
// a synthesised SoA batch, for the raw-CBOR -> verdict bench leg and tests:
// the host-built template (bench.raw_template: the golden body re-encoded with
// a 4-byte slot and counter = kesPeriod = 0) gets this header's prevHash seed,
// keys, VRF certificates (outputs = proof_to_hash of the proofs), sigma and a
// slot in KES period t; then the header_body bytes are KES-signed in place.
struct RawOffsets {
  uint32_t body, body_len, slot, prev, issuer, vrf, eta_out, eta_proof, lead_out, lead_proof,
      hot, sigma, sig;
};
__device__ void proof_output(uint8_t* dst, const uint8_t* proof) {
  uint32_t G[8];
  for (int k = 0; k < 8; k++)
    G[k] = proof[4 * k] | (proof[4 * k + 1] << 8) | (proof[4 * k + 2] << 16) |
           ((uint32_t)proof[4 * k + 3] << 24);
  ge_p3 Gamma;
  ge_decode(&Gamma, G, false);
  ge_p3 G8 = ge_mul8(Gamma);
  uint32_t enc[8];
  ge_encode_with_inv(enc, G8.X, G8.Y, fe_invert(G8.Z));
  uint32_t bp[9];
  bp[0] = 0x04u | (0x03u << 8) | (enc[0] << 16);
  for (int k = 1; k < 8; k++) bp[k] = (enc[k - 1] >> 16) | (enc[k] << 16);
  bp[8] = enc[7] >> 16;
  uint64_t H[8];
  sha512_prefixed<34>(H, bp, ShaNoTail{}, 0);
  uint32_t w[16];
  sha512_digest_words(w, H);
  for (int k = 0; k < 64; k++) dst[k] = (uint8_t)byte_of(w, k);
}
__global__ void __launch_bounds__(kBlock) k_synth_raw(
    size_t n, uint64_t first, int npools, Tag tbody, Tag tkes, const uint32_t* nodes,
    const uint8_t* tmpl, uint32_t raw_len, RawOffsets o, uint64_t spkp, const uint8_t* issuer_vk,
    const uint8_t* vrf_vk, const uint8_t* eta_proof, const uint8_t* leader_proof,
    const uint8_t* hot_vk, const uint8_t* sigma, const uint32_t* kes_t, uint8_t* raw,
    int32_t* scratch, const int32_t* btab) {
  const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t nth = (size_t)gridDim.x * blockDim.x;
  const Slot lane = slot_of(scratch, tid, kLaneWords);
  for (size_t i = tid; i < n; i += nth) {
    const uint64_t g = first + i;
    const int j = (int)(g % (uint64_t)npools);
    const uint32_t t = kes_t[i];
    uint8_t* r = raw + i * (size_t)raw_len;
    for (uint32_t b = 0; b < raw_len; b++) r[b] = tmpl[b];
    const uint32_t slot = (uint32_t)(t * spkp + g % 1000);
    for (int b = 0; b < 4; b++) r[o.slot + b] = (uint8_t)(slot >> (24 - 8 * b));
    uint32_t ph[8];
    seed_of(ph, tbody, g);
    for (int b = 0; b < 32; b++) r[o.prev + b] = (uint8_t)byte_of(ph, b);
    for (int b = 0; b < 32; b++) {
      r[o.issuer + b] = issuer_vk[32 * i + b];
      r[o.vrf + b] = vrf_vk[32 * i + b];
      r[o.hot + b] = hot_vk[32 * i + b];
    }
    for (int b = 0; b < 80; b++) {
      r[o.eta_proof + b] = eta_proof[80 * i + b];
      r[o.lead_proof + b] = leader_proof[80 * i + b];
    }
    for (int b = 0; b < 64; b++) r[o.sigma + b] = sigma[64 * i + b];
    proof_output(r + o.eta_out, eta_proof + 80 * i);
    proof_output(r + o.lead_out, leader_proof + 80 * i);
    // KES: leaf t of pool j signs the header_body bytes; Merkle pairs bottom-up
    uint32_t ts[8], ls[8];
    seed_of(ts, tkes, (uint64_t)j);
    kes_leaf_seed(ls, ts, t);
    ExpandedKey leaf;
    expand_seed(leaf, ls, lane, btab);
    uint32_t lsig[16];
    ed25519_sign_lane(lsig, leaf, ShaGlobalTail{r + o.body}, o.body_len, lane, btab);
    uint8_t* ks = r + o.sig;
    for (int b = 0; b < 64; b++) ks[b] = (uint8_t)byte_of(lsig, b);
    const uint32_t* nb = nodes + (size_t)j * 127 * 8;
    for (int k = 1; k <= 6; k++) {
      const int idx = (int)(t >> (k - 1)) & ~1;
      const uint32_t* pair = nb + node_index(k - 1, idx) * 8;  // vk0 || vk1
      for (int b = 0; b < 64; b++) ks[64 + 64 * (k - 1) + b] = (uint8_t)byte_of(pair, b);
    }
  }
}

// ---- host launchers (device pointers; synchronous) ---------------------------
namespace {
Tag make_tag(const char* s) {
  Tag t{{0, 0, 0}};
  uint8_t b[12] = {0};
  for (int i = 0; i < 12 && s[i]; i++) b[i] = (uint8_t)s[i];
  for (int w = 0; w < 3; w++)
    t.w[w] = b[4 * w] | (b[4 * w + 1] << 8) | (b[4 * w + 2] << 16) | ((uint32_t)b[4 * w + 3] << 24);
  return t;
}
struct Ctx {
  int32_t* btab = nullptr;
  int32_t* scratch = nullptr;
  size_t lanes = 0;
};
Ctx g_ctx;
int grid_for(size_t items) {
  size_t b = (items + kBlock - 1) / kBlock;
  if (b > 4096) b = 4096;
  return b ? (int)b : 1;
}
int prepare(size_t items) {
  if (!g_ctx.btab) {
    std::vector<int32_t> tab(kBTabWords);
    build_btab(tab.data());
    const size_t bytes = tab.size() * sizeof(int32_t);
    if (hipMalloc(&g_ctx.btab, bytes) != hipSuccess) return -2;
    if (hipMemcpy(g_ctx.btab, tab.data(), bytes, hipMemcpyHostToDevice) != hipSuccess) return -2;
  }
  size_t lanes = (size_t)grid_for(items) * kBlock;
  if (lanes > g_ctx.lanes) {
    if (g_ctx.scratch) (void)hipFree(g_ctx.scratch);
    if (hipMalloc(&g_ctx.scratch, lanes * kLaneWords * sizeof(int32_t)) != hipSuccess) return -2;
    g_ctx.lanes = lanes;
  }
  return 0;
}
int done() { return hipDeviceSynchronize() == hipSuccess && hipGetLastError() == hipSuccess ? 0 : -2; }
}  // namespace

// v_mad_u64_u32 throughput (the roofline peak of DESIGN.md; same kernel as
// tools/microbench/int_rates.hip)
constexpr int kPeakIters = 4096;
__global__ void k_peak_mad_u64(uint64_t* out, uint32_t seed) {
  uint32_t a = seed ^ threadIdx.x, b = a * 2654435761u;
  uint64_t c0 = a, c1 = b, c2 = a + 1, c3 = b + 1, c4 = a + 2, c5 = b + 2, c6 = a + 3, c7 = b + 3;
  uint64_t cc;
  for (int i = 0; i < kPeakIters; ++i) {
#define OURO_MAD(c) asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(c), "=s"(cc) : "v"(a), "v"(b));
    OURO_MAD(c0) OURO_MAD(c1) OURO_MAD(c2) OURO_MAD(c3) OURO_MAD(c4) OURO_MAD(c5) OURO_MAD(c6) OURO_MAD(c7)
#undef OURO_MAD
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = c0 ^ c1 ^ c2 ^ c3 ^ c4 ^ c5 ^ c6 ^ c7;
}

extern "C" {

double ouro_peak_mad_u64_tmacs(void) {
  hipDeviceProp_t p;
  if (hipGetDeviceProperties(&p, 0) != hipSuccess) return -1.0;
  const int threads = 256, blocks = p.multiProcessorCount * 8;
  uint64_t* d = nullptr;
  if (hipMalloc(&d, sizeof(uint64_t) * threads * blocks) != hipSuccess) return -1.0;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  hipLaunchKernelGGL(k_peak_mad_u64, dim3(blocks), dim3(threads), 0, 0, d, 1u);
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(e0, 0);
  for (int r = 0; r < 10; r++) hipLaunchKernelGGL(k_peak_mad_u64, dim3(blocks), dim3(threads), 0, 0, d, 2u + r);
  (void)hipEventRecord(e1, 0);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  (void)hipFree(d);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  const double macs = 10.0 * blocks * threads * kPeakIters * 8;
  return macs / (ms * 1e-3) / 1e12;
}

int ouro_synth_ed25519(size_t n, uint64_t first, uint8_t* pk, uint8_t* sig, uint8_t* msg) {
  if (prepare(n)) return -2;
  hipLaunchKernelGGL(k_synth_ed25519, dim3(grid_for(n)), dim3(kBlock), 0, 0, n, first,
                     make_tag("ed"), make_tag("msg"), pk, sig, msg, g_ctx.scratch, g_ctx.btab);
  return done();
}

int ouro_synth_vrf(size_t n, uint64_t first, uint8_t* pk, uint8_t* proof, uint8_t* alpha) {
  if (prepare(n)) return -2;
  hipLaunchKernelGGL(k_synth_vrf, dim3(grid_for(n)), dim3(kBlock), 0, 0, n, first,
                     make_tag("vrf"), make_tag("alpha"), pk, proof, alpha, g_ctx.scratch,
                     g_ctx.btab);
  return done();
}

// work buffers: nodes = npools*127*8 u32, pool = npools*56 u32 (device)
int ouro_synth_headers(size_t n, uint64_t first, int npools, const uint8_t* body_tmpl, uint32_t body_len,
                       uint32_t* nodes, uint32_t* pool, uint8_t* issuer_vk, uint8_t* vrf_vk,
                       uint8_t* eta_proof, uint8_t* leader_proof, uint8_t* eta_alpha,
                       uint8_t* leader_alpha, uint8_t* hot_vk, uint64_t* counter, uint64_t* c0,
                       uint8_t* sigma, uint32_t* kes_t, uint8_t* kes_sig, uint8_t* body,
                       uint64_t* body_off, uint32_t* body_lens) {
  if (npools <= 0 || body_len < 37) return -3;
  if (prepare(n > (size_t)npools * 64 ? n : (size_t)npools * 64)) return -2;
  hipLaunchKernelGGL(k_synth_kes_leaves, dim3(grid_for((size_t)npools * 64)), dim3(kBlock), 0, 0,
                     npools, make_tag("kes"), nodes, g_ctx.scratch, g_ctx.btab);
  if (done()) return -2;
  hipLaunchKernelGGL(k_synth_kes_tree, dim3((npools + kBlock - 1) / kBlock), dim3(kBlock), 0, 0,
                     npools, nodes);
  if (done()) return -2;
  hipLaunchKernelGGL(k_synth_pools, dim3(grid_for(npools)), dim3(kBlock), 0, 0, npools,
                     make_tag("cold"), make_tag("vrfpool"), nodes, pool, g_ctx.scratch, g_ctx.btab);
  if (done()) return -2;
  hipLaunchKernelGGL(k_synth_headers, dim3(grid_for(n)), dim3(kBlock), 0, 0, n, first, npools,
                     make_tag("eta"), make_tag("lead"), make_tag("body"), make_tag("kes"), pool,
                     nodes, body_tmpl, body_len, issuer_vk, vrf_vk, eta_proof, leader_proof,
                     eta_alpha, leader_alpha, hot_vk, counter, c0, sigma, kes_t, kes_sig, body,
                     body_off, body_lens, g_ctx.scratch, g_ctx.btab);
  return done();
}

// the node configuration (k_synth_seeded) of a batch ouro_synth_headers made
// with the same n, first, npools, pool; eta0 a device pointer or NULL
int ouro_synth_seeded(size_t n, uint64_t first, int npools, const uint32_t* pool, uint64_t slot0,
                      const uint8_t* eta0, uint64_t* slot, uint8_t* eta_alpha,
                      uint8_t* leader_alpha, uint8_t* eta_proof, uint8_t* leader_proof,
                      uint8_t* eta_out, uint8_t* lead_out) {
  if (npools <= 0) return -3;
  if (prepare(n)) return -2;
  hipLaunchKernelGGL(k_synth_seeded, dim3(grid_for(n)), dim3(kBlock), 0, 0, n, first, npools,
                     pool, slot0, eta0, slot, eta_alpha, leader_alpha, eta_proof, leader_proof,
                     eta_out, lead_out, g_ctx.scratch, g_ctx.btab, (const uint64_t*)nullptr);
  return done();
}

// the same at given slots (slot_in, device, n entries): the raw-CBOR bench's
// node configuration, whose raw headers carry k_synth_raw's slots
int ouro_synth_seeded_at(size_t n, uint64_t first, int npools, const uint32_t* pool,
                         const uint64_t* slot_in, const uint8_t* eta0, uint64_t* slot,
                         uint8_t* eta_alpha, uint8_t* leader_alpha, uint8_t* eta_proof,
                         uint8_t* leader_proof, uint8_t* eta_out, uint8_t* lead_out) {
  if (npools <= 0 || !slot_in) return -3;
  if (prepare(n)) return -2;
  hipLaunchKernelGGL(k_synth_seeded, dim3(grid_for(n)), dim3(kBlock), 0, 0, n, first, npools,
                     pool, (uint64_t)0, eta0, slot, eta_alpha, leader_alpha, eta_proof,
                     leader_proof, eta_out, lead_out, g_ctx.scratch, g_ctx.btab, slot_in);
  return done();
}

// raw wire headers for a batch made by ouro_synth_headers (same n, first,
// npools, nodes); offs = 13 uint32 (RawOffsets order), tmpl on the device
int ouro_synth_raw_headers(size_t n, uint64_t first, int npools, const uint32_t* nodes,
                           const uint8_t* tmpl, uint32_t raw_len, const uint32_t* offs,
                           uint64_t slots_per_kes_period, const uint8_t* issuer_vk,
                           const uint8_t* vrf_vk, const uint8_t* eta_proof,
                           const uint8_t* leader_proof, const uint8_t* hot_vk,
                           const uint8_t* sigma, const uint32_t* kes_t, uint8_t* raw) {
  if (npools <= 0 || slots_per_kes_period == 0) return -3;
  RawOffsets o;
  memcpy(&o, offs, sizeof(o));
  if (o.body + o.body_len > raw_len || o.sig + 448 > raw_len) return -3;
  if (prepare(n)) return -2;
  hipLaunchKernelGGL(k_synth_raw, dim3(grid_for(n)), dim3(kBlock), 0, 0, n, first, npools,
                     make_tag("body"), make_tag("kes"), nodes, tmpl, raw_len, o,
                     slots_per_kes_period, issuer_vk, vrf_vk, eta_proof, leader_proof, hot_vk,
                     sigma, kes_t, raw, g_ctx.scratch, g_ctx.btab);
  return done();
}
}
