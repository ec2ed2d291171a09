// hostpath_asan_shim.cpp -- TEST-ONLY: the product's host path (host_path.hip
// + task_pool.cpp) in a library of its own, built under AddressSanitizer +
// UBSan (Makefile lib/libouro_hostpath_asan.so) and driven by
// tests/test_sanitizers.py; the product library does not contain this file.
#include "host_path.h"

extern "C" {
int hp_ed_batch(size_t n, const uint8_t* pk, const uint8_t* sig, const uint8_t* msg,
                const uint64_t* off, const uint32_t* len, uint8_t* verdict, uint32_t byron) {
  return ouro_host::ed_batch(n, pk, sig, msg, off, len, verdict, byron);
}
int hp_vrf_batch(size_t n, const uint8_t* pk, const uint8_t* proof, const uint8_t* alpha,
                 const uint64_t* off, const uint32_t* len, uint8_t* beta, uint8_t* verdict,
                 uint32_t flags) {
  return ouro_host::vrf_batch(n, pk, proof, alpha, off, len, beta, verdict, flags);
}
int hp_kes_batch(size_t n, const uint8_t* vk, const uint32_t* t, const uint8_t* msg,
                 const uint64_t* off, const uint32_t* len, const uint8_t* sig, uint8_t* verdict) {
  return ouro_host::kes_batch(n, vk, t, msg, off, len, sig, verdict);
}
int hp_hdr_batch(const ouro_tpraos_batch* b, uint8_t* verdict, uint8_t* beta_eta,
                 uint8_t* beta_leader) {
  return ouro_host::hdr_batch(b, verdict, beta_eta, beta_leader);
}
}
