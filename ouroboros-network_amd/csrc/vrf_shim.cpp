// vrf_shim.cpp -- OPT-IN link shim (lib/libouro_vrf_shim.so): the
// cardano-crypto-praos symbol names PraosVRF binds with `foreign import ccall`
// (crypto_vrf_ietfdraft03_verify / _proof_to_hash, and the fork's
// version-less crypto_vrf_* aliases of draft-03), served by the product
// library's single-item entry points.  It is a separate library so that
// nothing takes over the fork's symbols unless a maintainer links it on
// purpose, ahead of the fork.
//
// Error convention.  These names follow libsodium's: 0 = valid, -1 = invalid,
// and PraosVRF reads ANY nonzero as an invalid proof.  A device or runtime
// failure (OURO_EDEVICE / OURO_ENODEV / OURO_EINVAL) must therefore not be
// returned as is: it would reject valid headers as cryptographically invalid.
// By default the shim aborts the process with the error on stderr (a node
// must not silently fork off on a GPU fault); OURO_SHIM_ON_ERROR=invalid
// selects the libsodium reading (error -> -1) for callers that accept it.
#include "shim_common.h"

extern "C" {

__attribute__((visibility("default"))) int crypto_vrf_ietfdraft03_verify(
    unsigned char* output, const unsigned char* pk, const unsigned char* proof,
    const unsigned char* m, unsigned long long mlen) {
  return shim_rc(ouro_vrf03_verify(output, pk, proof, m, mlen), "crypto_vrf_ietfdraft03_verify");
}

__attribute__((visibility("default"))) int crypto_vrf_ietfdraft03_proof_to_hash(
    unsigned char* output, const unsigned char* proof) {
  return shim_rc(ouro_vrf03_proof_to_hash(output, proof), "crypto_vrf_ietfdraft03_proof_to_hash");
}

__attribute__((visibility("default"))) int crypto_vrf_verify(unsigned char* output,
                                                             const unsigned char* pk,
                                                             const unsigned char* proof,
                                                             const unsigned char* m,
                                                             unsigned long long mlen) {
  return shim_rc(ouro_vrf03_verify(output, pk, proof, m, mlen), "crypto_vrf_verify");
}

__attribute__((visibility("default"))) int crypto_vrf_proof_to_hash(unsigned char* output,
                                                                    const unsigned char* proof) {
  return shim_rc(ouro_vrf03_proof_to_hash(output, proof), "crypto_vrf_proof_to_hash");
}

}  // extern "C"
