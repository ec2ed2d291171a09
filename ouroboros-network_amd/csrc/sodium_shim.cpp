// sodium_shim.cpp -- OPT-IN link shim (lib/libouro_sodium_shim.so): libsodium
// 1.0.18's crypto_sign_ed25519_verify_detached, the symbol cardano-crypto-class
// Ed25519DSIGN.verifyDSIGN binds ("alias
// crypto_sign_ed25519_verify_detached behind a link option"), served by the
// product's ouro_ed25519_verify (same signature and acceptance rules,
// bit-exact with libsodium: tests/test_gpu_parity.py).  Linked ahead of
// libsodium it takes that one symbol over; every other libsodium symbol (key
// generation, hashing) still resolves to libsodium.  Error policy:
// shim_common.h.  Each call is one GPU round trip (include/ouro_verify.h
// routes per-item callers to libsodium itself; this shim is for callers that
// accept that latency).
#include "shim_common.h"

extern "C" {

__attribute__((visibility("default"))) int crypto_sign_ed25519_verify_detached(
    const unsigned char* sig, const unsigned char* m, unsigned long long mlen,
    const unsigned char* pk) {
  return shim_rc(ouro_ed25519_verify(sig, m, mlen, pk), "crypto_sign_ed25519_verify_detached");
}

}  // extern "C"
