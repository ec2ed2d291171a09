// shim_common.h -- the error policy of the opt-in link shims (vrf_shim.cpp,
// sodium_shim.cpp).  Their symbols follow libsodium's convention (0 valid,
// -1 invalid) and the Haskell callers read ANY nonzero as "invalid": a device
// or runtime failure returned as is would reject valid headers as
// cryptographically invalid.  By default the shim aborts with the error on
// stderr (a node must not silently fork off on a GPU fault);
// OURO_SHIM_ON_ERROR=invalid selects the libsodium reading (error -> -1).
#pragma once
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "../../include/ouro_verify.h"

namespace {
inline int shim_rc(int rc, const char* what) {
  if (rc == OURO_OK || rc == OURO_INVALID) return rc;
  const char* mode = getenv("OURO_SHIM_ON_ERROR");
  if (mode && strcmp(mode, "invalid") == 0) return OURO_INVALID;
  fprintf(stderr, "libouro shim: %s failed with %d (%s); aborting rather than "
                  "reporting a valid proof as invalid (OURO_SHIM_ON_ERROR=invalid to "
                  "return -1 instead)\n", what, rc, ouro_last_error());
  abort();
}
}  // namespace
