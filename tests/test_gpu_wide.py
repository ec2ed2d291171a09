"""The wave-wide arithmetic of the latency mode (csrc/wide.h) against the
lane-local routines it replaces, on the device: conversions, products,
squaring chains, z^(2^252-3), doubling, addition/subtraction, [s]P against
double-and-add, the identity, and the latency mode's [s]H item (wide_vrf.h).  One wave per case (random + edge field
elements: p - 1, 0); csrc/wide_test.hip is a test-only library."""
import ctypes
import os

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "ouroboros-network_amd", "lib", "libouro_wide_test.so")
NAMES = ["convert", "mul", "sq_chain", "pow22523", "dbl", "add_sub", "scalarmult", "identity",
         "vrf_sh_H", "vrf_sh_V"]


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [1, 0x5eed])
def test_wide_arithmetic_matches_lane_routines(gpu_lib, seed):
    lib = ctypes.CDLL(LIB)
    lib.ouro_wide_selftest.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]
    waves = 512
    out = np.zeros(waves * len(NAMES), dtype=np.int32)
    dbg = np.zeros(24, dtype=np.int32)
    assert lib.ouro_wide_selftest(waves, seed, out.ctypes.data, dbg.ctypes.data) == 0
    res = out.reshape(waves, len(NAMES))
    bad = {NAMES[t]: int((res[:, t] != 1).sum()) for t in range(len(NAMES))}
    assert all(v == 0 for v in bad.values()), (bad, dbg.tolist())
