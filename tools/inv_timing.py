"""Timing probe of the wave inversion (csrc/wide_inv.h) on the GPU: us per
inversion with and without the early exit, one wave per SIMD, and the cost of
one inversion's 18 batches of divstep matrices alone (lib/libouro_wide_test.so
ouro_wide_invert_us, ouro_wide_divsteps_us).
    python tools/inv_timing.py [waves] [iters]"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    waves = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    lib = ctypes.CDLL(os.path.join(ROOT, "ouroboros-network_amd", "lib", "libouro_wide_test.so"))
    lib.ouro_wide_invert_us.restype = ctypes.c_double
    lib.ouro_wide_invert_us.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_uint64]
    res = {}
    for rep in range(3):
        for early in (1, 0):
            us = lib.ouro_wide_invert_us(waves, iters, early, 1234 + rep)
            res.setdefault("early" if early else "all_25_batches", []).append(round(us, 3))
    lib.ouro_wide_divsteps_us.restype = ctypes.c_double
    lib.ouro_wide_divsteps_us.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                          ctypes.c_uint64]
    ds = {}
    for rep in range(3):
        for cap10 in (1, 0):
            us = lib.ouro_wide_divsteps_us(waves, iters, cap10, 99 + rep)
            ds.setdefault("cap10" if cap10 else "cap30", []).append(round(us, 3))
    print(json.dumps({"waves": waves, "iters": iters, "us_per_inversion": res,
                      "us_per_18_divstep_matrices": ds}))


if __name__ == "__main__":
    main()
