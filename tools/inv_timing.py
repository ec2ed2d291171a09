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
    inv_modes = {0: "all_25_batches_cap30", 1: "early_cap30", 2: "early_cap10",
                 3: "early_cap10_branchfree", 4: "early_cap30_branchfree",
                 5: "early_cap30_valu", 6: "early_cap10_valu"}
    ds_modes = {0: "cap30", 1: "cap10", 2: "cap10_branchfree", 3: "cap30_branchfree",
                4: "cap30_valu", 5: "cap10_valu", 6: "cap30_branchfree_spec"}
    res, ds = {}, {}
    lib.ouro_wide_divsteps_us.restype = ctypes.c_double
    lib.ouro_wide_divsteps_us.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                          ctypes.c_uint64]
    for rep in range(3):
        for m, name in inv_modes.items():
            res.setdefault(name, []).append(round(lib.ouro_wide_invert_us(waves, iters, m,
                                                                          1234 + rep), 3))
        for m, name in ds_modes.items():
            ds.setdefault(name, []).append(round(lib.ouro_wide_divsteps_us(waves, iters, m,
                                                                           99 + rep), 3))
    print(json.dumps({"waves": waves, "iters": iters, "us_per_inversion": res,
                      "us_per_18_divstep_matrices": ds}))


if __name__ == "__main__":
    main()
