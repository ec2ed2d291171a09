#!/usr/bin/env python3
"""A/B timing of build variants of the verifier in ONE process, interleaved
rounds (cdna_hip_programming.md §5.4 rule 24).  Each variant is a separately
built libouro_verify*.so; all run the header kernel on the same device-resident
synthetic batch and must produce identical verdicts/outputs.

  python tools/ab_variants.py lib1.so lib2.so ... [--headers N] [--rounds R]
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--headers", type=int, default=1 << 20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--kes", action="store_true", help="also time the Sum6KES batch kernel")
    args = ap.parse_args()
    import torch

    import bench
    from ouroboros_network_amd import _native

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    t, _ = bench.synth_headers(args.headers, 1024, dev)
    s = _native.TPraosBatch()
    s.n = args.headers
    for k, v in t.items():
        setattr(s, k, v.data_ptr())
    libs = []
    for path in args.libs:
        lib = ctypes.CDLL(os.path.abspath(path))
        fn = lib.ouro_tpraos_verify_batch_device
        fn.restype = ctypes.c_int
        fn.argtypes = [ctypes.c_void_p, ctypes.POINTER(_native.TPraosBatch), ctypes.c_void_p,
                       ctypes.c_void_p, ctypes.c_void_p]
        libs.append((path, fn))
    n = args.headers
    outs = {p: (torch.zeros(n, dtype=torch.uint8, device=dev),
                torch.zeros(n * 64, dtype=torch.uint8, device=dev),
                torch.zeros(n * 64, dtype=torch.uint8, device=dev)) for p, _ in libs}
    st = torch.cuda.current_stream()
    times = {p: [] for p, _ in libs}
    for r in range(args.rounds + 1):
        for p, fn in libs:
            v, be, bl = outs[p]
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            rc = fn(ctypes.c_void_p(st.cuda_stream), ctypes.byref(s), v.data_ptr(), be.data_ptr(),
                    bl.data_ptr())
            e1.record(st)
            torch.cuda.synchronize()
            assert rc == 0, (p, rc)
            if r > 0:
                times[p].append(e0.elapsed_time(e1))
    kes_times = {p: [] for p, _ in libs}
    if args.kes:
        kv = {p: torch.zeros(n, dtype=torch.uint8, device=dev) for p, _ in libs}
        kfns = []
        for path, _ in libs:
            lib = ctypes.CDLL(os.path.abspath(path))
            f = lib.ouro_sum6kes_verify_batch_device
            f.restype = ctypes.c_int
            kfns.append((path, f))
        for r in range(args.rounds + 1):
            for p, f in kfns:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                rc = f(ctypes.c_void_p(st.cuda_stream), ctypes.c_size_t(n),
                       *[ctypes.c_void_p(t[k].data_ptr()) for k in
                         ("hot_vk", "kes_t", "body", "body_off", "body_len", "kes_sig")],
                       ctypes.c_void_p(kv[p].data_ptr()))
                e1.record(st)
                torch.cuda.synchronize()
                assert rc == 0, (p, rc)
                if r > 0:
                    kes_times[p].append(e0.elapsed_time(e1))
    ref = outs[libs[0][0]]
    res = {}
    for p, _ in libs:
        v, be, bl = outs[p]
        same = bool(torch.equal(v, ref[0]) and torch.equal(be, ref[1]) and torch.equal(bl, ref[2]))
        res[os.path.basename(p)] = {"median_ms": float(np.median(times[p])), "min_ms": float(np.min(times[p])),
                                    "headers_per_s": n / (np.median(times[p]) * 1e-3),
                                    "all_valid": bool((v == 15).all().item()), "same_as_first": same}
        if args.kes:
            res[os.path.basename(p)]["kes_median_ms"] = float(np.median(kes_times[p]))
            res[os.path.basename(p)]["kes_all_valid"] = bool((kv[p] == 1).all().item())
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
