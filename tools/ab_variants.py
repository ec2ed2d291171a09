#!/usr/bin/env python3
"""A/B timing of build variants of the verifier in ONE process, interleaved
rounds (cdna_hip_programming.md §5.4 rule 24).  Each variant is a separately
built libouro_verify*.so; all run the same device-resident synthetic batches
and must produce identical verdicts/outputs.

Legs (--legs, default hdr): hdr = the header kernel (configs[3]), ed = the
standalone Ed25519 kernel (32-byte messages), kes = Sum6KES over the headers'
bodies, vrf = the standalone VRF kernel over the headers' eta proofs.

  python tools/ab_variants.py lib1.so lib2.so ... [--headers N] [--rounds R] [--legs hdr,ed,kes,vrf]
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
    ap.add_argument("--legs", default="hdr")
    ap.add_argument("--kes", action="store_true", help="(old spelling of --legs hdr,kes)")
    args = ap.parse_args()
    legs = args.legs.split(",") + (["kes"] if args.kes else [])
    import torch

    import bench
    from ouroboros_network_amd import _native

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    n = args.headers
    t, _ = bench.synth_headers(n, 1024, dev)
    s = _native.TPraosBatch()
    s.n = n
    for k, v in t.items():
        setattr(s, k, v.data_ptr())
    u8 = dict(dtype=torch.uint8, device=dev)
    V = ctypes.c_void_p
    if "ed" in legs:
        syn = ctypes.CDLL(bench.SYNTH_SO)
        epk, esig, emsg = torch.empty(n * 32, **u8), torch.empty(n * 64, **u8), torch.empty(n * 32, **u8)
        assert syn.ouro_synth_ed25519(ctypes.c_size_t(n), ctypes.c_uint64(0), V(epk.data_ptr()),
                                      V(esig.data_ptr()), V(emsg.data_ptr())) == 0
        eoff = torch.arange(n, dtype=torch.int64, device=dev) * 32
        elen = torch.full((n,), 32, dtype=torch.int32, device=dev)
    aoff = torch.arange(n, dtype=torch.int64, device=dev) * 32
    alen = torch.full((n,), 32, dtype=torch.int32, device=dev)
    st = torch.cuda.current_stream()
    S = lambda: V(st.cuda_stream)  # noqa: E731

    def leg_call(lib, leg, out):
        if leg == "hdr":
            f = lib.ouro_tpraos_verify_batch_device
            f.argtypes = [V, ctypes.POINTER(_native.TPraosBatch), V, V, V]
            return f(S(), ctypes.byref(s), V(out[0].data_ptr()), V(out[1].data_ptr()),
                     V(out[2].data_ptr()))
        if leg == "ed":
            return lib.ouro_ed25519_verify_batch_device(
                S(), ctypes.c_size_t(n), *[V(x.data_ptr()) for x in (epk, esig, emsg, eoff, elen)],
                V(out[0].data_ptr()))
        if leg == "kes":
            return lib.ouro_sum6kes_verify_batch_device(
                S(), ctypes.c_size_t(n),
                *[V(t[k].data_ptr()) for k in ("hot_vk", "kes_t", "body", "body_off", "body_len",
                                               "kes_sig")], V(out[0].data_ptr()))
        if leg == "vrf":
            return lib.ouro_vrf03_verify_batch_device(
                S(), ctypes.c_size_t(n),
                *[V(x.data_ptr()) for x in (t["vrf_vk"], t["eta_proof"], t["eta_alpha"], aoff, alen)],
                V(out[1].data_ptr()), V(out[0].data_ptr()))
        raise ValueError(leg)

    libs = [(p, ctypes.CDLL(os.path.abspath(p))) for p in args.libs]
    res = {os.path.basename(p): {} for p, _ in libs}
    for leg in legs:
        outs = {p: (torch.zeros(n, **u8), torch.zeros(n * 64, **u8), torch.zeros(n * 64, **u8))
                for p, _ in libs}
        times = {p: [] for p, _ in libs}
        for r in range(args.rounds + 1):
            for p, lib in libs:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                rc = leg_call(lib, leg, outs[p])
                e1.record(st)
                torch.cuda.synchronize()
                assert rc == 0, (p, leg, rc)
                if r > 0:
                    times[p].append(e0.elapsed_time(e1))
        ref = outs[libs[0][0]]
        want = 15 if leg == "hdr" else 1
        for p, _ in libs:
            o = outs[p]
            same = all(torch.equal(a, b) for a, b in zip(o, ref))
            res[os.path.basename(p)][leg] = {
                "median_ms": round(float(np.median(times[p])), 4),
                "min_ms": round(float(np.min(times[p])), 4),
                "items_per_s": round(n / (np.median(times[p]) * 1e-3), 1),
                "all_valid": bool((o[0] == want).all().item()), "same_as_first": same}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
