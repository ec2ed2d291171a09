#!/usr/bin/env python3
"""A/B of the configs[4] latency path's launch shape in ONE process: a
64-header hipGraph plan per value of a launch-shape variable read when the
plan's graph is captured (OURO_LAT_BLOCK: latency-mode workgroup size;
OURO_LAT_QUAD: cores on lane quads or one lane each), interleaved rounds,
p50 wall latency.

  python tools/ab_latency.py [--iters N] [--rounds R] [--var NAME --values a,b]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=500)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--var", default="OURO_LAT_BLOCK")
    ap.add_argument("--values", default="256,128,64")
    ap.add_argument("--combos", default=None,
                    help="instead of --var/--values: ';'-separated plans, each a '+'-joined "
                         "list of VAR=value set while that plan is created")
    ap.add_argument("--nonce", action="store_true",
                    help="(--libs) request the eta nonce output as a node would")
    ap.add_argument("--node", action="store_true",
                    help="the node configuration: claimed outputs, VRF inputs from (slot, eta0) "
                         "by mkSeed on the device (bench.synth_node_config)")
    ap.add_argument("--libs", nargs="*", default=None,
                    help="A/B build variants of libouro_verify.so instead of an env variable")
    args = ap.parse_args()
    import torch

    import bench
    from ouroboros_network_amd import _native
    from ouroboros_network_amd.tpraos import HeaderPlan

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    if args.node:
        t, _, pool = bench.synth_headers(args.batch, 1024, dev, keep_pool=True)
        bench.synth_node_config(t, args.batch, 1024, pool, bytes(range(7, 39)), dev)
        hb = bench.DeviceHeaders(t, args.batch, dev).host_sample(args.batch)
    else:
        t, _ = bench.synth_headers(4096, 1024, dev)
        hdr = bench.DeviceHeaders(t, 4096, dev)
        hb = hdr.host_sample(args.batch)
    body = int(hb.body_len.astype(np.int64).sum())
    plans, ref = {}, None
    if args.libs:
        return lib_variants(args, hb, body)
    if args.combos:
        values = args.combos.split(";")
        for combo in values:
            kv = [c.split("=", 1) for c in combo.split("+")]
            for k, v in kv:
                os.environ[k] = v
            _native.reload_knobs()  # the library reads its switches once (knobs.h)
            plans[combo] = HeaderPlan(args.batch, body)
            for k, _ in kv:
                del os.environ[k]
    else:
        values = args.values.split(",")
        for v in values:
            os.environ[args.var] = v
            _native.reload_knobs()
            plans[v] = HeaderPlan(args.batch, body)
    lat = {k: [] for k in plans}
    outs = {}
    for r in range(args.rounds + 1):
        for k, p in plans.items():
            out = p.run(hb)
            outs[k] = out
            for _ in range(args.iters):
                t0 = time.perf_counter()
                p.run(hb, out)
                if r:
                    lat[k].append(time.perf_counter() - t0)
    first = outs[values[0]]
    res = {}
    for k, v in lat.items():
        a = np.array(v) * 1e3
        same = all((outs[k][i] == first[i]).all() for i in range(3))
        res[k if args.combos else f"{args.var}={k}"] = {"p50_ms": round(float(np.percentile(a, 50)), 4),
                            "p99_ms": round(float(np.percentile(a, 99)), 4),
                            "all_valid": bool(((outs[k][0] & 15) == 15).all()), "same_as_first": same}
    for p in plans.values():
        p.close()
    print(json.dumps(res, indent=1))


def lib_variants(args, hb, body):
    """One 64-header plan per library build (same batch), interleaved rounds."""
    import ctypes

    from ouroboros_network_amd import _native

    P = ctypes.c_void_p
    plans = {}
    for path in args.libs:
        lib = ctypes.CDLL(os.path.abspath(path))
        lib.ouro_tpraos_plan_create.restype = P
        lib.ouro_tpraos_plan_create.argtypes = [ctypes.c_size_t, ctypes.c_size_t]
        lib.ouro_tpraos_plan_run.restype = ctypes.c_int
        lib.ouro_tpraos_plan_run.argtypes = [P, ctypes.POINTER(_native.TPraosBatch), P, P, P]
        plan = lib.ouro_tpraos_plan_create(args.batch, body)
        assert plan, path
        plans[os.path.basename(path)] = (lib, plan)
    n = len(hb)
    en = np.zeros((n, 32), np.uint8)
    s = hb.c_struct(eta_nonce=en) if args.nonce else hb.c_struct()
    outs = {k: (np.zeros(n, np.uint8), np.zeros((n, 64), np.uint8), np.zeros((n, 64), np.uint8))
            for k in plans}
    ptr = lambda a: a.ctypes.data_as(P)  # noqa: E731
    lat = {k: [] for k in plans}
    for r in range(args.rounds + 1):
        for k, (lib, plan) in plans.items():
            o = outs[k]
            for _ in range(args.iters):
                t0 = time.perf_counter()
                rc = lib.ouro_tpraos_plan_run(plan, ctypes.byref(s), ptr(o[0]), ptr(o[1]), ptr(o[2]))
                if r:
                    lat[k].append(time.perf_counter() - t0)
                assert rc == 0, (k, rc)
    first = outs[next(iter(plans))]
    res = {}
    for k, v in lat.items():
        a = np.array(v) * 1e3
        same = all((outs[k][i] == first[i]).all() for i in range(3))
        res[k] = {"p50_ms": round(float(np.percentile(a, 50)), 4),
                  "p99_ms": round(float(np.percentile(a, 99)), 4),
                  "all_valid": bool(((outs[k][0] & 15) == 15).all()), "same_as_first": same}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
