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
    args = ap.parse_args()
    import torch

    import bench
    from ouroboros_network_amd.tpraos import HeaderPlan

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    t, _ = bench.synth_headers(4096, 1024, dev)
    hdr = bench.DeviceHeaders(t, 4096, dev)
    hb = hdr.host_sample(args.batch)
    body = int(hb.body_len.astype(np.int64).sum())
    plans, ref = {}, None
    values = args.values.split(",")
    for v in values:
        os.environ[args.var] = v
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
        res[f"{args.var}={k}"] = {"p50_ms": round(float(np.percentile(a, 50)), 4),
                            "p99_ms": round(float(np.percentile(a, 99)), 4),
                            "all_valid": bool((outs[k][0] == 15).all()), "same_as_first": same}
    for p in plans.values():
        p.close()
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
