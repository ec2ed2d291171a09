#!/usr/bin/env python3
"""Where a configs[4] window's wall time goes, per plan variant: bench.py's
_plan_phases (submit = copy into the pinned block + graph launch, wait, the
graph's GPU time from events) on a 64-header window in the node
configuration, once per value of an environment variable read when the plan
is captured (default OURO_PLAN_STAGE 0 / 2).

  python tools/lat_phases.py [--iters N] [--var NAME --values a,b]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=2000)
    ap.add_argument("--var", default="OURO_PLAN_STAGE")
    ap.add_argument("--values", default="0,2")
    args = ap.parse_args()
    import torch

    import bench
    from ouroboros_network_amd import _native

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    nt, _, npool = bench.synth_headers(64, 1024, dev, keep_pool=True)
    bench.synth_node_config(nt, 64, 1024, npool, bytes(range(7, 39)), dev)
    nb = bench.DeviceHeaders(nt, 64, dev).host_sample(64)
    out = {}
    for v in args.values.split(","):
        os.environ[args.var] = v
        _native.reload_knobs()  # the library reads its switches once (knobs.h)
        out[f"{args.var}={v}"] = bench._plan_phases(nb, args.iters, nonce=True)
        del os.environ[args.var]
        _native.reload_knobs()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
