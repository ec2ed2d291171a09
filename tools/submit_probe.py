"""Where ouro_tpraos_plan_submit's rare slow calls come from (VERDICT r05
item 1): per-window submit / wait times at the C ABI over many windows, in
passes that differ in one thing each, with the spikes' window indices so a
period (a runtime pool that wraps) shows as equal gaps.

  python tools/submit_probe.py [--iters 20000] [--out FILE]

Passes (each its own plan, node configuration, 64 headers):
  plain   -- the product's form (no events)
  timed   -- OURO_PLAN_TIMING: two events recorded around each window's
             launches (the bench's phases pass)
  synced  -- plain, plus a hipStreamSynchronize-equivalent after each wait
             (the plan's stream drained: the kernel's end-of-pipe seen)
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def run_pass(nb, iters, env, drain=False):
    from ouroboros_network_amd import _native
    from ouroboros_network_amd.tpraos import HeaderPlan

    saved = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    getattr(_native, "reload_knobs", lambda: None)()
    body_bytes = int(nb.body_len.astype(np.int64).sum())
    plan = HeaderPlan(len(nb), body_bytes)
    try:
        out = plan.run(nb, nonce=True)
        s = nb.c_struct(out[3])
        P = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
        lib = plan._lib
        sub, wait = lib.ouro_tpraos_plan_submit, lib.ouro_tpraos_plan_wait
        drain_fn = getattr(lib, "ouro_debug_plan_drain", None)
        for _ in range(100):
            assert sub(plan._p, ctypes.byref(s)) == 0
            assert wait(plan._p, P(out[0]), P(out[1]), P(out[2])) == 0
        ph = np.empty((iters, 4))
        gms = ctypes.c_float()
        pc = time.perf_counter
        for k in range(iters):
            t0 = pc()
            rc = sub(plan._p, ctypes.byref(s))
            t1 = pc()
            rc |= wait(plan._p, P(out[0]), P(out[1]), P(out[2]))
            t2 = pc()
            if drain and drain_fn is not None:
                drain_fn(plan._p)
            lib.ouro_debug_plan_timing(plan._p, ctypes.byref(gms), None, None)
            ph[k] = (t1 - t0, t2 - t1, pc(), gms.value * 1e-3)
            assert rc == 0
    finally:
        plan.close()
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
        getattr(_native, "reload_knobs", lambda: None)()
    us = lambda a, q: round(float(np.percentile(a, q)) * 1e6, 1)  # noqa: E731
    st = lambda a: {"p50": us(a, 50), "p99": us(a, 99), "p99_9": us(a, 99.9),  # noqa: E731
                    "max": us(a, 100)}
    wall = ph[:, 0] + ph[:, 1]
    slow_sub = np.nonzero(ph[:, 0] > 40e-6)[0]
    slow_wall = np.nonzero(wall > np.percentile(wall, 99.9))[0]
    return {"submit_us": st(ph[:, 0]), "wait_us": st(ph[:, 1]), "wall_us": st(wall),
            "gpu_us": st(ph[:, 3]) if (ph[:, 3] > 0).all() else None,
            "n_submit_over_40us": int(slow_sub.size),
            "submit_over_40us_at": slow_sub[:40].tolist(),
            "gaps_between": np.diff(slow_sub)[:40].tolist(),
            "their_submit_us": [round(ph[i, 0] * 1e6, 1) for i in slow_sub[:40]],
            "slowest_walls_at": slow_wall[:20].tolist(),
            "slowest_walls": [{"submit": round(ph[i, 0] * 1e6, 1), "wait": round(ph[i, 1] * 1e6, 1)}
                              for i in slow_wall[:20]],
            "elapsed_s_at_slow_submits": [round(ph[i, 2] - ph[0, 2], 4) for i in slow_sub[:40]]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20000)
    ap.add_argument("--passes", default="plain,timed,synced")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import torch

    import bench

    torch.cuda.init()
    dev = torch.device("cuda:0")
    t, _, pool = bench.synth_headers(64, 64, dev, keep_pool=True)
    t = bench.synth_node_config(t, 64, 64, pool, bytes(range(32)), dev)
    nb = bench.DeviceHeaders(t, 64, dev).host_sample(64)
    res = {"iters": a.iters}
    forms = {"plain": ({}, False), "timed": ({"OURO_PLAN_TIMING": "1"}, False),
             "synced": ({}, True)}
    for name in a.passes.split(","):
        env, drain = forms[name]
        res[name] = run_pass(nb, a.iters, env, drain)
        print(name, json.dumps(res[name]["submit_us"]), json.dumps(res[name]["wall_us"]),
              res[name]["n_submit_over_40us"], flush=True)
    txt = json.dumps(res, indent=1)
    if a.out:
        with open(a.out, "w") as f:
            f.write(txt)
    print(txt)


if __name__ == "__main__":
    main()
