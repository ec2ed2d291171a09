#!/usr/bin/env python3
"""Timing probe of the fused configs[4] launch: a library built with
-DOURO_LAT_STAMPS=1 (tools/build_variant.sh stamps -DOURO_LAT_STAMPS=1), run
with OURO_LAT_STAMPS set, prints header 0's item start/end times
(s_memrealtime, 100 MHz); this runs a 64-header plan R times on that library
(OURO_VERIFY_LIB) and prints, per item, the median start and end in us
relative to the earliest start of each launch.  Items: 0/8 OCERT points/
scalars, 1/9 KES points/scalars, 2/3 U eta/leader, 4/5 V, 6/7 Gamma.

  python tools/lat_stamps.py [--runs R] [--lib PATH]
"""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import os, sys
sys.path.insert(0, %r)
import numpy as np, torch
torch.cuda.init()
import bench
from ouroboros_network_amd.tpraos import HeaderPlan
dev = torch.device("cuda", 0)
t, _ = bench.synth_headers(256, 64, dev)
hb = bench.DeviceHeaders(t, 256, dev).host_sample(64)
plan = HeaderPlan(64, int(hb.body_len.astype(np.int64).sum()))
for r in range(%d):
    out = plan.run(hb)
    torch.cuda.synchronize()
    print("run-end", flush=True)
assert (out[0] == 15).all()
plan.close()
"""


def main():
    runs = int(sys.argv[sys.argv.index("--runs") + 1]) if "--runs" in sys.argv else 20
    lib = sys.argv[sys.argv.index("--lib") + 1] if "--lib" in sys.argv else os.path.join(
        ROOT, "ouroboros-network_amd", "lib", "variants", "stamps.so")
    env = dict(os.environ, OURO_LAT_STAMPS="1", OURO_VERIFY_LIB=os.path.abspath(lib))
    p = subprocess.run([sys.executable, "-c", CHILD % (ROOT, runs)], env=env, capture_output=True,
                       text=True, timeout=600)
    if p.returncode:
        sys.exit(p.stderr[-2000:])
    launches, cur, vst, kst = [], [], {}, {}
    for line in p.stdout.splitlines():
        if line.startswith("kstamp "):
            f = line.split()
            kst.setdefault(len(launches), {})[int(f[1])] = [int(x) for x in f[2:]]
        if line.startswith("vstamp "):
            ts = [int(x) for x in line.split()[1:]]
            tags = ["start", "sha", "elligator", "table", "chain", "combine-add", "encoded"]
            vst.setdefault(len(launches), []).extend(zip(tags, ts))
        if line.startswith("stamp "):
            _, item, what, t0, t1 = line.split()
            cur.append((int(item), what, int(t0), int(t1)))
        elif line == "run-end":
            launches.append(cur)
            cur = []
    rows = {}
    for st in launches[2:]:  # skip warm-up launches
        base = min(t0 for _, _, t0, _ in st)
        for item, what, t0, t1 in st:
            rows.setdefault((item, what), []).append(((t0 - base) / 100.0, (t1 - base) / 100.0))
    print(f"{len(launches) - 2} launches; median start / end (us) per item of header 0")
    for (item, what), v in sorted(rows.items(), key=lambda kv: np.median([e for _, e in kv[1]])):
        a = np.array(v)
        print(f"item {item:2d} {what:5s} start {np.median(a[:, 0]):7.1f}  end {np.median(a[:, 1]):7.1f}")
    # phases of header 0's eta V item (vstamp), relative to its start
    phases = {}
    for k, st in vst.items():
        if k < 2:
            continue
        t0 = dict(st).get("start")
        for tag, t in st:
            if t0 is not None:
                phases.setdefault(tag, []).append((t - t0) / 100.0)
    if phases:
        print("eta V item phases (us after its start):",
              ", ".join(f"{k} {np.median(v):.1f}" for k, v in phases.items()))
    # header 0's KES items (kstamp): phases relative to the earlier start of the two
    tags = ["start", "walk", "prep", "arrive", "chain", "sha", "reduce", "lattice"]
    kph = {}
    for k, st in kst.items():
        if k < 2 or 1 not in st or 9 not in st:
            continue
        t0 = min(st[1][0], st[9][0])
        for item in (1, 9):
            for tag, t in zip(tags, st[item]):
                if t:
                    kph.setdefault((item, tag), []).append((t - t0) / 100.0)
    for item, name in ((1, "KES points"), (9, "KES scalars")):
        row = [f"{tag} {np.median(kph[(item, tag)]):.1f}" for tag in tags if (item, tag) in kph]
        if row:
            print(f"{name} item phases (us):", ", ".join(row))


if __name__ == "__main__":
    main()
