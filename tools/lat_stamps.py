#!/usr/bin/env python3
"""Timing probe of the fused configs[4] launch (split form).

A library built with -DOURO_LAT_STAMPS=1 (tools/build_lat_variant.sh stamps
-DOURO_LAT_STAMPS=1) records, without printf, s_memrealtime (100 MHz) at tagged
points of header 0's items into device memory (wide_cores.h lstamp); this
runs a 64-header plan R times on that library (OURO_VERIFY_LIB), reads the
stamps after each launch (ouro_debug_lat_stamps) and prints, per item and
tag, the median time in us after the earliest start of the launch.
Items: 0/8/10 OCERT points/scalars/doubling, 1/9/11 KES, 2/3 U eta/leader,
4/5 V, 6/7 Gamma, 12/13 V2, 14/15 V3 (OURO_LAT_V3 builds).  Tags: 0 start, 1 own part done, 2/3 chain X/Y
done, 4..7 VRF combination (start, adds, inverted, encoded), 8 end, 9/10/11
tail (start, challenges, end), 12..18 V/V2 phases (hash, exp start, exp end,
H, H128, table, chain).

  python tools/lat_stamps.py [--runs R] [--lib PATH]
"""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ITEMS = {0: "OCERT P", 8: "OCERT S", 10: "OCERT D", 1: "KES P", 9: "KES S", 11: "KES D",
         2: "U eta", 3: "U leader", 4: "V eta", 5: "V leader", 6: "Gamma eta",
         7: "Gamma leader", 12: "V2 eta", 13: "V2 leader", 14: "V3 eta", 15: "V3 leader"}
TAGS = {0: "start", 1: "part", 2: "chainX", 3: "chainY", 4: "comb0", 5: "combAdd",
        6: "combInv", 7: "combEnc", 8: "end", 9: "tail0", 10: "tailChal", 11: "tailEnd",
        12: "hash", 13: "exp0", 14: "exp1", 15: "H", 16: "H128", 17: "table", 18: "chain"}

CHILD = r"""
import ctypes, json, os, sys
sys.path.insert(0, %r)
import numpy as np, torch
torch.cuda.init()
import bench
from ouroboros_network_amd.tpraos import HeaderPlan
from ouroboros_network_amd import _native
dev = torch.device("cuda", 0)
t, _ = bench.synth_headers(256, 64, dev)
hb = bench.DeviceHeaders(t, 256, dev).host_sample(64)
plan = HeaderPlan(64, int(hb.body_len.astype(np.int64).sum()))
lib = _native.load()
buf = (ctypes.c_ulonglong * (16 * 24))()
rows = []
for r in range(%d):
    ctypes.memset(buf, 0, ctypes.sizeof(buf))
    out = plan.run(hb)
    torch.cuda.synchronize()
    assert lib.ouro_debug_lat_stamps(buf) == 16 * 24
    rows.append(list(buf))
assert os.environ.get("OURO_LAT_SKIP") or ((out[0] & 15) == 15).all()
plan.close()
print(json.dumps(rows))
"""


def main():
    runs = int(sys.argv[sys.argv.index("--runs") + 1]) if "--runs" in sys.argv else 30
    lib = sys.argv[sys.argv.index("--lib") + 1] if "--lib" in sys.argv else os.path.join(
        ROOT, "ouroboros-network_amd", "lib", "variants", "stamps.so")
    env = dict(os.environ, OURO_LAT_STAMPS="1", OURO_VERIFY_LIB=os.path.abspath(lib))
    p = subprocess.run([sys.executable, "-c", CHILD % (ROOT, runs)], env=env, capture_output=True,
                       text=True, timeout=600)
    if p.returncode:
        sys.exit(p.stderr[-2000:])
    import json
    rows = json.loads(p.stdout.strip().splitlines()[-1])[2:]  # skip warm-up launches
    a = np.array(rows, dtype=np.float64).reshape(len(rows), 16, 24)
    base = np.where(a[:, :, 0] > 0, a[:, :, 0], np.inf).min(axis=1)
    rel = (a - base[:, None, None]) / 100.0
    print(f"{len(rows)} launches; header 0, median us after the launch's first item start")
    ents = []
    for item, name in ITEMS.items():
        for tag, tname in TAGS.items():
            v = rel[:, item, tag][a[:, item, tag] > 0]
            if len(v) >= len(rows) // 2:
                ents.append((float(np.median(v)), name, tname, len(v)))
    for t, name, tname, n in sorted(ents):
        print(f"{t:8.1f}  {name:13s} {tname:9s} (n={n})")


if __name__ == "__main__":
    main()
