#!/usr/bin/env python3
"""HBM bytes per item of each kernel for each variant of a
tools/pmc_variants.sh run: 2 x FETCH_SIZE (gfx950 correction,
MI355X_MICROARCH.md) + WRITE_SIZE, per dispatch, divided by the items.

  python tools/summarize_vpmc.py TAG [--items 262144]
"""
import argparse
import collections
import csv
import glob
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNELS = ("k_tpraos_verify", "k_ed25519_verify", "k_sum6kes_verify", "k_vrf03_verify")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("--items", type=int, default=262144)
    args = ap.parse_args()
    out = collections.defaultdict(dict)
    for d in sorted(glob.glob(os.path.join(ROOT, "gpurun_out", f"vpmc_{args.tag}_*"))):
        base = os.path.basename(d)[len(f"vpmc_{args.tag}_"):]
        name, ctr = base.rsplit("_", 2)[0], "_".join(base.rsplit("_", 2)[1:])
        agg, disp = collections.defaultdict(float), collections.defaultdict(set)
        for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(p) as f:
                for r in csv.DictReader(f):
                    k = r["Kernel_Name"].split("(")[0].strip()
                    if k in KERNELS:
                        agg[k] += float(r["Counter_Value"])
                        disp[k].add(r["Dispatch_Id"])
        for k in agg:
            per = agg[k] * 1024 / len(disp[k]) / args.items
            out[name].setdefault(k, {})[ctr] = per
    res = {}
    for name, ks in out.items():
        res[name] = {k: round(2 * v.get("FETCH_SIZE", 0) + v.get("WRITE_SIZE", 0))
                     for k, v in ks.items()}
    print(json.dumps(res, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
