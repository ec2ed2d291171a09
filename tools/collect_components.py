#!/usr/bin/env python3
"""Copy one tools/profile_components.sh run (gpurun_out/c*_<TAG>, merged back
by gpurun) into profiles/<TAG>/components/ and summarise it per kernel:
average launch time (kernel trace), HBM bytes per item (FETCH_SIZE doubled per
the gfx950 correction of MI355X_MICROARCH.md + WRITE_SIZE, separate passes),
SQ shares and VALU instructions per item.  Writes summary.json there and
profiles/pmc_traffic_components.json (read by bench.py to stamp the ed25519 /
vrf / kes legs' traffic, with the source hash the passes measured).

  python tools/collect_components.py r03a [--items 262144]
"""
import argparse
import collections
import csv
import json
import os
import shutil

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNELS = {"k_ed25519_verify": "ed25519", "k_sum6kes_verify": "kes", "k_vrf03_verify": "vrf",
           "k_tpraos_verify": "header"}
# canonical limb-MACs per item (bench.py)
MACS = {"ed25519": 190_912, "kes": 190_912, "vrf": 468_800, "header": 1_319_424}


def per_kernel(path):
    """{kernel: {counter: mean value per dispatch}}"""
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r["Kernel_Name"].split("(")[0].strip()
            if name in KERNELS:
                agg[name][r["Counter_Name"]] += float(r["Counter_Value"])
                disp[name].add(r["Dispatch_Id"])
    return {k: {c: v / max(1, len(disp[k])) for c, v in cs.items()} for k, cs in agg.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("--items", type=int, default=262144)
    args = ap.parse_args()
    g = os.path.join(ROOT, "gpurun_out")
    d = os.path.join(ROOT, "profiles", args.tag, "components")
    os.makedirs(d, exist_ok=True)
    t = args.tag
    copies = {f"cprof_{t}/run_kernel_stats.csv": "kernel_stats.csv",
              f"cprof_{t}.bench.json": "bench_under_rocprof.json",
              f"cpmc_fetch_{t}/run_counter_collection.csv": "pmc_fetch_size.csv",
              f"cpmc_write_{t}/run_counter_collection.csv": "pmc_write_size.csv",
              f"cpmc_sq_{t}/run_counter_collection.csv": "pmc_sq.csv",
              f"cpmc_wait_{t}/run_counter_collection.csv": "pmc_wait.csv"}
    for src, dst in copies.items():
        if os.path.exists(os.path.join(g, src)):
            shutil.copy(os.path.join(g, src), os.path.join(d, dst))
    out = {"tag": t, "pmc_items_per_dispatch": args.items, "kernels": {}}
    with open(os.path.join(d, "kernel_stats.csv")) as f:
        for r in csv.DictReader(f):
            name = r["Name"].split("(")[0].strip()
            if name in KERNELS:
                leg = KERNELS[name]
                ms = float(r["AverageNs"]) / 1e6
                out["kernels"][name] = {"leg": leg, "calls": int(r["Calls"]), "avg_ms": ms,
                                        "items_per_launch": 1 << 20 if leg != "header" else None}
    fetch = per_kernel(os.path.join(d, "pmc_fetch_size.csv"))
    write = per_kernel(os.path.join(d, "pmc_write_size.csv"))
    sq = collections.defaultdict(dict)
    for name in ("pmc_sq.csv", "pmc_wait.csv"):
        p = os.path.join(d, name)
        if os.path.exists(p):
            for k, cs in per_kernel(p).items():
                sq[k].update(cs)
    src = None
    bj = os.path.join(d, "bench_under_rocprof.json")
    if os.path.exists(bj):
        with open(bj) as f:
            lines = [ln for ln in f.read().splitlines() if ln.startswith("{")]
        if lines:
            src = json.loads(lines[-1]).get("source_hash")
    out["source_hash"] = src
    traffic = {"tag": t, "source_hash": src}
    for name, rec in out["kernels"].items():
        fb = fetch.get(name, {}).get("FETCH_SIZE", 0.0) * 1024
        wb = write.get(name, {}).get("WRITE_SIZE", 0.0) * 1024
        hbm = 2 * fb + wb
        rec["hbm_bytes_per_item"] = hbm / args.items
        s = sq.get(name, {})
        if "SQ_WAVE_CYCLES" in s:
            w = s["SQ_WAVE_CYCLES"]
            rec["sq_shares"] = {k: s[k] / w for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
                                                      "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU")
                                if k in s}
        if "SQ_INSTS_VALU" in s:
            # SQ_INSTS_VALU counts wave instructions: x64 lanes / items = per item
            rec["valu_lane_insts_per_item"] = s["SQ_INSTS_VALU"] * 64 / args.items
            rec["vmem_rd_wave_insts_per_item"] = s.get("SQ_INSTS_VMEM_RD", 0) / args.items
        rec["sq"] = dict(s)
        if rec["items_per_launch"]:
            rec["achieved_tmacs"] = MACS[rec["leg"]] * rec["items_per_launch"] / (rec["avg_ms"] * 1e-3) / 1e12
        traffic[rec["leg"]] = {"kernel": name, "hbm_bytes_per_item": rec["hbm_bytes_per_item"]}
    with open(os.path.join(d, "summary.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    with open(os.path.join(ROOT, "profiles", "pmc_traffic_components.json"), "w") as f:
        json.dump(traffic, f, indent=1, sort_keys=True)
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
