#!/usr/bin/env python3
"""Summarise a round's rocprofv3 output (profiles/<round>/) into summary.json
and profiles/pmc_traffic.json (read by bench.py for roofline.traffic).

HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE (KiB,
memory-side L2 request counters) from separate --pmc passes; on gfx950
FETCH_SIZE reads half of a wide streaming read, so it is doubled (the scratch
tables here are read with 16-B-per-lane loads); WRITE_SIZE is taken as is.
The PMC passes ran bench.py --headers H --steps 1 --warmup 0, i.e. exactly one
k_tpraos_verify dispatch over H headers.

  python tools/summarize_profile.py r01 [--pmc-headers 262144]
"""
import argparse
import collections
import csv
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def counters(path, kernel="k_tpraos_verify"):
    agg = collections.defaultdict(float)
    n = collections.Counter()
    with open(path) as f:
        for r in csv.DictReader(f):
            if kernel in r["Kernel_Name"]:
                agg[r["Counter_Name"]] += float(r["Counter_Value"])
                n[r["Dispatch_Id"]] += 1
    return dict(agg), len(n)


def clock_ghz(path, kernel="k_tpraos_verify"):
    """GRBM_GUI_ACTIVE / 8 (rocprofv3 sums the 8 XCDs) / dispatch wall time:
    the clock the kernel ran at (MI355X_MICROARCH.md "DVFS give-back"; within
    3 % of the in-kernel clock for dispatches of 10 ms or more)."""
    with open(path) as f:
        for r in csv.DictReader(f):
            if kernel in r["Kernel_Name"] and r["Counter_Name"] == "GRBM_GUI_ACTIVE":
                ns = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
                return float(r["Counter_Value"]) / 8 / ns
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("round")
    ap.add_argument("--pmc-headers", type=int, default=262144)
    args = ap.parse_args()
    d = os.path.join(ROOT, "profiles", args.round)
    out = {"round": args.round, "pmc_headers_per_dispatch": args.pmc_headers}
    with open(os.path.join(d, "kernel_stats.csv")) as f:
        for r in csv.DictReader(f):
            name = r["Name"].split("(")[0]
            out.setdefault("kernels", {})[name] = {
                "calls": int(r["Calls"]), "avg_ms": float(r["AverageNs"]) / 1e6,
                "pct": float(r["Percentage"])}
    fetch, nd = counters(os.path.join(d, "pmc_fetch_size.csv"))
    write, _ = counters(os.path.join(d, "pmc_write_size.csv"))
    fetch_b = fetch.get("FETCH_SIZE", 0.0) * 1024 / max(nd, 1)
    write_b = write.get("WRITE_SIZE", 0.0) * 1024 / max(nd, 1)
    hbm = 2 * fetch_b + write_b
    out["hbm"] = {"fetch_size_bytes_raw": fetch_b, "write_size_bytes": write_b,
                  "hbm_bytes_per_dispatch": hbm, "per_header": hbm / args.pmc_headers,
                  "note": "FETCH_SIZE doubled per the gfx950 correction"}
    for name in ("pmc_sq.csv", "pmc_wait.csv"):
        p = os.path.join(d, name)
        if os.path.exists(p):
            c, _ = counters(p)
            out.setdefault("sq", {}).update(c)
    sq = out.get("sq", {})
    if "SQ_WAVE_CYCLES" in sq:
        w = sq["SQ_WAVE_CYCLES"]
        out["sq_shares"] = {k: sq[k] / w for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
                                                   "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU")
                            if k in sq}
        out["valu_insts_per_header"] = sq.get("SQ_INSTS_VALU", 0) * 64 / args.pmc_headers / 64
        out["valu_lane_insts_per_header"] = sq.get("SQ_INSTS_VALU", 0) * 64 / args.pmc_headers
    if os.path.exists(os.path.join(d, "pmc_sq.csv")):
        out["clock_ghz"] = clock_ghz(os.path.join(d, "pmc_sq.csv"))
    # the source the PMC passes measured: bench.py stamps it into its JSON line
    src = None
    bj = os.path.join(d, "bench_under_rocprof.json")
    if os.path.exists(bj):
        with open(bj) as f:
            lines = [ln for ln in f.read().splitlines() if ln.startswith("{")]
        if lines:
            src = json.loads(lines[-1]).get("roofline", {}).get("source_hash")
    out["source_hash"] = src
    with open(os.path.join(d, "summary.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    with open(os.path.join(ROOT, "profiles", "pmc_traffic.json"), "w") as f:
        json.dump({"round": args.round, "source_hash": src,
                   "k_tpraos_verify_bytes_per_launch_per_header": hbm / args.pmc_headers,
                   "valu_lane_insts_per_header": out.get("valu_lane_insts_per_header"),
                   "clock_ghz": out.get("clock_ghz")}, f, indent=1)
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
