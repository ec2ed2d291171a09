"""Tuning sweep of the raw-CBOR pipeline (ouro_tpraos_verify_cbor /
ouro_integrity_verify_cbor) on one GPU: chunk size, chunks in flight and
gather threads (OURO_CBOR_CHUNK / _SLOTS / _COPY_THREADS, read per call),
over n synthetic node-configuration raw headers in pageable host memory.
Prints one JSON object per configuration (best of `reps` calls).
CBOR_SWEEP_RAMP_AB=1: instead, the chunk ramp (OURO_CBOR_RAMP) on and off at
the default chunk / slots / threads, alternated.
    python tools/cbor_sweep.py [n] [reps]"""
import ctypes
import itertools
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import bench
    from ouroboros_network_amd import _native

    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    dev = torch.device("cuda", 0)
    lib = _native.load()
    lib.ouro_bind_thread_to_device(0)
    if os.environ.get("CBOR_SWEEP_BYRON"):  # ouro_byron_verify_cbor (round 6)
        return byron_sweep(lib, n, reps)
    eta0 = bytes(range(101, 133))
    raw, rl = bench.synth_raw_node_headers(n, 1024, dev, eta0)
    buf = raw.cpu().numpy()
    del raw
    torch.cuda.empty_cache()
    P = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    off = np.arange(n, dtype=np.uint64) * rl
    ln = np.full(n, rl, np.uint32)
    e0 = np.frombuffer(eta0, np.uint8).copy()
    st = np.zeros(n, np.uint8)
    v = np.zeros(n, np.uint8)
    be = np.zeros((n, 64), np.uint8)
    bl = np.zeros((n, 64), np.uint8)
    stats = np.zeros(6)

    def hdr():
        return lib.ouro_tpraos_verify_cbor(P(buf), buf.size, P(off), P(ln), n, 129600, P(e0),
                                           None, None, P(st), P(v), P(be), P(bl), None)

    def kes():
        return lib.ouro_integrity_verify_cbor(P(buf), buf.size, P(off), P(ln), n, 129600, P(st),
                                              P(v))

    grid = {
        "hdr": [(65536, 5, 8), (65536, 6, 8), (65536, 7, 8), (98304, 4, 8), (98304, 5, 8),
                (131072, 3, 8), (131072, 4, 8), (49152, 8, 8)],
        "kes": [(65536, 2, 8), (65536, 3, 8), (65536, 4, 8), (49152, 4, 8), (98304, 3, 8)],
    }
    if os.environ.get("CBOR_SWEEP_RAMP_AB"):  # the chunk ramp on / off at the defaults
        for kind, fn in (("hdr", hdr), ("kes", kes)):
            for ramp in ("1", "0", "1", "0"):
                os.environ["OURO_CBOR_RAMP"] = ramp
                _native.reload_knobs()  # the library reads its switches once (knobs.h)
                assert fn() == 0, lib.ouro_last_error()
                ts = []
                for _ in range(reps):
                    t0 = time.perf_counter()
                    assert fn() == 0, lib.ouro_last_error()
                    ts.append(time.perf_counter() - t0)
                lib.ouro_debug_cbor_stats(stats.ctypes.data)
                ok = bool((st == 0).all() and (((v & 0x3F) == 0x3F) if kind == "hdr" else v == 1).all())
                print(json.dumps({"kind": kind, "ramp": int(ramp), "ms": round(min(ts) * 1e3, 2),
                                  "M_per_s": round(n / min(ts) / 1e6, 3),
                                  "chunks": int(stats[3]), "all_valid": ok}), flush=True)
        return
    if os.environ.get("CBOR_SWEEP_GRID"):  # "kind:chunk:slots:threads,..." in order
        order = [g.split(":") for g in os.environ["CBOR_SWEEP_GRID"].split(",")]
        plan = [(k, {"hdr": hdr, "kes": kes}[k], [(int(c), int(s_), int(t))])
                for k, c, s_, t in order]
    else:
        plan = [(kind, fn, grid[kind]) for kind, fn in (("hdr", hdr), ("kes", kes))]
    for kind, fn, configs in plan:
        for chunk, slots, threads in configs:
            os.environ["OURO_CBOR_CHUNK"] = str(chunk)
            os.environ["OURO_CBOR_SLOTS"] = str(slots)
            os.environ["OURO_CBOR_COPY_THREADS"] = str(threads)
            _native.reload_knobs()
            assert fn() == 0, lib.ouro_last_error()
            ts, ss = [], []
            for _ in range(reps):
                t0 = time.perf_counter()
                assert fn() == 0, lib.ouro_last_error()
                ts.append(time.perf_counter() - t0)
                lib.ouro_debug_cbor_stats(stats.ctypes.data)
                ss.append(stats.copy())
            k = int(np.argmin(ts))
            ok = bool((st == 0).all() and (((v & 0x3F) == 0x3F) if kind == "hdr" else v == 1).all())
            print(json.dumps({"kind": kind, "chunk": chunk, "slots": slots, "threads": threads,
                              "ms": round(ts[k] * 1e3, 2), "M_per_s": round(n / ts[k] / 1e6, 3),
                              "gather_ms": round(ss[k][1], 2), "wait_ms": round(ss[k][2], 2),
                              "all_valid": ok}), flush=True)


def byron_sweep(lib, n, reps):
    """The golden Byron wire forms repeated to n (bench.py byron_leg), raw ->
    verdicts over chunk x slots x gather threads."""
    from ouroboros_network_amd import _native
    from ouroboros_network_amd import byron as B

    with open(os.path.join(ROOT, "tests", "golden", "reference_kats.json")) as f:
        wires = [bytes.fromhex(w["raw"]) for w in json.load(f)["byron_wire"]]
    raws = [wires[i % len(wires)] for i in range(n)]
    ln = np.array([len(r) for r in raws], np.uint32)
    off = np.zeros(n, np.uint64)
    off[1:] = np.cumsum(ln[:-1], dtype=np.uint64)
    arg = (np.frombuffer(b"".join(raws), np.uint8), off, ln)
    stats = np.zeros(6)
    grid = list(itertools.product((32768, 65536, 131072, 262144), (2, 4, 6, 8), (8, 16)))
    if os.environ.get("CBOR_SWEEP_GRID"):  # "chunk:slots:threads,..." repeated in order
        grid = [tuple(int(x) for x in g.split(":")) for g in
                os.environ["CBOR_SWEEP_GRID"].split(",")]
    for chunk, slots, threads in grid:
        os.environ["OURO_CBOR_CHUNK"] = str(chunk)
        os.environ["OURO_CBOR_SLOTS"] = str(slots)
        os.environ["OURO_CBOR_COPY_THREADS"] = str(threads)
        _native.reload_knobs()
        v, st = B.verify_byron_cbor(arg, B.HEADER_MAGIC)
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            v, st = B.verify_byron_cbor(arg, B.HEADER_MAGIC)
            ts.append(time.perf_counter() - t0)
        lib.ouro_debug_cbor_stats(stats.ctypes.data)
        print(json.dumps({"kind": "byron", "chunk": chunk, "slots": slots, "threads": threads,
                          "ms": round(min(ts) * 1e3, 2), "M_per_s": round(n / min(ts) / 1e6, 3),
                          "gather_ms": round(stats[1], 2), "wait_ms": round(stats[2], 2),
                          "all_valid": bool(v.all())}), flush=True)


if __name__ == "__main__":
    main()
