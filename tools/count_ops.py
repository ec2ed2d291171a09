#!/usr/bin/env python3
"""Count the GF(2^255-19) multiplications/squarings the kernels' lane routines
actually execute per unit (host build of verify.h with -DOURO_COUNT_OPS).

Used for DESIGN.md's work table: the roofline numerator stays SURVEY.md
§8(d)'s canonical figure; this shows how much of it the implementation does.
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

SO = os.path.join(ROOT, "ouroboros-network_amd", "lib", "libouro_devhost_test.so")


def main():
    print(json.dumps(counts(), indent=1))


def counts(header_only: bool = False):
    """header_only: just the golden header through the throughput schedule
    (no oracle-synthesised inputs; what bench.py reports)."""
    d = ctypes.CDLL(SO)
    nm, ns = ctypes.c_ulonglong(), ctypes.c_ulonglong()

    def measure(fn):
        d.dh_count_reset()
        fn()
        d.dh_count_get(ctypes.byref(nm), ctypes.byref(ns))
        return {"mul": nm.value, "sq": ns.value, "M": nm.value + ns.value}

    kats = json.load(open(os.path.join(ROOT, "tests", "golden", "reference_kats.json")))
    from ouroboros_network_amd import header as H
    import numpy as np

    hd = H.parse_header(bytes.fromhex(kats["headers"][0]["raw"]))
    # one golden header through tpraos.h's throughput schedule (shared key table,
    # single-inversion finish)
    batch = H.pack([hd], [bytes.fromhex(kats["headers"][0]["eta_alpha"])],
                   [bytes.fromhex(kats["headers"][0]["leader_alpha"])], slots_per_kes_period=100)
    st = batch.c_struct()
    v, be, bl = np.zeros(1, np.uint8), np.zeros((1, 64), np.uint8), np.zeros((1, 64), np.uint8)
    d.dh_tpraos_verify.argtypes = [ctypes.c_void_p, ctypes.c_int] + [ctypes.c_void_p] * 3
    d.dh_tpraos_verify(ctypes.addressof(st), 0, v.ctypes.data, be.ctypes.data, bl.ctypes.data)
    hdr = measure(lambda: d.dh_tpraos_verify(ctypes.addressof(st), 0, v.ctypes.data,
                                             be.ctypes.data, bl.ctypes.data))
    assert int(v[0]) & 0x0F == 15
    if header_only:
        return {"tpraos_header (throughput schedule)": hdr}
    import oracle_ffi as O

    pk, sig, msg = O.synth_ed25519(1, first=0)
    # build the host copy of the fixed-base table outside the counted region
    d.dh_ed25519_verify(bytes(sig[0]), bytes(msg[0]), 32, bytes(pk[0]))
    ed = measure(lambda: d.dh_ed25519_verify(bytes(sig[0]), bytes(msg[0]), 32, bytes(pk[0])))
    vpk, proof, alpha = O.synth_vrf(1, first=0)
    out = ctypes.create_string_buffer(64)
    vrf = measure(lambda: d.dh_vrf03_verify(out, bytes(vpk[0]), bytes(proof[0]), bytes(alpha[0]), 32))
    kats = json.load(open(os.path.join(ROOT, "tests", "golden", "reference_kats.json")))
    from ouroboros_network_amd import header as H

    hd = H.parse_header(bytes.fromhex(kats["headers"][0]["raw"]))
    kes = measure(lambda: d.dh_sum6kes_verify(hd.hot_vk, 0, hd.body, len(hd.body), hd.kes_sig))
    return {"ed25519_verify": ed, "vrf03_verify": vrf, "sum6kes_verify": kes,
            "tpraos_header (throughput schedule)": hdr,
            "canonical_M (SURVEY.md §8(d))": {"ed25519": 2983, "vrf": 7325, "header": 20616}}


if __name__ == "__main__":
    main()
