#!/usr/bin/env python3
"""bench.py -- TPraos header-crypto throughput on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[3]): full TPraos header batches -- per header
the opcert Ed25519, Sum6KES (6 Blake2b Merkle levels + Ed25519 leaf over the
544-byte body) and the eta + leader draft-03 VRF verifies with their outputs.
At N = 1 one GPU verifies a batch of 1,048,576 synthetic headers per step.  At
N > 1 the default is configs[3] as written -- ONE batch of 1,048,576 headers
per step cut into N/G contiguous shards (strong scaling; no data-path
collective) -- and the step ends with the one RCCL all-gather of verdicts and
VRF outputs the north star names; the weak-scaling figure (1,048,576 headers
per GPU) is reported beside it as `weak`.  --weak makes weak scaling the line.

Inputs are synthesised on the device (lib/libouro_synth.so, deterministic
seeds) and are resident in HBM before timing starts.  The
CPU baseline is the oracle (oracle/build/liboracle.so, a C port) on a bounded
sample of the same headers, at the box's CPU share of threads.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--headers H]
"""
from __future__ import annotations

import argparse
import ctypes
import hashlib
import json
import math
import os
import subprocess
import socket
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "TPraos header verifies/sec (VRF+KES+Ed25519) at 1/2/4/8 MI355X; Ed25519 ver/s"
# algorithmic work per unit, SURVEY.md §8(d) / BASELINE.md (limb-MACs)
MACS_PER_HEADER = 1_319_424
MACS_PER_ED25519 = 190_912
SYNTH_SO = os.path.join(ROOT, "ouroboros-network_amd", "lib", "libouro_synth.so")


def body_template() -> bytes:
    """The golden Shelley header body (544 B) from the committed fixtures."""
    with open(os.path.join(ROOT, "tests", "golden", "reference_kats.json")) as f:
        kats = json.load(f)
    from ouroboros_network_amd import header as H

    return H.parse_header(bytes.fromhex(kats["headers"][0]["raw"])).body


def synth_headers(n: int, npools: int, device, first: int = 0, keep_nodes: bool = False,
                  keep_pool: bool = False):
    """Device-resident SoA header batch (torch uint8 tensors)."""
    import torch

    lib = ctypes.CDLL(SYNTH_SO)
    tmpl = body_template()
    blen = len(tmpl)
    u8 = dict(dtype=torch.uint8, device=device)
    t = {
        "issuer_vk": torch.empty(n * 32, **u8), "vrf_vk": torch.empty(n * 32, **u8),
        "eta_proof": torch.empty(n * 80, **u8), "leader_proof": torch.empty(n * 80, **u8),
        "eta_alpha": torch.empty(n * 32, **u8), "leader_alpha": torch.empty(n * 32, **u8),
        "hot_vk": torch.empty(n * 32, **u8), "ocert_counter": torch.empty(n * 8, **u8),
        "ocert_kes_period": torch.empty(n * 8, **u8), "ocert_sigma": torch.empty(n * 64, **u8),
        "kes_t": torch.empty(n * 4, **u8), "kes_sig": torch.empty(n * 448, **u8),
        "body": torch.empty(n * blen, **u8), "body_off": torch.empty(n * 8, **u8),
        "body_len": torch.empty(n * 4, **u8),
    }
    nodes = torch.empty(npools * 127 * 32, **u8)
    pool = torch.empty(npools * 56 * 4, **u8)
    dtmpl = torch.frombuffer(bytearray(tmpl), dtype=torch.uint8).to(device)
    P = ctypes.c_void_p
    fn = lib.ouro_synth_headers
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_size_t, ctypes.c_uint64, ctypes.c_int, P, ctypes.c_uint32] + [P] * 17
    order = ["issuer_vk", "vrf_vk", "eta_proof", "leader_proof", "eta_alpha", "leader_alpha",
             "hot_vk", "ocert_counter", "ocert_kes_period", "ocert_sigma", "kes_t", "kes_sig",
             "body", "body_off", "body_len"]
    rc = fn(n, first, npools, dtmpl.data_ptr(), blen, nodes.data_ptr(), pool.data_ptr(),
            *[t[k].data_ptr() for k in order])
    if rc != 0:
        raise RuntimeError(f"ouro_synth_headers failed: {rc}")
    torch.cuda.synchronize()
    if keep_nodes and keep_pool:
        return t, blen, nodes, pool
    if keep_nodes:
        return t, blen, nodes
    if keep_pool:
        return t, blen, pool
    return t, blen


def synth_node_config(t, n: int, npools: int, pool, eta0: bytes, device, slot0: int = 4_492_800):
    """Turn a synth_headers batch into the node's configuration:
    slots (slot0 + i), VRF proofs re-made over mkSeed seedEta / seedL slot eta0
    (the device then derives the alphas itself), and the headers' claimed
    outputs.  Adds "slot", "epoch_nonce", "eta_output", "leader_output"."""
    import torch

    lib = ctypes.CDLL(SYNTH_SO)
    u8 = dict(dtype=torch.uint8, device=device)
    t["slot"] = torch.empty(n * 8, **u8)
    t["epoch_nonce"] = torch.frombuffer(bytearray(eta0), dtype=torch.uint8).to(device)
    t["eta_output"] = torch.empty(n * 64, **u8)
    t["leader_output"] = torch.empty(n * 64, **u8)
    P = ctypes.c_void_p
    fn = lib.ouro_synth_seeded
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_size_t, ctypes.c_uint64, ctypes.c_int, P, ctypes.c_uint64] + [P] * 8
    rc = fn(n, 0, npools, pool.data_ptr(), slot0, t["epoch_nonce"].data_ptr(),
            *[t[k].data_ptr() for k in ("slot", "eta_alpha", "leader_alpha", "eta_proof",
                                        "leader_proof", "eta_output", "leader_output")])
    if rc != 0:
        raise RuntimeError(f"ouro_synth_seeded failed: {rc}")
    torch.cuda.synchronize()
    return t


RAW_OFFSET_NAMES = ["body", "body_len", "slot", "prev", "issuer", "vrf", "eta_out", "eta_proof",
                    "lead_out", "lead_proof", "hot", "sigma", "sig"]


def raw_template():
    """Wire-header template for synthesised raw headers:
    #6.24(bytes .cbor [header_body, kes_sig]) with the golden Shelley body
    re-encoded -- slot as a 4-byte uint, counter = kesPeriod = 0 (the synthetic
    opcerts sign counter 0, period 0), the other fields at fixed offsets that
    the device fills (ouro_synth_raw_headers).  Returns (bytes, offsets)."""
    from ouroboros_network_amd import header as H

    golden = body_template()
    f = H.array_items(golden, 0)
    raw = lambda k: golden[f[k][0]:f[k][1]]  # noqa: E731
    body = bytearray(b"\x8f")
    offs = {}

    def put(name, head, size):
        body.extend(head)
        offs[name] = len(body)
        body.extend(b"\0" * size)

    body += raw(0)                                   # blockNo
    put("slot", b"\x1a", 4)                          # slot (4-byte uint)
    put("prev", b"\x58\x20", 32)                     # prevHash
    put("issuer", b"\x58\x20", 32)
    put("vrf", b"\x58\x20", 32)
    body += b"\x82"
    put("eta_out", b"\x58\x40", 64)
    put("eta_proof", b"\x58\x50", 80)
    body += b"\x82"
    put("lead_out", b"\x58\x40", 64)
    put("lead_proof", b"\x58\x50", 80)
    body += raw(7) + raw(8)                          # bodySize, bodyHash
    put("hot", b"\x58\x20", 32)
    body += b"\x00\x00"                              # counter 0, kesPeriod 0
    put("sigma", b"\x58\x40", 64)
    body += raw(13) + raw(14)                        # protocol version
    inner = b"\x82" + bytes(body) + b"\x59\x01\xc0" + b"\0" * 448
    prefix = b"\xd8\x18\x59" + len(inner).to_bytes(2, "big")
    base = len(prefix) + 1                           # header_body starts after 0x82
    out = {k: base + v for k, v in offs.items()}
    out["body"] = base
    out["body_len"] = len(body)
    out["sig"] = len(prefix) + len(inner) - 448
    return prefix + inner, [out[k] for k in RAW_OFFSET_NAMES]


def synth_raw_headers(n: int, npools: int, device, first: int = 0,
                      slots_per_kes_period: int = 129600):
    """Synthetic SoA batch plus the same headers as raw wire CBOR on the device
    (n x raw_len bytes, uint8 tensor): (t, raw, raw_len)."""
    import torch

    t, _blen, nodes = synth_headers(n, npools, device, first, keep_nodes=True)
    tmpl, offs = raw_template()
    lib = ctypes.CDLL(SYNTH_SO)
    raw = torch.empty(n * len(tmpl), dtype=torch.uint8, device=device)
    dt = torch.frombuffer(bytearray(tmpl), dtype=torch.uint8).to(device)
    o = (ctypes.c_uint32 * 13)(*offs)
    P = ctypes.c_void_p
    fn = lib.ouro_synth_raw_headers
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_size_t, ctypes.c_uint64, ctypes.c_int, P, P, ctypes.c_uint32, P,
                   ctypes.c_uint64] + [P] * 8
    rc = fn(n, first, npools, nodes.data_ptr(), dt.data_ptr(), len(tmpl), o,
            slots_per_kes_period, *[t[k].data_ptr() for k in (
                "issuer_vk", "vrf_vk", "eta_proof", "leader_proof", "hot_vk", "ocert_sigma",
                "kes_t")], raw.data_ptr())
    if rc != 0:
        raise RuntimeError(f"ouro_synth_raw_headers failed: {rc}")
    torch.cuda.synchronize()
    return t, raw, len(tmpl)


def synth_raw_node_headers(n: int, npools: int, device, eta0: bytes,
                           slots_per_kes_period: int = 129600):
    """Raw wire headers in the node's configuration: each header's VRF proofs
    are over mkSeed seedEta / seedL of ITS OWN slot (the slot the raw bytes
    carry, k_synth_raw's) and eta0, so the verifier derives the VRF inputs on
    the device as the OVERLAY rule does.  Returns (raw uint8 device tensor,
    raw_len)."""
    import torch

    t, _blen, nodes, pool = synth_headers(n, npools, device, keep_nodes=True, keep_pool=True)
    kt = t["kes_t"].view(torch.int32).to(torch.int64)
    slots = kt * slots_per_kes_period + torch.arange(n, device=device, dtype=torch.int64) % 1000
    e0 = torch.frombuffer(bytearray(eta0), dtype=torch.uint8).to(device)
    u8 = dict(dtype=torch.uint8, device=device)
    slot_out = torch.empty(n * 8, **u8)
    eo, lo = torch.empty(n * 64, **u8), torch.empty(n * 64, **u8)
    lib = ctypes.CDLL(SYNTH_SO)
    P = ctypes.c_void_p
    fn = lib.ouro_synth_seeded_at
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_size_t, ctypes.c_uint64, ctypes.c_int, P, P, P] + [P] * 7
    rc = fn(n, 0, npools, pool.data_ptr(), slots.data_ptr(), e0.data_ptr(), slot_out.data_ptr(),
            *[t[k].data_ptr() for k in ("eta_alpha", "leader_alpha", "eta_proof", "leader_proof")],
            eo.data_ptr(), lo.data_ptr())
    if rc != 0:
        raise RuntimeError(f"ouro_synth_seeded_at failed: {rc}")
    tmpl, offs = raw_template()
    raw = torch.empty(n * len(tmpl), **u8)
    dt = torch.frombuffer(bytearray(tmpl), dtype=torch.uint8).to(device)
    o = (ctypes.c_uint32 * 13)(*offs)
    fn = lib.ouro_synth_raw_headers
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_size_t, ctypes.c_uint64, ctypes.c_int, P, P, ctypes.c_uint32, P,
                   ctypes.c_uint64] + [P] * 8
    rc = fn(n, 0, npools, nodes.data_ptr(), dt.data_ptr(), len(tmpl), o, slots_per_kes_period,
            *[t[k].data_ptr() for k in ("issuer_vk", "vrf_vk", "eta_proof", "leader_proof",
                                        "hot_vk", "ocert_sigma", "kes_t")], raw.data_ptr())
    if rc != 0:
        raise RuntimeError(f"ouro_synth_raw_headers failed: {rc}")
    torch.cuda.synchronize()
    return raw, len(tmpl)


class DeviceHeaders:
    """Binds a device SoA to the C ABI's ouro_tpraos_batch."""

    def __init__(self, t, n, device):
        import torch

        from ouroboros_network_amd import _native

        self.lib = _native.load()
        self.n = n
        self.t = t
        self.s = _native.TPraosBatch()
        self.s.n = n
        for k, v in t.items():
            setattr(self.s, k, v.data_ptr())
        # two output sets: the all-gather of step k reads one while step k+1
        # writes the other (bench.py overlaps the collective with compute)
        self.sets = [(torch.zeros(n, dtype=torch.uint8, device=device),
                      torch.zeros(n * 64, dtype=torch.uint8, device=device),
                      torch.zeros(n * 64, dtype=torch.uint8, device=device)) for _ in range(2)]
        self.use(0)

    def use(self, k: int) -> None:
        self.verdict, self.beta_eta, self.beta_leader = self.sets[k]

    def launch(self, stream) -> None:
        from ouroboros_network_amd import _native

        rc = self.lib.ouro_tpraos_verify_batch_device(
            ctypes.c_void_p(stream.cuda_stream), ctypes.byref(self.s), self.verdict.data_ptr(),
            self.beta_eta.data_ptr(), self.beta_leader.data_ptr())
        _native.check(rc, "ouro_tpraos_verify_batch_device")

    def host_sample(self, m: int):
        """First m headers copied to host as a HeaderBatch (for the CPU leg)."""
        from ouroboros_network_amd.tpraos import HeaderBatch

        def h(k, dt, w=None):
            a = self.t[k].cpu().numpy().view(dt)
            return a.reshape(-1, w)[:m] if w else a[:m]

        blen = int(h("body_len", np.uint32)[0])
        body = self.t["body"][: m * blen].cpu().numpy()
        opt = {}
        if "slot" in self.t:  # the node configuration (synth_node_config)
            opt = dict(slot=h("slot", np.uint64), epoch_nonce=self.t["epoch_nonce"].cpu().numpy(),
                       eta_output=h("eta_output", np.uint8, 64),
                       leader_output=h("leader_output", np.uint8, 64))
        return HeaderBatch(**opt,
            issuer_vk=h("issuer_vk", np.uint8, 32), vrf_vk=h("vrf_vk", np.uint8, 32),
            eta_proof=h("eta_proof", np.uint8, 80), leader_proof=h("leader_proof", np.uint8, 80),
            eta_alpha=h("eta_alpha", np.uint8, 32), leader_alpha=h("leader_alpha", np.uint8, 32),
            hot_vk=h("hot_vk", np.uint8, 32), ocert_counter=h("ocert_counter", np.uint64),
            ocert_kes_period=h("ocert_kes_period", np.uint64),
            ocert_sigma=h("ocert_sigma", np.uint8, 64), kes_t=h("kes_t", np.uint32),
            kes_sig=h("kes_sig", np.uint8, 448), body=body, body_off=h("body_off", np.uint64),
            body_len=h("body_len", np.uint32))


def source_hash() -> str:
    """sha256 over the sources the header kernel k_tpraos_verify is built from
    (csrc/ and include/ headers, kernels.hip): ties a committed PMC traffic
    figure to the code it was measured on.  The latency-mode translation unit
    (kernels_lat.hip, wide*.h) and the test/synthesis sources do not enter
    that kernel and are left out."""
    h = hashlib.sha256()
    for d in (os.path.join(ROOT, "ouroboros-network_amd", "csrc"), os.path.join(ROOT, "include")):
        for name in sorted(os.listdir(d)):
            if (name.endswith((".h", ".hip"))
                    and not name.startswith(("devhost", "synth", "wide", "kernels_lat"))):
                with open(os.path.join(d, name), "rb") as f:
                    h.update(name.encode() + b"\0" + f.read())
    return h.hexdigest()[:16]


def host_cpu_info() -> dict:
    """The host the CPU baselines run on: model, nproc, the
    CPUs this process may run on (affinity) and the cgroup CPU quota; `usable`
    = the cores the baselines use (the box gives a job a share of a larger
    machine, so nproc alone would oversubscribe it)."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    nproc = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = nproc
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                quota = int(q) / int(per)
    except (OSError, ValueError):
        pass
    usable = min(aff, math.ceil(quota)) if quota else aff
    return {"model": model, "nproc": nproc, "affinity_cpus": aff, "cgroup_cpu_quota": quota,
            "usable": max(1, usable)}


def native_oracle(O) -> str:
    """Load the oracle built -O3 -march=native on THIS host (make -C oracle
    native); falls back to the shipped x86-64-v2 build."""
    try:
        r = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "native"],
                           capture_output=True, timeout=180)
        path = os.path.join(ROOT, "oracle", "build", "liboracle_native.so")
        if r.returncode == 0 and os.path.exists(path):
            O.lib(path)
            return "gcc -O3 -march=native (built on this host)"
    except (OSError, subprocess.SubprocessError):
        pass
    O.lib()
    return "gcc -O3 -march=x86-64-v2 (native build failed)"


def measure_peak_mac(device) -> float:
    """Live v_mad_u64_u32 rate (TMAC/s) from the microbenchmark kernel."""
    lib = ctypes.CDLL(SYNTH_SO)
    fn = lib.ouro_peak_mad_u64_tmacs
    fn.restype = ctypes.c_double
    return float(fn())


CLOCK_SO = os.path.join(ROOT, "ouroboros-network_amd", "lib", "libouro_verify_clock.so")
DEVHOST_SO = os.path.join(ROOT, "ouroboros-network_amd", "lib", "libouro_devhost_test.so")


def kernel_clock_ghz(hdr, stream, launches: int = 36):
    """The shader clock k_tpraos_verify itself runs at on THIS box: the
    diagnostic build lib/libouro_verify_clock.so (-DOURO_CLOCK_STAMPS=1: the
    same kernel with s_memtime / s_memrealtime stamps at each workgroup's entry
    and exit, MI355X_MICROARCH.md "DVFS give-back" item 6) run back to back on
    the same device-resident batch; median over workgroups of the last launch.
    The timed product launches never execute a stamp."""
    import torch

    if not os.path.exists(CLOCK_SO):
        return None, "lib/libouro_verify_clock.so not built"
    lib = ctypes.CDLL(CLOCK_SO)
    P = ctypes.c_void_p
    lib.ouro_tpraos_verify_batch_device.argtypes = [P, P, P, P, P]
    lib.ouro_debug_clock_stamps.argtypes = [P, ctypes.c_int]
    lib.ouro_set_device.argtypes = [ctypes.c_int]
    lib.ouro_set_device(torch.cuda.current_device())
    t0 = time.perf_counter()
    for _ in range(launches):
        rc = lib.ouro_tpraos_verify_batch_device(P(stream.cuda_stream), ctypes.byref(hdr.s),
                                                 P(hdr.verdict.data_ptr()),
                                                 P(hdr.beta_eta.data_ptr()),
                                                 P(hdr.beta_leader.data_ptr()))
        if rc != 0:
            return None, f"diagnostic launch failed ({rc})"
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    buf = np.zeros((8192, 4), np.uint64)
    rows = lib.ouro_debug_clock_stamps(P(buf.ctypes.data), 8192)
    if rows <= 0:
        return None, "no stamps"
    st = buf[:rows].astype(np.float64)
    ok = (st[:, 3] > st[:, 2]) & (st[:, 1] > st[:, 0])
    ghz = (st[ok, 1] - st[ok, 0]) / (st[ok, 3] - st[ok, 2]) * 0.1
    return float(np.median(ghz)), f"median of {int(ok.sum())} workgroups, last of {launches} " \
                                  f"back-to-back launches ({wall:.2f} s)"


def executed_work_per_header():
    """Field operations the kernels' lane routines execute for one header in
    the throughput schedule (the host build with operation counters,
    lib/libouro_devhost_test.so -- the same source), as v_mad_u64_u32 counts:
    100 per multiply, 55 per squaring (csrc/fe25519.h)."""
    if not os.path.exists(DEVHOST_SO):
        return None
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    try:
        import count_ops
        r = count_ops.counts(header_only=True)["tpraos_header (throughput schedule)"]
    except Exception:  # noqa: BLE001
        return None
    return {"field_mul": r["mul"], "field_sq": r["sq"],
            "executed_mads_per_header": 100 * r["mul"] + 55 * r["sq"]}


def ed25519_rate(device, n: int, reps: int):
    """Ed25519 verifies/s on n device-resident synthetic signatures; returns
    (result, (pk, sig, msg) device tensors)."""
    import torch

    from ouroboros_network_amd import _native

    lib = ctypes.CDLL(SYNTH_SO)
    u8 = dict(dtype=torch.uint8, device=device)
    pk, sig, msg = torch.empty(n * 32, **u8), torch.empty(n * 64, **u8), torch.empty(n * 32, **u8)
    lib.ouro_synth_ed25519.argtypes = [ctypes.c_size_t, ctypes.c_uint64] + [ctypes.c_void_p] * 3
    if lib.ouro_synth_ed25519(n, 0, pk.data_ptr(), sig.data_ptr(), msg.data_ptr()) != 0:
        raise RuntimeError("ouro_synth_ed25519 failed")
    off = torch.arange(n, dtype=torch.int64, device=device) * 32
    ln = torch.full((n,), 32, dtype=torch.int32, device=device)
    ver = torch.zeros(n, **u8)
    v = _native.load()
    st = torch.cuda.current_stream()

    def go():
        rc = v.ouro_ed25519_verify_batch_device(ctypes.c_void_p(st.cuda_stream), n, pk.data_ptr(),
                                                 sig.data_ptr(), msg.data_ptr(), off.data_ptr(),
                                                 ln.data_ptr(), ver.data_ptr())
        _native.check(rc, "ed25519 device batch")

    go()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        go()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    ok = int(ver.sum().item())
    out = {"value": n / (ms * 1e-3), "unit": "verifies/s", "n": n, "ms_per_launch": ms,
           "all_valid": ok == n,
           "roofline_frac": (n * MACS_PER_ED25519 / (ms * 1e-3) / 1e12)}
    return out, (pk, sig, msg)


SODIUM_SO = "/opt/conda/lib/libsodium.so.23"


def libsodium_ed25519_rate(pk, sig, msg, cpu: dict, n: int):
    """the function the reference calls for Ed25519,
    libsodium 1.0.18's crypto_sign_ed25519_verify_detached (the CI pin), timed
    on the host cores over the first n of the same synthetic signatures the
    GPU leg verified, by the oracle library's C pthread pool (dlopen of the
    library; no Python per item).  A CPU baseline only -- never the measured
    path."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_ffi as O

    if not os.path.exists(SODIUM_SO):
        return {"error": f"{SODIUM_SO} absent on this host"}
    pk, sig, msg = (np.ascontiguousarray(x[: n * w].cpu().numpy()) for x, w in
                    ((pk, 32), (sig, 64), (msg, 32)))
    ver = np.zeros(n, np.uint8)

    def timed(k, threads):
        t0 = time.perf_counter()
        rc = O.lib().orc_sodium_ed25519_verify_batch(SODIUM_SO.encode(), k, O.p(pk), O.p(sig),
                                                     O.p(msg), O.p(ver), threads)
        dt = time.perf_counter() - t0
        if rc != 0:
            raise RuntimeError("dlopen of libsodium failed")
        return k / dt, int(ver[:k].sum())

    threads = cpu["usable"]
    timed(min(n, 4096), threads)  # warm: pages, library init
    rate, acc = timed(n, threads)
    n1 = max(1, n // 16)
    rate1, acc1 = timed(n1, 1)
    return {"value": round(rate, 1), "unit": "verifies/s", "cores": threads, "kind": "reference",
            "sample": f"first {n} of the same synthetic signatures (32-B messages), libsodium "
                      f"1.0.18 crypto_sign_ed25519_verify_detached from a C pthread pool",
            "one_core": round(rate1, 1), "one_core_sample": n1,
            "thread_scaling": round(rate / rate1, 2),
            "accepts_all": acc == n and acc1 == n1}


def component_rates(hdr, n: int, reps: int = 3):
    """configs[1] and configs[2]: VRF verify + output and Sum6KES verify over
    the n device-resident items of the synthetic header batch (its eta proofs
    and its KES signatures), timed with HIP events on the launch stream."""
    import torch

    from ouroboros_network_amd import _native

    v = _native.load()
    dev = hdr.verdict.device
    st = torch.cuda.current_stream()
    t = hdr.t
    a_off = torch.arange(n, dtype=torch.int64, device=dev) * 32
    a_len = torch.full((n,), 32, dtype=torch.int32, device=dev)
    beta = torch.zeros(n * 64, dtype=torch.uint8, device=dev)
    ver = torch.zeros(n, dtype=torch.uint8, device=dev)
    S = ctypes.c_void_p

    def vrf():
        rc = v.ouro_vrf03_verify_batch_device(S(st.cuda_stream), n, t["vrf_vk"].data_ptr(),
                                               t["eta_proof"].data_ptr(), t["eta_alpha"].data_ptr(),
                                               a_off.data_ptr(), a_len.data_ptr(), beta.data_ptr(),
                                               ver.data_ptr())
        _native.check(rc, "vrf device batch")

    def kes():
        rc = v.ouro_sum6kes_verify_batch_device(S(st.cuda_stream), n, t["hot_vk"].data_ptr(),
                                                 t["kes_t"].data_ptr(), t["body"].data_ptr(),
                                                 t["body_off"].data_ptr(), t["body_len"].data_ptr(),
                                                 t["kes_sig"].data_ptr(), ver.data_ptr())
        _native.check(rc, "kes device batch")

    # checkLeaderValue on the batch's leader outputs:
    # synthetic relative stakes ~ 1/1024 per pool, f = 1/20 given as its
    # unActiveSlotLog = floor(10^34 ln(0.95)) (a constant input, as the
    # reference's ActiveSlotCoeff stores it)
    sig_num = (torch.arange(n, dtype=torch.int64, device=dev) % 997 + 1)
    sig_den = torch.full((n,), 1024 * 1000, dtype=torch.int64, device=dev)
    act_log = -512932943875505334261961442500000
    a_lo, a_hi = act_log & ((1 << 64) - 1), act_log >> 64
    lead = torch.zeros(n, dtype=torch.uint8, device=dev)

    def leader():
        rc = v.ouro_leader_check_batch_device(S(st.cuda_stream), n, hdr.beta_leader.data_ptr(),
                                               sig_num.data_ptr(), sig_den.data_ptr(),
                                               ctypes.c_int64(a_hi), ctypes.c_uint64(a_lo), 0,
                                               lead.data_ptr())
        _native.check(rc, "leader device batch")

    out = {}
    leader()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(reps):
        leader()
    e1.record(st)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    out["leader"] = {"value": round(n / (ms * 1e-3), 1), "unit": "checks/s", "n": n,
                     "ms_per_launch": round(ms, 3),
                     "leaders": int((lead == 1).sum().item()),
                     "badarg": int((lead == 0xFF).sum().item())}
    for name, fn, macs in (("vrf", vrf, 468_800), ("kes", kes, 190_912)):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(reps):
            fn()
        e1.record(st)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        out[name] = {"value": round(n / (ms * 1e-3), 1), "unit": "verifies/s", "n": n,
                     "ms_per_launch": round(ms, 3), "all_valid": bool((ver == 1).all().item()),
                     "achieved_tmacs": round(n * macs / (ms * 1e-3) / 1e12, 3)}
        if name == "vrf":
            # the computed outputs must equal the header kernel's eta outputs
            out[name]["beta_equals_header_kernel"] = bool(torch.equal(beta, hdr.beta_eta))
    return out


def cpu_baseline(hb, threads: int):
    """The oracle (C port) on a bounded sample; returns (rate, results)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_ffi as O

    O.lib()
    t0 = time.perf_counter()
    res = O.tpraos_verify_batch(hb, threads=threads)
    dt = time.perf_counter() - t0
    return len(hb) / dt, dt, res


def _plan_latency(hb, iters: int, nonce: bool):
    """Wall-clock latency of ouro_tpraos_plan_run on one batch, timed at the C
    ABI as an FFI caller drives it (a prepared batch struct; the Python
    wrapper's per-call marshalling, ~tens of us, is not the product's
    latency).  Returns (latencies s, outputs)."""
    from ouroboros_network_amd.tpraos import HeaderPlan

    body_bytes = int(hb.body_len.astype(np.int64).sum())
    plan = HeaderPlan(len(hb), body_bytes)
    try:
        out = plan.run(hb, nonce=nonce)
        s = hb.c_struct(out[3] if nonce else None)
        P = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
        run = plan._lib.ouro_tpraos_plan_run
        args = (plan._p, ctypes.byref(s), P(out[0]), P(out[1]), P(out[2]))
        for _ in range(min(50, iters)):
            assert run(*args) == 0
        lat = np.empty(iters)
        for k in range(iters):
            t0 = time.perf_counter()
            rc = run(*args)
            lat[k] = time.perf_counter() - t0
            assert rc == 0
    finally:
        plan.close()
    return lat, out


def _plan_phases(hb, iters: int, nonce: bool):
    """Where a window's wall time goes, to explain the latency tail (VERDICT
    r03 item 5): the plan's submit (copy into pinned staging + the launch
    calls) and wait (until the results are in the caller's buffers) timed on
    the host, and the GPU time of the window (input copy kernel's start to
    the last header's end; "gpu_graph" keeps its round-4 name) from
    s_memrealtime stamps the kernels write into the plan's pinned done block
    (OURO_PLAN_TIMING at plan create; since round 6 no runtime events: an
    event pair per window made the runtime stall one submit in ~250 for
    ~125 us, profiles/r06b/submit_probe.json).  host_gap = wall - gpu:
    launch latency + completion wake-up + the host copies."""
    from ouroboros_network_amd.tpraos import HeaderPlan

    from ouroboros_network_amd import _native

    body_bytes = int(hb.body_len.astype(np.int64).sum())
    with _native.knob_env(OURO_PLAN_TIMING="1"):  # read when the plan is created
        plan = HeaderPlan(len(hb), body_bytes)
    try:
        out = plan.run(hb, nonce=nonce)
        s = hb.c_struct(out[3] if nonce else None)
        P = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
        lib = plan._lib
        sub, wait = lib.ouro_tpraos_plan_submit, lib.ouro_tpraos_plan_wait
        gms, cus, lus = ctypes.c_float(), ctypes.c_float(), ctypes.c_float()
        for _ in range(min(50, iters)):
            assert sub(plan._p, ctypes.byref(s)) == 0
            assert wait(plan._p, P(out[0]), P(out[1]), P(out[2])) == 0
        ph = np.empty((iters, 5))
        for k in range(iters):
            t0 = time.perf_counter()
            assert sub(plan._p, ctypes.byref(s)) == 0
            t1 = time.perf_counter()
            assert wait(plan._p, P(out[0]), P(out[1]), P(out[2])) == 0
            t2 = time.perf_counter()
            lib.ouro_debug_plan_timing(plan._p, ctypes.byref(gms), ctypes.byref(cus),
                                       ctypes.byref(lus))
            ph[k] = (t1 - t0, t2 - t1, gms.value * 1e-3, cus.value * 1e-6, lus.value * 1e-6)
    finally:
        plan.close()
    wall = ph[:, 0] + ph[:, 1]
    gap = wall - ph[:, 2]
    us = lambda a, q: round(float(np.percentile(a, q)) * 1e6, 1)  # noqa: E731
    pc = lambda a: {"p50_us": us(a, 50), "p99_us": us(a, 99), "p99_9_us": us(a, 99.9),  # noqa: E731
                    "max_us": us(a, 100)}
    worst = np.argsort(wall)[-5:][::-1]
    return {"iters": iters, "wall": pc(wall), "submit": pc(ph[:, 0]),
            "submit_copy": pc(ph[:, 3]), "submit_graph_launch": pc(ph[:, 4]), "wait": pc(ph[:, 1]),
            "gpu_graph": pc(ph[:, 2]), "host_gap": pc(gap),
            "slowest_windows_us": [{"wall": round(wall[i] * 1e6, 1),
                                    "submit": round(ph[i, 0] * 1e6, 1),
                                    "wait": round(ph[i, 1] * 1e6, 1),
                                    "gpu_graph": round(ph[i, 2] * 1e6, 1)} for i in worst],
            "note": "GPU span from the kernels' s_memrealtime stamps in the plan's done block "
                    "(OURO_PLAN_TIMING, a separate pass; no runtime events); host_gap = wall - "
                    "gpu_graph (launch latency, completion wake-up, host copies)"}


def _pcts(lat):
    ms = lambda q: round(float(np.percentile(lat, q)) * 1e3, 4)  # noqa: E731
    return {"p50_ms": ms(50), "p99_ms": ms(99), "p99_9_ms": ms(99.9), "max_ms": ms(100)}


def latency_leg(hdr, batch: int, iters: int, cpu_threads: int, cpu_iters: int, node=None):
    """configs[4]: ChainSync small-batch path.  `batch` headers from host
    memory through a plan (pinned staging, its input copy kernel and the fused
    latency kernel writing into pinned memory), wall-clock per call over `iters` windows (p50 / p99 / p99.9); next to
    the CPU oracle on the same batch on 1 core and on `cpu_threads` cores.
    `node` (a DeviceHeaders in the node's configuration, synth_node_config):
    the same timing with claimed outputs, (slot, eta0) seeds derived on the
    device and the eta nonce requested -- the configuration a node runs --
    beside the minimal one (caller-supplied alphas, no claims, no nonce)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_ffi as O
    from ouroboros_network_amd.tpraos import HDR_ALL_OK, HDR_STRICT_OK, HeaderPlan

    hb = hdr.host_sample(batch)
    body_bytes = int(hb.body_len.astype(np.int64).sum())
    lat, out = _plan_latency(hb, iters, nonce=False)
    # windows in flight: 4 plans (e.g. 4 ChainSync peers) submitted round-robin,
    # each waited for just before its next submit
    plans = [HeaderPlan(batch, body_bytes) for _ in range(4)]
    try:
        for p in plans:
            p.submit(hb)
        t0 = time.perf_counter()
        rounds = max(1, iters // 4)
        for _ in range(rounds):
            for p in plans:
                p.wait(out)
                p.submit(hb)
        for p in plans:
            p.wait(out)
        inflight_s = time.perf_counter() - t0
    finally:
        for p in plans:
            p.close()
    cv, cbe, cbl = O.tpraos_verify_batch(hb, threads=1)
    same = bool((out[0] == cv).all() and (out[1] == cbe).all() and (out[2] == cbl).all())

    def cpu_lat(threads):
        O.tpraos_verify_batch(hb, threads=threads)
        t = np.empty(cpu_iters)
        for k in range(cpu_iters):
            t0 = time.perf_counter()
            O.tpraos_verify_batch(hb, threads=threads)
            t[k] = time.perf_counter() - t0
        return t

    c1, cn = cpu_lat(1), cpu_lat(cpu_threads)
    ms = lambda a, q: round(float(np.percentile(a, q)) * 1e3, 3)  # noqa: E731
    res = {"workload": f"configs[4]: {batch}-header batches from host memory, plan "
                       "(minimal configuration: caller alphas, no claimed outputs, no nonce)",
           "iters": iters, **_pcts(lat),
           "headers_per_s_at_p50": round(batch / (np.percentile(lat, 50)), 1),
           "in_flight_4_plans_headers_per_s": round(batch * (4 * rounds + 4) / inflight_s, 1),
           "all_valid": bool(((out[0] & HDR_ALL_OK) == HDR_ALL_OK).all()), "gpu_equals_cpu": same,
           "cpu_1core": {"p50_ms": ms(c1, 50), "p99_ms": ms(c1, 99), "iters": cpu_iters},
           "cpu_ncores": {"cores": cpu_threads, "p50_ms": ms(cn, 50), "p99_ms": ms(cn, 99),
                          "iters": cpu_iters}}
    if node is not None:
        nb = node.host_sample(batch)
        nlat, nout = _plan_latency(nb, iters, nonce=True)
        wv, wbe, wbl, wen = O.tpraos_verify_batch_nonce(nb, threads=1)
        res["node"] = {
            "workload": f"{batch}-header windows as a node runs them: claimed outputs checked "
                        "(*_CLAIM_OK), VRF inputs from (slot, eta0) by mkSeed on the device, "
                        "eta nonce output requested",
            "iters": iters, **_pcts(nlat),
            "phases": _plan_phases(nb, iters, nonce=True),
            "all_strict_ok": bool(((nout[0] & HDR_STRICT_OK) == HDR_STRICT_OK).all()),
            "gpu_equals_cpu": bool((nout[0] == wv).all() and (nout[1] == wbe).all()
                                   and (nout[2] == wbl).all() and (nout[3] == wen).all())}
    return res


def e2e_leg(hdr, n: int, reps: int = 3):
    """Host buffers in, host buffers out (SURVEY.md §8(d) "end-to-end"): the
    whole n-header batch from pageable host memory through the C ABI's
    ouro_tpraos_verify_batch -- PCIe H2D, the header kernel, D2H of verdicts
    and both VRF outputs -- wall clock per call.  The default path pipelines
    chunks over two streams; OURO_HOST_CHUNK=0 (one-piece staging) is timed
    beside it.  Never `value` (inputs are not HBM-resident here)."""
    from ouroboros_network_amd.tpraos import verify_headers

    hb = hdr.host_sample(n)
    in_bytes = sum(getattr(hb, k).nbytes for k in hb.__dataclass_fields__
                   if getattr(hb, k) is not None)
    dv = hdr.verdict.cpu().numpy()
    dbe = hdr.beta_eta.cpu().numpy().reshape(n, 64)
    dbl = hdr.beta_leader.cpu().numpy().reshape(n, 64)
    res = {"workload": f"configs[3] batch of {n} headers in pageable host memory, "
                       "ouro_tpraos_verify_batch (H2D + kernel + D2H)",
           "h2d_bytes": int(in_bytes), "d2h_bytes": int(129 * n)}
    from ouroboros_network_amd import _native

    for name, chunk in (("pipelined", os.environ.get("OURO_HOST_CHUNK")), ("one_piece", "0")):
        with _native.knob_env(OURO_HOST_CHUNK=chunk):
            v, be, bl = verify_headers(hb)  # warm: device/pinned buffers grown
            t = []
            for _ in range(reps):
                t0 = time.perf_counter()
                v, be, bl = verify_headers(hb)
                t.append(time.perf_counter() - t0)
            best = min(t)
        res[name] = {"headers_per_s": round(n / best, 1), "ms": round(best * 1e3, 2),
                     "equals_device_path": bool((v == dv).all() and (be == dbe).all()
                                                and (bl == dbl).all())}
    return res


def inproc_leg(hdr, n: int, devices, reps: int = 3):
    """One process, several GPUs: the
    one-process Haskell node's path, ouro_tpraos_verify_batch_multi over the
    listed devices -- contiguous shards on persistent per-device workers, each
    NUMA-bound with its own pinned staging, results straight into the host
    buffers -- against ouro_tpraos_verify_batch on one device, both from
    pageable host memory (PCIe-inclusive; never `value`).  A device listed
    twice runs two pipelines on it (the one-GPU rehearsal)."""
    from ouroboros_network_amd import _native
    from ouroboros_network_amd.tpraos import verify_headers, verify_headers_multi

    hb = hdr.host_sample(n)
    dv = hdr.verdict.cpu().numpy()
    res = {"workload": f"configs[3] batch of {n} headers in pageable host memory",
           "devices": list(devices)}
    for name, fn in (("single_device", lambda: verify_headers(hb)),
                     ("multi", lambda: verify_headers_multi(hb, devices=list(devices)))):
        v, _, _ = fn()  # warm: workers, streams, pinned staging
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            v, _, _ = fn()
            ts.append(time.perf_counter() - t0)
        res[name] = {"headers_per_s": round(n / min(ts), 1), "ms": round(min(ts) * 1e3, 2),
                     "equals_device_path": bool((v == dv).all())}
    workers = np.zeros(64, np.int32), np.zeros(64, np.int32), np.zeros(64, np.int32)
    k = _native.load().ouro_debug_multi_workers(*[w.ctypes.data for w in workers], 64)
    res["workers"] = [{"device": int(workers[0][i]), "numa_node": int(workers[1][i]),
                       "bound_cpus": int(workers[2][i])} for i in range(min(k, 64))]
    return res


def h2d_gbps(device, mib: int = 256, reps: int = 5) -> float:
    """This rank's pinned host -> HBM copy rate (GB/s, best of reps)."""
    import torch

    h = torch.empty(mib << 20, dtype=torch.uint8).pin_memory()
    d = torch.empty(mib << 20, dtype=torch.uint8, device=device)
    best = 1e9
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        d.copy_(h, non_blocking=True)
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1))
    return round((mib << 20) / (best * 1e-3) / 1e9, 2)


def pci_bus_id(device) -> str:
    import torch

    p = torch.cuda.get_device_properties(device)
    dom, bus, dev = (getattr(p, k, None) for k in ("pci_domain_id", "pci_bus_id", "pci_device_id"))
    if bus is None:
        return f"device{device.index}"
    return f"{dom or 0:04x}:{bus:02x}:{dev or 0:02x}.0"


def raw_leg(n: int, npools: int, device, threads: int, chunk: int = 0, reps: int = 3):
    """Raw wire CBOR -> verdicts: n synthetic headers as
    the bytes ChainSync hands over (#6.24-wrapped [header_body, kes_sig],
    bench.raw_template).  Three forms, never `value`:
      device    raw headers resident in HBM -> the device slicer
                (ouro_tpraos_pack_cbor_device) -> the header kernel, one stream;
      pcie      raw headers in pinned host memory, uploaded in chunks on a
                copy stream overlapping the slicer + kernel of the previous
                chunk, results copied back;
      host      pageable host memory -> the C slicer on `threads` host threads
                -> ouro_tpraos_verify_batch (H2D + kernel + D2H), slicing chunk
                k+1 behind the verification of chunk k."""
    import threading

    import torch

    from ouroboros_network_amd import _native

    t, raw, rl = synth_raw_headers(n, npools, device)
    lib = _native.load()
    P = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    V = ctypes.c_void_p
    res = {"raw_bytes_per_header": rl}

    # ---- device: raw in HBM -> device slicer -> kernel ---------------------
    doff = torch.arange(n, dtype=torch.int64, device=device) * rl
    dlen = torch.full((n,), rl, dtype=torch.int32, device=device)
    nbd = int(lib.ouro_tpraos_pack_bytes(n))
    darena = torch.empty(nbd, dtype=torch.uint8, device=device)
    dstatus = torch.empty(n, dtype=torch.uint8, device=device)
    dv = torch.empty(n, dtype=torch.uint8, device=device)
    dbe = torch.empty(n * 64, dtype=torch.uint8, device=device)
    dbl = torch.empty(n * 64, dtype=torch.uint8, device=device)
    st = torch.cuda.current_stream()
    S = V(st.cuda_stream)

    def dev_batch(lo, m, arena_t, out):
        rc = lib.ouro_tpraos_pack_cbor_device(
            S, V(raw.data_ptr()), raw.numel(), V(doff.data_ptr() + 8 * lo), V(dlen.data_ptr() + 4 * lo),
            m, 129600, V(arena_t.data_ptr()), arena_t.numel(), ctypes.byref(out), None, None,
            V(dstatus.data_ptr() + lo))
        _native.check(rc, "ouro_tpraos_pack_cbor_device")
        out.eta_alpha = t["eta_alpha"].data_ptr() + 32 * lo
        out.leader_alpha = t["leader_alpha"].data_ptr() + 32 * lo
        rc = lib.ouro_tpraos_verify_batch_device(S, ctypes.byref(out), V(dv.data_ptr() + lo),
                                                 V(dbe.data_ptr() + 64 * lo),
                                                 V(dbl.data_ptr() + 64 * lo))
        _native.check(rc, "ouro_tpraos_verify_batch_device")

    out = _native.TPraosBatch()
    dev_batch(0, n, darena, out)  # warm
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        dev_batch(0, n, darena, out)
        e1.record(st)
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    pk = []
    for _ in range(reps):  # the device slicer alone
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        _native.check(lib.ouro_tpraos_pack_cbor_device(
            S, V(raw.data_ptr()), raw.numel(), V(doff.data_ptr()), V(dlen.data_ptr()), n, 129600,
            V(darena.data_ptr()), nbd, ctypes.byref(_native.TPraosBatch()), None, None,
            V(dstatus.data_ptr())), "pack")
        e1.record(st)
        torch.cuda.synchronize()
        pk.append(e0.elapsed_time(e1))
    dev_ok = bool((dstatus == 0).all().item() and (dv == 0x3F).all().item())
    res["device"] = {"headers_per_s": round(n / (min(ts) * 1e-3), 1), "ms": round(min(ts), 3),
                     "slicer_ms": round(min(pk), 3), "all_valid": dev_ok}

    # ---- pcie: pinned host raw, chunked upload overlapping slice + kernel ---
    rawh = raw.cpu().pin_memory()
    pch = 1 << 17
    nchp = (n + pch - 1) // pch
    arenas = [torch.empty(int(lib.ouro_tpraos_pack_bytes(pch)), dtype=torch.uint8, device=device)
              for _ in range(2)]
    copy_st = torch.cuda.Stream()
    vh = torch.empty(n, dtype=torch.uint8).pin_memory()
    beh = torch.empty(n * 64, dtype=torch.uint8).pin_memory()
    blh = torch.empty(n * 64, dtype=torch.uint8).pin_memory()

    def run_pcie():
        evs = []
        for k in range(nchp):
            lo, m = k * pch, min(pch, n - k * pch)
            with torch.cuda.stream(copy_st):
                raw[lo * rl:(lo + m) * rl].copy_(rawh[lo * rl:(lo + m) * rl], non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(copy_st)
            evs.append(ev)
        for k in range(nchp):
            lo, m = k * pch, min(pch, n - k * pch)
            st.wait_event(evs[k])
            dev_batch(lo, m, arenas[k % 2], _native.TPraosBatch())
        vh.copy_(dv, non_blocking=True)
        beh.copy_(dbe, non_blocking=True)
        blh.copy_(dbl, non_blocking=True)
        torch.cuda.synchronize()

    run_pcie()
    best = min(_timed(run_pcie) for _ in range(reps))
    res["pcie"] = {"headers_per_s": round(n / best, 1), "ms": round(best * 1e3, 2),
                   "h2d_bytes": int(n * rl), "chunk": pch,
                   "all_valid": bool((vh == 0x3F).all().item())}
    del rawh, arenas, darena

    # ---- host: pageable raw -> C slicer -> host-buffer verify ---------------
    rawh = raw.cpu().numpy()
    del raw
    ea = t["eta_alpha"].cpu().numpy()
    la = t["leader_alpha"].cpu().numpy()
    del t
    chunk = chunk or max(1, (n + 1) // 2)
    off = np.arange(n, dtype=np.uint64) * rl
    ln = np.full(n, rl, np.uint32)
    nch = (n + chunk - 1) // chunk
    harenas = [np.zeros(lib.ouro_tpraos_pack_bytes(chunk), np.uint8) for _ in range(2)]
    status = np.zeros(n, np.uint8)
    verdict = np.zeros(n, np.uint8)
    be = np.zeros((n, 64), np.uint8)
    bl = np.zeros((n, 64), np.uint8)
    structs = [_native.TPraosBatch() for _ in range(nch)]

    def pack(k):
        lo = k * chunk
        m = min(chunk, n - lo)
        a = harenas[k % 2]
        rc = lib.ouro_tpraos_pack_cbor(P(rawh), rawh.size, P(off[lo:]), P(ln[lo:]), m, 129600,
                                       P(a), a.size, ctypes.byref(structs[k]), None, None,
                                       P(status[lo:]), threads)
        assert rc == 0, rc
        structs[k].eta_alpha = ea.ctypes.data + 32 * lo
        structs[k].leader_alpha = la.ctypes.data + 32 * lo

    def verify(k):
        lo = k * chunk
        rc = lib.ouro_tpraos_verify_batch(ctypes.byref(structs[k]), P(verdict[lo:]), P(be[lo:]),
                                          P(bl[lo:]))
        _native.check(rc, "ouro_tpraos_verify_batch")

    def run_host():
        pack(0)
        for k in range(nch):
            th = None
            if k + 1 < nch:
                # arena (k+1) % 2 is free: chunk k-1's verify has returned
                th = threading.Thread(target=pack, args=(k + 1,))
                th.start()
            verify(k)
            if th:
                th.join()

    run_host()  # warm: device buffers, pinned staging, arena pages
    best = min(_timed(run_host) for _ in range(reps))
    ok = bool((status == 0).all() and ((verdict & 0x3F) == 0x3F).all())
    pk_t = []
    for _ in range(reps):
        t0 = time.perf_counter()
        for k in range(nch):
            pack(k)
        pk_t.append(time.perf_counter() - t0)
    res["host"] = {"headers_per_s": round(n / best, 1), "ms": round(best * 1e3, 2),
                   "slicer_headers_per_s": round(n / min(pk_t), 1), "slicer_threads": threads,
                   "chunk": chunk, "all_valid": ok}
    res["workload"] = (f"{n} raw wire headers ({rl} B each): device = HBM-resident raw -> device "
                       "slicer -> header kernel; pcie = pinned host raw uploaded in 128K-header "
                       "chunks overlapping slice + kernel, results back; host = pageable raw -> "
                       "C slicer -> ouro_tpraos_verify_batch")
    return res


def integrity_leg(n: int, npools: int, device, reps: int = 3):
    """Storage integrity straight from raw CBOR: the
    KES-only verifyHeaderIntegrity
    (ouroboros-consensus-shelley/src/Ouroboros/Consensus/Shelley/Ledger/Integrity.hs:20-44)
    that the VolatileDB parser runs on every block at open (Storage/VolatileDB/
    Impl/Parser.hs:66-85) and ImmutableDB chunk validation on every block of a
    chunk (Storage/ImmutableDB/Impl/Validation.hs:358-365), over n synthetic
    raw headers: HBM-resident (ouro_integrity_verify_cbor_device: device
    slicer + Sum6KES kernel) and from pageable host memory in one call
    (ouro_integrity_verify_cbor: host slicer, H2D, kernel, D2H).  Never `value`."""
    import torch

    from ouroboros_network_amd import _native

    t, raw, rl = synth_raw_headers(n, npools, device)
    lib = _native.load()
    V = ctypes.c_void_p
    st = torch.cuda.current_stream()
    S = V(st.cuda_stream)
    doff = torch.arange(n, dtype=torch.int64, device=device) * rl
    dlen = torch.full((n,), rl, dtype=torch.int32, device=device)
    nb = int(lib.ouro_tpraos_pack_bytes(n))
    arena = torch.empty(nb, dtype=torch.uint8, device=device)
    status = torch.empty(n, dtype=torch.uint8, device=device)
    ver = torch.empty(n, dtype=torch.uint8, device=device)

    def go():
        _native.check(lib.ouro_integrity_verify_cbor_device(
            S, V(raw.data_ptr()), raw.numel(), V(doff.data_ptr()), V(dlen.data_ptr()), n, 129600,
            V(arena.data_ptr()), nb, V(status.data_ptr()), V(ver.data_ptr())),
            "ouro_integrity_verify_cbor_device")

    go()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        go()
        e1.record(st)
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    dms = min(ts)
    all_ok = bool((ver == 1).all().item()) and bool((status == 0).all().item())
    hraw = raw.cpu().numpy()
    hoff = doff.cpu().numpy().astype(np.uint64)
    hlen = dlen.cpu().numpy().astype(np.uint32)
    hst = np.zeros(n, np.uint8)
    hv = np.zeros(n, np.uint8)
    P = lambda a: a.ctypes.data_as(V)  # noqa: E731

    def host():
        _native.check(lib.ouro_integrity_verify_cbor(P(hraw), hraw.size, P(hoff), P(hlen), n,
                                                     129600, P(hst), P(hv)),
                      "ouro_integrity_verify_cbor")

    host()
    th = min(_timed(host) for _ in range(reps))
    return {"workload": f"{n} synthetic raw Shelley headers ({rl} B each), KES-only "
                        "verifyHeaderIntegrity from raw CBOR",
            "device_resident": {"headers_per_s": round(n / (dms * 1e-3), 1),
                                "ms": round(dms, 3), "all_valid": all_ok},
            "host_buffers_one_call": {"headers_per_s": round(n / th, 1), "ms": round(th * 1e3, 2),
                                      "equals_device": bool((hv == ver.cpu().numpy()).all()),
                                      "note": "host slicer + PCIe + kernel + D2H"}}


def cbor_abi_leg(n: int, npools: int, device, reps: int = 3, multi_devices=None):
    """Raw wire CBOR in PAGEABLE host memory -> verdicts in ONE C-ABI call, no
    torch in the timed region: what
    the reference's bulk callers -- ChainDB suffix re-validation
    (ouroboros-consensus/src/Ouroboros/Consensus/Storage/ChainDB/Impl/LgrDB.hs:350-368),
    ChainSync windows (.../MiniProtocol/ChainSync/Client.hs:792), storage
    integrity (.../Storage/VolatileDB/Impl/Parser.hs:66-85) -- get through the
    FFI.  n synthetic headers in the node's configuration (VRF inputs derived
    on the device from each header's slot and eta0; claimed outputs checked;
    both VRF outputs and the eta nonce returned):
      tpraos     ouro_tpraos_verify_cbor (the raw-CBOR pipeline: gather into
                 pinned staging, upload, device slicer, header kernel, results)
      integrity  ouro_integrity_verify_cbor on the same bytes (Sum6KES only)
    and, as res["inproc_cbor"], the one-process multi-device forms
    (ouro_tpraos_verify_cbor_multi / ouro_integrity_verify_cbor_multi) over
    `multi_devices` -- every visible device; [0, 0] on a one-GPU box, two
    pooled workers sharing it.
    Wall clock around the ctypes call; never `value` (PCIe-inclusive)."""
    import torch

    from ouroboros_network_amd import _native

    eta0 = bytes(range(101, 133))
    raw, rl = synth_raw_node_headers(n, npools, device, eta0)
    buf = raw.cpu().numpy()  # pageable host memory, as the caller's ByteStrings
    del raw
    torch.cuda.empty_cache()
    lib = _native.load()
    P = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    off = np.arange(n, dtype=np.uint64) * rl
    ln = np.full(n, rl, np.uint32)
    e0 = np.frombuffer(eta0, np.uint8).copy()
    status = np.zeros(n, np.uint8)
    verdict = np.zeros(n, np.uint8)
    be = np.zeros((n, 64), np.uint8)
    bl = np.zeros((n, 64), np.uint8)
    en = np.zeros((n, 32), np.uint8)
    stats = np.zeros(6)

    def tpraos():
        _native.check(lib.ouro_tpraos_verify_cbor(
            P(buf), buf.size, P(off), P(ln), n, 129600, P(e0), None, None, P(status),
            P(verdict), P(be), P(bl), P(en)), "ouro_tpraos_verify_cbor")

    def integrity():
        _native.check(lib.ouro_integrity_verify_cbor(P(buf), buf.size, P(off), P(ln), n, 129600,
                                                     P(status), P(verdict)),
                      "ouro_integrity_verify_cbor")

    res = {"workload": f"{n} raw wire headers ({rl} B each, {n * rl / 2**30:.2f} GiB) in pageable "
                       "host memory, node configuration (mkSeed on the device from each "
                       "header's slot and eta0), one C-ABI call each",
           "raw_bytes_per_header": rl}
    devs = np.ascontiguousarray(multi_devices or [0], np.int32)

    def tpraos_multi():
        _native.check(lib.ouro_tpraos_verify_cbor_multi(
            P(devs), int(devs.size), P(buf), buf.size, P(off), P(ln), n, 129600, P(e0), None,
            None, P(status), P(verdict), P(be), P(bl), P(en)), "ouro_tpraos_verify_cbor_multi")

    def integrity_multi():
        _native.check(lib.ouro_integrity_verify_cbor_multi(
            P(devs), int(devs.size), P(buf), buf.size, P(off), P(ln), n, 129600, P(status),
            P(verdict)), "ouro_integrity_verify_cbor_multi")

    multi = {"devices": devs.tolist(),
             "note": "one process, contiguous shards on pooled NUMA-bound workers, one per "
                     "listed device (SURVEY.md §8(e)); on a one-GPU box [0, 0] (two shards "
                     "sharing the GPU)"}
    for name, fn, ok in (("tpraos", tpraos_multi, lambda: ((verdict & 0x3F) == 0x3F).all()),
                         ("integrity", integrity_multi, lambda: (verdict == 1).all())):
        fn()
        verdict[:] = 0
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        multi[name] = {"headers_per_s": round(n / min(ts), 1), "ms": round(min(ts) * 1e3, 2),
                       "all_valid": bool(ok() and (status == 0).all())}
    for name, fn, ok in (("tpraos", tpraos, lambda: ((verdict & 0x3F) == 0x3F).all()),
                         ("integrity", integrity, lambda: (verdict == 1).all())):
        fn()  # warm: pinned staging and device buffers grown, pool threads started
        verdict[:] = 0
        ts, st = [], []
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
            lib.ouro_debug_cbor_stats(stats.ctypes.data)
            st.append(stats.copy())
        k = int(np.argmin(ts))
        res[name] = {"headers_per_s": round(n / ts[k], 1), "ms": round(ts[k] * 1e3, 2),
                     "gather_ms": round(st[k][1], 2), "wait_ms": round(st[k][2], 2),
                     "chunks": int(st[k][3]), "slots": int(st[k][4]),
                     "copy_threads": int(st[k][5]),
                     "all_valid": bool(ok() and (status == 0).all())}
    res["inproc_cbor"] = multi
    return res


def byron_leg(n: int, threads: int, reps: int = 3):
    """Raw Byron header CBOR -> verdicts: the golden
    Byron headers (tests/golden/reference_kats.json "byron_wire": N2N v1 and
    Cardano HFC forms, regular and epoch-boundary) repeated to n, host memory.
      pack        the C slicer alone (ouro_byron_pack_cbor, `threads` host threads)
      verify_cbor slicer + ByronDSIGN batch verify on the GPU in one call
                  (ouro_byron_verify_cbor: H2D of the messages, kernel, D2H)
      python      the per-header Python slicer (byron.parse_byron_header) on a
                  sample, for contrast
    Real keys and signatures (the golden ones, so every row is the same
    work); never `value`."""
    from ouroboros_network_amd import byron as B

    with open(os.path.join(ROOT, "tests", "golden", "reference_kats.json")) as f:
        wires = [bytes.fromhex(w["raw"]) for w in json.load(f)["byron_wire"]]
    raws = [wires[i % len(wires)] for i in range(n)]
    ln = np.array([len(r) for r in raws], np.uint32)
    off = np.zeros(n, np.uint64)
    off[1:] = np.cumsum(ln[:-1], dtype=np.uint64)
    arg = (np.frombuffer(b"".join(raws), np.uint8), off, ln)
    magic = B.HEADER_MAGIC  # the golden wire forms carry the test network's own magic
    B.pack_byron_cbor(arg, magic, nthreads=threads)  # warm
    tp = min(_timed(lambda: B.pack_byron_cbor(arg, magic, nthreads=threads)) for _ in range(reps))
    v, st = B.verify_byron_cbor(arg, magic)  # warm
    tv = min(_timed(lambda: B.verify_byron_cbor(arg, magic)) for _ in range(reps))
    import torch

    ndev = torch.cuda.device_count()
    mdevs = list(range(ndev)) if ndev > 1 else [0, 0]
    vm, _ = B.verify_byron_cbor(arg, magic, devices=mdevs)  # warm
    tm = min(_timed(lambda: B.verify_byron_cbor(arg, magic, devices=mdevs)) for _ in range(reps))
    m = min(n, 4096)
    t0 = time.perf_counter()
    for r in raws[:m]:
        B.byron_status(r)
    tpy = time.perf_counter() - t0
    # delegation certificates: the golden regular header's own certificate
    # repeated to n (ouro_byron_dlg_cert_verify_batch: messages built on the
    # host, ByronDSIGN kernel), every eighth with one signature bit flipped
    h = next(x for x in (B.byron_status(w)[1] for w in wires) if x is not None)
    iss = np.tile(np.frombuffer(h.issuer_xpub, np.uint8), (n, 1))
    dlg = np.tile(np.frombuffer(h.delegate_xpub, np.uint8), (n, 1))
    sig = np.tile(np.frombuffer(h.cert_sig, np.uint8), (n, 1))
    sig[::8, 5] ^= 0x20
    ep = np.full(n, h.cert_epoch, np.uint64)
    dv = B.verify_delegation_certs(iss, dlg, ep, sig, h.magic)  # warm
    td = min(_timed(lambda: B.verify_delegation_certs(iss, dlg, ep, sig, h.magic))
             for _ in range(reps))
    bad = np.zeros(n, bool)
    bad[::8] = True
    dlg_out = {"certificates": n, "certs_per_s": round(n / td, 1),
               "verdicts_as_expected": bool((dv == ~bad).all()),
               "note": "golden certificate repeated, 1/8 with a flipped signature bit; host "
                       "arrays in, verdicts out"}
    return {"headers": n, "all_valid": bool(v.all()),
            "boundary_headers": int((st == B.PACK_EBB).sum()),
            "pack_headers_per_s": round(n / tp, 1), "pack_threads": threads,
            "verify_cbor_headers_per_s": round(n / tv, 1),
            "verify_cbor_multi": {"devices": mdevs, "headers_per_s": round(n / tm, 1),
                                  "equals_one_device": bool((vm == v).all())},
            "python_slicer_headers_per_s": round(m / tpy, 1),
            "delegation_certificates": dlg_out,
            "note": "golden Byron headers repeated; pageable host memory in, verdicts out; "
                    "since round 6 on the raw-CBOR pipeline (pinned staging, device Byron "
                    "slicer, ByronDSIGN kernel, 5 chunks in flight)"}


def _timed(fn) -> float:
    t0 = time.perf_counter()
    fn()
    return time.perf_counter() - t0


def load_pmc_traffic():
    """HBM bytes per header of one header-kernel launch from the committed PMC
    run (profiles/pmc_traffic.json, tools/summarize_profile.py), with whether
    that run measured THIS source (its stamped source_hash), and the same
    run's box-independent counters: VALU lane-instructions per header
    (SQ_INSTS_VALU) and the clock it ran at (GRBM_GUI_ACTIVE / 8 / wall)."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None, {}
    return d.get("k_tpraos_verify_bytes_per_launch_per_header"), {
        "traffic_round": d.get("round"), "traffic_source_hash": d.get("source_hash"),
        "traffic_matches_source": d.get("source_hash") == source_hash(),
        "valu_lane_insts_per_header": d.get("valu_lane_insts_per_header"),
        "pmc_clock_ghz": d.get("clock_ghz")}


def load_component_traffic():
    """HBM bytes per item of the standalone kernels from the committed
    component PMC run (profiles/pmc_traffic_components.json,
    tools/collect_components.py), with whether it measured THIS source."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic_components.json")
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return {}
    meta = {"traffic_tag": d.get("tag"), "traffic_source_hash": d.get("source_hash"),
            "traffic_matches_source": d.get("source_hash") == source_hash()}
    return {leg: {"traffic_per_item": round(v["hbm_bytes_per_item"], 1), "traffic_kernel": v["kernel"],
                  **meta}
            for leg, v in d.items() if isinstance(v, dict) and "hbm_bytes_per_item" in v}


def single_item_leg(ed, hdr, iters: int = 300):
    """Per-call wall latency of the ABI-identical single-item symbols -- the
    number a per-item Haskell FFI caller sees -- on both routes: the library's
    host path (the default since round 4: the kernels' lane routines compiled
    for the CPU) and the GPU (OURO_SINGLE_ITEM=gpu: a one-item batch, H2D,
    one wave, D2H), next to the reference's own libsodium call on the host;
    host_path_lanes = the round-4 host path (the kernels' lane routines
    compiled for the CPU, OURO_HOST_IMPL=lanes) for comparison."""
    from ouroboros_network_amd import _native

    lib = _native.load()
    pk, sig, msg = (x[: iters * w].cpu().numpy().tobytes() for x, w in
                    ((ed[0], 32), (ed[1], 64), (ed[2], 32)))
    items = [(sig[64 * i:64 * i + 64], msg[32 * i:32 * i + 32], pk[32 * i:32 * i + 32])
             for i in range(iters)]
    vk = hdr.t["vrf_vk"][: iters * 32].cpu().numpy().tobytes()
    pi = hdr.t["eta_proof"][: iters * 80].cpu().numpy().tobytes()
    al = hdr.t["eta_alpha"][: iters * 32].cpu().numpy().tobytes()
    vitems = [(vk[32 * i:32 * i + 32], pi[80 * i:80 * i + 80], al[32 * i:32 * i + 32])
              for i in range(iters)]
    out = ctypes.create_string_buffer(64)

    def lat(fn):
        fn(0)
        t = np.empty(iters)
        for i in range(iters):
            t0 = time.perf_counter()
            rc = fn(i)
            t[i] = time.perf_counter() - t0
            if rc != 0:
                raise RuntimeError(f"single-item call rejected a valid item ({rc})")
        return {"p50_us": round(float(np.percentile(t, 50)) * 1e6, 1),
                "p99_us": round(float(np.percentile(t, 99)) * 1e6, 1)}

    shim = _native.load_shim()

    def route(r):
        with _native.knob_env(OURO_SINGLE_ITEM=r):
            return {
                "ouro_ed25519_verify": lat(lambda i: lib.ouro_ed25519_verify(
                    items[i][0], items[i][1], 32, items[i][2])),
                "ouro_vrf03_verify": lat(lambda i: lib.ouro_vrf03_verify(
                    out, vitems[i][0], vitems[i][1], vitems[i][2], 32)),
                "crypto_vrf_ietfdraft03_verify (opt-in shim)": lat(
                    lambda i: shim.crypto_vrf_ietfdraft03_verify(out, vitems[i][0], vitems[i][1],
                                                                 vitems[i][2], 32))}

    def lanes_route():
        with _native.knob_env(OURO_HOST_IMPL="lanes"):
            return route("host")

    res = {"workload": f"{iters} single-item calls, valid synthetic items, one thread",
           "routing": "single items run on the library's host path by default "
                      "(include/ouro_verify.h; since round 5 its own 5 x 51-bit CPU arithmetic, "
                      "csrc/host_fast.h); OURO_SINGLE_ITEM=gpu sends them to the device",
           "host_path": route("host"), "host_path_lanes": lanes_route(), "gpu": route("gpu")}
    # the default route's figures at the top level (the names the ABI exports)
    res.update(res["host_path"])
    if os.path.exists(SODIUM_SO):
        so = ctypes.CDLL(SODIUM_SO)
        so.sodium_init()
        fn = so.crypto_sign_ed25519_verify_detached
        fn.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_ulonglong, ctypes.c_char_p]
        res["libsodium_ed25519_host"] = lat(lambda i: fn(items[i][0], items[i][1], 32,
                                                         items[i][2]))
        res["libsodium_ed25519_host"]["kind"] = "reference (ctypes per call, ~1 us of it)"
    return res


def step_shards(world: int, rank: int, headers: int, global_headers: int, weak: bool):
    """This rank's share of a step: (strong, n, first, n_global).  N = 1: one
    batch of `headers`.  N > 1: configs[3] as written by default -- ONE batch
    of 1,048,576 (or global_headers) headers cut into N/G contiguous shards
     -- or, with `weak` / global_headers = 0, `headers`
    per rank (global headers [rank*n, (rank+1)*n))."""
    from ouroboros_network_amd.shard import shard_range

    if global_headers < 0:
        global_headers = 0 if (world == 1 or weak) else (1 << 20)
    if global_headers > 0:
        lo, hi = shard_range(global_headers, world, rank)
        if hi == lo:
            raise SystemExit("more ranks than headers")
        return True, hi - lo, lo, global_headers
    return False, headers, rank * headers, headers * world


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--headers", type=int, default=1 << 20,
                    help="headers per GPU per step (weak scaling; the N = 1 batch)")
    ap.add_argument("--global-headers", type=int, default=-1,
                    help="strong scaling: ONE batch of this many headers per step, cut into "
                         "N/G contiguous shards (default for N > 1: 1,048,576, configs[3] as "
                         "written; 0 = weak scaling)")
    ap.add_argument("--weak", action="store_true",
                    help="N > 1: weak scaling (--headers per GPU) as the line")
    ap.add_argument("--pools", type=int, default=1024)
    ap.add_argument("--cpu-sample", type=int, default=65536)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-extras", action="store_true")
    ap.add_argument("--no-latency", action="store_true")
    ap.add_argument("--no-e2e", action="store_true",
                    help="skip the host-buffer (PCIe-inclusive) end-to-end leg")
    ap.add_argument("--lat-iters", type=int, default=10000,
                    help="configs[4] 64-header plan launches timed for p50/p99/p99.9 "
                         "(SURVEY.md §8(d) C5: >= 10,000)")
    ap.add_argument("--lat-cpu-iters", type=int, default=50)
    ap.add_argument("--components-only", action="store_true",
                    help="time only the standalone Ed25519 / VRF / Sum6KES kernels over --headers "
                         "items (the profiling run of tools/profile_components.sh)")
    ap.add_argument("--inproc", default=None,
                    help="comma-separated device list (e.g. 0,1,2,3 or 0,0): also time "
                         "ouro_tpraos_verify_batch_multi over those devices in this one process "
                         "(the one-process node's multi-GPU path; key `inproc`)")
    ap.add_argument("--dist-backend", default="nccl",
                    help="nccl (RCCL over xGMI, the real path) or gloo (rehearsal of the "
                         "multi-rank path on fewer GPUs: ranks share devices, gather via host)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            raise SystemExit("--gpus > 1 must be launched with torch.distributed.run")
    gpu = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(gpu)
    device = torch.device("cuda", gpu)
    from ouroboros_network_amd import _native

    _native.load().ouro_set_device(gpu)
    # this rank's host side on its GPU's NUMA node: threads
    # created from here on inherit the binding; -1 = unknown (left alone)
    numa_node = _native.load().ouro_bind_thread_to_device(gpu)
    if world > 1:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group(args.dist_backend)
        # a multi-GPU line only from a real N-GPU world: N ranks, each on its
        # own GPU (the gloo rehearsal may share one); fails loudly otherwise
        from ouroboros_network_amd.shard import check_rank_devices

        topo = [None] * world
        dist.all_gather_object(topo, {"rank": rank, "device": gpu, "bus_id": pci_bus_id(device),
                                      "host": socket.gethostname()})
        check_rank_devices(topo, args.gpus, allow_shared=args.dist_backend != "nccl")

    from ouroboros_network_amd.shard import all_gather_results, pack_results

    strong, n, first, n_global = step_shards(world, rank, args.headers, args.global_headers,
                                             args.weak)
    t_syn = time.perf_counter()
    tensors, blen = synth_headers(n, args.pools, device, first=first)
    syn_s = time.perf_counter() - t_syn
    hdr = DeviceHeaders(tensors, n, device)
    stream = torch.cuda.current_stream()
    if args.components_only:
        # one header launch (the VRF leg compares its outputs), then each
        # standalone kernel: 1 warm + --steps timed launches over n items
        hdr.launch(stream)
        torch.cuda.synchronize()
        out = {"components_only": True, "n": n, "steps": args.steps, "source_hash": source_hash()}
        out["ed25519"], _ = ed25519_rate(device, n, args.steps)
        out.update(component_rates(hdr, n, args.steps))
        print(json.dumps(out))
        return

    def gather():
        # the one collective of the path: every rank receives all verdicts and
        # VRF outputs (RCCL all-gather over xGMI), SURVEY.md §8(e)
        local = pack_results(hdr.verdict, hdr.beta_eta, hdr.beta_leader)
        if args.dist_backend != "nccl":
            local = local.cpu()
        return all_gather_results(local, n_global, world)

    # the collective of step k runs on its own stream, overlapped with the
    # kernel of step k+1 (double-buffered outputs); a set is rewritten only
    # after the gather that read it has finished
    comm = torch.cuda.Stream(device) if world > 1 else None
    gdone = [None, None]

    def step(k: int) -> None:
        s = k % 2
        if gdone[s] is not None:
            stream.wait_event(gdone[s])
        hdr.use(s)
        hdr.launch(stream)
        if world > 1:
            kev = torch.cuda.Event()
            kev.record(stream)
            with torch.cuda.stream(comm):
                comm.wait_event(kev)
                gather()
                done = torch.cuda.Event()
                done.record(comm)
                gdone[s] = done

    for w in range(args.warmup):
        step(w)
    torch.cuda.synchronize()
    # correctness gate: every synthetic header must verify
    all_ok = bool(((hdr.verdict & 15) == 15).all().item())  # masks: ouro_verify.h

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.steps)]
    t0 = time.perf_counter()
    for k in range(args.steps):
        s = (args.warmup + k) % 2
        if gdone[s] is not None:
            stream.wait_event(gdone[s])
        hdr.use(s)
        ev[k][0].record(stream)
        hdr.launch(stream)
        ev[k][1].record(stream)
        if world > 1:
            with torch.cuda.stream(comm):
                comm.wait_event(ev[k][1])
                gather()
                done = torch.cuda.Event()
                done.record(comm)
                gdone[s] = done
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    if world > 1:
        red_dev = device if args.dist_backend == "nccl" else torch.device("cpu")
        tt = torch.tensor([elapsed], dtype=torch.float64, device=red_dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
        ok_t = torch.tensor([1 if all_ok else 0], dtype=torch.int32, device=red_dev)
        dist.all_reduce(ok_t, op=dist.ReduceOp.MIN)
        all_ok = bool(ok_t.item())

    total = n_global * args.steps
    value = total / elapsed
    ms_per_step = elapsed / args.steps * 1e3
    dist_info = None
    if world > 1:
        # what the process group itself reports, and every rank's kernel time
        per_rank = [None] * world
        try:
            bw = h2d_gbps(device)
        except Exception:  # noqa: BLE001
            bw = None
        dist.all_gather_object(per_rank, {"rank": rank, "device": gpu, "headers": n,
                                          "bus_id": pci_bus_id(device),
                                          "kernel_ms": round(kern_ms, 3),
                                          "numa_node": numa_node, "h2d_gb_per_s": bw})
        dist_info = {"world_size_seen": dist.get_world_size(), "backend": dist.get_backend(),
                     "per_rank": per_rank}
        if strong:
            # the weak-scaling figure beside the strong line: each rank
            # re-verifies its N/G shard G times per step (1,048,576 headers of
            # kernel work per GPU per step when G divides it), then gathers
            torch.cuda.synchronize()
            dist.barrier()
            tw = time.perf_counter()
            for k in range(args.steps):
                hdr.use(0)
                for _ in range(world):
                    hdr.launch(stream)
                gather()
            torch.cuda.synchronize()
            dist.barrier()
            ew = time.perf_counter() - tw
            red_dev = device if args.dist_backend == "nccl" else torch.device("cpu")
            tt = torch.tensor([ew], dtype=torch.float64, device=red_dev)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            ew = float(tt.item())
            dist_info["weak"] = {
                "value": round(n * world * world * args.steps / ew, 1), "unit": "headers/s",
                "headers_per_gpu_per_step": n * world, "ms_per_step": round(ew / args.steps * 1e3, 3),
                "how": "each rank verifies its N/G shard G times per step, then the all-gather"}

    if rank == 0:
        peak = None
        try:
            peak = measure_peak_mac(device)
        except Exception as e:  # noqa: BLE001
            print(f"# peak microbench failed: {e}", file=sys.stderr)
        achieved = n * MACS_PER_HEADER / (kern_ms * 1e-3) / 1e12
        traffic_per_header, traffic_meta = load_pmc_traffic()
        # box-independent companions of frac: the clock
        # the header kernel itself ran at on this box (diagnostic stamp
        # build), the INT32 issue ceiling at that clock, the MADs the code
        # executes, and the committed SQ / traffic counters per header
        clk, clk_how = None, "not measured (--no-extras: the profiling runs)"
        if not args.no_extras:
            try:
                clk, clk_how = kernel_clock_ghz(hdr, stream)
            except Exception as e:  # noqa: BLE001
                clk, clk_how = None, f"clock probe failed: {e}"
        cus = torch.cuda.get_device_properties(device).multi_processor_count
        ceiling = cus * 64 * clk * 1e9 / 1e12 if clk else None
        work = executed_work_per_header()
        exec_mads = work["executed_mads_per_header"] if work else None
        roof = {
            "bound": "valu",
            "kernel": "k_tpraos_verify",
            "achieved": round(achieved, 3),
            "peak": round(peak, 3) if peak else None,
            "unit": "TMAC/s",
            "frac": round(achieved / peak, 4) if peak else None,
            "frac_clock": round(achieved / ceiling, 4) if ceiling else None,
            "clock_ghz": round(clk, 4) if clk else None,
            "clock_how": clk_how,
            "int32_ceiling_at_clock": round(ceiling, 3) if ceiling else None,
            "int32_ceiling_note": f"{cus} CU x 64 lanes x clock_ghz: one 32-bit VALU op "
                                  "per lane per clock",
            "executed_mads_per_header": exec_mads,
            "executed_mad_rate": (round(n * exec_mads / (kern_ms * 1e-3) / 1e12, 3)
                                  if exec_mads else None),
            "frac_clock_executed": (round(n * exec_mads / (kern_ms * 1e-3) / 1e12 / ceiling, 4)
                                    if exec_mads and ceiling else None),
            "field_ops_per_header": ({"mul": work["field_mul"], "sq": work["field_sq"]}
                                     if work else None),
            "traffic": (round(traffic_per_header * n) if traffic_per_header else None),
            "traffic_note": "HBM bytes per launch from the committed PMC pass named by "
                            "traffic_round (FETCH_SIZE x 2 + WRITE_SIZE per the guide's gfx950 "
                            "correction); traffic_matches_source says whether it measured this "
                            "source",
            "traffic_per_header": (round(traffic_per_header, 1) if traffic_per_header else None),
            "algorithmic_bytes_per_header": 1537,
            "traffic_ratio": (round(traffic_per_header / 1537, 1) if traffic_per_header else None),
            "macs_per_header": MACS_PER_HEADER,
            "kernel_ms_per_launch": round(kern_ms, 3),
            "source_hash": source_hash(),
            **traffic_meta,
        }
        out = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "headers/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None,
            "dtype": "u32/u64 (GF(2^255-19) int limbs)",
            "data": "synthetic (device-signed, deterministic seeds)",
            "config": {"workload": "tpraos_header_batch (configs[3])",
                       "headers_per_gpu": n, "global_batch": n_global,
                       "pools": args.pools, "body_bytes": blen,
                       "parallelism": f"shard{world}"},
            "all_valid": all_ok,
            "numa_node": numa_node,
            "synth_s": round(syn_s, 2),
            "roofline": roof,
        }
        if dist_info:
            out["distributed"] = dist_info
        cpu = host_cpu_info()
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle_ffi as O

        oracle_build = native_oracle(O) if not args.no_cpu else None
        ed = None
        if not args.no_extras:
            try:
                out["ed25519"], ed = ed25519_rate(device, 1 << 20, 3)
                if peak:
                    out["ed25519"]["roofline_frac"] = round(out["ed25519"]["roofline_frac"] / peak, 4)
                if not args.no_cpu and world == 1:
                    out["ed25519"]["cpu_libsodium"] = libsodium_ed25519_rate(*ed, cpu, 262144)
            except Exception as e:  # noqa: BLE001
                out["ed25519"] = {"error": str(e)}
            try:
                comp = component_rates(hdr, n)
                for k, val in comp.items():
                    if peak and "achieved_tmacs" in val:
                        val["roofline_frac"] = round(val["achieved_tmacs"] / peak, 4)
                    out[k] = val
            except Exception as e:  # noqa: BLE001
                out["components_error"] = str(e)
            # each standalone kernel's HBM traffic per item from its committed
            # rocprofv3 PMC run (profiles/r03*/components), stamped with the
            # source hash it measured
            for leg, tr in load_component_traffic().items():
                if leg in out and isinstance(out[leg], dict) and "error" not in out[leg]:
                    out[leg]["traffic"] = tr
            if ed is not None and world == 1:
                try:
                    out["single_item"] = single_item_leg(ed, hdr)
                except Exception as e:  # noqa: BLE001
                    out["single_item"] = {"error": str(e)}
        if not args.no_e2e and world == 1:
            try:
                out["e2e"] = e2e_leg(hdr, n)
            except Exception as e:  # noqa: BLE001
                out["e2e"] = {"error": str(e)}
        if not args.no_e2e and world == 1:
            try:
                out["raw_cbor"] = raw_leg(n, args.pools, device, cpu["usable"])
            except Exception as e:  # noqa: BLE001
                out["raw_cbor"] = {"error": str(e)}
        if args.inproc and world == 1:
            try:
                out["inproc"] = inproc_leg(hdr, n, [int(x) for x in args.inproc.split(",")])
            except Exception as e:  # noqa: BLE001
                out["inproc"] = {"error": str(e)}
        if not args.no_e2e and world == 1:
            try:
                # the one-process multi-device entries over every visible
                # device ([0, 0] on a one-GPU box: two pooled workers)
                ndev = torch.cuda.device_count()
                mdevs = list(range(ndev)) if ndev > 1 else [0, 0]
                out["cbor_abi"] = cbor_abi_leg(n, args.pools, device, multi_devices=mdevs)
                out["inproc_cbor"] = out["cbor_abi"].pop("inproc_cbor")
            except Exception as e:  # noqa: BLE001
                out["cbor_abi"] = {"error": str(e)}
        if not args.no_e2e and world == 1:
            try:
                out["integrity_cbor"] = integrity_leg(n, args.pools, device)
            except Exception as e:  # noqa: BLE001
                out["integrity_cbor"] = {"error": str(e)}
        if not args.no_e2e and world == 1:
            try:
                out["byron_cbor"] = byron_leg(1 << 20, cpu["usable"])
            except Exception as e:  # noqa: BLE001
                out["byron_cbor"] = {"error": str(e)}
        if not args.no_latency and world == 1:
            try:
                nt, _, npool = synth_headers(64, args.pools, device, keep_pool=True)
                synth_node_config(nt, 64, args.pools, npool, bytes(range(7, 39)), device)
                node = DeviceHeaders(nt, 64, device)
                out["latency"] = latency_leg(hdr, 64, args.lat_iters, cpu["usable"],
                                             args.lat_cpu_iters, node=node)
            except Exception as e:  # noqa: BLE001
                out["latency"] = {"error": str(e)}
        if not args.no_cpu and world == 1:
            threads = cpu["usable"]
            m = min(args.cpu_sample, n)
            hb = hdr.host_sample(m)
            rate, dt, (cv, cbe, cbl) = cpu_baseline(hb, threads)
            m1 = min(2048, m)
            rate1, dt1, _ = cpu_baseline(hb.slice(0, m1), 1)
            gv = hdr.verdict[:m].cpu().numpy()
            gbe = hdr.beta_eta[: m * 64].cpu().numpy().reshape(m, 64)
            gbl = hdr.beta_leader[: m * 64].cpu().numpy().reshape(m, 64)
            out["cpu_baseline"] = {
                "value": round(rate, 1), "unit": "headers/s", "cores": threads,
                "kind": "port",
                "sample": f"first {m} of the same synthetic headers, oracle/ C port "
                          f"({oracle_build}), {threads} pthreads, {dt:.1f} s wall",
                "one_core": round(rate1, 1), "one_core_sample": m1,
                "thread_scaling": round(rate / rate1, 2),
                "host": cpu,
                "cores_note": (f"{threads} = the CPUs this job may use: the cgroup quota "
                               f"({cpu['cgroup_cpu_quota']}) / affinity of a {cpu['nproc']}-CPU "
                               "host -- a container limit, not the box's core count"),
                "why_port": "the reference's VRF C (cardano-crypto-praos) is not in the image; "
                            "the oracle restates it and is pinned to libsodium 1.0.18 + golden "
                            "vectors (DESIGN.md §2)",
                "gpu_equals_cpu_on_sample": bool((gv == cv).all() and (gbe == cbe).all()
                                                 and (gbl == cbl).all()),
            }
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
