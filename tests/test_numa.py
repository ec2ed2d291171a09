"""NUMA placement of each GPU's host side ("each GPU has its
own HIP stream and pinned-host staging (NUMA-local)"):
the device -> node mapping read from sysfs and the thread binding the
multi-device workers and bench.py's ranks get (csrc/numa.cpp), against a
mocked sysfs (OURO_SYSFS_ROOT).  CPU only: the binding logic is host code;
the GPU test checks the workers of ouro_tpraos_verify_batch_multi are bound
to their device's node on a real box.
"""
import ctypes
import os
import threading

import numpy as np
import pytest


def _sysfs(tmp_path, pci, nodes):
    for busid, node in pci.items():
        d = tmp_path / "bus" / "pci" / "devices" / busid
        d.mkdir(parents=True)
        (d / "numa_node").write_text(f"{node}\n")
    for node, cpulist in nodes.items():
        d = tmp_path / "devices" / "system" / "node" / f"node{node}"
        d.mkdir(parents=True)
        (d / "cpulist").write_text(cpulist + "\n")
    return str(tmp_path)


def _in_thread(fn):
    """Run fn in a fresh thread (a binding is per thread: pytest's own thread
    keeps its CPUs) and return its result."""
    out = {}

    def run():
        out["r"] = fn()

    t = threading.Thread(target=run)
    t.start()
    t.join()
    return out["r"]


def _thread_cpus(lib):
    buf = (ctypes.c_int * 1024)()
    k = lib.ouro_debug_thread_cpus(buf, 1024)
    return list(buf[:k])


@pytest.fixture(scope="module")
def lib():
    from ouroboros_network_amd import _native

    return _native.load()


def test_bind_to_a_pci_functions_node(lib, tmp_path):
    allowed = sorted(os.sched_getaffinity(0))
    if len(allowed) < 4:
        pytest.skip("needs 4 usable CPUs")
    want = allowed[1:3] + allowed[-1:]
    spec = ",".join(str(c) for c in want)
    root = _sysfs(tmp_path, {"0000:c1:00.0": 1, "0000:05:00.0": -1, "0000:06:00.0": 2,
                             "0000:07:00.0": 3},
                  {0: f"{allowed[0]}", 1: spec, 2: "100000-100003", 3: "0-x"})
    os.environ["OURO_SYSFS_ROOT"] = root
    try:
        def bind(busid):
            n = ctypes.c_int(-7)
            node = lib.ouro_debug_numa_bind_pci(busid.encode(), ctypes.byref(n))
            return node, n.value, _thread_cpus(lib)

        # upper-case bus ids as hipDeviceGetPCIBusId may return them
        node, n, cpus = _in_thread(lambda: bind("0000:C1:00.0"))
        assert (node, n, cpus) == (1, 3, want)
        # the firmware's -1 / no such device: nothing changes
        base = _in_thread(lambda: _thread_cpus(lib))
        assert _in_thread(lambda: bind("0000:05:00.0")) == (-1, 0, base)
        assert _in_thread(lambda: bind("0000:99:00.0")) == (-1, 0, base)
        # a node whose CPUs are all outside this process's cpuset: left alone
        assert _in_thread(lambda: bind("0000:06:00.0")) == (2, 0, base)
        # a malformed cpulist: left alone
        assert _in_thread(lambda: bind("0000:07:00.0")) == (3, 0, base)
    finally:
        del os.environ["OURO_SYSFS_ROOT"]
    # the caller's own thread was never touched
    assert sorted(os.sched_getaffinity(0)) == allowed


def test_cpulist_ranges(lib, tmp_path):
    allowed = sorted(os.sched_getaffinity(0))
    root = _sysfs(tmp_path, {"0000:0a:00.0": 0},
                  {0: ",".join(f"{c}-{c}" for c in allowed) + ", "})
    os.environ["OURO_SYSFS_ROOT"] = root
    try:
        n = ctypes.c_int()
        got = _in_thread(lambda: (lib.ouro_debug_numa_bind_pci(b"0000:0a:00.0", ctypes.byref(n)),
                                  _thread_cpus(lib)))
    finally:
        del os.environ["OURO_SYSFS_ROOT"]
    assert got == (0, allowed) and n.value == len(allowed)


@pytest.mark.gpu
def test_multi_device_workers_bound_to_their_node(gpu_lib, kats):
    """ouro_tpraos_verify_batch_multi's workers run on their GPU's node."""
    import hdr_cases as HC
    from ouroboros_network_amd import tpraos as T

    batch = HC.golden_variants(kats, stride=40)
    T.verify_headers_multi(batch, devices=[0, 0])
    dev = (ctypes.c_int * 16)()
    node = (ctypes.c_int * 16)()
    cpus = (ctypes.c_int * 16)()
    k = gpu_lib.ouro_debug_multi_workers(dev, node, cpus, 16)
    assert k >= 2
    for i in range(min(k, 16)):
        want = gpu_lib.ouro_device_numa_node(dev[i])
        assert node[i] == want
        if want >= 0:
            assert cpus[i] > 0, "worker not bound although the device has a NUMA node"
    assert np.all(np.array(node[:min(k, 16)]) >= -1)
