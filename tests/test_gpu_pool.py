"""Per-thread device contexts are pooled, not leaked (kernels.hip ThreadCtx /
Lease; include/ouro_verify.h "thread-safe and reentrant").  GHC runs `safe`
FFI calls on a worker pool that grows and churns, one thread per peer
(ouroboros-consensus/src/Ouroboros/Consensus/Network/NodeToNode.hs:173-176):
64 short-lived threads, one after another, each verify a 65,536-header batch
through the host-buffer ABI.  They must reuse the context the previous thread
returned at its exit -- no new context, device memory flat within one
context's size -- and every result equals the oracle's."""
import os
import sys
import threading

import numpy as np
import pytest

import oracle_ffi as O

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_short_lived_threads_reuse_pooled_contexts(gpu_lib):
    import ctypes

    import torch

    sys.path.insert(0, ROOT)
    import bench
    from ouroboros_network_amd import _native
    from ouroboros_network_amd.tpraos import verify_headers

    n = 1 << 16
    dev = torch.device("cuda:0")
    t, _ = bench.synth_headers(n, 256, dev)
    rng = torch.Generator().manual_seed(64)
    rows = torch.randint(0, n, (n // 8,), generator=rng)
    t["eta_proof"].view(n, 80)[rows.to(dev), 70] ^= 1  # some invalid eta proofs
    hb = bench.DeviceHeaders(t, n, dev).host_sample(n)
    del t
    torch.cuda.synchronize()
    sample = np.sort(np.random.default_rng(2).choice(n, 1024, replace=False))
    wv, wbe, wbl = O.tpraos_verify_batch(hb.rows(sample), threads=min(16, os.cpu_count() or 1))

    def counts():
        c, i = ctypes.c_size_t(), ctypes.c_size_t()
        _native.check(gpu_lib.ouro_debug_contexts(0, ctypes.byref(c), ctypes.byref(i)), "ctx")
        return c.value, i.value

    results, errors = [], []

    def one():
        try:
            _native.load().ouro_set_device(0)
            results.append(verify_headers(hb))
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    # one thread first: its context, grown to this batch, goes back to the pool
    th = threading.Thread(target=one)
    th.start()
    th.join()
    torch.cuda.synchronize()
    free0, _ = torch.cuda.mem_get_info(dev)
    created0, idle0 = counts()
    assert idle0 >= 1
    ref = results.pop()
    for _ in range(64):
        th = threading.Thread(target=one)
        th.start()
        th.join()
        assert not errors, errors
        v, be, bl = results.pop()
        np.testing.assert_array_equal(v, ref[0])
        np.testing.assert_array_equal(be, ref[1])
        np.testing.assert_array_equal(bl, ref[2])
    created1, idle1 = counts()
    free1, _ = torch.cuda.mem_get_info(dev)
    assert created1 == created0, (created0, created1)   # every thread reused one
    assert idle1 == idle0
    assert free0 - free1 < 64 << 20, (free0, free1)      # no device memory leaked
    np.testing.assert_array_equal(ref[0][sample], wv)
    np.testing.assert_array_equal(ref[1][sample], wbe)
    np.testing.assert_array_equal(ref[2][sample], wbl)
