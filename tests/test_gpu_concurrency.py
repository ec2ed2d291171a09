"""Concurrent C callers of the ABI (tests/c/concurrency.c): 8 pthreads mixing
single-item calls (ouro_ed25519_verify, crypto_vrf_ietfdraft03_verify and
crypto_vrf_proof_to_hash through the opt-in shim, ouro_sum6kes_verify) with
batch calls, every result checked against the oracle -- the header's
"thread-safe and reentrant" promise, under the reference's one-thread-per-peer
calling pattern (ouroboros-consensus/src/Ouroboros/Consensus/Network/NodeToNode.hs:173-176)
-- then 64 short-lived threads one after another, which must reuse one pooled
context (kernels.hip ThreadCtx / Lease) instead of leaking one each."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "c", "build", "concurrency")

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("single_route", ["host", "gpu"])
def test_eight_threads_mixed_calls(gpu_lib, single_route):
    """Single items on the host path (the default since round 4) and on the
    GPU (OURO_SINGLE_ITEM=gpu), concurrently with batch calls."""
    if not os.path.exists(EXE):
        subprocess.run(["make", "-C", os.path.join(ROOT, "tests", "c")], check=True)
    env = dict(os.environ, OURO_SINGLE_ITEM=single_route)
    r = subprocess.run([EXE, "8", "30", "64"], capture_output=True, text=True, timeout=100,
                       env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    ok, calls, created = r.stdout.split()
    assert (ok, calls) == ("ok", str(8 * 30))
    assert int(created) <= 1, r.stdout
